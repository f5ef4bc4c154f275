#!/bin/bash
# A/B of whole-library variants (build/lib_<name>.so): fixed-kernel parity subset, bench kernel
# time (two passes, interleaved) and one FETCH_SIZE pass per variant.  Usage: lib_ab.sh TAG name...
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-libab}
shift
mkdir -p $OUT
export TMPDIR=/tmp
for v in "$@"; do
  UFC_LIB=$R/build/lib_$v.so timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fixed" \
    > $OUT/parity_$v.log 2>&1
  rc=$?
  echo "$v parity rc=$rc $(tail -1 $OUT/parity_$v.log)"
  if [ $rc -ne 0 ]; then exit 1; fi
done
for rep in 1 2; do
  for v in "$@"; do
    UFC_LIB=$R/build/lib_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 > $OUT/$v.json 2>$OUT/$v.err \
      || { echo "$v bench failed"; tail -3 $OUT/$v.err; exit 1; }
    python3 -c "import json;j=json.load(open('$OUT/$v.json'));print('$v', j['roofline']['kernel_avg_ms'], 'ms', j['roofline']['achieved'], 'GB/s')"
  done
done
for v in "$@"; do
  UFC_LIB=$R/build/lib_$v.so timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_$v -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_$v.log 2>&1 || { echo "$v pmc failed"; exit 1; }
  echo "$v $(python3 tools/pmc_summary.py $OUT/pmc_$v "fixed_kernel<6, false" | tr -d '\n')"
done
