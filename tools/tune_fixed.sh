#!/bin/bash
# Sweep the fixed-length kernel configurations (UFC_FIXED_CFG="NS,JC"): parity subset + bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-tune}
mkdir -p $OUT
shift
for cfg in "$@"; do
  UFC_FIXED_JC=$cfg timeout -k 10 200 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "fixed or seal_fixed" > $OUT/parity_$cfg.log 2>&1
  rc=$?
  echo "cfg $cfg parity rc=$rc $(tail -1 $OUT/parity_$cfg.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
  UFC_FIXED_JC=$cfg timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $OUT/bench_$cfg.json 2>$OUT/bench_$cfg.err || { echo bench fail; tail -3 $OUT/bench_$cfg.err; exit 1; }
  python3 -c "import json;j=json.load(open('$OUT/bench_$cfg.json'));print('cfg $cfg', j['value'], 'GiB/s kernel', j['roofline']['kernel_avg_ms'], 'ms frac', j['roofline']['frac'])"
done
