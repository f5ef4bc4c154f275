#!/bin/bash
# Ablation runs of the fixed-length kernel (tuning build): full / loads-only / compute-only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-ablate}
mkdir -p $OUT
export UFC_LIB=$R/uflow_amd/libuflowcrc_tuning.so UFC_FIXED_JC=${CFG:-6}
for rep in 1 2; do
for ab in ${ABS:-0 8 16}; do
  UFC_ABLATE=$ab timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $OUT/ab_$ab.json 2>$OUT/ab_$ab.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "ablate $ab rc=$rc"; tail -3 $OUT/ab_$ab.err; exit 1; fi
  python3 -c "import json;j=json.load(open('$OUT/ab_$ab.json'));print('ablate $ab kernel', j['roofline']['kernel_avg_ms'], 'ms', j['roofline']['achieved'], 'GB/s')"
done
done
