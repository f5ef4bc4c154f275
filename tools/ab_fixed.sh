#!/bin/bash
# A/B of the fixed-length kernels on the bench workload: lean (default) vs generic.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-ab}
mkdir -p $OUT
for rep in 1 2; do
for k in lean generic; do
  UFC_FIXED_KERNEL=$k timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $OUT/$k.json 2>$OUT/$k.err
  rc=$?
  if [ $rc -ne 0 ]; then echo "$k rc=$rc"; tail -3 $OUT/$k.err; exit 1; fi
  python3 -c "import json;j=json.load(open('$OUT/$k.json'));print('$k kernel', j['roofline']['kernel_avg_ms'], 'ms', j['roofline']['achieved'], 'GB/s', 'value', j['value'])"
done
done
