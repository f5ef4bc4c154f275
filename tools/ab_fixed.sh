#!/bin/bash
# A/B of fixed-length kernel variants on the bench workload (kernel avg ms from bench.py).
# Variants: "name:ENV=VAL,ENV=VAL" ; the tuning library is used for UFC_LEAN_ABL variants.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-ab}
shift
mkdir -p $OUT
VARS=${@:-"lean3:UFC_LEAN_DEPTH=3 lean2:UFC_LEAN_DEPTH=2 generic:UFC_FIXED_KERNEL=generic"}
for rep in 1 2; do
for v in $VARS; do
  name=${v%%:*}; envs=${v#*:}
  env_args=$(echo $envs | tr ',' ' ')
  env $env_args timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $OUT/$name.json 2>$OUT/$name.err
  rc=$?
  if [ $rc -gt 1 ]; then echo "$name rc=$rc"; tail -3 $OUT/$name.err; exit 1; fi
  python3 -c "import json;j=json.load(open('$OUT/$name.json'));print('$name', j['roofline']['kernel_avg_ms'], 'ms', j['roofline']['achieved'], 'GB/s', 'value', j['value'], 'rc=$rc')"
done
done
