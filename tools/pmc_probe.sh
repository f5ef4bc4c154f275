#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 pass, no tracing domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
shift
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1
  rc=$?
  echo "group $i [$grp] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after rc=$rc"; exit 1; fi
done
