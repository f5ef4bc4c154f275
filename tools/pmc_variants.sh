#!/bin/bash
# One FETCH_SIZE (and optionally other counter) pass per kernel variant: "name:K=V,K=V".
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=$R/gpurun_out/${1:-pmcv}
shift
mkdir -p $OUT
export TMPDIR=/tmp
CNT=${CNT:-FETCH_SIZE}
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  (
    for kv in $(echo $envs | tr ',' ' '); do export "$kv"; done
    timeout -k 10 240 rocprofv3 --pmc $CNT --output-format csv -d $OUT/$name -o run -- \
        python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$name.log 2>&1
  )
  rc=$?
  echo "$name rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
  python3 tools/pmc_summary.py $OUT/$name frame_crc | tr -d '\n' ; echo
done
