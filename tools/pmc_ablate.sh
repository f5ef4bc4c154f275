#!/bin/bash
# PMC passes (one counter group per rocprofv3 pass) over the tuning build, per ablation mode.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmcab}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp UFC_LIB=$R/uflow_amd/libuflowcrc_tuning.so UFC_FIXED_JC=6
shift
for ab in ${ABS:-0 16}; do
i=0
for grp in "$@"; do
  i=$((i+1))
  UFC_ABLATE=$ab timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d $OUT/a${ab}_p$i -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/a${ab}_p$i.log 2>&1
  rc=$?
  echo "ablate $ab group $i [$grp] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
done
done
