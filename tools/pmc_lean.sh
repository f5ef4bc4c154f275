#!/bin/bash
# SQ/TA counter passes over the lean fixed kernel: product path (abl 0) and the loads-only
# ablation (abl 1) of the tuning build.  One counter group per rocprofv3 pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmclean}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp UFC_LIB=${UFC_LIB:-$R/uflow_amd/libuflowcrc_tuning.so}
shift
timeout -k 10 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
for ab in ${ABS:-0 1}; do
i=0
for grp in "$@"; do
  i=$((i+1))
  UFC_LEAN_ABL=$ab timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/a${ab}_p$i -o run -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/a${ab}_p$i.log 2>&1
  rc=$?
  echo "abl $ab group $i [$grp] rc=$rc"
  if [ $rc -gt 1 ]; then exit 1; fi
  python3 tools/pmc_summary.py $OUT/a${ab}_p$i "fixed_kernel<6, false" | python3 -c "import json,sys;d=json.load(sys.stdin);print({k:round(v['mean']) for k,v in d.items()})"
done
done
