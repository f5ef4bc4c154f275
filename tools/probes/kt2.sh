#!/bin/bash
# Kernel-trace stats of the 8-lane varlen path with two tuning libraries (per-kernel averages).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp
export TMPDIR=/tmp
i=0
for L in $1 $2; do
  i=$((i+1))
  UFC_LIB=$R/$L UFC_V8_WAVES=$3 UFC_V8_DEPTH=$4 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/gpurun_out/kt2_$i -o run -- python3 $R/tools/probes/v2run.py 6 6 > /dev/null 2>&1 || exit 1
  echo "== $L"
  grep -E "varlen8|sort_runs" $R/gpurun_out/kt2_$i/run_kernel_stats.csv | cut -d, -f1-4
done
