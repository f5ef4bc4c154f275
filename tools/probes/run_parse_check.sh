#!/bin/bash
# Parse kernels' trace (rocprofv3 --kernel-trace --stats) and the bench's per-step event cost
# (--event-every 1 vs 10), each step under its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/${1:-parse2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o run -- \
  python3 $R/tools/bench_configs.py --only parse --reps 10 > $O/ktrace.log 2>&1 || { tail -5 $O/ktrace.log; exit 1; }
find $O/ktrace -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -12
for ev in 1 10 1 10; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --event-every $ev > $O/bench_ev$ev.json 2>/dev/null || exit 1
  python3 -c "import json;j=json.load(open('$O/bench_ev$ev.json'));print('ev $ev', j['ms_per_step'], j['value'], j['roofline']['kernel_avg_ms'], j['roofline']['frac'])"
done
