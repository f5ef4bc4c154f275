#!/bin/bash
# GPU box: one clean rocprofv3 record per workload -- every workload in its own processes, so no
# kernel name mixes two workloads ("Make every roofline reproducible from profiles/"):
#   <w>_ktrace  rocprofv3 --kernel-trace --stats      (durations of every dispatch)
#   <w>_fetch   rocprofv3 --pmc FETCH_SIZE            (own pass: FETCH uses 3 TCC counters)
#   <w>_write   rocprofv3 --pmc WRITE_SIZE            (own pass)
# workloads: bench (config 2, bench.py), varlen (config 3), shard (config 4's per-GPU share), seal,
# seal_varlen, parse, parse_mtu (tools/bench_configs.py --only <w>).  Each step has its own time limit; the
# chain stops at the first failure.  Usage: tools/profile_workloads.sh <tag> [workloads]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
WL=${2:-bench varlen shard seal seal_varlen parse parse_mtu}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.log 2>&1 || { echo "$name failed"; tail -20 $OUT/$name.log; exit 1; }
  echo "$name ok"
}
for w in $WL; do
  if [ $w = bench ]; then
    run=(python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline)
    pmc=(python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 50 --no-ceiling)
  else
    run=(python3 $R/tools/bench_configs.py --only $w --reps 20)
    pmc=(python3 $R/tools/bench_configs.py --only $w --reps 10 --no-check)
  fi
  step ${w}_ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${w}_ktrace -o run -- "${run[@]}"
  step ${w}_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/${w}_fetch -o run -- "${pmc[@]}"
  step ${w}_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/${w}_write -o run -- "${pmc[@]}"
done
echo done
