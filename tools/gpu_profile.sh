#!/bin/bash
# GPU-box profiling sequence (rocprofv3, MI355X_MICROARCH.md "HBM" + "rocprofv3 PMC slots"):
#   1. kernel trace + stats of bench.py (the config-2 validate kernel of the bench line)
#   2. FETCH_SIZE and WRITE_SIZE of bench.py, each in its own --pmc pass
#   3. kernel trace + stats of tools/bench_configs.py (varlen, shard, seal, parse kernels)
#   4. FETCH_SIZE and WRITE_SIZE of tools/bench_configs.py, separate passes
# Every step has its own time limit; the chain stops at the first failure.
# Usage: tools/gpu_profile.sh <tag> [bench_configs --only list]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}
ONLY=${2:-varlen,shard,seal,parse}
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
step bench_ktrace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_ktrace -o run -- \
    python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline
step bench_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/bench_fetch -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline
step bench_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/bench_write -o run -- \
    python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline
step cfg_ktrace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/cfg_ktrace -o run -- \
    python3 $R/tools/bench_configs.py --only $ONLY --reps 10
step cfg_fetch 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cfg_fetch -o run -- \
    python3 $R/tools/bench_configs.py --only $ONLY --reps 3
step cfg_write 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cfg_write -o run -- \
    python3 $R/tools/bench_configs.py --only $ONLY --reps 3
step configs 600 python3 $R/tools/bench_configs.py --reps 20
cat $OUT/configs.log
timeout -k 10 300 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
echo done
