#!/bin/bash
# GPU-box check: the whole -m gpu suite, then the bench line.  Every GPU step has its own time
# limit and the chain stops at the first failure.  Usage: tools/gpu_check.sh <tag> [pytest -k expr]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-check}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
