#!/bin/bash
# GPU box: the multi-rank rehearsal on one device first (torch.distributed.run under its own time
# limit, so a stalled RCCL socket transport ends the step), then the shard and bench tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-shard}
mkdir -p $OUT
cd $R
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port 29612 tests/gpu_shard_worker.py > $OUT/worker2.log 2>&1
rc=$?
tail -3 $OUT/worker2.log
[ $rc -eq 0 ] || { grep -v "^\s*$" $OUT/worker2.log | tail -40; exit $rc; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_bench.py -x -v --timeout 300 \
    --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
exit $rc
