#!/bin/bash
# GPU box: the tuning-only kernels' parity tests against a tuning build of the library
# (UFC_LIB=uflow_amd/libuflowcrc_tuning.so, built here beforehand with
#  python -c "from uflow_amd._build import build_native; build_native(tuning=True, out='uflow_amd/libuflowcrc_tuning.so')").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-tuning}
mkdir -p $OUT
cd $R
UFC_LIB=uflow_amd/libuflowcrc_tuning.so timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py -x -v \
    --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
exit $rc
