#!/bin/bash
# varlen kernel experiments on the GPU box: timings of the product build and of the loads-only /
# compute-only builds, then two SQ counter passes of the product build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-v2x}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/prod.log 2>&1 || { tail $OUT/prod.log; exit 1; }
UFC_LIB=$R/tools/probes/lib_v2_loads.so timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/loads.log 2>&1 || { tail $OUT/loads.log; exit 1; }
UFC_LIB=$R/tools/probes/lib_v2_noloads.so timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/noloads.log 2>&1 || { tail $OUT/noloads.log; exit 1; }
timeout -k 10 120 python tools/probes/v2run.py 5 4 > $OUT/claim16.log 2>&1 || { tail $OUT/claim16.log; exit 1; }
tail -n2 $OUT/*.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 tools/probes/v2run.py 2 > $OUT/pmc1.log 2>&1 || { tail $OUT/pmc1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc2 -o run -- python3 tools/probes/v2run.py 2 > $OUT/pmc2.log 2>&1 || { tail $OUT/pmc2.log; exit 1; }
echo done
