#!/bin/bash
# SQ counters of the varlen kernel chosen by option value $2 (library $3, default the product).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-vlpmc}
MODE=${2:-0}
LIB=${3:-}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
[ -n "$LIB" ] && export UFC_AB=1 UFC_LIB=$R/$LIB
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc1 -o run -- python3 tools/probes/v2run.py 2 $MODE > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM --output-format csv -d $OUT/pmc2 -o run -- python3 tools/probes/v2run.py 2 $MODE > $OUT/pmc2.log 2>&1 || exit 1
echo done
