#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc pass per group, each under its own time limit) over one
# workload: bench (config 2, bench.py) or a tools/bench_configs.py workload (varlen, seal, ...).
# usage: tools/pmc_sq.sh <tag> <workload> ["<group 1>" "<group 2>" ...]
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; W=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
if [ $# -eq 0 ]; then
  set -- "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU" \
         "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA"
fi
if [ "$W" = bench ]; then
  run=(python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --settle-ms 50 --no-ceiling)
else
  run=(python3 $R/tools/bench_configs.py --only $W --reps 10 --no-check)
fi
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/${W}_p$i -o run -- "${run[@]}" > $OUT/${W}_p$i.log 2>&1
  rc=$?
  echo "$W group $i [$grp] rc=$rc"
  if [ $rc -gt 1 ]; then exit 1; fi
done
