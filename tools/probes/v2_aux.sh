#!/bin/bash
# varlen kernel: nt (product) vs default-policy block loads (lib_v2_noloads.so is built with
# UFC_V2_AUX=0 here), times and FETCH_SIZE of each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-v2aux}
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/nt.log 2>&1 || exit 1
UFC_LIB=$R/tools/probes/lib_v2_noloads.so timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/aux0.log 2>&1 || exit 1
UFC_LIB=$R/tools/probes/lib_v2_loads.so timeout -k 10 120 python tools/probes/v2run.py 5 > $OUT/aux0_loads.log 2>&1 || exit 1
timeout -k 10 120 python tools/probes/v2run.py 5 4 > $OUT/claim16.log 2>&1 || exit 1
tail -n1 $OUT/*.log
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_nt -o run -- python3 tools/probes/v2run.py 2 > /dev/null 2>&1 || exit 1
UFC_LIB=$R/tools/probes/lib_v2_noloads.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_aux0 -o run -- python3 tools/probes/v2run.py 2 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch_claim16 -o run -- python3 tools/probes/v2run.py 2 4 > /dev/null 2>&1 || exit 1
echo done
