#!/bin/bash
# 8-lane varlen kernel: waves/depth variants (tuning library) and SQ counters of the product one.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export TMPDIR=/tmp
T=$R/tools/probes/lib_tune.so
TAG=${1:-v8pmc}
for cfg in ${CFGS:-8,3 8,2 12,2}; do
  wv=${cfg%,*}; dp=${cfg#*,}
  echo -n "waves=$wv depth=$dp: "
  UFC_LIB=$T UFC_V8_WAVES=$wv UFC_V8_DEPTH=$dp timeout -k 10 120 python tools/probes/v2run.py 6 6 2>&1 | tail -2 | tr '\n' ' ' || exit 1
  echo
done
echo -n "sorted (4-lane): "; timeout -k 10 120 python tools/probes/v2run.py 6 2 2>&1 | tail -2 | tr '\n' ' '; echo
[ -n "$NOPMC" ] || bash tools/probes/vl_pmc.sh $TAG 6 > /dev/null 2>&1 || echo pmc failed
