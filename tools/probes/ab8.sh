#!/bin/bash
# A/B of two tuning libraries on the 8-lane varlen kernel (config 3 batch), alternating.
# Usage: tools/probes/ab8.sh <libA> <libB> <waves> <depth> [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in $(seq ${5:-3}); do
  for L in $1 $2; do
    echo -n "$L: "
    UFC_LIB=$R/$L UFC_V8_WAVES=$3 UFC_V8_DEPTH=$4 timeout -k 10 120 python tools/probes/v2run.py 6 6 2>&1 | tail -2 | tr '\n' ' ' || exit 1
    echo
  done
done
