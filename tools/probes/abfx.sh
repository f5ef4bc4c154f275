#!/bin/bash
# A/B of two libraries on the fixed validate kernel (config 2), alternating.  Usage: abfx.sh libA libB [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in $(seq ${3:-4}); do
  for L in $1 $2; do
    echo -n "$L: "
    UFC_LIB=$R/$L timeout -k 10 120 python tools/probes/fxrun.py 50 2>&1 | tail -1 || exit 1
  done
done
