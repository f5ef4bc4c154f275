#!/bin/bash
# A/B of two libraries on the config-3 varlen batch, alternating, in one GPU session.
# Usage: tools/probes/ab.sh <libA> <libB> [mode] [rounds]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in $(seq ${4:-3}); do
  for L in $1 $2; do
    echo -n "$L: "
    UFC_LIB=$R/$L timeout -k 10 120 python tools/probes/v2run.py 6 ${3:-0} 2>&1 | tail -2 | tr '\n' ' ' || exit 1
    echo
  done
done
