#!/bin/bash
# Run GPU steps in order, each "<seconds> <command...>" line of a step file under its own timeout.
# Continues past an ordinary failure (exit 1 / 2: a failed assertion or self-check), stops at
# anything else (fault, abort, segfault, time limit) so that nothing more touches the GPU.
# usage: tools/gpu/run_steps.sh <outdir> <stepfile>
out=$1; steps=$2
mkdir -p "$out"
i=0; worst=0
while IFS= read -r line; do
  [[ -z "$line" || "$line" == \#* ]] && continue
  i=$((i+1)); secs=${line%% *}; cmd=${line#* }
  echo "[step $i] ($secs s) $cmd" | tee -a "$out/steps.txt"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/step$i.log" 2>&1
  rc=$?
  echo "[step $i] rc=$rc in $(( $(date +%s) - start )) s" | tee -a "$out/steps.txt"
  tail -3 "$out/step$i.log"
  if [[ $rc -ne 0 && $rc -ne 1 && $rc -ne 2 ]]; then echo "stopping: rc $rc"; exit $rc; fi
  [[ $rc -ne 0 ]] && worst=$rc
done < "$steps"
exit $worst
