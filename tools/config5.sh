#!/bin/bash
# BASELINE.json config 5 (and 1) on the GPU box: the loopback harness with the CPU gate and with the
# GPU gate in the receive path, one JSON line each, appended to gpurun_out/config5.jsonl.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
B=$R/tools/loopback/ufc_loopback
timeout -k 10 60 $B --echo --port 18801 > gpurun_out/echo.log 2>&1 && tail -1 gpurun_out/echo.log >> gpurun_out/config5.jsonl || exit 1
for gate in cpu gpu; do
  for batch in ${BATCHES:-4096}; do
    timeout -k 10 120 $B --gate $gate --batch $batch --frames ${FRAMES:-3000000} --port 18802 --corrupt-every 1000 \
      >> gpurun_out/config5.jsonl 2> gpurun_out/config5_$gate.err || { echo "$gate failed"; tail -3 gpurun_out/config5_$gate.err; exit 1; }
  done
done
# Send side too: every flush built with zero trailers and batch-sealed (CPU per frame, or GPU).
for seal in cpu gpu; do
  timeout -k 10 120 $B --gate gpu --send-seal $seal --frames ${FRAMES:-3000000} --port 18803 --corrupt-every 1000 \
    >> gpurun_out/config5.jsonl 2> gpurun_out/config5_seal_$seal.err || { echo "seal $seal failed"; tail -3 gpurun_out/config5_seal_$seal.err; exit 1; }
done
cat gpurun_out/config5.jsonl
