#!/bin/bash
# BASELINE.json configs 1 and 5 on the GPU box, one JSON line per run in gpurun_out/<tag>/config5.jsonl:
#   1. the echo plumbing (config 1);
#   2. the inline receive loops (receive + gate + parse + payload check in one thread, the server
#      loop of server/mod.rs:591-602) on 1, 2, 4 threads, each fed by TXR sender threads, with the
#      CPU gate and with the asynchronous GPU gate overlapped with the next receive: paced senders
#      swept up to each arm's highest offered rate with loss <= 0.5 % (tools/config5_sweep.py), then
#      unpaced saturation runs with their loss;
#   3. the receiver/worker pipeline of round 1 (one receive thread, one worker) with both gates;
#   4. the send side: every flush built with zero trailers and batch-sealed (CPU per frame, or GPU).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-config5}
mkdir -p $OUT
B=$R/tools/loopback/ufc_loopback
J=$OUT/config5.jsonl
run() {  # run <name> <args...>
  local name=$1
  shift
  timeout -k 10 120 $B "$@" >> $J 2>> $OUT/$name.err || { echo "$name failed"; tail -5 $OUT/$name.err; exit 1; }
}
port=31000
timeout -k 10 60 $B --echo --port $port > $OUT/echo.log 2>&1 && tail -1 $OUT/echo.log >> $J || { echo "echo failed"; exit 1; }
# like-for-like (round 3): paced senders, each arm's highest offered rate with loss <= 0.5 %
timeout -k 10 400 python3 $R/tools/config5_sweep.py --threads ${THREADS:-1,2,4} --tx-per-rx ${TXR:-2} >> $J \
    2> $OUT/sweep.err || { echo "sweep failed"; tail -5 $OUT/sweep.err; exit 1; }
# unpaced saturation (loss reported in every line)
for th in ${THREADS_UNPACED:-1 2}; do
  for g in cpu gpu; do
    port=$((port + 20))
    run inline_${g}_$th --gate $g --rx-threads $th --tx-per-rx ${TXR:-2} --batch ${BATCH:-4096} --frames ${FRAMES:-2000000} \
      --corrupt-every 997 --port $port
  done
done
for g in cpu gpu; do
  port=$((port + 20))
  run pipeline_$g --gate $g --frames ${FRAMES:-2000000} --corrupt-every 1000 --port $port
done
for seal in cpu gpu; do
  port=$((port + 20))
  run seal_$seal --gate gpu --send-seal $seal --frames ${FRAMES:-2000000} --corrupt-every 1000 --port $port
done
cat $J
