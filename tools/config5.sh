#!/bin/bash
# Config 5 on the GPU box: the inline receive loops with the CPU and the GPU gate at 1, 2, 4 and 8
# receive threads (each with its own sender), 2M frames each; one JSON line per run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-config5}
mkdir -p $OUT
B=$R/tools/loopback/ufc_loopback
port=31000
for th in ${THREADS:-1 2 4 8}; do
  for g in cpu gpu; do
    port=$((port + 20))
    timeout -k 10 120 $B --gate $g --rx-threads $th --tx-per-rx ${TXR:-2} --frames ${FRAMES:-2000000} --corrupt-every 997 --port $port \
      >> $OUT/config5.jsonl 2>> $OUT/config5.err || { echo "run $g x$th failed"; tail -5 $OUT/config5.err; exit 1; }
  done
done
cat $OUT/config5.jsonl
