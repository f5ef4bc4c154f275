#!/bin/bash
# A/B of bench.py's untimed settle phase (fresh processes, alternating): does a longer settle
# reach the sustained launch time more reliably?  Usage: tools/probes/settle_ab.sh
set -o pipefail
mkdir -p gpurun_out/settle
for r in 1 2 3; do
  for s in ${ORDER:-50 300}; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --settle-ms $s > gpurun_out/settle/b_${s}_$r.json 2>/dev/null || exit 1
    python3 -c "import json;j=json.load(open('gpurun_out/settle/b_${s}_$r.json'));r=j['roofline'];print('settle=$s', r['kernel_avg_ms'], r['kernel_min_ms'], r['frac'])"
  done
done
