#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/parse
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "parse" > $O/pt1.log 2>&1
rc=$?; tail -15 $O/pt1.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pt.log 2>&1
rc=$?; tail -3 $O/pt.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_configs.py --only parse --reps 20 > $O/parse.txt 2>&1 || { tail -5 $O/parse.txt; exit 1; }
tail -1 $O/parse.txt
for ev in 1 10 1 10; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 100 --event-every $ev > $O/bench_ev$ev.json 2>/dev/null || exit 1
  python3 -c "import json;j=json.load(open('$O/bench_ev$ev.json'));print('ev $ev', j['ms_per_step'], j['value'], j['roofline']['kernel_avg_ms'], j['roofline']['frac'])"
done
