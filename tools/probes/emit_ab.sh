# Parse emit variants (tuning build): UFC_EMIT_U items per thread per round, UFC_EMIT_X4 16-byte header
# loads; the parse parity tests run against the tuning library in two variants first.  Tuning probe.
set -e
mkdir -p gpurun_out/emit
T=$PWD/uflow_amd/libuflowcrc_tuning.so
UFC_LIB=$T UFC_EMIT_U=4 UFC_EMIT_X4=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k parse -m gpu > gpurun_out/emit/pytest_u4x4.log 2>&1
tail -1 gpurun_out/emit/pytest_u4x4.log
UFC_LIB=$T UFC_EMIT_U=2 UFC_EMIT_X4=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k parse -m gpu > gpurun_out/emit/pytest_u2.log 2>&1
tail -1 gpurun_out/emit/pytest_u2.log
for r in 1 2; do for v in 1:0 2:0 4:0 1:1 4:1; do u=${v%:*}; x=${v#*:}
  UFC_LIB=$T UFC_EMIT_U=$u UFC_EMIT_X4=$x timeout -k 10 200 python -u tools/bench_configs.py --only parse > gpurun_out/emit/u${u}x${x}_r${r}.json 2>gpurun_out/emit/u${u}x${x}_r${r}.err
  echo "U=$u X4=$x r=$r $(python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d["ms"], d["items"], d["items_digest"])' gpurun_out/emit/u${u}x${x}_r${r}.json)"
done; done
