# A/B of the product library against another build of it (uflow_amd/libuflowcrc_ab.so, e.g. the
# previous commit's sources built with build_native(out=...)) on one bench_configs workload,
# alternating separate processes.  Usage: tools/probes/lib_ab.sh <workload> [rounds].  Tuning probe.
set -e
W=${1:-parse}
N=${2:-3}
mkdir -p gpurun_out/lib_ab
for r in $(seq 1 $N); do for v in ab prod; do
  if [ $v = ab ]; then L=$PWD/uflow_amd/libuflowcrc_ab.so; else L=$PWD/uflow_amd/libuflowcrc.so; fi
  UFC_LIB=$L timeout -k 10 200 python -u tools/bench_configs.py --only $W > gpurun_out/lib_ab/${v}_r${r}.json 2>gpurun_out/lib_ab/${v}_r${r}.err
  echo "$v r=$r $(python -c 'import sys,json; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d.get("ms"), d.get("items"), d.get("items_digest"))' gpurun_out/lib_ab/${v}_r${r}.json)"
done; done
