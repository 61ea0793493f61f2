set -o pipefail
timeout -k 10 200 python3 tools/probe_c8.py 8 80 > gpurun_out/probe_a.log 2>&1; echo "probe rc=$?"; tail -6 gpurun_out/probe_a.log
CLRSDP_SLAB_QSOLVE=0 timeout -k 10 200 python3 tools/probe_c8.py 8 80 > gpurun_out/probe_b.log 2>&1; tail -4 gpurun_out/probe_b.log
timeout -k 10 120 microbin/eig_split_bench 2>&1 | head -2
bash tools/gpu_tests.sh r4f || exit 1
mkdir -p gpurun_out/r4f
for a in "--config c2 --precision 2" "--config c5 --precision 4" ""; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 100 $a > gpurun_out/r4f/b.log 2>&1 || { echo "bench failed: $a"; tail -5 gpurun_out/r4f/b.log; exit 1; }
  tail -1 gpurun_out/r4f/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:40], d["dtype"], round(d["value"],1), "it/s")'
done
