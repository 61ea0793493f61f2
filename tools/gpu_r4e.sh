set -o pipefail
bash tools/gpu_tests.sh r4e || exit 1
mkdir -p gpurun_out/r4e
for a in "--config c2 --precision 2" "--config c5 --precision 4" ""; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 100 $a > gpurun_out/r4e/b.log 2>&1 || { echo "bench failed: $a"; tail -5 gpurun_out/r4e/b.log; exit 1; }
  tail -1 gpurun_out/r4e/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:40], d["dtype"], round(d["value"],1), "it/s", "host_enqueue_ms", round(d["host_enqueue_ms"],3), "eager_body_ms", round(d["eager_body_ms"],3), d["exchange_ranks"], d["exchange_backend_native"])'
done
timeout -k 10 200 python3 bench.py --no-cpu --steps 200 --clusters 8 > gpurun_out/r4e/b8.log 2>&1 && tail -1 gpurun_out/r4e/b8.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("clusters 8:", round(d["value"],1), "it/s", round(d["ms_per_step"],3), "ms; host_enqueue_ms", round(d["host_enqueue_ms"],3), "eager_body_ms", round(d["eager_body_ms"],3))'
