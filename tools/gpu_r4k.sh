set -o pipefail
mkdir -p gpurun_out/r4k
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_mw.py -k "qd or dd or gemm or mw" > gpurun_out/r4k/t.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r4k/t.log
for a in "--config c5 --precision 4" "--config c2 --precision 2" "--config c5 --precision 4" "--config c2 --precision 2"; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 100 $a > gpurun_out/r4k/b.log 2>&1 || { echo "bench failed: $a"; tail -5 gpurun_out/r4k/b.log; exit 1; }
  tail -1 gpurun_out/r4k/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:40], d["dtype"], round(d["value"],1), "it/s")'
done
