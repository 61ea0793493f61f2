set -o pipefail
mkdir -p gpurun_out/r4u
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "pipelined or iterate or golden or full" > gpurun_out/r4u/t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r4u/t.log
for rep in 1 2 3; do
  for gc in 1 0; do
    CLRSDP_GRAPH_COPY=$gc timeout -k 10 200 python3 bench.py --no-cpu --steps 300 > gpurun_out/r4u/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4u/b.log; exit 1; }
    tail -1 gpurun_out/r4u/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c3 graph_copy='$gc'", round(d["value"],1), "it/s", round(d["roofline"]["frac"],3))'
  done
done
