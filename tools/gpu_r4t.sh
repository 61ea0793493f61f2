set -o pipefail
mkdir -p gpurun_out/r4t
for rep in 1 2 3; do
  for lp in sync pipelined; do
    CLRSDP_NO_GRAPH=1 timeout -k 10 200 python3 bench.py --no-cpu --steps 300 --clusters 8 --loop $lp > gpurun_out/r4t/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4t/b.log; exit 1; }
    tail -1 gpurun_out/r4t/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c3/8 eager '$lp'", round(d["value"],1), "it/s")'
  done
done
