set -o pipefail
mkdir -p gpurun_out/r4s
for rep in 1 2 3; do
  for ng in 0 1; do
    CLRSDP_NO_GRAPH=$ng timeout -k 10 200 python3 bench.py --no-cpu --steps 200 --config c2 --precision 2 > gpurun_out/r4s/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4s/b.log; exit 1; }
    tail -1 gpurun_out/r4s/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c4 no_graph='$ng'", round(d["value"],1), "it/s")'
  done
done
for rep in 1 2; do
  for ng in 0 1; do
    CLRSDP_NO_GRAPH=$ng timeout -k 10 200 python3 bench.py --no-cpu --steps 300 --clusters 8 > gpurun_out/r4s/b.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/r4s/b.log; exit 1; }
    tail -1 gpurun_out/r4s/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("c3/8 no_graph='$ng'", round(d["value"],1), "it/s")'
  done
done
