set -o pipefail
mkdir -p gpurun_out/r4n
for rep in 1 2 3; do
  for lp in sync pipelined; do
    timeout -k 10 200 python3 bench.py --no-cpu --steps 200 --loop $lp > gpurun_out/r4n/b.log 2>&1 || { echo "bench failed: $lp"; tail -5 gpurun_out/r4n/b.log; exit 1; }
    tail -1 gpurun_out/r4n/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$lp'", round(d["value"],1), "it/s", round(d["ms_per_step"],4))'
  done
done
