set -o pipefail
mkdir -p gpurun_out/r4q
for rep in 1 2 3; do
  for ng in 0 1; do
    for cfg in "c5:--config c5 --precision 4" "c2:--config c2"; do
      name=${cfg%%:*}; args=${cfg#*:}
      CLRSDP_NO_GRAPH=$ng timeout -k 10 200 python3 bench.py --no-cpu --steps 200 $args > gpurun_out/r4q/b.log 2>&1 || { echo "bench failed: $ng $cfg"; tail -5 gpurun_out/r4q/b.log; exit 1; }
      tail -1 gpurun_out/r4q/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$name' no_graph='$ng'", round(d["value"],1), "it/s")'
    done
  done
done
