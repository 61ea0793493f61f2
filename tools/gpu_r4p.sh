set -o pipefail
mkdir -p gpurun_out/r4p
for rep in 1 2; do
  for cfg in "c5:--config c5 --precision 4" "c4:--config c2 --precision 2"; do
    for lp in sync pipelined; do
      name=${cfg%%:*}; args=${cfg#*:}
      timeout -k 10 200 python3 bench.py --no-cpu --steps 150 --loop $lp $args > gpurun_out/r4p/b.log 2>&1 || { echo "bench failed: $cfg $lp"; tail -5 gpurun_out/r4p/b.log; exit 1; }
      tail -1 gpurun_out/r4p/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$name' '$lp'", round(d["value"],1), "it/s", round(d["ms_per_step"],4))'
    done
  done
done
