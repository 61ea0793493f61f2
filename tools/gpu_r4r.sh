set -o pipefail
bash tools/gpu_tests.sh r4r || exit 1
for cfg in "c5:--config c5 --precision 4" "c5:--config c5 --precision 4" "c3:"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 200 python3 bench.py --no-cpu --steps 200 $args > gpurun_out/r4r/b.log 2>&1 || { echo "bench failed: $cfg"; tail -5 gpurun_out/r4r/b.log; exit 1; }
  tail -1 gpurun_out/r4r/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$name'", round(d["value"],1), "it/s", d["graph_replay"], d["host_loop"])'
done
