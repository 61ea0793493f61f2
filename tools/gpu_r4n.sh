set -o pipefail
mkdir -p gpurun_out/r4n
timeout -k 10 120 microbin/eig_mx_bench 64 32 > gpurun_out/r4n/eigmx.log 2>&1; echo "eigmx rc=$?"; grep -v "rejected\|stamps" gpurun_out/r4n/eigmx.log
for nb in 45 60; do
  CLRSDP_EIGMX_STATS=1 timeout -k 10 100 python3 tools/probe_eigmx.py c2 $nb 2 > gpurun_out/r4n/p.log 2>&1 || exit 1
  echo "bodies $nb: $(grep fallbacks gpurun_out/r4n/p.log)"
done
for a in "--config c2 --precision 2" "--config c5 --precision 4"; do
  timeout -k 10 200 python3 bench.py --no-cpu --steps 100 $a > gpurun_out/r4n/b.log 2>&1 || { echo "bench failed: $a"; tail -5 gpurun_out/r4n/b.log; exit 1; }
  tail -1 gpurun_out/r4n/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["workload"][:40], d["dtype"], round(d["value"],1), "it/s")'
done
for rep in 1 2; do
  for v in "sync:0" "pipelined:0" "pipelined:1"; do
    lp=${v%%:*}; og=${v#*:}
    CLRSDP_PIPE_ONE_GRAPH=$og timeout -k 10 200 python3 bench.py --no-cpu --steps 200 --loop $lp > gpurun_out/r4n/b.log 2>&1 || { echo "bench failed: $v"; tail -5 gpurun_out/r4n/b.log; exit 1; }
    tail -1 gpurun_out/r4n/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("'$v'", round(d["value"],1), "it/s", round(d["ms_per_step"],4))'
  done
done
