set -o pipefail
mkdir -p gpurun_out/r4m
for nb in 2 5 10 15 20 30 45 60; do
  CLRSDP_EIGMX_STATS=1 timeout -k 10 100 python3 tools/probe_eigmx.py c2 $nb 2 > gpurun_out/r4m/p.log 2>&1 || exit 1
  echo "bodies $nb: $(grep fallbacks gpurun_out/r4m/p.log)"
done
CLRSDP_EIGMX_STATS=1 timeout -k 10 100 python3 tools/probe_eigmx.py c2 5 2 > gpurun_out/r4m/p5.log 2>&1; grep "^  block" gpurun_out/r4m/p5.log | head -32
