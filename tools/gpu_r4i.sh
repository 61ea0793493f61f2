set -o pipefail
mkdir -p gpurun_out/r4i
for c in "c2 8 2" "c2 60 2"; do
  CLRSDP_EIG_MX=1 CLRSDP_EIGMX_STATS=1 timeout -k 10 200 python3 tools/probe_eigmx.py $c > gpurun_out/r4i/p.log 2>&1; echo "probe $c rc=$?"; grep -v "^  block" gpurun_out/r4i/p.log | tail -2; grep "^  block" gpurun_out/r4i/p.log | head -40
done
