set -o pipefail
mkdir -p gpurun_out/r4h
timeout -k 10 120 microbin/eig_mx_bench 64 32 > gpurun_out/r4h/eigmx.log 2>&1; echo "eigmx rc=$?"; grep -v rejected gpurun_out/r4h/eigmx.log; grep rejected gpurun_out/r4h/eigmx.log | head -6
CLRSDP_EIG_MX=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_steplength.py tests/test_gpu_keywords.py tests/test_gpu_parity.py -k "eigmin or keyword or c4 or c5 or dd or qd" > gpurun_out/r4h/t_eig.log 2>&1; echo "tests rc=$?"; tail -5 gpurun_out/r4h/t_eig.log
for a in "--config c2 --precision 2" "--config c5 --precision 4"; do
  for mx in 1 0; do
    CLRSDP_EIG_MX=$mx timeout -k 10 200 python3 bench.py --no-cpu --steps 100 $a > gpurun_out/r4h/b.log 2>&1 || { echo "bench failed: $a"; tail -5 gpurun_out/r4h/b.log; exit 1; }
    tail -1 gpurun_out/r4h/b.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("mx='$mx'", d["config"]["workload"][:40], d["dtype"], round(d["value"],1), "it/s")'
  done
done
