set -o pipefail
mkdir -p gpurun_out/sweep
for d in 10 12 14 16 20; do
  timeout -k 10 120 python tools/sphere_packing_run.py --words 4 --gap 1e-30 --d $d --maxit 400 --json gpurun_out/sweep/sp_qd_d$d.json > gpurun_out/sweep/sp_qd_d$d.log 2>&1 || echo "d=$d failed rc=$?"
done
for J in 8 16 32; do
  timeout -k 10 120 python bench.py --clusters $J --no-cpu > gpurun_out/sweep/bench_J$J.log 2>&1 || exit 1
done
grep -h "bound\|status" gpurun_out/sweep/*.log
