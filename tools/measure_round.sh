#!/bin/bash
# Round-end measurement set on the GPU box (run through gpurun from the repo root):
#   1. tools/profile_round.sh: kernel trace + the FETCH_SIZE / WRITE_SIZE passes of the Schur
#      launches; its counter summary is copied to profiles/${TAG}_schur_pmc.json first, so the
#      bench lines below carry `traffic` from a counter pass of this very build;
#   2. bench lines C3 (default, with the CPU baseline), C2, C4 (C2 shape, double-double),
#      C5 (sphere-packing shape, quad-double);
#   3. the C3 body at 8/16/32 clusters (the per-rank share of the strong-scaling shards), and a
#      kernel trace of the 8-cluster body.
# Outputs: gpurun_out/meas_$TAG/ and gpurun_out/prof_$TAG/.
set -euo pipefail
TAG=${1:-r03}
OUT=gpurun_out/meas_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
bash tools/profile_round.sh $TAG > $OUT/profile.log 2>&1
cp gpurun_out/prof_$TAG/schur_pmc.json profiles/${TAG}_schur_pmc.json
cp gpurun_out/prof_$TAG/schur_pmc.json $OUT/schur_pmc.json
cp gpurun_out/prof_$TAG/kernels_pmc.json profiles/${TAG}_kernels_pmc.json
cp gpurun_out/prof_$TAG/kernel_summary.txt profiles/${TAG}_c3_kernel_summary.txt
timeout -k 10 200 python3 bench.py > $OUT/bench_c3_fp64.log 2>&1
timeout -k 10 200 python3 bench.py --config c2 > $OUT/bench_c2_fp64.log 2>&1
timeout -k 10 200 python3 bench.py --config c2 --precision 2 > $OUT/bench_c4_dd.log 2>&1
timeout -k 10 200 python3 bench.py --config c5 --precision 4 > $OUT/bench_c5_qd.log 2>&1
# kernel summaries of the multi-word lines (C4 double-double, C5 quad-double)
for cfg in "c4_dd:--config c2 --precision 2" "c5_qd:--config c5 --precision 4"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$name -o run -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu $args > $OUT/kt_$name.log 2>&1
  python3 tools/prof_summary.py $OUT/kt_$name/run_kernel_stats.csv > $OUT/${name}_kernel_summary.txt
done
for c in 8 16 32; do
  timeout -k 10 120 python3 bench.py --clusters $c --no-cpu --steps 300 > $OUT/clusters_$c.log 2>&1
done
# kernel summary and per-body listing of the 8-cluster shard (the N = 8 rank's body)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_clusters8 -o run -- \
  python3 bench.py --clusters 8 --steps 20 --warmup 3 --no-cpu > $OUT/kt_clusters8.log 2>&1
python3 tools/prof_summary.py $OUT/kt_clusters8/run_kernel_stats.csv > $OUT/clusters8_kernel_summary.txt
python3 tools/iter_trace.py $OUT/kt_clusters8/run_kernel_trace.csv > $OUT/clusters8_body_trace.txt
echo done
