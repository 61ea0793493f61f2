#!/bin/bash
# Copy the judged outputs of `tools/gpu_job.sh TAG measure` (gpurun_out/meas_TAG, prof_TAG) into
# profiles/ under the round's names (run in the container after the gpurun call).
#   bash tools/collect_round.sh r06
set -euo pipefail
T=$1; M=gpurun_out/meas_$T; P=gpurun_out/prof_$T
for c in c3_fp64 c2_fp64 c4_dd c5_qd; do tail -1 $M/bench_$c.log > profiles/${T}_bench_$c.json; done
for c in 8 16 32; do tail -1 $M/clusters_$c.log > profiles/${T}_clusters_$c.json; done
cp $M/c4_dd_kernel_summary.txt $M/c5_qd_kernel_summary.txt $M/clusters8_kernel_summary.txt \
   $M/clusters8_body_trace.txt profiles/ 2>/dev/null || true
for f in c4_dd_kernel_summary c5_qd_kernel_summary clusters8_kernel_summary clusters8_body_trace; do
  mv profiles/$f.txt profiles/${T}_$f.txt
done
cp $P/schur_pmc.json profiles/${T}_schur_pmc.json
cp $P/kernels_pmc.json profiles/${T}_kernels_pmc.json
cp $P/kernel_summary.txt profiles/${T}_c3_kernel_summary.txt
cp $P/body_trace.txt profiles/${T}_c3_body_trace.txt
cp $P/copy_census.txt profiles/${T}_c3_copy_census.txt
cp $P/kt/run_kernel_stats.csv profiles/${T}_c3_kernel_stats.csv
ls profiles/${T}_*
