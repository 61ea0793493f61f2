#!/bin/bash
# Profile the C3 bench on the GPU box (run through gpurun from the repo root):
#   1. rocprofv3 --kernel-trace --stats      -> per-kernel durations (rocprof agrees with bench.py's events)
#   2. rocprofv3 --pmc FETCH_SIZE            -> HBM read bytes per dispatch   (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE            -> HBM write bytes per dispatch  (own pass)
#   4. rocprofv3 --pmc SQ_* GRBM_GUI_ACTIVE  -> per-kernel MFMA / stall / LDS counters (own pass)
# Outputs go to gpurun_out/prof_$TAG; copy the summaries into profiles/ afterwards.
set -euo pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu > $OUT/bench_write.log 2>&1
python3 tools/pmc_traffic.py $OUT/fetch/run_counter_collection.csv \
  $OUT/write/run_counter_collection.csv $OUT/schur_pmc.json > /dev/null
# 4. one SQ + GRBM pass for the kernels that set the body (GEMMs and strip chains, Cholesky
#    inverse, eigen-solver, Schur): fp64 MFMA instructions, MFMA busy cycles, the wave-cycle split
#    and LDS bank conflicts (8 SQ slots, 1 GRBM slot: within one pass's limits); only counters
#    this rocprofv3 lists are requested
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
PMC=""
for c in SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
         SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE; do
  if grep -qw "$c" $OUT/counters_list.txt; then PMC="$PMC $c"; fi
done
echo "SQ pass counters:$PMC"
timeout -s KILL 180 rocprofv3 --pmc $PMC --output-format csv -d $OUT/sq -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS:-} > $OUT/bench_sq.log 2>&1
python3 tools/pmc_kernels.py $OUT/sq/run_counter_collection.csv $OUT/kt/run_kernel_stats.csv \
  $OUT/kernels_pmc.json > /dev/null
python3 tools/prof_summary.py $OUT/kt/run_kernel_stats.csv > $OUT/kernel_summary.txt
python3 tools/copy_census.py $OUT/kt/run_kernel_trace.csv > $OUT/copy_census.txt
python3 tools/iter_trace.py $OUT/kt/run_kernel_trace.csv > $OUT/body_trace.txt
echo done
