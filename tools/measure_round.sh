#!/bin/bash
# Round-end measurement set on the GPU box (run through gpurun from the repo root):
#   bench lines C3 (default, with the CPU baseline), C2, C4 (C2 shape, double-double),
#   C5 (sphere-packing shape, quad-double), then tools/profile_round.sh (kernel trace + the
#   FETCH_SIZE / WRITE_SIZE passes of the Schur launches).  Outputs: gpurun_out/meas_$TAG/.
set -euo pipefail
TAG=${1:-r02}
OUT=gpurun_out/meas_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py > $OUT/bench_c3_fp64.log 2>&1
timeout -k 10 200 python3 bench.py --config c2 > $OUT/bench_c2_fp64.log 2>&1
timeout -k 10 200 python3 bench.py --config c2 --precision 2 > $OUT/bench_c4_dd.log 2>&1
timeout -k 10 200 python3 bench.py --config c5 --precision 4 > $OUT/bench_c5_qd.log 2>&1
bash tools/profile_round.sh $TAG > $OUT/profile.log 2>&1
echo done
