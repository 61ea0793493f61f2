# kernel traces of the C3 bench and the 8-cluster body; one body dumped per trace
set -o pipefail
OUT=gpurun_out/${1:-trace}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu > $OUT/bench_kt.log 2>&1 || exit 1
python3 tools/iter_trace.py $OUT/kt/run_kernel_trace.csv > $OUT/body_c3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt8 -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu --clusters 8 > $OUT/bench_kt8.log 2>&1 || exit 1
python3 tools/iter_trace.py $OUT/kt8/run_kernel_trace.csv > $OUT/body_c8.txt
wc -l $OUT/body_c3.txt $OUT/body_c8.txt
