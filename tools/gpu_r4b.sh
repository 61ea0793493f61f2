set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 120 microbin/eig_split_stamps 128 > gpurun_out/r4b/stamps128.log 2>&1; echo "st rc=$?"
timeout -k 10 120 microbin/eig_split_stamps 16 > gpurun_out/r4b/stamps16.log 2>&1; echo "st rc=$?"
cat gpurun_out/r4b/stamps128.log gpurun_out/r4b/stamps16.log
timeout -k 10 300 python -u tools/dd_gap_probe.py 70 > gpurun_out/r4b/ddgap.log 2>&1; echo "dd rc=$?"
tail -25 gpurun_out/r4b/ddgap.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4b/kt -o run -- \
  python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/r4b/bench_kt.log 2>&1; echo "kt rc=$?"
python3 tools/copy_census.py gpurun_out/r4b/kt/run_kernel_trace.csv > gpurun_out/r4b/census.txt 2>&1
python3 tools/prof_summary.py gpurun_out/r4b/kt/run_kernel_stats.csv 33 > gpurun_out/r4b/kernel_summary.txt 2>&1
head -30 gpurun_out/r4b/census.txt; head -12 gpurun_out/r4b/kernel_summary.txt; tail -1 gpurun_out/r4b/bench_kt.log | cut -c1-400
