set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_mw
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mw/c4 -o run -- python3 bench.py --config c2 --precision 2 --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_mw/c4.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mw/c5 -o run -- python3 bench.py --config c5 --precision 4 --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_mw/c5.log 2>&1
python3 tools/prof_summary.py gpurun_out/prof_mw/c4/run_kernel_stats.csv 13 > gpurun_out/prof_mw/c4_summary.txt
python3 tools/prof_summary.py gpurun_out/prof_mw/c5/run_kernel_stats.csv 13 > gpurun_out/prof_mw/c5_summary.txt
