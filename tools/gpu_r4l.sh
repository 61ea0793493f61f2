set -o pipefail
bash tools/gpu_tests.sh r4l || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4l/smoke.log 2>&1; echo "smoke rc=$?"; tail -3 gpurun_out/r4l/smoke.log
timeout -k 10 300 python3 bench.py > gpurun_out/r4l/bench.log 2>&1; echo "bench rc=$?"; tail -1 gpurun_out/r4l/bench.log | cut -c1-300
