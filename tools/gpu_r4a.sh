set -o pipefail
mkdir -p gpurun_out/r4a
timeout -k 10 120 microbin/eig_split_bench > gpurun_out/r4a/eig.log 2>&1; echo "eig rc=$?"
tail -20 gpurun_out/r4a/eig.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4a/gputests.log 2>&1; echo "tests rc=$?"
tail -15 gpurun_out/r4a/gputests.log
