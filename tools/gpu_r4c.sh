set -o pipefail
mkdir -p gpurun_out/r4c
timeout -k 10 120 microbin/eig_ops_probe > gpurun_out/r4c/ops.log 2>&1; echo "ops rc=$?"
cat gpurun_out/r4c/ops.log
timeout -k 10 120 microbin/eig_split_bench > gpurun_out/r4c/eig.log 2>&1; echo "eig rc=$?"
cat gpurun_out/r4c/eig.log
timeout -k 10 120 microbin/eig_split_stamps 128 > gpurun_out/r4c/stamps.log 2>&1; echo "st rc=$?"
cat gpurun_out/r4c/stamps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4c/gputests.log 2>&1; echo "tests rc=$?"
tail -15 gpurun_out/r4c/gputests.log
