set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 120 microbin/eig_split_stamps 128 > gpurun_out/r4b/stamps128.log 2>&1; echo "st rc=$?"
timeout -k 10 120 microbin/eig_split_stamps 16 > gpurun_out/r4b/stamps16.log 2>&1; echo "st rc=$?"
cat gpurun_out/r4b/stamps128.log gpurun_out/r4b/stamps16.log
timeout -k 10 300 python -u tools/dd_gap_probe.py 70 > gpurun_out/r4b/ddgap.log 2>&1; echo "dd rc=$?"
tail -25 gpurun_out/r4b/ddgap.log
