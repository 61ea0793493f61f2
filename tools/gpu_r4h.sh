set -o pipefail
mkdir -p gpurun_out/r4h
timeout -k 10 60 microbin/eig_mx_dump > gpurun_out/r4h/dump.log 2>&1; echo "dump rc=$?"; cat gpurun_out/r4h/dump.log
