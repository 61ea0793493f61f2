set -o pipefail
mkdir -p gpurun_out/c4split
export TMPDIR=/tmp
timeout -k 10 500 bash tools/env_sweep.sh "--config c2 --precision 2" NONE CLRSDP_MW_SPLIT=0 CLRSDP_TRSV_NW4=1 NONE CLRSDP_MW_SPLIT=0 > gpurun_out/c4split/sweep.log 2>&1 || exit 1
cat gpurun_out/c4split/sweep.log
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/c4split/tests.log 2>&1; rc=$?
tail -3 gpurun_out/c4split/tests.log; exit $rc
