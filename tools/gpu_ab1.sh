set -o pipefail
timeout -k 10 120 microbin/eig_split_bench 2>&1 | head -2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 -k "full_run or newton or pipelined or stage" > gpurun_out/ab1_tests.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/ab1_tests.log
bash tools/ab.sh "CLRSDP_SLAB_QSOLVE=0" 3 --steps 300
bash tools/ab.sh "CLRSDP_SLAB_QSOLVE=0" 3 --steps 300 --clusters 8
