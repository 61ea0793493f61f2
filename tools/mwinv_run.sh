#!/bin/bash
# Multi-word explicit-inverse A/B (CLRSDP_MW_INV_S / _Q): C5 qd and C4 dd bench lines under each
# setting, then the whole -m gpu suite with both on.  Usage: bash tools/mwinv_run.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 bash tools/env_sweep.sh "--config c2 --precision 2" NONE "CLRSDP_MW_INV_S=1 CLRSDP_MW_INV_Q=1" NONE "CLRSDP_MW_INV_S=1 CLRSDP_MW_INV_Q=1" > $OUT/sweep_c4.log 2>&1 || exit 1
cat $OUT/sweep_c4.log
CLRSDP_MW_INV_S=1 CLRSDP_MW_INV_Q=1 timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; exit $rc
