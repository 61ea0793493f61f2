#!/bin/bash
# Multi-word split-form A/B (CLRSDP_MW_SPLIT=1: potrf + L^-1 by four-wave solves of the
# identity, GEMV solves) against the explicit-inverse default: C5 qd and C4 dd bench lines, then
# the -m gpu suite with the split form on.  Usage: bash tools/mwsplit_run.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 bash tools/env_sweep.sh "--config c5 --precision 4" NONE CLRSDP_MW_SPLIT=1 NONE CLRSDP_MW_SPLIT=1 > $OUT/sweep_c5.log 2>&1 || exit 1
cat $OUT/sweep_c5.log
timeout -k 10 300 bash tools/env_sweep.sh "--config c2 --precision 2" NONE CLRSDP_MW_SPLIT=1 > $OUT/sweep_c4.log 2>&1 || exit 1
cat $OUT/sweep_c4.log
CLRSDP_MW_SPLIT=1 timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?
tail -5 $OUT/tests.log; exit $rc
