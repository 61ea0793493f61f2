#!/bin/bash
# Several microbenchmark runs in one GPU call, one log each (gpu_job.sh's micro step keeps one
# log per binary).  Usage: bash tools/micro_runs.sh TAG "BIN ARGS" ["BIN ARGS" ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for run in "$@"; do
  set -- $run
  b=$1; shift
  log=$OUT/${b}_$(echo "$*" | tr ' ' '_').log
  timeout -k 10 120 microbin/$b "$@" > $log 2>&1; rc=$?
  echo "== $b $* rc=$rc"; tail -12 $log
  [ $rc = 0 ] || exit $rc
done
