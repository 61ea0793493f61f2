#!/bin/bash
# One parametrised GPU-box job runner (replaces the per-lease one-off scripts of round 4).
# Run from the repo root through gpurun; every step has its own time limit and the first
# failing step ends the job (no GPU step runs after a failure, a timeout or an abort).
#
#   bash tools/gpu_job.sh TAG STEP [STEP ...]
#
# TAG names the output directory gpurun_out/TAG.  Each STEP is one of
#   tests[:PYTEST_K]        the -m gpu suite (optionally -k PYTEST_K), log tests.log
#   testfile:FILE[:K]       one test file (optionally -k K), log tests_<file>.log
#   micro:BIN[:ARGS]        a microbenchmark binary in microbin/ (hipcc line at the top of its tools/micro/*.hip)
#   bench[:ARGS]            one bench.py line (ARGS with ',' for spaces), log bench_<n>.log
#   ab:ENV:R[:ARGS]         tools/ab.sh alternating A/B of ENV (ARGS with ',' for spaces)
#   sweep:ARGS:ENV:ENV...   tools/env_sweep.sh: one bench run per setting (NONE = none)
#   dist2                   2-rank bench rehearsal on one GPU (CLRSDP_BENCH_ONE_GPU=1)
#   trace[:ARGS]            rocprofv3 kernel trace of a bench line + per-body listing
#   measure                 tools/measure_round.sh TAG (PMC passes, bench lines, summaries)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  kind=${step%%:*}
  rest=""; [ "$kind" != "$step" ] && rest=${step#*:}
  case $kind in
    tests)
      k=(); [ -n "$rest" ] && k=(-k "$rest")
      timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        "${k[@]}" > $OUT/tests.log 2>&1; rc=$?
      echo "tests rc=$rc"; grep -E "passed|failed|Error|FAILED" $OUT/tests.log | tail -15 ;;
    testfile)
      f=${rest%%:*}; k=(); [ "$f" != "$rest" ] && k=(-k "${rest#*:}")
      log=$OUT/tests_$(basename $f .py).log
      timeout -k 10 900 python3 -u -m pytest "$f" -m gpu -x -v --timeout 300 --timeout-method thread \
        "${k[@]}" > $log 2>&1; rc=$?
      echo "$f rc=$rc"; grep -E "passed|failed|Error|FAILED" $log | tail -15 ;;
    micro)
      b=${rest%%:*}; a=""; [ "$b" != "$rest" ] && a=${rest#*:}
      timeout -k 10 120 microbin/$b ${a//,/ } > $OUT/micro_$b.log 2>&1; rc=$?
      echo "micro $b rc=$rc"; tail -25 $OUT/micro_$b.log ;;
    bench)
      timeout -k 10 240 python3 bench.py ${rest//,/ } > $OUT/bench_$n.log 2>&1; rc=$?
      echo "bench ${rest//,/ } rc=$rc"; tail -1 $OUT/bench_$n.log | cut -c1-600 ;;
    ab)
      envb=${rest%%:*}; r2=${rest#*:}; R=${r2%%:*}; a=""; [ "$R" != "$r2" ] && a=${r2#*:}
      timeout -k 10 900 bash tools/ab.sh "$envb" $R ${a//,/ } > $OUT/ab_$n.log 2>&1; rc=$?
      echo "ab $envb ${a//,/ } rc=$rc"; cat $OUT/ab_$n.log ;;
    sweep)
      # sweep:ARGS:ENV1:ENV2:... (ARGS with ',' for spaces; NONE = no setting)
      a=${rest%%:*}; envs=${rest#*:}
      timeout -k 10 1000 bash tools/env_sweep.sh "${a//,/ }" ${envs//:/ } > $OUT/sweep_$n.log 2>&1; rc=$?
      echo "sweep ${a//,/ } rc=$rc"; cat $OUT/sweep_$n.log ;;
    dist2)
      CLRSDP_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 \
        --steps 20 --warmup 3 > $OUT/dist2.log 2>&1; rc=$?
      echo "dist2 rc=$rc"; tail -1 $OUT/dist2.log | cut -c1-400 ;;
    trace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$n -o run -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu ${rest//,/ } > $OUT/trace_$n.log 2>&1; rc=$?
      if [ $rc = 0 ]; then
        python3 tools/iter_trace.py $OUT/kt_$n/run_kernel_trace.csv > $OUT/body_$n.txt
        python3 tools/prof_summary.py $OUT/kt_$n/run_kernel_stats.csv > $OUT/summary_$n.txt
        head -30 $OUT/summary_$n.txt
      fi
      echo "trace ${rest//,/ } rc=$rc" ;;
    measure)
      timeout -k 10 1100 bash tools/measure_round.sh $TAG > $OUT/measure.log 2>&1; rc=$?
      echo "measure rc=$rc"; tail -5 $OUT/measure.log ;;
    *)
      echo "unknown step $step"; rc=2 ;;
  esac
  [ $rc = 0 ] || exit $rc
done
