# the -m gpu suite on the box, log under gpurun_out/$1
set -o pipefail
OUT=gpurun_out/${1:-tests}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ${2:-} > $OUT/gputests.log 2>&1; rc=$?
echo "tests rc=$rc"
grep -E "passed|failed|Error|FAILED" $OUT/gputests.log | tail -15
exit $rc
