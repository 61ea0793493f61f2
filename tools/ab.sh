#!/bin/bash
# A/B timing on the GPU box: alternate `python bench.py` runs with and without an environment
# setting, R rounds, printing iterations/s per run (bench args after the setting).
#   bash tools/ab.sh "CLRSDP_NO_GRAPH=1" 3 --steps 600
set -uo pipefail
ENVB=${1//,/ }; R=$2; shift 2  # (several settings: comma-separated)
export TMPDIR=/tmp
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = A ]; then cmd="python3 bench.py --no-cpu $*"; else cmd="env $ENVB python3 bench.py --no-cpu $*"; fi
    out=$(timeout -k 10 120 $cmd 2>&1 | tail -1) || { echo "run failed: $out"; exit 1; }
    echo "$v $(echo "$out" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],1), round(d["roofline"]["schur_ms_per_iteration"]*1e3,1))')"
  done
done
