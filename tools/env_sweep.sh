#!/bin/bash
# One bench.py configuration under a list of environment settings, one run each (a numerical
# regression hunt / quick sweep): prints the setting, exit code and iterations/s.  A run that
# ends with a library error (exit 1) does not stop the sweep; any other failure (a time limit,
# an abort, a fault) ends it at once.
#   bash tools/env_sweep.sh "--clusters 8 --steps 300" NONE CLRSDP_DY_DOT=0 CLRSDP_CHAIN=0 ...
set -uo pipefail
ARGS=$1; shift
export TMPDIR=/tmp
for e in "$@"; do
  if [ "$e" = NONE ]; then cmd="python3 bench.py --no-cpu $ARGS"; else cmd="env $e python3 bench.py --no-cpu $ARGS"; fi
  out=$(timeout -k 10 150 $cmd 2>&1); rc=$?
  val=$(echo "$out" | tail -1 | python3 -c 'import json,sys
try: print(round(json.loads(sys.stdin.read())["value"],1))
except Exception: print("-")' 2>/dev/null)
  err=$(echo "$out" | grep -o "clrsdp error.*" | tail -1)
  echo "$e rc=$rc value=$val $err"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
