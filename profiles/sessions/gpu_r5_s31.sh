#!/bin/bash
# Round 5, session 31: the seeded random parameter sweep (tests/test_gpu_sweep.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=40 step r05_s31_sweep 600 python -u -m pytest tests/test_gpu_sweep.py -v --timeout 300 --timeout-method thread
echo "session done"
