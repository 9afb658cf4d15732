#!/bin/bash
# Round 5, session 38: the final tree with both libraries rebuilt (in-place
# pinning back in the measurement build, off by default): every GPU test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s38_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s38_measure_forms.log
echo "session done"
