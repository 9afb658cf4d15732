#!/bin/bash
# Round 3 (second session): the restored tree on a fresh box — smoke, every
# GPU test, the headline bench.  Each GPU step time-limited; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r03b_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step r03b_bench 600 python bench.py
echo "session done"
