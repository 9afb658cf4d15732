#!/bin/bash
# Round 6, session 16: the exact final tree once more, as the driver runs it:
# every GPU test, smoke, the default bench line (after the block-pair form left).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s16_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r06_s16_measure_forms.log
step r06_s16_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step r06_s16_bench 600 python bench.py
# the suite once more (round 6 session 10 read RS(4,2,8) decode 0.752
# against 0.78-0.80 in round 5's three suites: box noise or not)
TAILN=2 step r06_s16_suite 600 python tools/bench_suite.py --skip-cpu
echo "session done"
