#!/bin/bash
# Round 6, session 7: the round's final tree: every GPU test, smoke, the bench
# line, the traced bench with its host leg (kept in profiles/ as the round's
# kernel summary), and the queue forms of the measurement build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s7_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r06_s7_measure_forms.log
step r06_s7_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step r06_s7_bench 600 python bench.py
cd /tmp && export TMPDIR=/tmp
step r06_s7_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06_s7_bench_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5
echo "session done"
