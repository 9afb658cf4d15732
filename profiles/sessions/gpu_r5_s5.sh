#!/bin/bash
# Round 5, session 5: the shipped liberation policy (libb_apply for w >= 11,
# libb_dec_apply with 64 lanes for every syndrome decode / repair, coding
# blocks repaired through syndromes) in the product library: smoke, every
# GPU test, the suite of every config (rocprof kernel trace of it too), the
# bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s5_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r05_s5_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s5_measure_forms.log
step r05_s5_suite 600 python tools/bench_suite.py --skip-cpu
cd /tmp && export TMPDIR=/tmp
step r05_s5_suite_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s5_suite_prof -o run -- python $ROOT/tools/bench_suite.py --skip-cpu
cd $ROOT
step r05_s5_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
