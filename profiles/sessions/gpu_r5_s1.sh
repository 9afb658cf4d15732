#!/bin/bash
# Round 5, session 1: the inherited tree on a fresh box (smoke, GPU tests,
# the driver-style bench line, its rocprof kernel summary), then the issue
# counters of the liberation kernels beside gf8_apply (tools/pmc_r5_issue.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s1_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r05_s1_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step r05_s1_bench 600 python bench.py --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
step r05_s1_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s1_prof -o run -- python $ROOT/bench.py --steps 20 --warmup 5 --no-cpu
cd $ROOT
step r05_s1_pmc_issue 900 bash tools/pmc_r5_issue.sh r05
echo "session done"
