#!/bin/bash
# Round 4: the driver's own round-end commands, verbatim, on the final tree
# (smoke, the GPU tests without a global timeout, the driver-style bench
# line), then the every-config suite with the reference's default cauchyrs
# parameters added.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s5_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s5_pytest 1100 python -m pytest tests/ -x -q -m gpu
step r04_s5_bench 600 python bench.py --steps 20 --warmup 5
step r04_s5_suite 600 python tools/bench_suite.py --skip-cpu
echo "session done"
