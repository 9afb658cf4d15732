#!/bin/bash
# Round 4, session 10: the driver's round-end commands on the tree with gf_init's
# warm-up (smoke, the GPU tests without a global timeout, the driver-style
# bench line), then the every-config suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s10_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s10_pytest 1100 python -m pytest tests/ -x -q -m gpu
step r04_s10_bench 600 python bench.py --steps 20 --warmup 5
step r04_s10_suite 600 python tools/bench_suite.py --skip-cpu
echo "session done"
