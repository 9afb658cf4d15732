#!/bin/bash
# Round 6, session 9: bench.py's host leg with native caller threads
# (tools/libhost_callers.so; the Python-thread figures beside them): the
# host-leg GPU test, then the bench line twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s9_host_leg_test 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "host_leg or thread_exit or warms"
TAILN=1 step r06_s9_bench_a 600 python bench.py
TAILN=1 step r06_s9_bench_b 600 python bench.py
echo "session done"
