#!/bin/bash
# Round 5, session 10: the pattern kernels' test (measurement process) and
# the bench line with the pattern ceiling's read / write halves.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
LEOEC_LIBRARY=measure step r05_s10b_pattern_test 300 python -u -m pytest tests/test_measure_forms.py -x -q -m measure_gpu -k pattern_kernels --timeout 120 --timeout-method thread
step r05_s10b_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
