#!/bin/bash
# Round 6, session 10: the 64 MiB cauchyrs launch through gfbk (parity), and
# the whole-suite record of every BASELINE config on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s10_gfbk_tests 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "gfbk"
TAILN=5 step r06_s10_suite 900 python tools/bench_suite.py
echo "session done"
