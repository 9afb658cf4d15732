#!/bin/bash
# Round 5, session 11: the suite of every config on the final tree (repair
# into per-object rows and into separate tensors), with its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s11_suite 600 python tools/bench_suite.py
cd /tmp && export TMPDIR=/tmp
step r05_s11_suite_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s11_suite_prof -o run -- python $ROOT/tools/bench_suite.py --skip-cpu
echo "session done"
