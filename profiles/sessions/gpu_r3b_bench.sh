#!/bin/bash
# Headline bench with the live access-pattern ceiling leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log" | cut -c1-400; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_bench_ceil 600 python bench.py
step r03b_bench64_ceil 600 python bench.py --workload 64MiB --no-cpu
echo "session done"
