#!/bin/bash
# Round 4, session 17 (final tree): rocprofv3 kernel-trace summaries of the
# headline bench and the 64 MiB workload, then the driver-style bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s17_bench_prof 600 rocprofv3 --kernel-trace --stats -d $OUT/r04_s17_bench_prof -- python bench.py --steps 20 --warmup 5 --no-cpu
step r04_s17_bench64_prof 600 rocprofv3 --kernel-trace --stats -d $OUT/r04_s17_bench64_prof -- python bench.py --workload 64MiB --steps 20 --warmup 5 --no-cpu
step r04_s17_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
