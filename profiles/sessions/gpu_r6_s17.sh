#!/bin/bash
# Round 6, session 17: the final tree's bench under the kernel tracer (host
# leg included), for the rocprof summary of the kernels the round ships.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=1 step r06_s17_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06_s17_bench_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5
cd "$ROOT"
python3 tools/rocprof_summary.py --by-launch $OUT/r06_s17_bench_prof > $OUT/r06_s17_bench_kernel_summary.txt
head -6 $OUT/r06_s17_bench_kernel_summary.txt
echo "session done"
