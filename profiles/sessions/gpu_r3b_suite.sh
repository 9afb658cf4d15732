#!/bin/bash
# Round 3 (second session): every BASELINE config and the other classes /
# widths in one process on the final tree (tools/bench_suite.py, the CPU
# configs[0] leg with the queued baseline), then the same suite under
# rocprofv3 --kernel-trace --stats.  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_suite 600 python tools/bench_suite.py --reps 20 --cpu-seconds 12
cd /tmp && export TMPDIR=/tmp
step r03b_suite_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/suite_prof" -o run -- python "$ROOT/tools/bench_suite.py" --reps 20 --skip-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/suite_prof" > "$OUT/r03b_suite_kernel_summary.txt"
python tools/rocprof_summary.py --by-launch "$OUT/suite_prof" > "$OUT/r03b_suite_kernel_summary_by_launch.txt"
echo "session done"
