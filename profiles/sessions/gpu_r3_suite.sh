#!/bin/bash
# Round 3: GPU tests on the final kernels, then every BASELINE config (and
# the other classes / widths) in one process (tools/bench_suite.py), then the
# same suite under rocprofv3 --kernel-trace --stats for per-kernel summaries.
# Each step time-limited; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step r03_pytest 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
fi
step r03_suite 600 python tools/bench_suite.py --reps 20 --cpu-seconds 12
cd /tmp && export TMPDIR=/tmp
step r03_suite_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/suite_prof" -o run -- python "$ROOT/tools/bench_suite.py" --reps 20 --skip-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/suite_prof" > "$OUT/r03_suite_kernel_summary.txt"
echo "session done"
