#!/bin/bash
# Round 4, last session on the final tree: every GPU test, the headline bench
# (CPU legs with warm-up passes), and the every-config suite with its rocprof
# summary (configs[0] on the CPU in both pass structures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s4_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
cp "$OUT/measure_forms.log" "$OUT/r04_s4_measure_forms.log" 2>/dev/null || true
step r04_s4_bench 600 python bench.py
step r04_s4_suite 600 python tools/bench_suite.py
cd /tmp && export TMPDIR=/tmp
step r04_s4_suite_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/r04_suite_prof" -o run -- python "$ROOT/tools/bench_suite.py" --skip-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/r04_suite_prof" > "$OUT/r04_suite_kernel_summary.txt"
python tools/rocprof_summary.py "$OUT/r04_suite_prof" --by-launch > "$OUT/r04_suite_kernel_summary_by_launch.txt" 2>/dev/null || true
echo "session done"
