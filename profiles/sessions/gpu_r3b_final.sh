#!/bin/bash
# Round 3 (second session) evidence on the final tree: smoke, every GPU test,
# the headline bench (with the live pattern ceiling) and its rocprof summary,
# configs[4] and its rocprof summary, a 2-rank rehearsal.  Each GPU step has
# its own time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_final_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r03b_final_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step r03b_final_bench 600 python bench.py
step r03b_final_bench64 600 python bench.py --workload 64MiB --no-cpu
step r03b_final_bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10 --no-cpu
cd /tmp && export TMPDIR=/tmp
step r03b_final_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python "$ROOT/bench.py" --no-cpu
step r03b_final_prof64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof64" -o run -- python "$ROOT/bench.py" --workload 64MiB --no-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/prof" > "$OUT/r03b_final_bench_kernel_summary.txt"
python tools/rocprof_summary.py "$OUT/prof64" > "$OUT/r03b_final_bench64_kernel_summary.txt"
echo "session done"
