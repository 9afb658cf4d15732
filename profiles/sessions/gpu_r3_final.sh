#!/bin/bash
# Round 3 evidence session on the final tree: smoke, every GPU test, the
# round-2 abort form's test with the runtime's diagnostics on, the access-
# pattern ceilings, the headline bench (and its rocprof summary), configs[4]
# (and its rocprof summary), a 2-rank rehearsal.  Every GPU step has its own
# time limit; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r03_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
LIBC_FATAL_STDERR_=1 AMD_LOG_LEVEL=1 step r03_cauchy_forms 300 python -u -X faulthandler -m pytest tests/test_gpu_parity.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "cauchy_kernel_forms"
step r03_order_ceiling_64MiB 240 ./tools/order_ceiling 67108864 64 20
step r03_order_ceiling_1MiB 240 ./tools/order_ceiling 1048576 2048 20
step r03_bench 600 python bench.py
step r03_bench64 600 python bench.py --workload 64MiB --no-cpu
step r03_bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10 --no-cpu
cd /tmp && export TMPDIR=/tmp
step r03_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- python "$ROOT/bench.py" --no-cpu
step r03_prof64 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof64" -o run -- python "$ROOT/bench.py" --workload 64MiB --no-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/prof" > "$OUT/r03_bench_kernel_summary.txt"
python tools/rocprof_summary.py "$OUT/prof64" > "$OUT/r03_bench64_kernel_summary.txt"
echo "session done"
