#!/bin/bash
# Round 4: the bench's rocprof summaries (1 MiB and configs[4]), configs[4]'s
# bench line, and a 2-rank rehearsal on the one GPU showing the N > 1 line's
# node aggregate and per-rank fractions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s3_bench64 600 python bench.py --workload 64MiB --no-cpu
step r04_s3_bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10 --no-cpu
cd /tmp && export TMPDIR=/tmp
step r04_s3_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/r04_prof" -o run -- python "$ROOT/bench.py" --no-cpu
step r04_s3_prof64 600 rocprofv3 --kernel-trace --stats -d "$OUT/r04_prof64" -o run -- python "$ROOT/bench.py" --workload 64MiB --no-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/r04_prof" > "$OUT/r04_bench_kernel_summary.txt"
python tools/rocprof_summary.py "$OUT/r04_prof64" > "$OUT/r04_bench64_kernel_summary.txt"
echo "session done"
