#!/bin/bash
# Round 5, session 41: final-tree records — the bench's kernel trace
# (--no-host) and the every-config suite with its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s41_suite 600 python tools/bench_suite.py
cd /tmp && export TMPDIR=/tmp
step r05_s41_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s41_bench_prof -o run -- python $ROOT/bench.py --steps 20 --warmup 5 --no-host
step r05_s41_suite_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s41_suite_prof -o run -- python $ROOT/tools/bench_suite.py --skip-cpu
cd $ROOT
python tools/rocprof_summary.py $OUT/r05_s41_bench_prof > $OUT/r05_final_bench_kernel_summary.txt
python tools/rocprof_summary.py $OUT/r05_s41_suite_prof > $OUT/r05_final2_suite_kernel_summary.txt
echo "session done"
