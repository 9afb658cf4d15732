#!/bin/bash
# Round 5, session 6: the tree after the warm-up, drain and bench-leg work:
# smoke, every GPU test, the bench line (with the host-memory leg and its
# pinned link rate), a rocprof kernel trace of the bench, and a two-rank
# rehearsal of the bench on the one card (per-rank host legs summed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
# Second call: smoke, tests and the bench line passed in the first; rocprofv3
# 7.2 --kernel-trace aborted in its stream_stack.cpp:56 check once the
# host-memory leg's caller threads ran, so the traced run skips that leg.
cd /tmp && export TMPDIR=/tmp
step r05_s6_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s6_bench_prof -o run -- python $ROOT/bench.py --steps 20 --warmup 5 --no-host
cd $ROOT
step r05_s6_bench2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --oversubscribe
echo "session done"
