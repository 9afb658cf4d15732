#!/bin/bash
# Round 6, session 8: every GPU test after the reclaim list is drained on
# every host call; the bench's N > 1 path on the final tree, rehearsed on
# the one card (2 ranks, --oversubscribe: each rank its own host-leg child and
# warm-up thread; the driver's 8-GPU SCALE run takes the same code path).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s8_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=1 step r06_s8_bench_2rank 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --oversubscribe
TAILN=1 step r06_s8_bench_64MiB 600 python bench.py --workload 64MiB --steps 5 --warmup 2 --no-host
echo "session done"
