#!/bin/bash
# Round 5, session 32: two ranks on the one card (--oversubscribe) with the
# host leg's system-runtime child per rank; the widened random sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=1 step r05_s32_bench_2rank_one_card 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 3 --oversubscribe
step r05_s32_sweep 600 python -u -m pytest tests/test_gpu_sweep.py -q --timeout 300 --timeout-method thread
echo "session done"
