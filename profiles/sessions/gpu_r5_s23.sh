#!/bin/bash
# Round 5, session 23: the reference's basho_bench concurrency (1 and 4
# callers, 1 MiB RS(10,4,8)) now that batches overlap their copies: the
# shipped policy (up to 4 encode / 2 decode calls on the per-thread path
# while the queue is idle) against every call batched and against one
# direct call, alternating; then the batching-queue GPU tests (both stream
# forms).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for v in "LEOEC_HOSTQ_DIRECT=4" "LEOEC_HOSTQ_DIRECT=0,LEOEC_HOSTQ_DIRECT_MAP=0" "LEOEC_HOSTQ_DIRECT=1,LEOEC_HOSTQ_DIRECT_MAP=1"; do
    n=$(echo $v | tr ',=' '__')
    TAILN=7 step r05_s23_few_${n}_$r 180 tools/capi_bench $L few $v
  done
done
step r05_s23_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 120 --timeout-method thread -k "host_batching"
echo "session done"
