#!/bin/bash
# Round 5, session 20: the batching queue's copies on two dedicated copy
# streams (LEOEC_HOSTQ_STREAMS=1, now the default) against the per-slot
# stream form (=0), alternating, from plain C++ threads (system runtime);
# the product library's size sweep; every GPU test; the bench line (its
# host-memory leg runs on the torch-bundled runtime).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for st in 1 0; do
    TAILN=6 step r05_s20_callers_streams${st}_$r 120 tools/capi_bench $L callers LEOEC_HOSTQ_STREAMS=$st
  done
done
TAILN=12 step r05_s20_sizes_product 300 tools/capi_bench leo_erasure_amd/libleoec.so sizes
step r05_s20_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
TAILN=1 step r05_s20_bench 600 python bench.py
echo "session done"
