#!/bin/bash
# Round 5, session 29: large per-thread calls in column chunks with both link
# directions at once (LEOEC_LARGE_CHUNKS, engine.cpp large_chunked): parity
# (product and measurement forms), then the reference's eunit benchmark
# (one 100 MiB encode per class) at 8 / 4 / 1 (= the round-4 one-piece form)
# chunks, alternating, and on the product library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s29_product_large 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "above_zero_copy_cap"
step r05_s29_forms_large 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 200 --timeout-method thread -k "large_chunked or pinned_large or staging_forms"
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for c in 8 1 4; do
    TAILN=5 step r05_s29_ref_chunks${c}_$r 180 tools/capi_bench $L ref LEOEC_LARGE_CHUNKS=$c
  done
done
TAILN=5 step r05_s29_ref_product 180 tools/capi_bench leo_erasure_amd/libleoec.so ref
echo "session done"
