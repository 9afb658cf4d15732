#!/bin/bash
# Round 5, session 30: the bench line with its host-memory leg in a child
# process on the system HIP runtime (torch-free, as a NIF's VM), the torch
# runtime's leg beside it; the large-call tests after large_chunks went back
# to 1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=1 step r05_s30_bench 600 python bench.py
step r05_s30_product_large 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "above_zero_copy_cap"
step r05_s30_forms_large 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 200 --timeout-method thread -k "large_chunked or pinned_large"
echo "session done"
