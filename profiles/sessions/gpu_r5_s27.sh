#!/bin/bash
# Round 5, session 27: the product library with the new per-thread caps
# (16 / 8) and copy streams: 1-32 callers from plain C++, the sizes sweep,
# every GPU test, smoke, the bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
P=leo_erasure_amd/libleoec.so
# TAILN=8 step r05_s27_few_product 240 tools/capi_bench $P few
# TAILN=8 step r05_s27_mid_product 240 tools/capi_bench $P mid
# TAILN=5 step r05_s27_ref_product 240 tools/capi_bench $P ref
step r05_s27b_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step r05_s27b_smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r05_s27b_bench 600 python bench.py
echo "session done"
