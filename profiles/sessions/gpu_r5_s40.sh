#!/bin/bash
# Round 5, session 40: small batches back on the slot's stream
# (LEOEC_HOSTQ_SPLIT_KIB=1024, shipped) against splitting every batch (=0),
# alternating, 16 KiB - 1 MiB objects at 8 and 32 callers; then every GPU
# test and the bench line on the final tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for k in 1024 0; do
    TAILN=3 step r05_s40_small_split${k}_$r 240 tools/capi_bench $L small LEOEC_HOSTQ_SPLIT_KIB=$k
    TAILN=4 step r05_s40_callers_split${k}_$r 240 tools/capi_bench $L callers LEOEC_HOSTQ_SPLIT_KIB=$k
  done
done
step r05_s40_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s40_measure_forms.log
step r05_s40_smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r05_s40_bench 600 python bench.py
echo "session done"
