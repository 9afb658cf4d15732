#!/bin/bash
# Round 5, session 36: per-thread zero-copy calls with the caller's blocks
# pinned in place (LEOEC_ZC_PIN=1, now the default) against packing them
# (=0): every GPU test first, then 1-16 callers and a lone caller's
# microseconds, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s36_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s36_measure_forms.log
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for p in 1 0; do
    TAILN=9 step r05_s36_few_pin${p}_$r 240 tools/capi_bench $L few LEOEC_ZC_PIN=$p
    TAILN=3 step r05_s36_lone_pin${p}_$r 240 tools/capi_bench $L lone LEOEC_ZC_PIN=$p
  done
done
TAILN=9 step r05_s36_mid_product 240 tools/capi_bench leo_erasure_amd/libleoec.so mid
echo "session done"
