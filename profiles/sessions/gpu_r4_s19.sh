#!/bin/bash
# Round 4, session 19: the lone-caller A/B again on the final tree (one
# piece vs two column chunks, measurement library; the product library),
# interleaved processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  step r04_s19_lone_c1_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_ZC_CHUNKS=1
  step r04_s19_lone_c2_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_ZC_CHUNKS=2
  step r04_s19_lone_product_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec.so lone
done
echo "session done"
