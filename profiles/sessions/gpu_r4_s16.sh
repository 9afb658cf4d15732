#!/bin/bash
# Round 4, session 16: a lone caller's zero-copy launches (one object, ~26
# tiles of 4 KiB) with 64-lane, 1 KiB tiles instead (4x the workgroups
# issuing PCIe reads), interleaved processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  step r04_s16_lone_wg256_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone
  step r04_s16_lone_wg64_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_GF8_WG=64
  step r04_s16_lone_wg64_c1_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_GF8_WG=64,LEOEC_ZC_CHUNKS=1
done
echo "session done"
