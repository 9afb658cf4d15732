#!/bin/bash
# Round 4, session 20: a lone caller's zero-copy launches (kernel reading and
# writing pinned host memory over PCIe) with the gf8 variants that change
# the memory policy or occupancy: shipped (1), no non-temporal bit (12),
# 6 waves (16), 8 waves (17); interleaved processes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  for v in 1 12 16 17; do
    step r04_s20_lone_v${v}_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_GF8_VARIANT=$v
  done
done
echo "session done"
