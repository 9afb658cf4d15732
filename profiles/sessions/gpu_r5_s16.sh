#!/bin/bash
# Round 5, session 16: the completer unpacking small batches itself
# (LEOEC_HOSTQ_UNPACK_BYTES, default 1 MiB of outputs) against callers
# unpacking (=0) and a 4 MiB bound, alternating; then every GPU test.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for ub in 1048576 0 4194304; do
    TAILN=2 step r05_s16_small_unpack${ub}_$r 120 tools/capi_bench $L small LEOEC_HOSTQ_UNPACK_BYTES=$ub
  done
done
TAILN=6 step r05_s16_callers_unpack1m 120 tools/capi_bench $L callers LEOEC_HOSTQ_UNPACK_BYTES=1048576
TAILN=6 step r05_s16_callers_unpack0 120 tools/capi_bench $L callers LEOEC_HOSTQ_UNPACK_BYTES=0
step r05_s16_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
echo "session done"
