#!/bin/bash
# Round 5, session 15: the worker's spin for a closed batch's fills
# (LEOEC_HOSTQ_SPIN_US, default 30) against sleeping at once (=0), small
# objects and 1 MiB, alternating runs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for sp in 30 0 10 100; do
    TAILN=2 step r05_s15_small_spin${sp}_$r 120 tools/capi_bench $L small LEOEC_HOSTQ_SPIN_US=$sp
  done
done
TAILN=6 step r05_s15_callers_spin30 120 tools/capi_bench $L callers LEOEC_HOSTQ_SPIN_US=30
TAILN=6 step r05_s15_callers_spin0 120 tools/capi_bench $L callers LEOEC_HOSTQ_SPIN_US=0
echo "session done"
