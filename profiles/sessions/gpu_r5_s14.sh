#!/bin/bash
# Round 5, session 14: targeted queue wake-ups (LEOEC_HOSTQ_WAKE=1, the new
# default) against the round-4 broadcasts (=0), small objects and 1 MiB,
# alternating runs; the product library's size sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
TAILN=2 step r05_s14_small_wake1_a 120 tools/capi_bench $L small LEOEC_HOSTQ_WAKE=1
TAILN=2 step r05_s14_small_wake0_a 120 tools/capi_bench $L small LEOEC_HOSTQ_WAKE=0
TAILN=2 step r05_s14_small_wake1_b 120 tools/capi_bench $L small LEOEC_HOSTQ_WAKE=1
TAILN=2 step r05_s14_small_wake0_b 120 tools/capi_bench $L small LEOEC_HOSTQ_WAKE=0
TAILN=6 step r05_s14_callers_wake1 120 tools/capi_bench $L callers LEOEC_HOSTQ_WAKE=1
TAILN=6 step r05_s14_callers_wake0 120 tools/capi_bench $L callers LEOEC_HOSTQ_WAKE=0
echo "session done"
