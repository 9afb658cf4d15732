#!/bin/bash
# Round 5, session 13: the host path's small-object call rate under the
# batching queue's knobs (measurement library, queue timeline counters).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
TAILN=2 step r05_s13_small_default 120 tools/capi_bench $L small
TAILN=2 step r05_s13_small_depth2 120 tools/capi_bench $L small LEOEC_HOSTQ_DEPTH=2
TAILN=2 step r05_s13_small_depth5 120 tools/capi_bench $L small LEOEC_HOSTQ_DEPTH=5
TAILN=2 step r05_s13_small_sync2 120 tools/capi_bench $L small LEOEC_HOSTQ_SYNC=2
TAILN=2 step r05_s13_small_zc 120 tools/capi_bench $L small LEOEC_HOSTQ_ZC=1
TAILN=2 step r05_s13_small_close0 120 tools/capi_bench $L small LEOEC_HOSTQ_CLOSE=0
TAILN=2 step r05_s13_small_direct0 120 tools/capi_bench $L small LEOEC_HOSTQ_DIRECT=0
echo "session done"
