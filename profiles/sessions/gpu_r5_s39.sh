#!/bin/bash
# Round 5, session 39: the copy-stream form on another box (LEOEC_HOSTQ_STREAMS
# 1 / 0, alternating, 8-32 callers) and small objects (16 / 64 KiB, 32
# callers) in both forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for st in 1 0; do
    TAILN=9 step r05_s39_mid_streams${st}_$r 240 tools/capi_bench $L mid LEOEC_HOSTQ_STREAMS=$st
    TAILN=3 step r05_s39_small_streams${st}_$r 240 tools/capi_bench $L small LEOEC_HOSTQ_STREAMS=$st
  done
done
echo "session done"
