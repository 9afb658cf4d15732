#!/bin/bash
# Round 5, session 25: per-thread-path caps (LEOEC_HOSTQ_DIRECT encode /
# _MAP decode) from 4 to 32 callers: shipped 4 / 2 against 8 / 4, 8 / 8 and
# 16 / 16, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for v in "LEOEC_HOSTQ_DIRECT=4" "LEOEC_HOSTQ_DIRECT=8,LEOEC_HOSTQ_DIRECT_MAP=4" "LEOEC_HOSTQ_DIRECT=8,LEOEC_HOSTQ_DIRECT_MAP=8" "LEOEC_HOSTQ_DIRECT=16,LEOEC_HOSTQ_DIRECT_MAP=16"; do
    n=$(echo $v | tr ',=' '__')
    TAILN=9 step r05_s25_mid_${n}_$r 240 tools/capi_bench $L mid $v
  done
done
echo "session done"
