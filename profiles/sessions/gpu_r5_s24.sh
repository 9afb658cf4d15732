#!/bin/bash
# Round 5, session 24: how many calls may take the per-thread path while the
# queue is idle (LEOEC_HOSTQ_DIRECT encode / _MAP decode; shipped 4 / 2) at
# 1-8 callers, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for v in "LEOEC_HOSTQ_DIRECT=4" "LEOEC_HOSTQ_DIRECT_MAP=4" "LEOEC_HOSTQ_DIRECT=8,LEOEC_HOSTQ_DIRECT_MAP=8"; do
    n=$(echo $v | tr ',=' '__')
    TAILN=9 step r05_s24_few_${n}_$r 240 tools/capi_bench $L few $v
  done
done
echo "session done"
