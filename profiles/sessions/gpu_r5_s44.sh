#!/bin/bash
# Round 5, session 44: the decode per-thread cap, 8 (shipped) against 12 and
# 16 with the encode cap at 16, three rotated rounds, 1-32 callers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-1} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_DIRECT_MAP=8" "LEOEC_HOSTQ_DIRECT_MAP=12" "LEOEC_HOSTQ_DIRECT_MAP=16")
for r in 0 1 2; do
  for i in 0 1 2; do
    v=${V[$(( (i + r) % 3 ))]}
    n=$(echo $v | tr ',=' '__')
    step r05_s44_few_${n}_$r 240 tools/capi_bench $L few $v
    step r05_s44_mid_${n}_$r 240 tools/capi_bench $L mid $v
  done
done
echo "session done"
