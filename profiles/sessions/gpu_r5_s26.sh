#!/bin/bash
# Round 5, session 26: per-thread-path caps again, 1-32 callers, three rounds
# in rotated order: shipped 4 / 2, 8 / 4, 16 / 8, 16 / 16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_DIRECT=4" "LEOEC_HOSTQ_DIRECT=8,LEOEC_HOSTQ_DIRECT_MAP=4" "LEOEC_HOSTQ_DIRECT=16,LEOEC_HOSTQ_DIRECT_MAP=8" "LEOEC_HOSTQ_DIRECT=16,LEOEC_HOSTQ_DIRECT_MAP=16")
for r in 0 1 2; do
  for i in 0 1 2 3; do
    v=${V[$(( (i + r) % 4 ))]}
    n=$(echo $v | tr ',=' '__')
    TAILN=1 step r05_s26_few_${n}_$r 240 tools/capi_bench $L few $v
    TAILN=1 step r05_s26_mid_${n}_$r 240 tools/capi_bench $L mid $v
  done
done
echo "session done"
