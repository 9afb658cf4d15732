#!/bin/bash
# Round 5, session 21: with the copies on their own streams, the queue's
# batches in flight (LEOEC_HOSTQ_DEPTH 3 / 4) and its closing rule
# (LEOEC_HOSTQ_CLOSE 1 / 0), alternating; and the link leg's copies on
# runtime-created streams in a torch process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=6 step r05_s21_link_torch 300 python tools/link_torch.py 256
L=leo_erasure_amd/libleoec_measure.so
for r in a b; do
  for v in "LEOEC_HOSTQ_DEPTH=3" "LEOEC_HOSTQ_DEPTH=4" "LEOEC_HOSTQ_CLOSE=0" "LEOEC_HOSTQ_DEPTH=4,LEOEC_HOSTQ_CLOSE=0"; do
    n=$(echo $v | tr ',=' '__')
    TAILN=6 step r05_s21_callers_${n}_$r 120 tools/capi_bench $L callers $v
  done
done
echo "session done"
