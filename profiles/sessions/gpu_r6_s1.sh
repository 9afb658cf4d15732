#!/bin/bash
# Round 6, session 1: cauchyrs(10,4,8) forms at the bench's batch (verdict
# r5 item 4): the shipped gfbit_apply against gfbk_apply (64 lanes, 3 blocks
# ahead) and the one-wave compiled bitmatrix (CBM=6/7, encode only), encode /
# decode / repair, interleaved in one process at 1,024 / 2,048 / 4,096 objects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
V=";LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_WG=64,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_CBM=6;LEOEC_GFBIT_CBM=7"
for n in 2048 1024 4096; do
  TAILN=12 step r06_s1_ab_cauchy_$n 500 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects $n --rounds 4 --repair 0,5,10,13 --variants "$V"
done
echo "session done"
