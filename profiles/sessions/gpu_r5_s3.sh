#!/bin/bash
# Round 5, session 3: the liberation forms again on another box (session 2:
# libb_dec_apply with 64 lanes +5 / +10 % on decode of (7,2,7) / (10,2,11),
# libb_apply -3 to -7 % on encode), now with the old decode kernel at 64
# lanes for reference, the syndrome repair of coding blocks against the
# generic bitmatrix kernel (LEOEC_LIB_DEC_COD=0), and the pattern ceiling
# with a time-based warm-up.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s3_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 120 --timeout-method thread -k liberation
TAILN=16 step r05_s3_lib_ceiling_727 300 tools/lib_ceiling 1024 20 7
V=";LEOEC_LIB_DEC_WG=64;LEOEC_LIB_BUF=1;LEOEC_LIB_BUF=1,LEOEC_LIB_LA=4;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64,LEOEC_LIB_DEC_LA=4;LEOEC_LIB_DEC_COD=0"
for cfg in "7 2 7 0,7" "4 2 7 0,4" "10 2 11 0,10" "5 2 5 0,5" "13 2 13 0,13"; do
  set -- $cfg
  TAILN=24 step r05_s3_ab_lib_$1_$3 600 python tools/env_ab.py --coding liberation --k $1 --m $2 --w $3 --erased 0,1 --repair $4 --objects 1024 --rounds 4 --variants "$V"
done
TAILN=6 step r05_s3_ab_lib_727_repQ 600 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --erased "" --repair 8 --objects 1024 --rounds 4 --variants ";LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64;LEOEC_LIB_DEC_COD=0"
echo "session done"
