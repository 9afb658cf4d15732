#!/bin/bash
# liberation decode: lib_dec_apply with 4 / 6 packets of load look-ahead
# (LEOEC_LIB_DEC_LA) against the shipped 2; parity first, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_libdec_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "liberation_encode_forms"
step r03b_libdec_ab77 300 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --erased 0,1 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_LIB_DEC_LA=4;LEOEC_LIB_DEC_LA=6"
step r03b_libdec_ab1011 300 python tools/env_ab.py --coding liberation --k 10 --m 2 --w 11 --erased 0,1 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_LIB_DEC_LA=4;LEOEC_LIB_DEC_LA=6"
echo "session done"
