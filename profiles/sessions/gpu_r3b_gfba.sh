#!/bin/bash
# cauchyrs(10,4,8): gfba_apply (line-aligned copies into per-wave LDS slots,
# LEOEC_GFBIT_FORM=3) — parity first, then A/B against the shipped kernel in
# one process, 1,024 and 4,096 objects.  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_gfba_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cauchy_aligned_copy"
V=";LEOEC_GFBIT_FORM=3;LEOEC_GFBIT_FORM=3,LEOEC_GFBIT_PF=2;LEOEC_GFBIT_FORM=3,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_FORM=3,LEOEC_GFBIT_WG=256;LEOEC_GFBIT_FORM=3,LEOEC_GFBIT_PF=3,LEOEC_GFBIT_CEIL=1"
step r03b_gfba_ab 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step r03b_gfba_ab4096 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants "$V"
echo "session done"
