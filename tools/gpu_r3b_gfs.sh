#!/bin/bash
# vandrs RS(10,4,32) encode: the matrix compiled in (LEOEC_GFS_MODE=3,
# gfs_spec: per-input bodies with every coefficient test resolved at compile
# time; 235 VGPRs, 2 waves per SIMD) against the shipped kernel; parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_gfs_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gfw_kernel_forms"
step r03b_gfs_spec 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 32 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFS_MODE=3"
echo "session done"
