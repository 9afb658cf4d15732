#!/bin/bash
# vandrs RS(10,4,32) / RS(10,4,16): gfs_apply with two inputs in flight
# (LEOEC_GFS_PF=2) against the shipped one; parity of the form first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_gfs_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gfw_kernel_forms"
step r03b_gfs_pf32 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 32 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFS_PF=2"
step r03b_gfs_pf16 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 16 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFS_PF=2"
echo "session done"
