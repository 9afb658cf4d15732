#!/bin/bash
# w = 16 / 32 gfs_apply register and prefetch forms: parity, then one-process
# A/Bs of RS(10,4,w) 1 MiB x 1024.  Each step time-limited; a failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-12} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_gfw_forms 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gfw_kernel_forms"
V="${GV:-;LEOEC_GFS_FORM=1;LEOEC_GFS_FORM=2;LEOEC_GFS_FORM=3}"
step r03_gfs32 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 32 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step r03_gfs16 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 16 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
echo "session done"
