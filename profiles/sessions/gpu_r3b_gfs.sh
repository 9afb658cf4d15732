#!/bin/bash
# vandrs RS(10,4,32) encode: what the w = 32 kernel's time pays for
# (profiles/r03b_v8_gfs_branch_cost_w32.log).  LEOEC_GFS_MODE=1: every
# coefficient forced to 0xFFFFFFFF at run time through an opaque scalar (the
# shipped tests and branches run, all taken; 116 VGPRs as shipped); 2: the
# same VALU with no tests compiled in (128 VGPRs, 13 spilled).  Timing only:
# wrong bytes.  (The matrix-compiled-in form of r03b_v11 is at e6f694c.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_gfs_modes2 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 32 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFS_MODE=1;LEOEC_GFS_MODE=2"
echo "session done"
