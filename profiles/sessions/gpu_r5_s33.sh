#!/bin/bash
# Round 5, session 33: liberation's access pattern with line-aligned loads
# and the lanes rotated through LDS (lib_ceiling's sweep forms) against the
# misaligned and aligned-packet patterns, (4,2,7) and (7,2,7).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=20 step r05_s33_lib_sweep_427 300 tools/lib_ceiling 1024 20 4
TAILN=20 step r05_s33_lib_sweep_727 300 tools/lib_ceiling 1024 20 7
echo "session done"
