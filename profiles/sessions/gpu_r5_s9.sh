#!/bin/bash
# Round 5, session 9: the headline's byte stream with its reads and writes
# alone (tools/hbm_mix.hip) beside the bench line's kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=20 step r05_s9b_hbm_mix 240 tools/hbm_mix 2048 20

echo "session done"
