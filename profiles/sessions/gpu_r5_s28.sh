#!/bin/bash
# Round 5, session 28: duplex with caller memory: pinned in place
# (hipHostRegister) and pageable, alone, paired, and in 8 chunks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=20 step r05_s28_duplex_caller_memory 180 tools/duplex_probe 256 5 128
echo "session done"
