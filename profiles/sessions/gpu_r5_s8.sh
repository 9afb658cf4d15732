#!/bin/bash
# Round 5, session 8: the repair probe with the output-aliasing cases (four
# [n, bs] outputs end to end in one buffer, and at 2 MiB-aligned bases).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=14 step r05_s8_repair_probe 300 python tools/repair_probe.py
echo "session done"
