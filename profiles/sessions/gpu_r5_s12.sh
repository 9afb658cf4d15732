#!/bin/bash
# Round 5, session 12: the host path's per-call cost against object size
# (C ABI from plain C++ threads, system HIP runtime, 16 KiB - 4 MiB).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=25 step r05_s12_capi_sizes 300 tools/capi_bench leo_erasure_amd/libleoec.so sizes
echo "session done"
