#!/bin/bash
# Round 4, session 13: where a lone caller's 1 MiB encode spends its ~88 us
# (the per-thread zero-copy path): plain, then under a kernel + HIP API trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s13_lone 120 tools/capi_bench leo_erasure_amd/libleoec.so lone
step r04_s13_lone_trace 180 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $OUT/r04_s13_trace -- tools/capi_bench leo_erasure_amd/libleoec.so lone
echo "session done"
