#!/bin/bash
# Round 4, session 11: what a stream creation costs by order and thread
# (the per-thread path creates one per calling thread), and the first calls
# of new threads after gf_init ran on another (a VM's dirty schedulers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s11_streams 120 tools/stream_probe 8
step r04_s11_threads 120 tools/capi_bench leo_erasure_amd/libleoec.so threads
echo "session done"
