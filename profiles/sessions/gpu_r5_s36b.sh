#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-5} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s36b_dbg_gather 200 python tools/dbg_repair64.py LEOEC_HOST_STAGING=gather LEOEC_STAGE_CHUNK_KIB=256
step r05_s36b_dbg_default 200 python tools/dbg_repair64.py
step r05_s36b_dbg_gather_nopin 200 python tools/dbg_repair64.py LEOEC_HOST_STAGING=gather LEOEC_ZC_PIN=0
echo "session done"
