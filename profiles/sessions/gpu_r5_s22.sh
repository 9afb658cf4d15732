#!/bin/bash
# Round 5, session 22: the link's duplex through the system HIP runtime and
# through the torch wheel's bundled runtime, from Python, same copies.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s22_link_system 120 python tools/link_hip.py 256
step r05_s22_link_torch_runtime 300 python tools/link_hip.py --torch 256
echo "session done"
