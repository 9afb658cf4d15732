#!/bin/bash
# Round 5, session 19: the batching queue's copy shape against the link
# (duplex_probe's queue-shape cases), and the bench's torch link leg against
# raw hipMemcpyAsync on torch's and on hipHostMalloc'd pinned buffers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=14 step r05_s19_duplex_queue 120 tools/duplex_probe 256 5 128
TAILN=5 step r05_s19_link_torch 300 python tools/link_torch.py 256
L=leo_erasure_amd/libleoec_measure.so
TAILN=8 step r05_s19_callers 120 tools/capi_bench $L callers
echo "session done"
