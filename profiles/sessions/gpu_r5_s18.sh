#!/bin/bash
# Round 5, session 18: PCIe duplex probe (tools/duplex_probe.hip): DMA and
# kernel movers of each direction alone and paired, at three kernel grid
# sizes, and with the runtime's copies on blit kernels (HSA_ENABLE_SDMA=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=10 step r05_s18_duplex_512 120 tools/duplex_probe 256 5 512
TAILN=10 step r05_s18_duplex_128 120 tools/duplex_probe 256 5 128
TAILN=10 step r05_s18_duplex_2048 120 tools/duplex_probe 256 5 2048
TAILN=10 step r05_s18_duplex_nosdma 120 env HSA_ENABLE_SDMA=0 tools/duplex_probe 256 5 512
echo "session done"
