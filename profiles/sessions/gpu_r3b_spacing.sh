#!/bin/bash
# Diagnostic (not the reference's layout): does the 10 data blocks' spacing
# (bs, with 5*bs = 2^k + a few lines at the reference geometry) explain why
# the encode pattern reads less at 64 MiB than at 1 MiB?  The XOR-only
# pattern at the reference spacing and with extra bytes between blocks.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for pad in 0 4096 65536 1048576 3145728; do
  step r03b_spacing_64MiB_pad$pad 240 ./tools/order_ceiling 67108864 64 20 $pad quick
done
for pad in 0 4096 65536; do
  step r03b_spacing_1MiB_pad$pad 240 ./tools/order_ceiling 1048576 2048 20 $pad quick
done
echo "session done"
