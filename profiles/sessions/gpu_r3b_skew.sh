#!/bin/bash
# Pattern experiment at the reference's 64 MiB geometry: blocks 5..9 read at
# another column than blocks 0..4 (so no burst holds block j and block j+5
# of one column): +1 KiB, -1 KiB, and the two 1 KiB windows of a pair
# swapped (skew argument 1).  Not a code: the XOR then mixes columns.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for sk in 0 1024 6709888 1; do
  step r03b_skew2_64MiB_$sk 240 ./tools/order_ceiling 67108864 64 20 0 quick $sk
done
step r03b_skew2_1MiB_0 240 ./tools/order_ceiling 1048576 2048 20 0 quick 0
step r03b_skew2_1MiB_1 240 ./tools/order_ceiling 1048576 2048 20 0 quick 1
echo "session done"
