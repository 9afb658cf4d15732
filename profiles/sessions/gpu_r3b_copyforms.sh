#!/bin/bash
# RS(10,4,8) 1 MiB x 2048: the shipped encode against the XOR-for-GF (COPY)
# forms of gf8_apply — the candidates for bench.py's pattern ceiling.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_copyforms 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 1048576 --objects 2048 --rounds 6 --reps 10 --variants ";LEOEC_GF8_VARIANT=7;LEOEC_GF8_VARIANT=27;LEOEC_GF8_VARIANT=39;LEOEC_GF8_VARIANT=43"
step r03b_order_ceiling 240 ./tools/order_ceiling 1048576 2048 20
step r03b_bench_ceil 600 python bench.py --no-cpu
echo "session done"
