#!/bin/bash
# vandrs RS(10,4,8): gf8 variant 47 (pair-swapped block halves, LDS hand-over
# of half-sums) against the shipped kernel at 64 MiB and 1 MiB; parity first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_swap_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "pair_swap"
step r03b_swap_ab64 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 67108864 --objects 64 --rounds 6 --reps 6 --variants ";LEOEC_GF8_VARIANT=47"
step r03b_swap_ab1 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 1048576 --objects 2048 --rounds 6 --reps 10 --variants ";LEOEC_GF8_VARIANT=47"
echo "session done"
