#!/bin/bash
# cauchyrs(10,4,8): gfbit_apply with the uniform full-tile fast path
# (LEOEC_GFBIT_FAST=1: no per-lane guards in tiles inside every shard) against
# the default form; parity first, then A/B in one process at 1,024 and 4,096.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03b_fast_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cauchy"
step r03b_fast_ab 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFBIT_FAST=1"
step r03b_fast_ab4096 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants ";LEOEC_GFBIT_FAST=1"
echo "session done"
