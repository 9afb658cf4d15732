#!/bin/bash
# cauchyrs(10,4,8): the shipped kernel against its XOR-only memory ceiling
# (LEOEC_GFBIT_CEIL=1, not a code) and the bit-pair accumulation form, for
# encode and decode; parity of the forms first.  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_cauchy_forms 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cauchy_kernel_forms"
step r03_cauchy_ceil 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants ";LEOEC_GFBIT_CEIL=1;LEOEC_GFBIT_PAIRS=1"
step r03_cauchy_ceil4 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants ";LEOEC_GFBIT_CEIL=1;LEOEC_GFBIT_PAIRS=1"
echo "session done"
