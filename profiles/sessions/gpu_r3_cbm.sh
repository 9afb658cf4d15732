#!/bin/bash
# cauchyrs(10,4,8) encode with the bitmatrix compiled in (cbm_inst.hip):
# parity of every form, then one-process A/Bs against the shipped bitsliced
# kernel at 1 MiB x 1024 / x 4096.  Each step time-limited.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_cbm_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cauchy_kernel_forms or cauchy_compiled"
V="${CV:-;LEOEC_GFBIT_CBM=1;LEOEC_GFBIT_CBM=2;LEOEC_GFBIT_CBM=3;LEOEC_GFBIT_CBM=4;LEOEC_GFBIT_CBM=5}"
step r03_cbm_ab1 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step r03_cbm_ab4 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants "$V"
echo "session done"
