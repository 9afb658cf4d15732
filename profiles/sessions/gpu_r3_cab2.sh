#!/bin/bash
# cauchyrs(10,4,8) row-split form: its parity cases, then one-process A/Bs at
# 1 MiB x 1024 / x 4096.  Each step time-limited; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-12} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_cauchy_forms 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cauchy_kernel_forms"
V="${CV:-;LEOEC_GFBIT_RSPL=2;LEOEC_GFBIT_RSPL=2,LEOEC_GFBIT_PF=0}"
step r03_cab1 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step r03_cab4 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --size 1048576 --objects 4096 --rounds 4 --reps 6 --variants "$V"
echo "session done"
