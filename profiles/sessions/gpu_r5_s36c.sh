#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-5} "$OUT/$name.log"; if [ $rc -ne 0 ]; then return 0; fi; }
TAILN=12 step r05_s36c_forms_pin1 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -q --timeout 200 --timeout-method thread
TAILN=12 step r05_s36c_forms_pin0 600 env LEOEC_LIBRARY=measure LEOEC_ZC_PIN=0 python -u -m pytest tests/test_measure_forms.py -m measure_gpu -q --timeout 200 --timeout-method thread
echo "session done"
