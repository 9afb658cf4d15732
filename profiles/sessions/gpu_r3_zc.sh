#!/bin/bash
# Zero-copy staging of the host entry points' per-thread path: parity of
# every staging form, then the lone / few-caller rates against the default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_zc_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "host_staging_forms or host_batching or concurrent_callers"
step r03_zc_e2e 600 python tools/e2e_bench.py --forms "default:;zerocopy:LEOEC_HOST_STAGING=zerocopy;default2:;zerocopy2:LEOEC_HOST_STAGING=zerocopy" --threads 1,2,4,8
echo "session done"
