#!/bin/bash
# Round 4, session 9: do register + unregister cycles slow later pageable
# copies of the same memory (tools/large_copy_probe poison); the engine's
# 100 MiB host path with and without the pinned form (measurement build) and
# the product library with gf_init's warm-up; the host-path form tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s9_poison 120 tools/large_copy_probe 100 5 poison
step r04_s9_capi_ref_product 120 tools/capi_bench leo_erasure_amd/libleoec.so ref
step r04_s9_capi_ref_measure_default 120 tools/capi_bench leo_erasure_amd/libleoec_measure.so ref
step r04_s9_capi_ref_measure_pin 120 tools/capi_bench leo_erasure_amd/libleoec_measure.so ref LEOEC_HOST_PIN=1
step r04_s9_capi_ref_measure_pin5m 120 tools/capi_bench leo_erasure_amd/libleoec_measure.so ref LEOEC_HOST_PIN=1,LEOEC_HOST_PIN_KIB=5120
step r04_s9_capi_ref_measure_default2 120 tools/capi_bench leo_erasure_amd/libleoec_measure.so ref
step r04_s9_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "pinned or staging"
echo "session done"
