#!/bin/bash
# Round 4, session 15: the chunked zero-copy form with the decode's survivor
# copies overlapped, A/B against one piece (interleaved processes), and the
# product library with it shipped (2 chunks): lone caller, multi-caller,
# smoke, GPU tests, driver-style bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for r in 1 2 3; do
  for c in 1 2; do
    step r04_s15_lone_c${c}_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_ZC_CHUNKS=$c
  done
done
step r04_s15_lone_product 60 tools/capi_bench leo_erasure_amd/libleoec.so lone
step r04_s15_callers_product 180 tools/capi_bench leo_erasure_amd/libleoec.so callers
step r04_s15_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
step r04_s15_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s15_pytest 1100 python -m pytest tests/ -x -q -m gpu
step r04_s15_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
