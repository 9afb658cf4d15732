#!/bin/bash
# Round 4, session 14: the chunked zero-copy form (LEOEC_ZC_CHUNKS) for a
# lone caller's 1 MiB encode / decode, interleaved processes; its form tests
# (measurement library, own process); the product GPU tests and smoke.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s14_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "chunks or pinned or staging or mixed"
for r in 1 2; do
  for c in 1 2 3 4; do
    step r04_s14_lone_c${c}_r${r} 60 tools/capi_bench leo_erasure_amd/libleoec_measure.so lone LEOEC_ZC_CHUNKS=$c
  done
done
step r04_s14_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s14_pytest 1100 python -m pytest tests/ -x -q -m gpu
echo "session done"
