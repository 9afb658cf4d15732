#!/bin/bash
# Round 5, session 37: the final tree after the in-place pinning form went
# back to the measurement build: every GPU test twice (a state-dependent
# failure would show), smoke, the bench line, the product's host path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s37_pytest_a 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s37_measure_forms_a.log
step r05_s37_pytest_b 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s37_measure_forms_b.log
step r05_s37_smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r05_s37_bench 600 python bench.py
TAILN=9 step r05_s37_few_product 240 tools/capi_bench leo_erasure_amd/libleoec.so few
TAILN=9 step r05_s37_mid_product 240 tools/capi_bench leo_erasure_amd/libleoec.so mid
echo "session done"
