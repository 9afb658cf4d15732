#!/bin/bash
# Round 4, final tree (swap form removed, non-temporal packing for gathered
# inputs only): smoke, every GPU test, the headline bench, and the host path
# A/B (shipped packing against memcpy, interleaved) at 1 / 8 / 16 / 32
# callers, encode and decode.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s3_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s3_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
cp "$OUT/measure_forms.log" "$OUT/r04_s3_measure_forms.log" 2>/dev/null || true
step r04_s3_bench 600 python bench.py
step r04_s3_bench_driver 600 python bench.py --steps 20 --warmup 5
TAILN=6 step r04_s3_e2e_ab 600 python tools/e2e_bench.py --forms "shipped:;memcpy:LEOEC_HOSTQ_NTCOPY=0;shipped2:;memcpy2:LEOEC_HOSTQ_NTCOPY=0" --threads 1,8,16,32 --no-ceiling
echo "session done"
