#!/bin/bash
# Zero-copy batches (LEOEC_HOSTQ_ZC=1): parity, then 4-32 callers A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-2} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_zcq_parity 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "host_batching or host_staging or concurrent"
step r03_zcq_e2e 600 python tools/e2e_bench.py --forms "dma:;zc:LEOEC_HOSTQ_ZC=1;dma2:;zc2:LEOEC_HOSTQ_ZC=1" --threads 8,16,32
echo "session done"
