#!/bin/bash
# Round 4, session 12: gf_init now also creates the device's batching queue
# and pools of streams / mapped buffers: the first calls of new threads and
# the reference's one-call benchmark again, then the round-end commands
# (smoke, GPU tests, driver-style bench) and the 2-rank rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s12_threads 120 tools/capi_bench leo_erasure_amd/libleoec.so threads
step r04_s12_capi_ref 120 tools/capi_bench leo_erasure_amd/libleoec.so ref
step r04_s12_capi_callers 180 tools/capi_bench leo_erasure_amd/libleoec.so callers
step r04_s12_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s12_pytest 1100 python -m pytest tests/ -x -q -m gpu
step r04_s12_bench 600 python bench.py --steps 20 --warmup 5
step r04_s12_bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10 --no-cpu
echo "session done"
