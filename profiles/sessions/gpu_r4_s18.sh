#!/bin/bash
# Round 4, session 18: the round-end commands on the final tree (smoke, the
# GPU tests without a global timeout, the driver-style bench line), then a
# lone caller's 1 MiB calls.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s18_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s18_pytest 1100 python -m pytest tests/ -x -q -m gpu
step r04_s18_bench 600 python bench.py --steps 20 --warmup 5
step r04_s18_lone 60 tools/capi_bench leo_erasure_amd/libleoec.so lone
echo "session done"
