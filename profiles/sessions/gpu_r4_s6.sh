#!/bin/bash
# Round 4, session 6: the bench line with the scalar CPU leg, and the repair
# output-layout A/B (tools/repair_layout.py), the reference's own 100 MiB
# encode benchmark through the C ABI (tools/ref_encode_bench.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s6_repair_layout 300 python tools/repair_layout.py
step r04_s6_ref_encode 300 python tools/ref_encode_bench.py --forms
step r04_s6_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
