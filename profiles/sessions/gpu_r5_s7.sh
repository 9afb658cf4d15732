#!/bin/bash
# Round 5, session 7: where the RS(10,4,8) repair's gap to encode comes from
# (map density against output layout, tools/repair_probe.py), and the bench
# line with the host-memory leg's three-way PCIe copy rates.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TAILN=12 step r05_s7_repair_probe 300 python tools/repair_probe.py
step r05_s7_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
