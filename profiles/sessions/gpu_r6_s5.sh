#!/bin/bash
# Round 6, session 5: the round's tree (gfbk shipped for >= 4 GB cauchyrs
# launches, pinned forms and the combine A/B form removed): every GPU test,
# smoke, the bench line, the traced bench with its host leg, and the host
# path from 32 to 96 C-ABI callers (whether more callers' packing closes the
# H2D gaps the copy trace attributes to the next batch's packs).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s5_build_tools 300 bash -c "g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl"
step r06_s5_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r06_s5_measure_forms.log
step r06_s5_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 step r06_s5_bench 600 python bench.py
cd /tmp && export TMPDIR=/tmp
step r06_s5_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06_s5_bench_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5
cd $ROOT
TAILN=8 step r06_s5_many_product 400 tools/capi_bench leo_erasure_amd/libleoec.so many
echo "session done"
