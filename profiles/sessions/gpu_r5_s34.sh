#!/bin/bash
# Round 5, session 34: the final tree — every GPU test (the NIF shim's load
# default included), smoke, the bench line, a kernel trace of the bench's
# timed region (--no-host: rocprofv3 aborts once the host leg's callers
# call in), and the product's host path from 1 to 32 callers.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s34_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s34_measure_forms.log
step r05_s34_smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
TAILN=1 step r05_s34_bench 600 python bench.py
P=leo_erasure_amd/libleoec.so
TAILN=8 step r05_s34_few_product 240 tools/capi_bench $P few
TAILN=8 step r05_s34_mid_product 240 tools/capi_bench $P mid
cd /tmp && export TMPDIR=/tmp
step r05_s34_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r05_s34_bench_prof -o run -- python $ROOT/bench.py --steps 20 --warmup 5 --no-host
cd $ROOT
python tools/rocprof_summary.py $OUT/r05_s34_bench_prof > $OUT/r05_s34_bench_kernel_summary.txt
echo "session done"
