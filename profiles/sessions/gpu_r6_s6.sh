#!/bin/bash
# Round 6, session 6: progressive batch inputs (LEOEC_HOSTQ_PROGRESSIVE: the
# H2D of a batch in runs of packed jobs while its last callers still pack),
# alone and with the eager hand-off; parity of the queue forms first, then
# A/B at 32 callers (three rotated rounds), 32-96 callers, and a copy trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s6_build_tools 300 bash -c "g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl"
step r06_s6_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 300 --timeout-method thread -k "batching_mixed_callers"
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_PROGRESSIVE=0" "LEOEC_HOSTQ_PROGRESSIVE=1" "LEOEC_HOSTQ_PROGRESSIVE=1,LEOEC_HOSTQ_EAGER=1" "LEOEC_HOSTQ_PROGRESSIVE=1,LEOEC_HOSTQ_EAGER=1,LEOEC_HOSTQ_PROG_KIB=2048")
for r in 0 1 2; do
  for i in 0 1 2 3; do
    v=${V[$(( (i + r) % 4 ))]}
    n=$(echo $v | tr ',=' '__')
    TAILN=2 step r06_s6_c32_${n}_$r 120 tools/capi_bench $L c32 $v
  done
done
TAILN=8 step r06_s6_many_prog 400 tools/capi_bench $L many LEOEC_HOSTQ_PROGRESSIVE=1,LEOEC_HOSTQ_EAGER=1
TAILN=8 step r06_s6_many_base 400 tools/capi_bench $L many LEOEC_HOSTQ_PROGRESSIVE=0
cd /tmp && export TMPDIR=/tmp
step r06_s6_copytrace_prog 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/r06_s6_copytrace_prog -o run -- $ROOT/tools/capi_bench $ROOT/$L trace32 LEOEC_HOSTQ_PROGRESSIVE=1,LEOEC_HOSTQ_EAGER=1
echo "session done"
