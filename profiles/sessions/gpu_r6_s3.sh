#!/bin/bash
# Round 6, session 3: eager hand-off of complete batches (LEOEC_HOSTQ_EAGER,
# the fix the copy trace points at: verdict r5 item 3) A/B at 32 callers
# (three rotated rounds) and at 1-32 callers; its copy trace; the issue
# counters of liberation(4,2,7)'s syndrome decode beside its pattern (item 5).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s3_build_tools 300 bash -c "/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/lib_ceiling tools/lib_ceiling.hip && g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl"
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_EAGER=0" "LEOEC_HOSTQ_EAGER=1")
for r in 0 1 2; do
  for i in 0 1; do
    v=${V[$(( (i + r) % 2 ))]}
    n=$(echo $v | tr ',=' '__')
    TAILN=2 step r06_s3_c32_${n}_$r 120 tools/capi_bench $L c32 $v
  done
done
for v in "${V[@]}"; do
  n=$(echo $v | tr ',=' '__')
  TAILN=8 step r06_s3_few_${n} 200 tools/capi_bench $L few $v
  TAILN=8 step r06_s3_mid_${n} 200 tools/capi_bench $L mid $v
done
cd /tmp && export TMPDIR=/tmp
step r06_s3_capi_copytrace_eager 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/r06_s3_copytrace_eager -o run -- $ROOT/tools/capi_bench $ROOT/$L trace32 LEOEC_HOSTQ_EAGER=1
cd $ROOT
step r06_s3_pmc_libdec 600 bash tools/pmc_r6_libdec.sh r06
echo "session done"
