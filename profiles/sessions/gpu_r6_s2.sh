#!/bin/bash
# Round 6, session 2: the tree after the thread-exit reclaim (no HIP call
# from a thread_local destructor), the always-threaded warm-up and the
# measurement-only pinning forms: every GPU test; the traced bench WITH its
# host leg (verdict r5 item 1); the liberation decode ceiling (item 5) beside
# the engine's decode kernel; the host path's copy trace (item 3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s2_build_tools 300 bash -c "/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/lib_ceiling tools/lib_ceiling.hip && g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl"
step r06_s2_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
step r06_s2_bench_prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/r06_s2_bench_prof -o run -- python3 $ROOT/bench.py --steps 20 --warmup 5
step r06_s2_capi_copytrace 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/r06_s2_copytrace -o run -- $ROOT/tools/capi_bench $ROOT/leo_erasure_amd/libleoec_measure.so trace32
cd $ROOT
TAILN=12 step r06_s2_lib_ceiling_k4 300 tools/lib_ceiling 1024 20 4
TAILN=12 step r06_s2_lib_ceiling_k7 300 tools/lib_ceiling 1024 20 7
TAILN=6 step r06_s2_ab_lib427_dec 300 python tools/env_ab.py --coding liberation --k 4 --m 2 --w 7 --objects 1024 --rounds 4 --erased 0,1 --variants ""
TAILN=6 step r06_s2_ab_lib727_dec 300 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --objects 1024 --rounds 4 --erased 0,1 --variants ""
# the batching queue's batch capacity and depth at 32 callers (item 3's A/B),
# three rotated rounds, one process per run
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_SLOT_KIB=16384" "LEOEC_HOSTQ_SLOT_KIB=8192" "LEOEC_HOSTQ_SLOT_KIB=4096" "LEOEC_HOSTQ_SLOT_KIB=8192,LEOEC_HOSTQ_DEPTH=4" "LEOEC_HOSTQ_SLOT_KIB=4096,LEOEC_HOSTQ_DEPTH=4")
for r in 0 1 2; do
  for i in 0 1 2 3 4; do
    v=${V[$(( (i + r) % 5 ))]}
    n=$(echo $v | tr ',=' '__')
    TAILN=2 step r06_s2_slot_${n}_$r 120 tools/capi_bench $L c32 $v
  done
done
# cauchyrs(10,4,8) forms at more launch sizes (item 4)
V2=";LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_WG=64,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_CBM=6"
for n in 3072 8192; do
  TAILN=9 step r06_s2_ab_cauchy_$n 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects $n --rounds 3 --repair 0,5,10,13 --variants "$V2"
done
echo "session done"
