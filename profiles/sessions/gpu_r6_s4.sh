#!/bin/bash
# Round 6, session 4: the tree with gfbk_apply shipped for cauchyrs(10,4,8)
# launches of >= 4 GB (verdict r5 item 4) and the worker's H2D wait cut short
# by a handed-over batch: every GPU test (with the new large-launch parity
# test); the eager hand-off A/B again at 32 callers and its copy trace
# (item 3); the gfbk threshold against the old path at 2,048-3,072 objects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s4_build_tools 300 bash -c "g++ -O2 -std=c++17 -pthread -o tools/capi_bench tools/capi_bench.cpp -ldl"
step r06_s4_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread
L=leo_erasure_amd/libleoec_measure.so
V=("LEOEC_HOSTQ_EAGER=0" "LEOEC_HOSTQ_EAGER=1")
for r in 0 1 2; do
  for i in 0 1; do
    v=${V[$(( (i + r) % 2 ))]}
    n=$(echo $v | tr ',=' '__')
    TAILN=2 step r06_s4_c32_${n}_$r 120 tools/capi_bench $L c32 $v
  done
done
TAILN=8 step r06_s4_few_eager1 200 tools/capi_bench $L few LEOEC_HOSTQ_EAGER=1
TAILN=8 step r06_s4_mid_eager1 200 tools/capi_bench $L mid LEOEC_HOSTQ_EAGER=1
cd /tmp && export TMPDIR=/tmp
step r06_s4_capi_copytrace_eager 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/r06_s4_copytrace_eager -o run -- $ROOT/tools/capi_bench $ROOT/$L trace32 LEOEC_HOSTQ_EAGER=1
cd $ROOT
V2=";LEOEC_GFBK_MIN_MIB=99999999"
for n in 2048 2560 2816 3072; do
  TAILN=6 step r06_s4_ab_gfbk_$n 300 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects $n --rounds 4 --repair 0,5,10,13 --variants "$V2"
done
# liberation syndrome decode: masked vs set-bit combine (item 5's counters:
# the kernel issues 3.2x the pattern's VALU instructions, memory identical)
V3=";LEOEC_LIB_DEC_COMBINE=1"
TAILN=6 step r06_s4_ab_lib427_combine 300 python tools/env_ab.py --coding liberation --k 4 --m 2 --w 7 --objects 1024 --rounds 4 --erased 0,1 --variants "$V3"
TAILN=6 step r06_s4_ab_lib727_combine 300 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --objects 1024 --rounds 4 --erased 0,1 --repair 0,7 --variants "$V3"
echo "session done"
