#!/bin/bash
# Round 5, session 4: the syndrome kernel's block form (absent shards
# skipped by a uniform branch, LEOEC_LIB_DEC_LA=0) against the streaming
# form and the shipped lib_dec_apply, decode of two data blocks and repair
# of {data, P}, on the five liberation shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s4_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 120 --timeout-method thread -k "liberation or tile or host_batching"
V=";LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64,LEOEC_LIB_DEC_LA=0;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_LA=0;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64,LEOEC_LIB_DEC_LA=4"
for cfg in "7 2 7 0,7" "4 2 7 0,4" "10 2 11 0,10" "5 2 5 0,5" "13 2 13 0,13"; do
  set -- $cfg
  TAILN=2 step r05_s4_ab_lib_$1_$3 600 python tools/env_ab.py --coding liberation --k $1 --m $2 --w $3 --erased 0,1 --repair $4 --objects 1024 --rounds 5 --variants "$V"
done
# the bench line with this round's legs: host-memory C-ABI callers, the
# pattern ceiling in its own process, the max-leg CPU baseline
step r05_s4_bench 600 python bench.py --steps 20 --warmup 5
echo "session done"
