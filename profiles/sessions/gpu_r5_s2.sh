#!/bin/bash
# Round 5, session 2: the branch-free liberation kernels (libb_apply /
# libb_dec_apply, measurement build, LEOEC_LIB_BUF=1): every GPU test (the new
# forms in the measurement child), then interleaved A/B against the shipped
# lib_apply / lib_dec_apply on liberation (7,2,7), (4,2,7), (10,2,11) at
# 1,024 x 1 MiB, liberation's XOR-only access-pattern ceiling
# (tools/lib_ceiling.hip), then the issue counters of the new forms and of
# repair.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s2_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r05_s2_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
cp $OUT/measure_forms.log $OUT/r05_s2_measure_forms.log
TAILN=16 step r05_s2_lib_ceiling_727 300 tools/lib_ceiling 1024 20 7
TAILN=16 step r05_s2_lib_ceiling_427 300 tools/lib_ceiling 1024 20 4
V=";LEOEC_LIB_BUF=1;LEOEC_LIB_BUF=1,LEOEC_LIB_LA=4;LEOEC_LIB_BUF=1,LEOEC_LIB_LA=8;LEOEC_LIB_BUF=1,LEOEC_LIB_WG=256;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_LA=4;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64;LEOEC_LIB_BUF=1,LEOEC_LIB_DEC_WG=64,LEOEC_LIB_DEC_LA=4"
TAILN=16 step r05_s2_ab_lib727 600 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --erased 0,1 --objects 1024 --rounds 4 --variants "$V"
TAILN=16 step r05_s2_ab_lib427 600 python tools/env_ab.py --coding liberation --k 4 --m 2 --w 7 --erased 0,1 --objects 1024 --rounds 4 --variants "$V"
TAILN=16 step r05_s2_ab_lib10211 600 python tools/env_ab.py --coding liberation --k 10 --m 2 --w 11 --erased 0,1 --objects 1024 --rounds 4 --variants "$V"
export EXTRA="--knobs LEOEC_LIB_BUF=1" ENC_K=libb_apply DEC_K=libb_dec_apply GF8=0
step r05_s2_pmc_issue_buf 900 bash tools/pmc_r5_issue.sh r05buf
echo "session done"
