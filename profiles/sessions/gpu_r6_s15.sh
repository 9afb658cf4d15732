#!/bin/bash
# Round 6, session 15: gfbk_apply over block pairs (LEOEC_GFBIT_PAIR=1: the
# terms of two blocks for one coefficient bit added by one 3-input XOR,
# -27 % of the accumulating XORs on cauchyrs(10,4,8) encode) — parity first,
# then interleaved A/B against the shipped kernel and gfbk at 1,024 / 2,048 /
# 4,096 objects.  Session 14 ran an if / else-if form of the same
# arithmetic: 0.37-0.44 of 8 TB/s, its accumulators copied between paths
# (13,000 AGPR copies and 20,000 moves in the code object); this form has
# three independent triangles (739 / 549).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r06_s15_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 300 --timeout-method thread -k "16B_forms_batches"
V=";LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_WG=64,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_PAIR=1,LEOEC_GFBIT_PF=2;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_PAIR=1,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_PAIR=1,LEOEC_GFBIT_PF=4"
for n in 2048 1024 4096; do
  TAILN=15 step r06_s15_ab_pair_$n 500 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects $n --rounds 4 --repair 0,5,10,13 --variants "$V"
done
echo "session done"
