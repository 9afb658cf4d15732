#!/bin/bash
# Round 5, session 17: cauchyrs(10,4,8) in the register regime of the one
# access pattern that read 0.77 on its geometry (packet_ceiling pattern<4,128>:
# 16-byte lanes, K compiled in, 276 VGPRs = one wave per SIMD).  gfbk_apply
# (LEOEC_GFBIT_FORM=5: the shipped bitsliced arithmetic, K = 10 compiled in,
# branch-free buffer loads, 1..3 blocks in flight) and the compiled-bitmatrix
# encode at one wave per SIMD with 32 / 48 packets in flight (CBM=6..9),
# parity first, then interleaved A/B at 1,024 and 4,096 objects.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r05_s17_forms 600 env LEOEC_LIBRARY=measure python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 120 --timeout-method thread -k "16B_forms_batches or compiled_bitmatrix or cauchy_kernel_forms"
V=";LEOEC_GFBIT_FORM=5;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_PF=2;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_WG=64,LEOEC_GFBIT_PF=3;LEOEC_GFBIT_FORM=5,LEOEC_GFBIT_WG=256;LEOEC_GFBIT_CBM=1;LEOEC_GFBIT_CBM=6;LEOEC_GFBIT_CBM=7;LEOEC_GFBIT_CBM=8;LEOEC_GFBIT_CBM=9"
TAILN=24 step r05_s17_ab_cauchy_1024 600 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects 1024 --rounds 4 --variants "$V"
TAILN=24 step r05_s17_ab_cauchy_4096 600 python tools/env_ab.py --coding cauchyrs --k 10 --m 4 --w 8 --objects 4096 --rounds 3 --variants "$V"
echo "session done"
