#!/bin/bash
# Issue counters of the liberation kernels beside gf8_apply<10,4> (round-5
# verdict item 1): one rocprofv3 --pmc pass per counter group (tools/one_op.py,
# 1,024 x 1 MiB objects), plus a kernel-trace pass for the durations.
#   bash tools/pmc_r5_issue.sh <tag-prefix>
# EXTRA: more one_op.py arguments for the liberation runs (e.g. --knobs
# LEOEC_LIB_BUF=1); ENC_K / DEC_K: kernel-name fragments of their kernels;
# GF8=0 skips the gf8 reference run.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd); P=${1:-r05}
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS GRBM_COUNT"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
)
run() {
  local tag=$1; shift
  local OUT=$ROOT/gpurun_out/pmc_${P}_$tag; mkdir -p "$OUT"
  local i=0
  for g in "${GROUPS_[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p$i.log" 2>&1 || return $?
    i=$((i + 1))
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 20 > "$OUT/kt.log" 2>&1 || return $?
}
LIB="--coding liberation --k 7 --m 2 --w 7 --objects 1024"
if [ "${GF8:-1}" = 1 ]; then
  run gf8_enc --coding vandrs --k 10 --m 4 --w 8 --op encode --objects 1024 || exit $?
fi
run lib_enc $LIB --op encode ${EXTRA:-} || exit $?
run lib_dec $LIB --op decode --erased 0,1 ${EXTRA:-} || exit $?
run lib_rep $LIB --op repair --erased 0,7 ${EXTRA:-} || exit $?
cd "$ROOT"
if [ "${GF8:-1}" = 1 ]; then
  python tools/pmc_summary.py gpurun_out/pmc_${P}_gf8_enc gf8_apply > gpurun_out/pmc_${P}_gf8_enc.json
fi
python tools/pmc_summary.py gpurun_out/pmc_${P}_lib_enc ${ENC_K:-lib_apply} > gpurun_out/pmc_${P}_lib_enc.json
python tools/pmc_summary.py gpurun_out/pmc_${P}_lib_dec ${DEC_K:-lib_dec_apply} > gpurun_out/pmc_${P}_lib_dec.json
python tools/pmc_summary.py gpurun_out/pmc_${P}_lib_rep bit_apply > gpurun_out/pmc_${P}_lib_rep.json
echo pmc done
