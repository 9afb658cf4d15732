#!/bin/bash
# Issue counters of liberation(4,2,7)'s syndrome decode of {0,1}
# (libb_dec_apply<7,4,4,64>, tools/one_op.py) beside its XOR-only access
# pattern (tools/lib_ceiling.hip dec_pattern<4,4,64,false>, decode form 0):
# round-6 verdict item 5, the counter groups of tools/pmc_r5_issue.sh, one
# rocprofv3 --pmc pass per group, plus kernel-trace passes for durations.
#   bash tools/pmc_r6_libdec.sh <tag-prefix>
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd); P=${1:-r06}
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS GRBM_COUNT"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
)
run() {
  local tag=$1 reps=$2; shift 2
  local OUT=$ROOT/gpurun_out/pmc_${P}_$tag; mkdir -p "$OUT"
  local i=0
  for g in "${GROUPS_[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1 || return $?
    i=$((i + 1))
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- "$@" > "$OUT/kt.log" 2>&1 || return $?
}
run lib427_dec 20 python "$ROOT/tools/one_op.py" --coding liberation --k 4 --m 2 --w 7 --objects 1024 --op decode --erased 0,1 --reps 20 || exit $?
run lib427_decpat 20 "$ROOT/tools/lib_ceiling" 1024 20 4 0 || exit $?
cd "$ROOT"
python tools/pmc_summary.py gpurun_out/pmc_${P}_lib427_dec libb_dec_apply > gpurun_out/pmc_${P}_lib427_dec.json
python tools/pmc_summary.py gpurun_out/pmc_${P}_lib427_decpat dec_pattern > gpurun_out/pmc_${P}_lib427_decpat.json
echo pmc done
