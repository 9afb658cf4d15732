#!/bin/bash
# cauchyrs(10,4,8) encode at the reference's 1 MiB geometry (packets of
# 13,120 B: odd packets start mid line) against 1,054,720-B objects (13,184-B
# packets, line-aligned), and the vandrs gf8 encode for reference: SQ / TA /
# TCP / TD / TCC counters, one rocprofv3 pass per group (tools/one_op.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum"
  "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
  "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"
)
run() {
  local tag=$1; shift
  local OUT=$ROOT/gpurun_out/pmc_$tag; mkdir -p "$OUT"
  local i=0
  for g in "${GROUPS_[@]}"; do
    timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p$i.log" 2>&1 || return $?
    i=$((i + 1))
  done
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 20 > "$OUT/kt.log" 2>&1 || return $?
}
run cauchy_ref --coding cauchyrs --k 10 --m 4 --w 8 --op encode --size 1048576 || exit $?
run cauchy_aligned --coding cauchyrs --k 10 --m 4 --w 8 --op encode --size 1054720 || exit $?
run gf8_ref --coding vandrs --k 10 --m 4 --w 8 --op encode --size 1048576 || exit $?
cd "$ROOT"
for t in cauchy_ref cauchy_aligned; do python tools/pmc_summary.py gpurun_out/pmc_$t gfbit_apply > gpurun_out/pmc_$t.json; done
python tools/pmc_summary.py gpurun_out/pmc_gf8_ref gf8_apply > gpurun_out/pmc_gf8_ref.json
echo pmc done
