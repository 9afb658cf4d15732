#!/bin/bash
# PMC passes over one operation (tools/one_op.py), one rocprofv3 run per
# counter group (rocprofv3 does not split counters over passes), plus a
# kernel-trace run for the durations.
#   bash tools/pmc_passes.sh <tag> <one_op args...>
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd); TAG=$1; shift
OUT=$ROOT/gpurun_out/pmc_$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_WAIT_ANY"
  "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_INSTS SQ_INST_CYCLES_SALU SQ_INSTS_SMEM"
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ GRBM_GUI_ACTIVE GRBM_COUNT"
)
i=0
for g in "${GROUPS_[@]}"; do
  timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p$i.log" 2>&1 || exit $?
  i=$((i + 1))
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 20 > "$OUT/kt.log" 2>&1 || exit $?
echo pmc done
