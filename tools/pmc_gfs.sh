#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_gfs; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for op in encode decode; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA --output-format csv -d "$OUT/w32_$op" -o run -- python "$ROOT/tools/one_op.py" --coding vandrs --k 10 --m 4 --w 32 --op $op --reps 5 > "$OUT/w32_$op.log" 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/w32_${op}_kt" -o run -- python "$ROOT/tools/one_op.py" --coding vandrs --k 10 --m 4 --w 32 --op $op --reps 20 > "$OUT/w32_${op}_kt.log" 2>&1 || exit $?
done
echo pmc done
