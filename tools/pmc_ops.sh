#!/bin/bash
# PMC passes over single ops (tools/one_op.py), one counter group per pass,
# each pass under its own time limit; a failure ends the script.
#   OPS="name:one_op args;name2:args" bash tools/pmc_ops.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out/pmc_ops; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE")
IFS=';' read -ra LIST <<< "${OPS}"
for ent in "${LIST[@]}"; do
  name=${ent%%:*}; args=${ent#*:}
  gi=0
  for grp in "${GROUPS_[@]}"; do
    gi=$((gi+1))
    echo "=== $name g$gi: $grp"
    timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/${name}_g$gi" -o run -- python "$ROOT/tools/one_op.py" $args --reps 5 > "$OUT/${name}_g$gi.log" 2>&1
    rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$OUT/${name}_g$gi.log"; exit $rc; }
  done
done
echo "pmc done"
