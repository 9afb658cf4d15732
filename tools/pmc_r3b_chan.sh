#!/bin/bash
# vandrs RS(10,4,8) encode (gf8_apply), 1 MiB x 2048 against 64 MiB x 64:
# HBM requests, DRAM credit stalls and L2 busy (rocprofv3 reports these
# summed over the L2 channels).  One rocprofv3 pass per group.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
run() {
  local tag=$1; shift
  local OUT=$ROOT/gpurun_out/pmcch_$tag; mkdir -p "$OUT"
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ TCC_EA0_WRREQ --output-format csv -d "$OUT/p0" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p0.log" 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_CREDIT_STALL TCC_EA0_WRREQ_DRAM_CREDIT_STALL --output-format csv -d "$OUT/p1" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p1.log" 2>&1 || return $?
  timeout -s KILL 120 rocprofv3 --pmc TCC_BUSY TCC_CYCLE --output-format csv -d "$OUT/p2" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$OUT/p2.log" 2>&1 || return $?
}
run gf8_1MiB --coding vandrs --k 10 --m 4 --w 8 --op encode --size 1048576 --objects 2048 || exit $?
run gf8_64MiB --coding vandrs --k 10 --m 4 --w 8 --op encode --size 67108864 --objects 64 || exit $?
echo pmc done
