#!/bin/bash
# Round 3, session 1: (1) the configs[4] access-pattern ceiling over every
# workgroup order (tools/order_ceiling), output kept this time; (2) the
# cauchyrs kernel-form parity test that aborted in round 2, run ONCE with
# glibc's fatal messages and the HIP runtime's errors sent to stderr.  Each
# GPU step is time-limited; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-8} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r03_order_ceiling_64MiB 240 ./tools/order_ceiling 67108864 64 20
step r03_order_ceiling_1MiB 240 ./tools/order_ceiling 1048576 2048 20
export LIBC_FATAL_STDERR_=1 AMD_LOG_LEVEL=1
step r03_cauchy_forms 400 python -u -X faulthandler -m pytest tests/test_gpu_parity.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "cauchy_kernel_forms"
echo "session done"
