#!/bin/bash
# Round 4, session 8: the host path on the system HIP runtime (no torch in
# the process, as under an Erlang VM) against torch's bundled runtime: the
# large-object copy arrangements and the C ABI itself (tools/capi_bench.cpp).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
TL=$(python -c "import os, torch; print(os.path.join(os.path.dirname(torch.__file__), 'lib'))")
mkdir -p /tmp/torchhip && ln -sf "$TL/libamdhip64.so" /tmp/torchhip/libamdhip64.so.7
TORCHRT="env LD_LIBRARY_PATH=/tmp/torchhip:$TL"
step r04_s8_copy_sys 180 tools/large_copy_probe 100 5
step r04_s8_copy_torchrt 180 $TORCHRT tools/large_copy_probe 100 5
step r04_s8_capi_ref_sys 180 tools/capi_bench leo_erasure_amd/libleoec.so ref
step r04_s8_capi_ref_torchrt 180 $TORCHRT tools/capi_bench leo_erasure_amd/libleoec.so ref
step r04_s8_capi_callers_sys 180 tools/capi_bench leo_erasure_amd/libleoec.so callers
step r04_s8_capi_callers_torchrt 180 $TORCHRT tools/capi_bench leo_erasure_amd/libleoec.so callers
echo "session done"
