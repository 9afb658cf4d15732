#!/bin/bash
# liberation 64-lane tile form: parity tests, then one-process A/Bs at 1 MiB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "liberation_encode_forms or liberation_device_batch"
V="${LV:-;LEOEC_LIB_WG=256}"
step lab7 300 python tools/env_ab.py --coding liberation --k 7 --m 2 --w 7 --erased 0,1 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step lab11 300 python tools/env_ab.py --coding liberation --k 10 --m 2 --w 11 --erased 0,1 --objects 1024 --rounds 6 --reps 10 --variants "$V"
step lab4 300 python tools/env_ab.py --coding liberation --k 4 --m 2 --w 7 --erased 0,1 --objects 1024 --rounds 6 --reps 10 --variants "$V"
echo "session done"
