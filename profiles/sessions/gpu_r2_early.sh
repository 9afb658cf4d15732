#!/bin/bash
# gf8 early-load form A/B (variants 1 = shipped, 36 = loads before LDS
# staging, 37 = 36 + buffer ld/st) at 1 MiB x 2048 and 64 MiB x 64, one
# process each.  Each step time-limited; a failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
V="LEOEC_GF8_VARIANT=1;LEOEC_GF8_VARIANT=36;LEOEC_GF8_VARIANT=37"
step early1 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 1048576 --objects 2048 --rounds 8 --reps 10 --variants "$V"
step early64 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 67108864 --objects 64 --rounds 8 --reps 8 --variants "$V"
step early1b 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 1048576 --objects 2048 --rounds 8 --reps 10 --variants "LEOEC_GF8_VARIANT=36;LEOEC_GF8_VARIANT=1"
echo "session done"
