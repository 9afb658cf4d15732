#!/bin/bash
# Large-object tile-map session: parity tests touching the gf8 tile maps, then
# one-process A/Bs at 16 / 32 / 64 MiB and the configs[4] bench line.  Every
# GPU step is time-limited; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  -k "segment_map or 64MiB or xcd_object_map or tile_width or device_encode_batch"
V="LEOEC_GF8_TMAP=0;;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=64;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=256;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=512;LEOEC_GF8_VARIANT=35;LEOEC_GF8_VARIANT=35,LEOEC_GF8_TMAP=0"
step ab64 400 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 67108864 --objects 64 --rounds 6 --reps 8 --variants "$V"
step ab32 400 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 33554432 --objects 128 --rounds 6 --reps 8 --variants "LEOEC_GF8_TMAP=0;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=128;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=256"
step ab16 400 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --size 16777216 --objects 256 --rounds 6 --reps 8 --variants "LEOEC_GF8_TMAP=0;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=128;LEOEC_GF8_TMAP=4,LEOEC_GF8_TGROUP=256"
step bench64 300 python bench.py --workload 64MiB --steps 50 --warmup 10 --no-cpu
cd /tmp && export TMPDIR=/tmp
step prof64 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof64" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --workload 64MiB --steps 20 --warmup 5 --no-cpu
cd "$GRAFT_REPO_ROOT"
OPS="cauchyenc:--coding cauchyrs --op encode;gf8enc64:--coding vandrs --size 67108864 --objects 64 --op encode" step pmc 400 bash tools/pmc_ops.sh
echo "session done"
