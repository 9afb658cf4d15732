#!/bin/bash
# Round 4, session 7: where the first (cold) call of the reference's 100 MiB
# encode benchmark spends its time (plain run, then the HIP API + kernel
# trace of the same), and the HBM bytes of the liberation kernels (one PMC
# counter group per pass), and the copy arrangements a large-object host
# path could use (tools/large_copy_probe.cpp).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
step r04_s7_large_copy 120 tools/large_copy_probe 100 5
step r04_s7_cold 300 python tools/ref_encode_bench.py --cold-only
step r04_s7_cold_trace 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $OUT/r04_s7_trace -- python tools/ref_encode_bench.py --cold-only --reps 2
LIB="--coding liberation --k 7 --m 2 --w 7 --reps 5 --objects 1024"
step r04_s7_pmc_lib_enc_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04_s7_pmc_lib_enc_fetch -- python tools/one_op.py $LIB --op encode
step r04_s7_pmc_lib_enc_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04_s7_pmc_lib_enc_write -- python tools/one_op.py $LIB --op encode
step r04_s7_pmc_lib_dec_fetch 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/r04_s7_pmc_lib_dec_fetch -- python tools/one_op.py $LIB --op decode --erased 0,1
step r04_s7_pmc_lib_dec_write 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/r04_s7_pmc_lib_dec_write -- python tools/one_op.py $LIB --op decode --erased 0,1
echo "session done"
