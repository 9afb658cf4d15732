#!/bin/bash
# Round 4, cauchyrs 16-byte swap form (gfbs_apply, LEOEC_GFBIT_FORM=4): the
# measurement-form parity tests, an interleaved A/B against the shipped
# 8-byte-lane kernel at 1,024 and 4,096 objects, and the vector-memory
# instruction count of both (PMC, one pass per counter group); then (was
# gpu_r4_s3.sh) configs[4]'s bench line, a 2-rank rehearsal of the N > 1
# line, and the rocprof summaries of both bench workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
export LEOEC_LIBRARY=measure
step r04_s2_swap_forms 600 python -u -m pytest tests/test_measure_forms.py -m measure_gpu -x -q --timeout 120 --timeout-method thread -k "cauchy"
V=";LEOEC_GFBIT_FORM=4;LEOEC_GFBIT_FORM=4,LEOEC_GFBIT_PF=0;LEOEC_GFBIT_FORM=4,LEOEC_GFBIT_WG=128;LEOEC_GFBIT_FORM=4,LEOEC_GFBIT_WG=512"
TAILN=12 step r04_s2_ab_swap_1024 600 python tools/env_ab.py --coding cauchyrs --objects 1024 --rounds 5 --variants "$V"
TAILN=12 step r04_s2_ab_swap_4096 600 python tools/env_ab.py --coding cauchyrs --objects 4096 --rounds 3 --variants "$V"
# host path: non-temporal packing (now shipped) against memcpy, interleaved
TAILN=6 step r04_s2_e2e_ntcopy_ab 600 python tools/e2e_bench.py --forms "nt:;memcpy:LEOEC_HOSTQ_NTCOPY=0;nt2:;memcpy2:LEOEC_HOSTQ_NTCOPY=0" --threads 1,4,8,16,32 --no-ceiling
unset LEOEC_LIBRARY
cd /tmp && export TMPDIR=/tmp
pmc() {
  local tag=$1; shift
  local D=$OUT/pmc_$tag; mkdir -p "$D"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d "$D/p0" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$D/p0.log" 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$D/p1" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$D/p1.log" 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum --output-format csv -d "$D/p2" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 5 > "$D/p2.log" 2>&1 || return $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$D/kt" -o run -- python "$ROOT/tools/one_op.py" "$@" --reps 20 > "$D/kt.log" 2>&1 || return $?
}
pmc cauchy_shipped --coding cauchyrs --op encode || exit $?
pmc cauchy_swap --coding cauchyrs --op encode --knobs LEOEC_GFBIT_FORM=4 || exit $?
cd "$ROOT"
python tools/pmc_summary.py gpurun_out/pmc_cauchy_shipped gfbit_apply > gpurun_out/pmc_cauchy_shipped.json
python tools/pmc_summary.py gpurun_out/pmc_cauchy_swap gfbs_apply > gpurun_out/pmc_cauchy_swap.json
cd "$ROOT"
step r04_s3_bench64 600 python bench.py --workload 64MiB --no-cpu
step r04_s3_bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10 --no-cpu
cd /tmp && export TMPDIR=/tmp
step r04_s3_prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/r04_prof" -o run -- python "$ROOT/bench.py" --no-cpu
step r04_s3_prof64 600 rocprofv3 --kernel-trace --stats -d "$OUT/r04_prof64" -o run -- python "$ROOT/bench.py" --workload 64MiB --no-cpu
cd "$ROOT"
python tools/rocprof_summary.py "$OUT/r04_prof" > "$OUT/r04_bench_kernel_summary.txt"
python tools/rocprof_summary.py "$OUT/r04_prof64" > "$OUT/r04_bench64_kernel_summary.txt"
echo "session done"
