#!/bin/bash
# Experiment session: variant A/B + PMC traffic passes (each step time-limited;
# a crash or timeout ends the script).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p "$OUT"
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -15 "$OUT/$name.log"; if [ $rc -ne 0 ] && { [ $rc -ge 124 ] || [ $rc -gt 128 ]; }; then exit $rc; fi; return 0; }
IFS=',' read -ra PARTS <<< "${EXP:-variants,pmc}"
for p in "${PARTS[@]}"; do
  case $p in
    variants) step variants 600 python tools/kvariants.py ${KV_ARGS:-} ;;
    pytest) step pytest 1200 python -m pytest tests -x -q -m gpu ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} ;;
    suite) step suite 900 python tools/bench_suite.py ${SUITE_ARGS:-} ;;
    e2e) step e2e 600 python tools/e2e_bench.py ;;
    bench_driver) step bench_driver 600 python bench.py --steps 20 --warmup 5 ;;
    bench64) step bench64 600 python bench.py --workload 64MiB --no-cpu ;;
    prof64)
      cd /tmp && export TMPDIR=/tmp
      step prof64_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof64_csv" -o run -- python "$ROOT/bench.py" --workload 64MiB --no-cpu
      cd "$ROOT" ;;
    layout) step layout 600 python tools/layout_exp.py ${LAYOUT_ARGS:-} ;;
    ab) step ab 900 python tools/env_ab.py ${AB_ARGS:-} ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    counters)
      cd /tmp && export TMPDIR=/tmp
      step counters_list 300 rocprofv3 -L
      step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 1 --warmup-s 0 --no-cpu
      cd "$ROOT" ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 1 --warmup-s 0 --no-cpu
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 1 --warmup-s 0 --no-cpu
      step prof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_csv" -o run -- python "$ROOT/bench.py" --no-cpu
      cd "$ROOT" ;;
  esac
done
echo "exp done"
