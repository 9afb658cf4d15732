#!/bin/bash
# One GPU session on the MI355X box: smoke, parity tests, bench, rocprof.
# Every GPU step has its own time limit; a crash / fault / timeout stops the
# script (no further GPU work), an ordinary test failure does not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-smoke,test,bench1,prof}

fatal() {  # exit codes that mean the GPU step crashed or hung
  case "$1" in 124|134|137|139|143) return 0;; esac
  [ "$1" -gt 128 ] && return 0
  return 1
}

run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if fatal $rc; then echo "FATAL in $name, stopping"; exit $rc; fi
  return $rc
}

[[ $STEPS == *smoke* ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *test* ]] && run pytest 1200 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-}
[[ $STEPS == *bench1* ]] && run bench 600 python bench.py ${BENCH_ARGS:-}
[[ $STEPS == *bench2* ]] && run bench2 600 python bench.py --gpus 2 --oversubscribe --steps 50 --warmup 10
[[ $STEPS == *e2e* ]] && run e2e 900 python tools/e2e_bench.py ${E2E_ARGS:---quick}
[[ $STEPS == *bench64* ]] && run bench64 600 python bench.py --workload 64MiB --steps 50 --warmup 10 --no-cpu
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
      python "$ROOT/bench.py" --steps 10 --no-cpu
  cd "$ROOT"
fi
if [[ $STEPS == *pmc* ]]; then
  # HBM bytes of the bench kernel: FETCH_SIZE and WRITE_SIZE in separate
  # passes (TCC slots), 1 MiB x 2048 and configs[4]'s 64 x 64 MiB; the JSON
  # records are stamped with the gf8_apply<10,4> code object they ran on
  cd /tmp && export TMPDIR=/tmp
  for wl in 1MiB 64MiB; do
    for c in FETCH_SIZE WRITE_SIZE; do
      run pmc_${wl}_$c 120 rocprofv3 --pmc $c --output-format csv -d "$OUT/pmc_${wl}_$c" -o run -- \
          python "$ROOT/bench.py" --workload $wl --steps 3 --warmup 1 --warmup-s 0 --no-cpu
    done
  done
  cd "$ROOT"
  python tools/pmc_traffic.py "$OUT" --fetch pmc_1MiB_FETCH_SIZE --write pmc_1MiB_WRITE_SIZE \
      > "$OUT/pmc_traffic.json"
  python tools/pmc_traffic.py "$OUT" --objects 64 --object-bytes 67108864 \
      --fetch pmc_64MiB_FETCH_SIZE --write pmc_64MiB_WRITE_SIZE > "$OUT/pmc_traffic_64MiB.json"
fi
echo "session done"
