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
[[ $STEPS == *bench64* ]] && run bench64 600 python bench.py --workload 64MiB --steps 50 --warmup 10 --no-cpu
if [[ $STEPS == *prof* ]]; then
  cd /tmp && export TMPDIR=/tmp
  run rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run -- \
      python "$ROOT/bench.py" --steps 10 --no-cpu
  cd "$ROOT"
fi
echo "session done"
