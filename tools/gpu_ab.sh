#!/bin/bash
# Short GPU call: selected parity tests, then env A/Bs (each step time-limited,
# a crash / timeout ends the script).  TESTS = pytest -k expression ("" = skip),
# AB_n = env_ab.py argument strings, run in order.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -${TAILN:-25} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
if [ -n "${TESTS:-}" ]; then
  step tests 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "$TESTS"
fi
for i in 1 2 3 4 5 6; do
  v="AB_$i"; [ -n "${!v:-}" ] || continue
  eval "step ab$i 600 python tools/env_ab.py ${!v}"
done
echo "ab done"
