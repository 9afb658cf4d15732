#!/bin/bash
# Round 6, session 18: vandrs RS(10,4,8) encode / decode / repair of the
# shipped kernels at 1,024 and 2,048 objects in one process each (session
# 16's suite read decode 0.742 at 1,024 objects where the bench line on the
# same box read 0.794 at 2,048).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
for n in 1024 2048 4096; do
  TAILN=3 step r06_s18_vandrs_$n 300 python tools/env_ab.py --coding vandrs --k 10 --m 4 --w 8 --objects $n --rounds 4 --repair 0,5,10,13 --variants ""
done
echo "session done"
