#!/bin/bash
# Round 4, first session: the environment facts round 3's verdict asked for
# (can the test process open /dev/tty; which fatal-message route glibc has),
# then smoke, every GPU test and the headline bench on the inherited tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); OUT=$ROOT/gpurun_out; mkdir -p $OUT
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "=== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log"; if [ $rc -ne 0 ]; then exit $rc; fi; }
python - > "$OUT/r04_s1_tty.log" 2>&1 <<'PY'
import os, sys
print("isatty stdin/stdout/stderr:", [os.isatty(f) for f in (0, 1, 2)])
try:
    fd = os.open("/dev/tty", os.O_RDWR | os.O_NOCTTY)
    print("open /dev/tty: OK (fd %d) -> glibc fatal messages go to the tty" % fd)
    os.close(fd)
except OSError as e:
    print("open /dev/tty: FAILED (%s) -> glibc falls back to stderr" % e)
print("ctty (ps -o tty):", os.popen("ps -o tty= -p %d" % os.getpid()).read().strip())
print("sid/pgid:", os.getsid(0), os.getpgid(0))
PY
cat "$OUT/r04_s1_tty.log"
step r04_s1_packet_ceiling_1024 120 tools/packet_ceiling 1024 30
step r04_s1_packet_ceiling_4096 120 tools/packet_ceiling 4096 20
step r04_s1_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step r04_s1_pytest 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread
step r04_s1_bench 600 python bench.py
step r04_s1_e2e_enc_dec 600 python tools/e2e_bench.py --forms "default:;ntcopy:LEOEC_HOSTQ_NTCOPY=1;surv0:LEOEC_HOSTQ_SURVIVORS=0;surv2:LEOEC_HOSTQ_SURVIVORS=2;default2:" --threads 8,16,32 --no-ceiling
echo "session done"
