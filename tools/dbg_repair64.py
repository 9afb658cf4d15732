"""Debug (measurement only): a 64 MiB vandrs(10,4,8) host repair under a given
staging form, printing the engine's status."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
os.environ.setdefault("LEOEC_LIBRARY", "measure")
import leo_erasure_amd as le  # noqa: E402
from gpu_helpers import rand_bytes  # noqa: E402
from oracle import oracle  # noqa: E402

le.gf_init()
for kv in sys.argv[1:]:
    a, b = kv.split("=")
    le._lib.measure_set_knob(a, b)
k, m, w, size = 10, 4, 8, (64 << 20) + 5
data = rand_bytes(size, size + 17 * k)
ref = oracle.encode("vandrs", k, m, w, data)
lost = [0, k + m - 1]
avail = [b for b in range(k + m) if b not in lost]
for i in range(3):
    st, rep = le.nif_repair("vandrs", (k, m, w), [ref[b] for b in avail], avail, lost)
    print(i, st, rep if st != "ok" else (rep == [ref[b] for b in lost]), flush=True)
