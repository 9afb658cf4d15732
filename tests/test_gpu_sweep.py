"""Seeded random sweep of the parameter space the reference accepts
(c_src/common.cpp checkParams, every coding class, k / m / w / object size
drawn at random and kept when the oracle's check_params accepts them):
host-memory encode / decode / repair through the C ABI and device-resident
batches, each against the CPU oracle, bit-exact.  The fixed configuration
tables of test_gpu_parity.py cover the reference's own test configurations;
this covers the space between them (odd k, every w the classes take, sizes
from one byte to 3 MiB, random survivor orders and erasure sets).
"""
import random

import pytest

from gpu_helpers import batch as _batch
from gpu_helpers import rand_bytes

pytestmark = pytest.mark.gpu

N_CHUNKS, PER_CHUNK = 6, 20


def _draw(rng, oracle):
    """One accepted (class, k, m, w, size)."""
    while True:
        cls = rng.choice(["vandrs", "vandrs", "isars", "cauchyrs", "liberation"])
        if cls == "vandrs":
            w, k, m = rng.choice([8, 8, 16, 32]), rng.randint(1, 20), rng.randint(1, 6)
        elif cls == "isars":
            w, k, m = 8, rng.randint(1, 20), rng.randint(1, 6)
        elif cls == "cauchyrs":
            w, k, m = rng.randint(2, 16), rng.randint(1, 12), rng.randint(1, 5)
        else:
            w = rng.choice([3, 5, 7, 11, 13, 17])
            k, m = rng.randint(1, min(w, 12)), 2
        if oracle.check_params(cls, k, m, w) != 0:
            continue
        size = rng.choice([rng.randint(1, 4096), rng.randint(4097, 1 << 20),
                           rng.randint((1 << 20) + 1, 3 << 20)])
        return cls, k, m, w, size


@pytest.mark.parametrize("chunk", range(N_CHUNKS))
def test_host_random_sweep(gpu, le, oracle, chunk):
    rng = random.Random(0x5EED + chunk)
    for _ in range(PER_CHUNK):
        cls, k, m, w, size = _draw(rng, oracle)
        case = (cls, k, m, w, size)
        data = rand_bytes(size, rng.randrange(1 << 30))
        ref = oracle.encode(cls, k, m, w, data)
        st, blocks = le.nif_encode(cls, (k, m, w), data, size)
        assert st == "ok" and blocks == ref, case
        # decode from a random survivor set (k .. k + m blocks, random order)
        ids = rng.sample(range(k + m), rng.randint(k, k + m))
        st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, size)
        assert st == "ok" and out == data, (case, ids)
        # repair 1 .. m lost blocks from a random survivor set of >= k others
        lost = rng.sample(range(k + m), rng.randint(1, m))
        rest = [b for b in range(k + m) if b not in lost]
        avail = rng.sample(rest, rng.randint(k, len(rest)))
        st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
        assert st == "ok" and rep == [ref[b] for b in lost], (case, avail, lost)


@pytest.mark.parametrize("chunk", range(3))
def test_device_random_sweep(gpu, le, oracle, chunk):
    """Device-resident batches: random object counts, sizes and row strides
    (multiples of 16), encode against the oracle on sampled objects, then an
    in-place decode of a random erasure set of at most m blocks (data blocks
    poisoned first) restoring every byte of every object."""
    rng = random.Random(0xDE71CE + chunk)
    for _ in range(PER_CHUNK):
        cls, k, m, w, size = _draw(rng, oracle)
        size = min(size, (1 << 20) + 12345)
        case = (cls, k, m, w, size)
        bs, _ = le.layout(cls, (k, m, w), size)
        n = rng.randint(1, 24)
        stride = (max(size, k * bs) + 15) // 16 * 16 + 16 * rng.randint(0, 3)
        host, objs = _batch(gpu, n, size, stride, rng.randrange(1 << 30))
        objs[:, size:] = 0  # bytes past the object (none are read)
        ref_objs = objs.clone()
        parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
        le.device.encode(cls, (k, m, w), objs, size, parity)
        gpu.cuda.synchronize()
        par = parity.cpu().numpy()
        for o in sorted({0, n - 1, rng.randrange(n)}):
            r = oracle.encode(cls, k, m, w, host[o, :size].tobytes())
            assert par[o].tobytes() == b"".join(r[k:]), (case, o)
        erased = sorted(rng.sample(range(k + m), rng.randint(1, m)))
        for e in erased:
            if e < k and e * bs < size:
                objs[:, e * bs:min((e + 1) * bs, size)] = 0xA5
        le.device.decode(cls, (k, m, w), objs, size, parity, erased)
        gpu.cuda.synchronize()
        assert gpu.equal(objs[:, :size], ref_objs[:, :size]), (case, erased, n)
