"""GPU parity: the HIP engine (through libleoec.so's C ABI) against the CPU
oracle, on the reference's own test configurations (test/leo_erasure_tests.erl)
plus the BASELINE configs.  Bit-exact everywhere (integer / byte arithmetic).
"""
import itertools
import json
import os
import random
import subprocess
import sys

import numpy as np
import pytest

from gpu_helpers import batch as _batch
from gpu_helpers import mixed_callers, rand_bytes

pytestmark = pytest.mark.gpu

# (class, k, m, w) — suite_test_ / repair_test / parameters_test / bench_encode_test
# configurations of test/leo_erasure_tests.erl:33-83,118-143,207-212 and BASELINE.json
CONFIGS = [
    ("vandrs", 10, 4, 8), ("vandrs", 4, 2, 8), ("vandrs", 8, 3, 8), ("vandrs", 6, 2, 8),
    ("vandrs", 4, 1, 8), ("vandrs", 4, 2, 16), ("vandrs", 10, 4, 16), ("vandrs", 4, 2, 32),
    ("vandrs", 10, 4, 32), ("vandrs", 17, 5, 8),
    ("isars", 10, 4, 8), ("isars", 4, 2, 8), ("isars", 8, 3, 8),
    ("cauchyrs", 4, 2, 3), ("cauchyrs", 10, 4, 8), ("cauchyrs", 10, 4, 10), ("cauchyrs", 6, 3, 4),
    ("liberation", 4, 2, 7), ("liberation", 5, 2, 5), ("liberation", 10, 2, 11),
    ("liberation", 4, 2, 5),
    # chunked launches: >16 inputs (accumulating launches), >4 outputs,
    # cauchyrs beyond the bitsliced kernel's w <= 16 (masked bitmatrix kernel)
    ("vandrs", 20, 6, 8), ("isars", 18, 5, 8), ("cauchyrs", 5, 3, 17), ("liberation", 3, 2, 31),
    ("vandrs", 17, 3, 16),
]


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "%s-%d-%d-%d" % c)
@pytest.mark.parametrize("size", [1, 1000, 65536 + 7, 300001])
def test_encode_matches_oracle(gpu, le, oracle, cfg, size):
    cls, k, m, w = cfg
    data = rand_bytes(size, size * 31 + k)
    st, blocks = le.nif_encode(cls, (k, m, w), data, size)
    assert st == "ok", blocks
    ref = oracle.encode(cls, k, m, w, data)
    assert len(blocks) == k + m
    for i, (a, b) in enumerate(zip(blocks, ref)):
        assert a == b, f"block {i} differs"


def _check_decode_subsets(le, cls, k, m, w, data, blocks, failures, rng, limit=None):
    combos = list(itertools.combinations(range(k + m), k + m - failures))
    if limit and len(combos) > limit:
        combos = rng.sample(combos, limit)
    for avail in combos:
        order = list(avail)
        rng.shuffle(order)
        st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in order], order, len(data))
        assert st == "ok", (avail, out)
        assert out == data, f"decode mismatch for survivors {avail}"


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "%s-%d-%d-%d" % c)
def test_decode_every_erasure_pattern(gpu, le, cfg):
    """suite_test_: decode from every (K+M-F)-subset, shuffled, F = 0..M."""
    cls, k, m, w = cfg
    data = rand_bytes(40961, k * 7 + m)
    st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
    assert st == "ok"
    rng = random.Random(k * 100 + m)
    for f in range(m + 1):
        _check_decode_subsets(le, cls, k, m, w, data, blocks, f, rng, limit=300)


@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: "%s-%d-%d-%d" % c)
def test_repair_every_pair(gpu, le, cfg):
    """repair_test: every 2-erasure pair repaired equals the encoded blocks."""
    cls, k, m, w = cfg
    data = rand_bytes(33333, k + 5 * m)
    st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
    assert st == "ok"
    full = list(range(k + m))
    for lost in itertools.combinations(full, min(2, m)):
        avail = [i for i in full if i not in lost]
        st, rep = le.nif_repair(cls, (k, m, w), [blocks[i] for i in avail], avail, list(lost))
        assert st == "ok", rep
        assert rep == [blocks[i] for i in lost], f"repair of {lost} differs"


def test_repair_matches_oracle_with_extra_survivors(gpu, le, oracle):
    """More than k survivors, in arbitrary order: same survivor choice as the
    reference (first k intact ids ascending; isars: first k listed)."""
    for cls, k, m, w in [("vandrs", 10, 4, 8), ("isars", 10, 4, 8), ("cauchyrs", 10, 4, 8),
                         ("liberation", 4, 2, 7)]:
        data = rand_bytes(20000, 5)
        blocks = oracle.encode(cls, k, m, w, data)
        ids = [13 % (k + m), 2, 0, 7 % (k + m), 1, 5, 3, 4, 8 % (k + m), 9 % (k + m), 11 % (k + m)]
        ids = list(dict.fromkeys(ids))[: k + 1]
        lost = [i for i in range(k + m) if i not in ids]
        # corrupt-free: the map is unique, so also compare against the oracle
        st, rep = le.nif_repair(cls, (k, m, w), [blocks[i] for i in ids], ids, lost)
        assert st == "ok"
        assert rep == oracle.repair(cls, k, m, w, [blocks[i] for i in ids], ids, lost)


def test_padding_10MiB_plus_1(gpu, le, oracle):
    """TEST_SIZE = 10485760 + 1 (test/leo_erasure_tests.erl:28)."""
    data = rand_bytes(10485760 + 1, 28)
    for cls, k, m, w in [("vandrs", 10, 4, 8), ("isars", 10, 4, 8), ("cauchyrs", 4, 2, 3),
                         ("liberation", 4, 2, 7)]:
        st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
        assert st == "ok"
        assert blocks == oracle.encode(cls, k, m, w, data)
        rng = random.Random(1)
        _check_decode_subsets(le, cls, k, m, w, data, blocks, m, rng, limit=6)


def test_host_objects_above_zero_copy_cap(gpu, le, oracle):
    """Host calls whose span passes the 16 MiB zero-copy cap take the
    per-thread copy path (one pageable copy each way; the measurement build's
    column-chunked form is tested in test_measure_forms.py): encode, decode
    of lost data blocks and repair of a data and a coding block, bit-exact
    with the oracle, twice over the same buffers, for GF(2^8) / GF(2^16)
    Reed-Solomon and ISA-L maps, a bitmatrix class and ragged sizes."""
    for cls, k, m, w, size in [("vandrs", 10, 4, 8, (40 << 20) + 3), ("isars", 10, 4, 8, 24 << 20),
                               ("vandrs", 6, 3, 16, (20 << 20) + 1001),
                               ("cauchyrs", 10, 4, 8, (17 << 20) + 77)]:
        data = rand_bytes(size, size % 997)
        ref = oracle.encode(cls, k, m, w, data)
        for _ in range(2):
            st, blocks = le.nif_encode(cls, (k, m, w), data, size)
            assert st == "ok" and blocks == ref, (cls, k, m, w, size)
            ids = list(range(m, k + m))[::-1]
            st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, size)
            assert st == "ok" and out == data, (cls, k, m, w, size)
            lost = [0, k + m - 1]
            avail = [b for b in range(k + m) if b not in lost]
            st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
            assert st == "ok" and rep == [ref[b] for b in lost], (cls, k, m, w, size)


@pytest.mark.parametrize("km", [(10, 4), (8, 3), (6, 2), (4, 2), (4, 1)])
def test_correctness_5MiB(gpu, le, km):
    """correctness_test (test/leo_erasure_tests.erl:171-204), default coder."""
    k, m = km
    data = rand_bytes(5 * 1024 * 1024, k * m)
    st, id_blocks = le.encode((k, m), data)
    assert st == "ok" and len(id_blocks) == k + m
    st, out = le.decode((k, m), id_blocks, len(data))
    assert st == "ok" and out == data
    lost = (k * 7 + m) % (k + m)
    rest = [x for x in id_blocks if x[0] != lost]
    st, rep = le.repair((k, m), rest)
    assert st == "ok" and rep == [id_blocks[lost]]


def test_parameters(gpu, le):
    """parameters_test (test/leo_erasure_tests.erl:214-275)."""
    data = rand_bytes(1024, 3)
    assert le.encode("vandrs", (4, 2, 7), data)[0] == "error"
    for cls, p in [("vandrs", (4, 2, 8)), ("cauchyrs", (4, 2, 3)), ("liberation", (4, 2, 5)),
                   ("isars", (4, 2, 8))]:
        st, idb = le.encode(cls, p, data)
        assert st == "ok"
        blocks = [b for _, b in idb]
        assert le.decode(cls, p, blocks, [0, 1, 2], len(data))[0] == "error"
        # genuinely too few blocks (3 blocks with 3 ids)
        assert le.decode(cls, p, blocks[:3], [0, 1, 2], len(data)) == \
            ("error", "Not Enough Blocks")
        assert le.decode(cls, p, blocks[:4] + blocks[:1], [0, 1, 2, 3, 0], len(data)) == \
            ("error", "Blocks should be unique")
    assert le.encode("cauchyrs", (10, 4, 3), data)[0] == "error"
    assert le.encode("liberation", (4, 2, 6), data)[0] == "error"
    assert le.encode("liberation", (4, 2, 3), data)[0] == "error"
    assert le.encode("isars", (4, 2, 7), data)[0] == "error"
    assert le.encode("unkown", (4, 2, 3), data) == ("error", "Invalid Coding")
    assert le.encode("liberation", ("troll",), data)[0] == "error"
    assert le.encode((4, 2, 5), "liberation", data)[0] == "error"
    for km, n in [((10, 4), 14), ((8, 3), 11), ((6, 2), 8)]:
        st, idb = le.encode(km, data)
        assert st == "ok" and len(idb) == n
        assert le.decode(km, idb, len(data)) == ("ok", data)


def test_edge_sizes(gpu, le, oracle):
    """Empty and ragged objects; trailing data blocks that are pure padding
    (the reference's fast-path overflow case, rscoding.cpp:116-120)."""
    for size in [0, 1, 15, 16, 17, 127, 128, 129, 1024, 1279, 1281]:
        data = rand_bytes(size, size + 1)
        for cls, k, m, w in [("vandrs", 10, 4, 8), ("cauchyrs", 10, 4, 8), ("isars", 4, 2, 8)]:
            st, blocks = le.nif_encode(cls, (k, m, w), data, size)
            assert st == "ok"
            assert blocks == oracle.encode(cls, k, m, w, data)
            ids = list(range(k))
            st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in ids], ids, size)
            assert st == "ok" and out == data
            ids = list(range(m, k + m))
            st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in ids], ids, size)
            assert st == "ok" and out == data


# ---------------------------------------------------------------------------
# device-resident batched API


@pytest.mark.parametrize("cfg", [("vandrs", 10, 4, 8), ("vandrs", 4, 2, 8), ("isars", 10, 4, 8),
                                 ("cauchyrs", 10, 4, 8), ("liberation", 4, 2, 7),
                                 ("vandrs", 10, 4, 16), ("vandrs", 6, 3, 32)],
                         ids=lambda c: "%s-%d-%d-%d" % c)
def test_device_encode_batch(gpu, le, oracle, cfg):
    cls, k, m, w = cfg
    n, size = 24, 200003
    bs, _ = le.layout(cls, (k, m, w), size)
    host, objs = _batch(gpu, n, size, size + 62, 11)  # stride not a multiple of 16 -> rejected
    parity = gpu.empty((n, m * bs), dtype=gpu.uint8, device="cuda")
    with pytest.raises(le.LeoecError):
        le.device.encode(cls, (k, m, w), objs, size, parity)
    host, objs = _batch(gpu, n, size, size + 77 - (size + 77) % 16, 12)
    le.device.encode(cls, (k, m, w), objs, size, parity)
    gpu.cuda.synchronize()
    par = parity.cpu().numpy()
    for o in range(n):
        ref = oracle.encode(cls, k, m, w, host[o, :size].tobytes())
        assert par[o].tobytes() == b"".join(ref[k:]), f"object {o}"


def test_device_decode_all_1001_patterns(gpu, le):
    """vandrs RS(10,4,8): every 4-erasure pattern, rebuilt in place."""
    k, m, w = 10, 4, 8
    n, size = 8, 1048576
    bs, _ = le.layout("vandrs", (k, m, w), size)
    host, objs = _batch(gpu, n, size, size, 99)
    parity = gpu.empty((n, m * bs), dtype=gpu.uint8, device="cuda")
    le.device.encode("vandrs", (k, m, w), objs, size, parity)
    ref = objs.clone()
    work = objs.clone()
    for erased in itertools.combinations(range(k + m), m):
        work.copy_(ref)
        for e in erased:
            if e < k:
                lo, hi = e * bs, min((e + 1) * bs, size)
                work[:, lo:hi] = 0xA5
        le.device.decode("vandrs", (k, m, w), work, size, parity, list(erased))
        if not gpu.equal(work, ref):
            raise AssertionError(f"in-place decode wrong for erasures {erased}")


def test_device_repair(gpu, le, oracle):
    for cls, k, m, w in [("vandrs", 10, 4, 8), ("cauchyrs", 10, 4, 8), ("isars", 10, 4, 8)]:
        n, size = 16, 123457
        bs, _ = le.layout(cls, (k, m, w), size)
        host = np.random.Generator(np.random.PCG64(3)).integers(0, 256, (n, size), dtype=np.uint8)
        blocks = np.zeros((k + m, n, bs), dtype=np.uint8)
        for o in range(n):
            ref = oracle.encode(cls, k, m, w, host[o].tobytes())
            for b in range(k + m):
                blocks[b, o] = np.frombuffer(ref[b], dtype=np.uint8)
        dev = [gpu.from_numpy(blocks[b]).cuda() for b in range(k + m)]
        lost = [0, 5, 10, 13]
        avail = [None if b in lost else dev[b] for b in range(k + m)]
        out = [gpu.empty((n, bs), dtype=gpu.uint8, device="cuda") for _ in lost]
        le.device.repair(cls, (k, m, w), avail, bs, lost, out, n)
        gpu.cuda.synchronize()
        for r, b in enumerate(lost):
            assert np.array_equal(out[r].cpu().numpy(), blocks[b]), (cls, b)


def test_device_roundtrip_bench_shape(gpu, le):
    """Size-independent property at the bench configuration: 1 MiB objects,
    RS(10,4,8), encode then in-place decode of {0,1,2,3} restores every byte."""
    k, m, w = 10, 4, 8
    n, size = 256, 1048576
    bs, _ = le.layout("vandrs", (k, m, w), size)
    g = gpu.Generator(device="cuda").manual_seed(0x1E0E)
    objs = gpu.randint(0, 256, (n, size), dtype=gpu.uint8, device="cuda", generator=g)
    parity = gpu.empty((n, m * bs), dtype=gpu.uint8, device="cuda")
    le.device.encode("vandrs", (k, m, w), objs, size, parity)
    ref = objs.clone()
    objs[:, : 4 * bs] = 0
    le.device.decode("vandrs", (k, m, w), objs, size, parity, [0, 1, 2, 3])
    assert gpu.equal(objs, ref)


@pytest.mark.parametrize("cls,k,m,w", [("vandrs", 4, 2, 8), ("vandrs", 10, 4, 8),
                                       ("cauchyrs", 10, 4, 8), ("isars", 10, 4, 8)],
                         ids=lambda v: str(v))
def test_baseline_configs_1MiB_device_batches(gpu, le, oracle, cls, k, m, w):
    """BASELINE configs[0]-[3] on the product library: batches of 13 whole
    1 MiB objects (13: the XCD object map's tail of fewer than 8 objects
    keeps dispatch order), device-resident.  Encode parity against the oracle
    for objects in and past the last whole group of 8; in-place decode of
    the worst-case data erasures over poisoned blocks; repair of a
    data + parity mix against the encoded blocks."""
    n, size = 13, 1048576
    bs, _ = le.layout(cls, (k, m, w), size)
    host, objs = _batch(gpu, n, size, size, 0xB0 + k + m + w)
    parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
    le.device.encode(cls, (k, m, w), objs, size, parity)
    gpu.cuda.synchronize()
    par = parity.cpu().numpy()
    for o in (0, 5, 7, 8, 12):
        ref = oracle.encode(cls, k, m, w, host[o].tobytes())
        assert par[o].tobytes() == b"".join(ref[k:]), f"object {o}"
    ref = objs.clone()
    erased = list(range(m))
    objs[:, :m * bs] = 0xA5
    le.device.decode(cls, (k, m, w), objs, size, parity, erased)
    gpu.cuda.synchronize()
    assert gpu.equal(objs, ref)
    pad = gpu.zeros((n, k * bs), dtype=gpu.uint8, device="cuda")
    pad[:, :size] = objs
    blocks = [pad[:, b * bs:(b + 1) * bs] if b < k else parity[:, (b - k) * bs:(b - k + 1) * bs]
              for b in range(k + m)]
    blocks = [b.contiguous() for b in blocks]
    lost = sorted({0, k // 2, k, k + m - 1})[:m]
    avail = [None if b in lost else blocks[b] for b in range(k + m)]
    out = [gpu.full((n, bs), 0x3C, dtype=gpu.uint8, device="cuda") for _ in lost]
    le.device.repair(cls, (k, m, w), avail, bs, lost, out, n)
    gpu.cuda.synchronize()
    for r, b in enumerate(lost):
        assert gpu.equal(out[r], blocks[b]), (cls, b)


@pytest.mark.parametrize("n,size", [(2800, 1048576), (2720, 1048576 + 77)])
def test_cauchy_large_launch_gfbk(gpu, le, oracle, n, size):
    """cauchyrs(10,4,8) launches of at least kGfbkMinBytes (4.0 GB of
    algorithmic bytes) take gfbk_apply (gfbit_impl.hpp, round 6): 2,800 x
    1 MiB (4.11 GB) takes it for encode, decode of 4 data blocks and repair
    of 4 blocks; 2,720 ragged objects (3.99 GB) stay on gfbit_apply.  Encode
    parity against the oracle for objects at both ends and in the middle;
    decode over poisoned blocks back to the objects; repair against the
    encoded blocks."""
    k, m, w, cls = 10, 4, 8, "cauchyrs"
    bs, _ = le.layout(cls, (k, m, w), size)
    stride = (size + 15) // 16 * 16
    g = gpu.Generator(device="cuda")
    g.manual_seed(0x6FB4 + n)
    objs = gpu.randint(0, 256, (n, stride), dtype=gpu.uint8, device="cuda", generator=g)
    parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
    le.device.encode(cls, (k, m, w), objs, size, parity)
    gpu.cuda.synchronize()
    for o in (0, 1, n // 2, n - 2, n - 1):
        ref = oracle.encode(cls, k, m, w, objs[o, :size].cpu().numpy().tobytes())
        assert parity[o].cpu().numpy().tobytes() == b"".join(ref[k:]), f"object {o}"
    ref = objs.clone()
    objs[:, :m * bs] = 0xA5
    le.device.decode(cls, (k, m, w), objs, size, parity, list(range(m)))
    gpu.cuda.synchronize()
    assert gpu.equal(objs[:, :size], ref[:, :size])
    del ref
    pad = gpu.zeros((n, k * bs), dtype=gpu.uint8, device="cuda")
    pad[:, :size] = objs[:, :size]
    lost = [0, 5, 10, 13]
    blocks = [pad[:, b * bs:(b + 1) * bs] if b < k else parity[:, (b - k) * bs:(b - k + 1) * bs]
              for b in range(k + m)]
    avail = [None if b in lost else blocks[b].contiguous() for b in range(k + m)]
    out = [gpu.full((n, bs), 0x3C, dtype=gpu.uint8, device="cuda") for _ in lost]
    le.device.repair(cls, (k, m, w), avail, bs, lost, out, n)
    gpu.cuda.synchronize()
    for r, b in enumerate(lost):
        assert gpu.equal(out[r], blocks[b]), b


def test_cauchy_64MiB_objects_gfbk(gpu, le, oracle):
    """configs[4]'s shape in cauchyrs(10,4,8): 64 x 64 MiB objects (+ 77 B,
    ragged) are 6.0 GB of algorithmic bytes per launch, so encode and
    decode take gfbk_apply with 6.7 MB blocks (820 tiles per object):
    encode parity of the first and last objects against the oracle, decode
    of data blocks 0-3 over poisoned blocks back to every object."""
    k, m, w, cls = 10, 4, 8, "cauchyrs"
    n, size = 64, (64 << 20) + 77
    bs, _ = le.layout(cls, (k, m, w), size)
    stride = (size + 15) // 16 * 16
    g = gpu.Generator(device="cuda")
    g.manual_seed(0x64CA)
    objs = gpu.randint(0, 256, (n, stride), dtype=gpu.uint8, device="cuda", generator=g)
    parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
    le.device.encode(cls, (k, m, w), objs, size, parity)
    gpu.cuda.synchronize()
    for o in (0, n - 1):
        ref = oracle.encode(cls, k, m, w, objs[o, :size].cpu().numpy().tobytes())
        assert parity[o].cpu().numpy().tobytes() == b"".join(ref[k:]), f"object {o}"
    ref = objs.clone()
    objs[:, :m * bs] = 0xA5
    le.device.decode(cls, (k, m, w), objs, size, parity, list(range(m)))
    gpu.cuda.synchronize()
    assert gpu.equal(objs[:, :size], ref[:, :size])


def test_host_above_zero_copy_cap(gpu, le, oracle):
    """Host calls whose span passes the per-thread zero-copy cap (16 MiB) and
    the batch cap: the per-thread copy path (one pageable copy each way, or
    the gather buffer for k separate survivor binaries): encode / decode /
    repair bit-exact with the oracle, twice over the same buffers, for every
    class (ragged sizes; a 64 MiB + 5 B object)."""
    cases = [("vandrs", 10, 4, 8, (64 << 20) + 5), ("isars", 10, 4, 8, (20 << 20) - 4095),
             ("cauchyrs", 10, 4, 8, (17 << 20) + 77), ("vandrs", 5, 3, 32, 17 << 20),
             ("liberation", 4, 2, 7, (17 << 20) + 1)]
    for cls, k, m, w, size in cases:
        data = rand_bytes(size, size + 19 * k)
        ref = oracle.encode(cls, k, m, w, data)
        for _ in range(2):
            st, blocks = le.nif_encode(cls, (k, m, w), data, size)
            assert st == "ok" and blocks == ref, (cls, k, m, w, size)
            ids = list(range(m, k + m))[::-1]
            st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, size)
            assert st == "ok" and out == data, (cls, k, m, w, size)
            lost = [0, k + m - 1]
            avail = [b for b in range(k + m) if b not in lost]
            st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
            assert st == "ok" and rep == [ref[b] for b in lost], (cls, k, m, w, size,
                                                                  rep if st != "ok" else "")


def test_golden_fixtures_gpu(gpu, le):
    """The committed restatement-derived fixtures, through the GPU engine."""
    import json
    import os
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "index.json")) as fh:
        index = json.load(fh)
    for ent in index:
        z = np.load(os.path.join(here, ent["file"]), allow_pickle=False)
        st, blocks = le.nif_encode(ent["class"], (ent["k"], ent["m"], ent["w"]),
                                   z["data"].tobytes(), ent["size"])
        assert st == "ok" and b"".join(blocks) == z["blocks"].tobytes(), ent["file"]


def test_file_helpers(gpu, le, tmp_path, monkeypatch):
    """file_test (test/leo_erasure_tests.erl:98-116): encode_file, delete blocks
    0/2/4/6, decode_file, compare."""
    monkeypatch.chdir(tmp_path)
    data = rand_bytes(10485760 + 1, 98)
    (tmp_path / "testbin").write_bytes(data)
    assert le.encode_file("vandrs", (10, 4, 8), "testbin") == 14
    for i in (0, 2, 4, 6):
        (tmp_path / "blocks" / ("testbin.%d" % i)).unlink()
    assert le.decode_file("vandrs", (10, 4, 8), "testbin", len(data)) == "ok"
    assert (tmp_path / "testbin.dec").read_bytes() == data


def test_device_64MiB_objects(gpu, le, oracle):
    """BASELINE configs[4] geometry: RS(10,4,8) on 64 MiB objects (bs =
    6,710,912, 256 B of zero pad in block 9), device-resident batch.  Parity of
    two objects against the oracle, then the size-independent round trips:
    in-place decode of {0,1,2,3} and repair of a data+parity mix."""
    k, m, w = 10, 4, 8
    n, size = 3, 64 * 1024 * 1024
    bs, _ = le.layout("vandrs", (k, m, w), size)
    assert bs == 6710912
    g = gpu.Generator(device="cuda").manual_seed(0x64)
    objs = gpu.randint(0, 256, (n, size), dtype=gpu.uint8, device="cuda", generator=g)
    parity = gpu.empty((n, m * bs), dtype=gpu.uint8, device="cuda")
    le.device.encode("vandrs", (k, m, w), objs, size, parity)
    gpu.cuda.synchronize()
    for o in (0, n - 1):
        ref = oracle.encode("vandrs", k, m, w, objs[o].cpu().numpy().tobytes())
        assert parity[o].cpu().numpy().tobytes() == b"".join(ref[k:]), f"object {o}"
    ref = objs.clone()
    objs[:, : 4 * bs] = 0x5A
    le.device.decode("vandrs", (k, m, w), objs, size, parity, [0, 1, 2, 3])
    assert gpu.equal(objs, ref)
    # repair {0, 5, 10, 13} from the other ten blocks, as separate shards
    pad = gpu.zeros((n, k * bs), dtype=gpu.uint8, device="cuda")
    pad[:, :size] = objs
    blocks = [pad[:, b * bs:(b + 1) * bs] if b < k else parity[:, (b - k) * bs:(b - k + 1) * bs]
              for b in range(k + m)]
    blocks = [b.contiguous() for b in blocks]
    lost = [0, 5, 10, 13]
    avail = [None if b in lost else blocks[b] for b in range(k + m)]
    out = [gpu.empty((n, bs), dtype=gpu.uint8, device="cuda") for _ in lost]
    le.device.repair("vandrs", (k, m, w), avail, bs, lost, out, n)
    gpu.cuda.synchronize()
    for r, b in enumerate(lost):
        assert gpu.equal(out[r], blocks[b]), b


def test_concurrent_callers(gpu, le, oracle):
    """The NIF is callable from any scheduler thread at once (basho_bench t4,
    test/basho_bench_leo_erasure_rs_10_4_8_1M_w_t4.config): 8 threads each
    run encode / decode / repair of their own objects through the C ABI
    (ctypes drops the GIL), over every class; all results match the oracle."""
    import concurrent.futures as cf

    cases = [("vandrs", 10, 4, 8), ("cauchyrs", 10, 4, 8), ("isars", 10, 4, 8),
             ("liberation", 4, 2, 7), ("vandrs", 4, 2, 16), ("vandrs", 6, 3, 32)]
    expect = {}
    for i, (cls, k, m, w) in enumerate(cases):
        data = rand_bytes(1048576 + 333 * i, 500 + i)
        expect[i] = (data, oracle.encode(cls, k, m, w, data))

    def worker(t):
        for r in range(6):
            i = (t + r) % len(cases)
            cls, k, m, w = cases[i]
            data, ref = expect[i]
            st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
            if st != "ok" or blocks != ref:
                return f"encode {cls}{(k, m, w)} thread {t}"
            ids = list(range(m, k + m))[::-1]
            st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, len(data))
            if st != "ok" or out != data:
                return f"decode {cls}{(k, m, w)} thread {t}"
            lost = [t % (k + m), (t + 3) % (k + m)]
            lost = sorted(set(lost))
            avail = [b for b in range(k + m) if b not in lost]
            st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
            if st != "ok" or rep != [ref[b] for b in lost]:
                return f"repair {cls}{(k, m, w)} {lost} thread {t}"
        return None

    with cf.ThreadPoolExecutor(8) as ex:
        errs = [e for e in ex.map(worker, range(8)) if e]
    assert not errs, errs


def test_thread_exit_releases_staging(gpu, le, oracle):
    """Caller threads that come and go (dirty schedulers, pools) give back their
    per-thread stream, device buffer and pinned buffers: an exiting thread
    hands them off without a HIP call (engine.cpp Staging::hand_off) and the
    next call of a live thread frees them (reclaim_drain).  160 short-lived
    threads each run a decode (gather staging) + encode of an 8 MiB object;
    device memory must not drift by their buffers (~19 MB each would be
    ~3 GB)."""
    import threading

    import torch

    k, m, w, size = 10, 4, 8, 8 << 20
    data = rand_bytes(size, 4242)
    ref = oracle.encode("vandrs", k, m, w, data)
    ids = list(range(4, k + m))
    errs = []

    def one():
        st, out = le.nif_decode("vandrs", (k, m, w), [ref[b] for b in ids], ids, size)
        if st != "ok" or out != data:
            errs.append("decode")
        st, blocks = le.nif_encode("vandrs", (k, m, w), data, size)
        if st != "ok" or blocks != ref:
            errs.append("encode")

    def wave(n):
        ths = [threading.Thread(target=one) for _ in range(n)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()

    wave(8)  # runtime warm-up
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    for _ in range(20):
        wave(8)
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert not errs, errs[:4]
    assert free0 - free1 < (512 << 20), (free0 - free1) / 2**20


def test_default_w_substitution(gpu, le):
    """suite_test_'s W = -1 and W = 0 cases (test/leo_erasure_tests.erl:40-48):
    encode/3 and decode/4 substitute ?coding_params_w(Class)
    (src/leo_erasure.erl:155-156,203-204); the blocks equal an explicit-W
    encode and decode with the substituted W round-trips."""
    data = rand_bytes(300001, 40)
    for cls, k, m in [("vandrs", 10, 4), ("cauchyrs", 4, 2), ("liberation", 4, 2), ("isars", 10, 4)]:
        w = le.api.coding_params_w(cls)
        st, ref = le.encode(cls, (k, m, w), data)
        assert st == "ok"
        for bad_w in (-1, 0):
            st, idb = le.encode(cls, (k, m, bad_w), data)
            assert st == "ok" and idb == ref, (cls, bad_w)
            keep = idb[m:]  # lose the first m blocks
            assert le.decode(cls, (k, m, bad_w), keep, len(data)) == ("ok", data), (cls, bad_w)


def test_bench_encode_100MiB_zero(gpu, le):
    """bench_encode_test (test/leo_erasure_tests.erl:207-212,304-336): one
    encode of a 100 MiB all-zero binary per class.  Every code is linear, so
    every block is zero; a decode from the last k blocks returns the object."""
    size = 100 << 20
    data = bytes(size)
    for cls, k, m, w in [("vandrs", 10, 4, 8), ("cauchyrs", 4, 2, 3), ("liberation", 4, 2, 7),
                         ("isars", 10, 4, 8)]:
        st, blocks = le.nif_encode(cls, (k, m, w), data, size)
        assert st == "ok" and len(blocks) == k + m
        assert all(not any(b[::4096]) and b.count(0) == len(b) for b in blocks[k:]), cls
        ids = list(range(m, k + m))
        st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in ids], ids, size)
        assert st == "ok" and out == data, cls


def test_host_batching_mixed_callers(gpu, le, oracle):
    """Cross-call batching under the product library's own policy
    (gpu_helpers.mixed_callers: 24 threads, mixed classes / widths / sizes /
    erasure patterns, every result equal to the oracle's).  The queue
    policies forced one way or the other, 4 dispatcher lanes and the
    injected per-job failures are test_measure_forms.py's."""
    errs, _ = mixed_callers(le, oracle)
    assert not errs, errs


@pytest.mark.timeout(900)
def test_measurement_forms_in_own_process(gpu):
    """Every measurement-build form test (tests/test_measure_forms.py) in a
    child process that loads libleoec_measure.so alone (LEOEC_LIBRARY=measure):
    this process, the product tests', never loads a second HIP library.  The
    child's output goes to gpurun_out/measure_forms.log when that directory
    exists (the GPU box), else to a temporary file; a failure shows its tail."""
    import tempfile
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "leo_erasure_amd", "libleoec_measure.so")):
        pytest.skip("measurement build absent (make -C leo_erasure_amd/csrc measure)")
    outdir = os.path.join(root, "gpurun_out")
    if os.path.isdir(outdir):
        log = os.path.join(outdir, "measure_forms.log")
    else:
        log = os.path.join(tempfile.mkdtemp(prefix="leoec_measure_"), "measure_forms.log")
    env = dict(os.environ, LEOEC_LIBRARY="measure", LIBC_FATAL_STDERR_="1")
    cmd = [sys.executable, "-u", "-m", "pytest", os.path.join(root, "tests", "test_measure_forms.py"),
           "-m", "measure_gpu", "-x", "-q", "-p", "no:cacheprovider",
           "--timeout", "120", "--timeout-method", "thread"]
    with open(log, "w") as fh:
        rc = subprocess.call(cmd, cwd=root, env=env, stdout=fh, stderr=subprocess.STDOUT,
                             timeout=840)
    with open(log) as fh:
        tail = fh.read()[-4000:]
    assert rc == 0, f"measurement-form tests failed (rc {rc}), {log}:\n{tail}"
    summary = tail.strip().splitlines()[-1]
    assert "passed" in summary and "skipped" not in summary, summary



def test_host_spread_opt_in(gpu, le, oracle):
    """leoec_host_spread: host-memory calls run on the caller's current device
    by default; spreading over an explicit device set is opt-in, a device the
    process cannot use is refused (the setting unchanged), and the empty set
    restores the default.  Every call in every mode is bit-exact."""
    devs = le._lib.host_lanes()
    assert devs and len(devs) == gpu.cuda.device_count()
    data = rand_bytes(1048576 + 77, 4321)
    ref = oracle.encode("vandrs", 10, 4, 8, data)
    try:
        assert le._lib.host_spread(devs) == len(devs)
        st, blocks = le.nif_encode("vandrs", (10, 4, 8), data, len(data))
        assert st == "ok" and blocks == ref
        with pytest.raises(le.LeoecError):
            le._lib.host_spread([len(devs) + 7])
        st, blocks = le.nif_encode("vandrs", (10, 4, 8), data, len(data))
        assert st == "ok" and blocks == ref
    finally:
        assert le._lib.host_spread([]) == 0
    ids = list(range(4, 14))
    st, out = le.nif_decode("vandrs", (10, 4, 8), [ref[i] for i in ids], ids, len(data))
    assert st == "ok" and out == data


_WARM_CHILD = r"""
import json, sys, time
sys.path[:0] = [sys.argv[1], sys.argv[2]]
import torch
import leo_erasure_amd as le
from oracle import oracle as O
torch.cuda.set_device(0)
before = le._lib.measure_warm_state(0)
free0, _ = torch.cuda.mem_get_info()
t0 = time.perf_counter()
n = le._lib.host_spread([0])
t_spread = time.perf_counter() - t0
after = le._lib.measure_warm_state(0)
reclaim = le._lib.measure_reclaim_state()
data = bytes(range(256)) * 4096 + b"tail"
t0 = time.perf_counter()
st, blocks = le.nif_encode("vandrs", (10, 4, 8), data, len(data))
t_first = time.perf_counter() - t0
final = le._lib.measure_warm_state(0)
le._lib.host_spread([])
torch.cuda.synchronize()
free1, _ = torch.cuda.mem_get_info()
print(json.dumps({"n": n, "before": before, "after": after, "final": final,
                  "reclaim": reclaim, "leak_MiB": (free0 - free1) / 2**20,
                  "t_spread": t_spread, "t_first": t_first, "ok": st == "ok",
                  "parity": blocks == O.encode("vandrs", 10, 4, 8, data)}))
"""


def test_host_spread_warms_its_devices(gpu):
    """leoec_host_spread warms every device of its set before returning (as
    gf_init warms the caller's device): in a fresh process that never called
    gf_init, host_spread([0]) builds device 0's batching queue and pools, and
    the first host call afterwards builds no queue and pays no start-up.
    The warm-up runs on a thread of its own even for a one-device set
    (engine.cpp warm_devices), so this is the branch a multi-GPU node's NIF
    load takes: the thread ran and ended, handed its staging back while alive
    (its stream joined the pool), and the device memory the warm-up keeps is
    bounded as in test_thread_exit_releases_staging.  Child process on the
    measurement build (its warm-state and reclaim counters)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists(os.path.join(root, "leo_erasure_amd", "libleoec_measure.so")):
        pytest.skip("measurement build absent (make -C leo_erasure_amd/csrc measure)")
    env = dict(os.environ, LEOEC_LIBRARY="measure")
    r = subprocess.run([sys.executable, "-c", _WARM_CHILD, root, os.path.join(root, "tests")],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["n"] == 1
    assert not out["before"]["queue"] and out["before"]["queues_built"] == 0
    assert out["after"]["queue"] and out["after"]["queues_built"] == 1
    assert out["after"]["pool_streams"] >= 1 and out["after"]["pool_mapped"] >= 1
    rc = out["reclaim"]
    assert rc["warm_threads_started"] == 1 and rc["warm_threads_done"] == 1, rc
    # the warm thread's own staging: handed off and freed before it ended
    assert rc["handed_off"] == 1 and rc["drained"] == 1 and rc["busy"] == 0, rc
    assert out["leak_MiB"] < 512, out
    assert out["final"]["queues_built"] == 1, "the first call after host_spread built a queue"
    assert out["ok"] and out["parity"]
    # a cold first call pays ~150-250 ms of runtime and queue set-up
    assert out["t_first"] < 0.05, out


def test_bench_host_leg_on_the_system_runtime(gpu):
    """bench.py's host-memory leg runs in a torch-free child process, so
    libleoec.so binds the system HIP runtime an Erlang VM would load; its
    record carries that runtime, outputs equal to the GPU's device parity,
    and the bench process's own (torch-runtime) figures beside it."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LEOEC_LIBRARY")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--objects", "64",
                        "--steps", "2", "--warmup", "1", "--warmup-s", "0.1", "--no-cpu",
                        "--no-ceiling", "--host-callers", "8", "--host-seconds", "0.2"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["verified"] is True
    hp = rec["host_path"]["per_rank"][0]
    assert "child_error" not in hp, hp.get("child_error")
    assert hp["runtime"].startswith("system HIP runtime")
    assert hp["parity_vs_gpu"] == {"objects": 8, "encode_equal": True, "decode_equal": True}
    assert hp["encode_GiBps"] > 0 and hp["decode_GiBps"] > 0
    assert hp["torch_runtime"]["parity_vs_gpu"]["encode_equal"] is True
