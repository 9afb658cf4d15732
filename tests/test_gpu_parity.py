"""GPU parity: the HIP engine (through libleoec.so's C ABI) against the CPU
oracle, on the reference's own test configurations (test/leo_erasure_tests.erl)
plus the BASELINE configs.  Bit-exact everywhere (integer / byte arithmetic).
"""
import itertools
import random

import numpy as np
import pytest

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


def rand_bytes(n, seed):
    return np.random.Generator(np.random.PCG64(seed)).integers(0, 256, n, dtype=np.uint8).tobytes()


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
def _batch(gpu, n, size, stride, seed):
    rng = np.random.Generator(np.random.PCG64(seed))
    host = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    return host, gpu.from_numpy(host).cuda()


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


@pytest.mark.parametrize("env", [{"LEOEC_BITMATRIX": "1"}, {"LEOEC_GFBIT_LW": "1"},
                                 {"LEOEC_GFBIT_LW": "4"}, {"LEOEC_GFBIT_PF": "0"},
                                 {"LEOEC_GFBIT_PF": "0", "LEOEC_GFBIT_LW": "1"},
                                 {"LEOEC_GFBIT_LDS": "1"}, {"LEOEC_GFBIT_PF": "2"},
                                 {"LEOEC_GFBIT_PF": "3", "LEOEC_GFBIT_LW": "1"},
                                 {"LEOEC_BITMATRIX": "1", "LEOEC_BIT_FORM": "0"},
                                 {"LEOEC_BITMATRIX": "1", "LEOEC_BIT_FORM": "1"},
                                 {"LEOEC_BITMATRIX": "1", "LEOEC_BIT_FORM": "2"},
                                 {"LEOEC_GFBIT_FORM": "1"},  # gfb2_apply, next block in flight
                                 {"LEOEC_GFBIT_FORM": "1", "LEOEC_GFBIT_PF": "0"},
                                 {"LEOEC_GFBIT_FORM": "1", "LEOEC_GFBIT_LW": "1"},
                                 {"LEOEC_GFBIT_WG": "128"},
                                 {"LEOEC_GFBIT_WG": "128", "LEOEC_GFBIT_PF": "0"},
                                 {"LEOEC_GFBIT_LW": "4", "LEOEC_GFBIT_PF": "0"},
                                 {"LEOEC_GFBIT_FORM": "1", "LEOEC_GFBIT_WG": "128"},
                                 {"LEOEC_GFBIT_WAVES": "4"}, {"LEOEC_GFBIT_WAVES": "5"},
                                 {"LEOEC_GFBIT_CBM": "1"}, {"LEOEC_GFBIT_CBM": "2"},
                                 {"LEOEC_GFBIT_CBM": "3"}, {"LEOEC_GFBIT_CBM": "4"},
                                 {"LEOEC_GFBIT_CBM": "5"},
                                 {"LEOEC_GFBIT_FORM": "2"}],  # gfbx_apply (LDS-shared, split rows)
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_cauchy_kernel_forms_agree(gpu, le, oracle, env, measure):
    """cauchyrs through the generic masked-bitmatrix kernel and through every
    lane width of the bitsliced GF kernel gives the oracle's bytes."""
    for k, v in env.items():
        measure.setenv(k, v)
    for cls, k, m, w in [("cauchyrs", 10, 4, 8), ("cauchyrs", 6, 3, 4), ("cauchyrs", 4, 2, 3)]:
        data = rand_bytes(100003, k + m + w)
        st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
        assert st == "ok" and blocks == oracle.encode(cls, k, m, w, data)
        ids = list(range(m, k + m))
        st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in ids], ids, len(data))
        assert st == "ok" and out == data


@pytest.mark.parametrize("form", ["0", "1", "2", "3", "4", "5", "6", "7", "8"])
def test_bitmatrix_kernel_forms_agree(gpu, le, oracle, form, measure):
    """liberation (and >32 output packets: w = 17 cauchy) through every form of
    the bitmatrix kernel: masked / branchy, with and without look-ahead."""
    measure.setenv("LEOEC_BIT_FORM", form)
    for cls, k, m, w in [("liberation", 7, 2, 7), ("liberation", 3, 2, 31),
                         ("cauchyrs", 5, 3, 17)]:
        data = rand_bytes(150001, k + w)
        st, blocks = le.nif_encode(cls, (k, m, w), data, len(data))
        assert st == "ok" and blocks == oracle.encode(cls, k, m, w, data)
        ids = list(range(m, k + m))
        st, out = le.nif_decode(cls, (k, m, w), [blocks[i] for i in ids], ids, len(data))
        assert st == "ok" and out == data
        st, rep = le.nif_repair(cls, (k, m, w), [blocks[i] for i in ids], ids, [0, k])
        assert st == "ok" and rep == [blocks[0], blocks[k]]


@pytest.mark.parametrize("form", ["0", "1", "1-wg256", "1-la4", "1-decwg64"])
def test_liberation_encode_forms(gpu, le, oracle, form, measure):
    """lib_apply (the liberation bitmatrix structure compiled in, LEOEC_LIB_FORM=1,
    shipped with 64-lane, 1 KiB tiles; "1-wg256": the 256-lane, 4 KiB-tile
    form; "1-la4": 4 packets of look-ahead, 256 lanes) and the generic masked
    bitmatrix kernel (0): every instantiated w, k from 1 to w, sizes with
    ragged tails, against the oracle; decode and repair (generic kernel) of
    what was encoded."""
    measure.setenv("LEOEC_LIB_FORM", form[0])
    if form.endswith("wg256"):
        measure.setenv("LEOEC_LIB_WG", "256")
    if form.endswith("la4"):
        measure.setenv("LEOEC_LIB_LA", "4")
    if form.endswith("decwg64"):
        measure.setenv("LEOEC_LIB_DEC_WG", "64")
    for w in (3, 5, 7, 11, 13):
        for k in sorted({1, 2, (w + 1) // 2, w}):
            for size in (1, 4097, 150001):
                data = rand_bytes(size, k * 100 + w + size)
                st, blocks = le.nif_encode("liberation", (k, 2, w), data, size)
                assert st == "ok", blocks
                assert blocks == oracle.encode("liberation", k, 2, w, data), (k, w, size)
            ids = list(range(2, k + 2))
            st, out = le.nif_decode("liberation", (k, 2, w), [blocks[i] for i in ids], ids, size)
            assert st == "ok" and out == data, (k, w)
            st, rep = le.nif_repair("liberation", (k, 2, w), [blocks[i] for i in ids], ids, [0, k, k + 1])
            assert st == "ok" and rep == [blocks[0], blocks[k], blocks[k + 1]], (k, w)
            # syndrome decode (lib_dec_apply) shapes: one data block lost with P
            # (solved through Q alone), and one of two lost data blocks wanted
            lost = [k - 1, k]
            ids = [i for i in range(k + 2) if i not in lost]
            st, out = le.nif_decode("liberation", (k, 2, w), [blocks[i] for i in ids], ids, size)
            assert st == "ok" and out == data, (k, w, lost)
            if k >= 2:
                ids = list(range(2, k + 2))
                st, rep = le.nif_repair("liberation", (k, 2, w), [blocks[i] for i in ids], ids, [1])
                assert st == "ok" and rep == [blocks[1]], (k, w)


def test_liberation_device_batch_forms(gpu, le, oracle, measure):
    """Device-resident batch (ragged object size, 37 objects) through both
    liberation encode forms: identical parity, equal to the oracle."""
    k, m, w = 7, 2, 7
    n, size = 37, 300007
    bs, _ = le.layout("liberation", (k, m, w), size)
    host, objs = _batch(gpu, n, size, size + 9 - (size + 9) % 16 + 16, 21)
    outs = []
    for form in ("1", "0"):
        measure.setenv("LEOEC_LIB_FORM", form)
        parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
        le.device.encode("liberation", (k, m, w), objs, size, parity)
        gpu.cuda.synchronize()
        outs.append(parity.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    for o in range(0, n, 6):
        ref = oracle.encode("liberation", k, m, w, host[o, :size].tobytes())
        assert outs[0][o].tobytes() == b"".join(ref[k:]), f"object {o}"


@pytest.mark.parametrize("wg", ["64", "256"])
def test_gf8_tile_width_forms(gpu, le, oracle, wg, measure):
    """gf8_apply at both tile widths (64-lane workgroups are shipped for blocks
    above 160 KiB, 256-lane below; LEOEC_GF8_WG forces one): sizes either side
    of the switch, encode against the oracle, a 4-data-erasure decode round
    trip and a data+parity repair."""
    measure.setenv("LEOEC_GF8_WG", wg)
    for cls, k, m in [("vandrs", 10, 4), ("isars", 10, 4), ("vandrs", 4, 2), ("vandrs", 17, 5)]:
        for size in (1, 5000, 1048576, 2097152 + 12345):
            data = rand_bytes(size, size + k)
            st, blocks = le.nif_encode(cls, (k, m, 8), data, size)
            assert st == "ok" and blocks == oracle.encode(cls, k, m, 8, data), (cls, k, m, size)
            ids = list(range(m, k + m))
            st, out = le.nif_decode(cls, (k, m, 8), [blocks[i] for i in ids], ids, size)
            assert st == "ok" and out == data, (cls, k, m, size)
            st, rep = le.nif_repair(cls, (k, m, 8), [blocks[i] for i in ids], ids, [0, k])
            assert st == "ok" and rep == [blocks[0], blocks[k]], (cls, k, m, size)


@pytest.mark.parametrize("cls,k,m,w", [("vandrs", 10, 4, 8), ("cauchyrs", 10, 4, 8),
                                       ("liberation", 7, 2, 7)])
def test_xcd_object_map_batches(gpu, le, oracle, measure, cls, k, m, w):
    """The object-interleaved XCD map (objects of <= 64 tiles) on batches that
    are not a multiple of 8 objects (the tail keeps dispatch order): parity
    identical with the map off, equal to the oracle, and decode in place."""
    n, size = 13, 1048576 - 333
    bs, _ = le.layout(cls, (k, m, w), size)
    host, objs = _batch(gpu, n, size, max(k, m) * bs, 31)
    ref = objs.clone()
    outs = []
    for env in (None, "0"):
        for var in ("LEOEC_GF8_TMAP", "LEOEC_GFBIT_XMAP", "LEOEC_LIB_XMAP"):
            if env is None:
                measure.delenv(var, raising=False)
            else:
                measure.setenv(var, env)
        parity = gpu.zeros((n, max(k, m) * bs), dtype=gpu.uint8, device="cuda")
        le.device.encode(cls, (k, m, w), objs, size, parity)
        objs[:, :2 * bs] = 0
        le.device.decode(cls, (k, m, w), objs, size, parity, [0, 1])
        gpu.cuda.synchronize()
        assert gpu.equal(objs, ref), env
        outs.append(parity.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    for o in (0, 7, 8, 12):
        r = oracle.encode(cls, k, m, w, host[o, :size].tobytes())
        assert outs[0][o, :m * bs].tobytes() == b"".join(r[k:]), f"object {o}"


@pytest.mark.parametrize("form", ["1", "2", "3", "4", "5"])
def test_cauchy_compiled_bitmatrix_batches(gpu, le, oracle, measure, form):
    """cauchyrs(10,4,8) encode with its bitmatrix compiled in (cbm_inst.hip,
    LEOEC_GFBIT_CBM): batches of whole and ragged 1 MiB objects (a short last
    data block, odd packets starting mid line), 13 objects (not a multiple of
    the XCD map's 8): parity identical to the bitsliced kernel's for every
    object and to the oracle's for some."""
    k, m, w = 10, 4, 8
    for size in (1048576, 1048576 - 333, 77777):
        n = 13
        bs, _ = le.layout("cauchyrs", (k, m, w), size)
        host, objs = _batch(gpu, n, size, max(k, m) * bs, 57 + size % 97)
        outs = []
        for env in ("0", form):
            measure.setenv("LEOEC_GFBIT_CBM", env)
            parity = gpu.full((n, max(k, m) * bs), 0x5A, dtype=gpu.uint8, device="cuda")
            le.device.encode("cauchyrs", (k, m, w), objs, size, parity)
            gpu.cuda.synchronize()
            outs.append(parity.cpu().numpy())
        assert np.array_equal(outs[0], outs[1]), size
        for o in (0, 7, 12):
            r = oracle.encode("cauchyrs", k, m, w, host[o, :size].tobytes())
            assert outs[1][o, :m * bs].tobytes() == b"".join(r[k:]), (size, o)


@pytest.mark.parametrize("env", [{}, {"LEOEC_GFBIT_WG": "256"}, {"LEOEC_GFBIT_PF": "2"},
                                 {"LEOEC_GFBIT_PF": "3"}, {"LEOEC_GFBIT_PF": "4"}, {"LEOEC_GFBIT_PF": "5"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "default")
def test_cauchy_aligned_copy_batches(gpu, le, oracle, measure, env):
    """cauchyrs through gfba_apply (LEOEC_GFBIT_FORM=3: line-aligned 16-byte
    copies into per-wave LDS slots, read back at each packet's phase): object
    rows at every 16-byte phase mod 128 (row stride = k*bs + 48), sizes whose
    blocks are full, short (last block 103,936 of 104,960 B), one packet of
    16 B, and empty (size 1,040: block 9 holds nothing); encode parity equal
    to the shipped kernel's and to the oracle's, decode and repair of
    erased data and parity blocks in place."""
    measure.setenv("LEOEC_GFBIT_FORM", "3")
    for key, v in env.items():
        measure.setenv(key, v)
    for k, m, size in [(10, 4, 1048576), (10, 4, 1048576 - 16 * 21), (10, 4, 77776),
                       (10, 4, 1040), (6, 3, 300000), (4, 2, 262144 + 4096)]:
        w, n = 8, 11
        bs, _ = le.layout("cauchyrs", (k, m, w), size)
        stride = max(k, m) * bs + 48
        host, objs = _batch(gpu, n, size, stride, 91 + size % 89)
        ref = objs.clone()
        outs = []
        for form in ("0", "3"):
            measure.setenv("LEOEC_GFBIT_FORM", form)
            parity = gpu.full((n, m * bs + 48), 0x5A, dtype=gpu.uint8, device="cuda")
            le.device.encode("cauchyrs", (k, m, w), objs, size, parity)
            gpu.cuda.synchronize()
            outs.append(parity.cpu().numpy())
        assert np.array_equal(outs[0], outs[1]), (k, m, size)
        for o in (0, 5, n - 1):
            r = oracle.encode("cauchyrs", k, m, w, host[o, :size].tobytes())
            assert outs[1][o, :m * bs].tobytes() == b"".join(r[k:]), (k, m, size, o)
        er = list(range(min(m, k)))
        objs[:, :len(er) * bs] = 0
        le.device.decode("cauchyrs", (k, m, w), objs, size,
                         gpu.from_numpy(outs[1]).cuda(), er)
        gpu.cuda.synchronize()
        assert gpu.equal(objs, ref), (k, m, size)


@pytest.mark.parametrize("tgroup", ["5", "128"])
def test_gf8_segment_map_forms(gpu, le, oracle, measure, tgroup):
    """gf8 tile map 4 (XCD-interleaved runs of consecutive tiles, shipped for
    blocks of >= 4096 tiles) forced on smaller objects, with run lengths that
    straddle object boundaries and a batch whose tail is not a whole group of
    8 runs: parity identical to tile-major order and to the oracle, and an
    in-place decode round trip."""
    k, m, w = 10, 4, 8
    n, size = 7, 3 * 1048576 + 4321
    bs, _ = le.layout("vandrs", (k, m, w), size)
    host, objs = _batch(gpu, n, size, max(k, m) * bs, 77)
    ref = objs.clone()
    outs = []
    measure.setenv("LEOEC_GF8_TGROUP", tgroup)
    for tmap in ("0", "4"):
        measure.setenv("LEOEC_GF8_TMAP", tmap)
        parity = gpu.zeros((n, max(k, m) * bs), dtype=gpu.uint8, device="cuda")
        le.device.encode("vandrs", (k, m, w), objs, size, parity)
        objs[:, :4 * bs] = 0xA5
        le.device.decode("vandrs", (k, m, w), objs, size, parity, [0, 1, 2, 3])
        gpu.cuda.synchronize()
        assert gpu.equal(objs, ref), tmap
        outs.append(parity.cpu().numpy())
    assert np.array_equal(outs[0], outs[1])
    for o in (0, n - 1):
        r = oracle.encode("vandrs", k, m, w, host[o, :size].tobytes())
        assert outs[1][o, :m * bs].tobytes() == b"".join(r[k:]), f"object {o}"


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


@pytest.mark.parametrize("w", [16, 32])
@pytest.mark.parametrize("env", [
    {},                                        # shipped: bitsliced planes (gfs_apply)
    {"LEOEC_GFW_FORM": "0"},                   # byte-plane v_perm, 2 columns per lane
    {"LEOEC_GFW_FORM": "0", "LEOEC_GFP_CPT": "1"},  # byte-plane, 1 column per lane
    {"LEOEC_GFW_FORM": "0", "LEOEC_GFP_BPC": "1"},  # byte-plane, 1 block per CU: long walks
    {"LEOEC_GFW_FORM": "1"},                   # w=16: 2-bit-field v_perm; w=32: shift-and-add
    {"LEOEC_GFW_FORM": "2"},                   # shift-and-add
    {"LEOEC_GFS_PF": "2"},                     # gfs_apply, two inputs in flight
])
def test_gfw_kernel_forms_agree(gpu, le, oracle, w, env, measure):
    """w = 16 / 32 through every kernel form: encode vs the oracle, decode
    and repair round trips, including > 16 inputs (accumulating launches,
    whose outputs are re-read into byte planes) and ragged tails."""
    for key, val in env.items():
        measure.setenv(key, val)
    for k, m, size in [(10, 4, 200011), (4, 2, 77777), (17, 5, 123457), (3, 3, 1000)]:
        data = rand_bytes(size, k * m + w)
        st, blocks = le.nif_encode("vandrs", (k, m, w), data, len(data))
        assert st == "ok" and blocks == oracle.encode("vandrs", k, m, w, data)
        ids = list(range(m, k + m))
        st, out = le.nif_decode("vandrs", (k, m, w), [blocks[i] for i in ids], ids, len(data))
        assert st == "ok" and out == data
        ids = list(range(1, k + 1))
        st, rep = le.nif_repair("vandrs", (k, m, w), [blocks[i] for i in ids], ids, [0, k + m - 1])
        assert st == "ok" and rep == [blocks[0], blocks[k + m - 1]]
        # the first parity alone: a row of ones, so every column is 0/1
        # (gfs_apply's word-domain columns only, no bitsliced input)
        ids = list(range(k))
        st, rep = le.nif_repair("vandrs", (k, m, w), [blocks[i] for i in ids], ids, [k])
        assert st == "ok" and rep == [blocks[k]]


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


@pytest.mark.parametrize("staging,chunk_kib", [("pinned", "16"), ("pinned", "256"),
                                               ("pinned", "8192"), ("pageable", "256"),
                                               ("gather", "256"), ("auto", "256"),
                                               ("zerocopy", "256")])
def test_host_staging_forms(gpu, le, oracle, staging, chunk_kib, measure):
    """Host entry points (the NIF path) under every staging form: the plain
    pageable copies, the default (auto: gather for several host buffers),
    the gather form (one pinned copy per direction,
    engine.cpp stage_h2d_segs / stage_d2h_sync) and the pinned-ring
    measurement form with chunks small enough to wrap the 8-slot ring many
    times within one call, and one chunk per object, and the zero-copy form
    (kernels on a pinned, device-mapped buffer; spans above its 16 MiB cap
    take the copy forms).  Encode / decode / repair bit-exact with the
    oracle, including ragged sizes and a 64 MiB + 5 object."""
    measure.setenv("LEOEC_HOST_STAGING", staging)
    measure.setenv("LEOEC_STAGE_CHUNK_KIB", chunk_kib)
    cases = [("vandrs", 10, 4, 8, 1048576), ("vandrs", 10, 4, 8, 300001),
             ("cauchyrs", 10, 4, 8, 1048576 + 77), ("isars", 4, 2, 8, 65536 + 7),
             ("liberation", 4, 2, 7, 777777), ("vandrs", 6, 3, 32, 123457)]
    if chunk_kib == "16" or staging in ("gather", "auto", "zerocopy"):
        # gather: a span above its 16 MiB pinned cap takes the pageable copies
        cases.append(("vandrs", 10, 4, 8, (64 << 20) + 5))
    if staging in ("gather", "auto", "zerocopy"):  # spans either side of the 16 MiB cap, D2H > H2D
        cases += [("vandrs", 10, 4, 8, 16 << 20), ("vandrs", 4, 6, 8, 5000),
                  ("vandrs", 2, 8, 8, 3000000)]
    for cls, k, m, w, size in cases:
        data = rand_bytes(size, size + 17 * k)
        ref = oracle.encode(cls, k, m, w, data)
        st, blocks = le.nif_encode(cls, (k, m, w), data, size)
        assert st == "ok" and blocks == ref, (cls, k, m, w, size)
        ids = list(range(m, k + m))[::-1]
        st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, size)
        assert st == "ok" and out == data, (cls, k, m, w, size)
        lost = [0, k + m - 1] if m > 1 else [0]
        avail = [b for b in range(k + m) if b not in lost]
        st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
        assert st == "ok" and rep == [ref[b] for b in lost], (cls, k, m, w, size)


def test_thread_exit_releases_staging(gpu, le, oracle):
    """Caller threads that come and go (dirty schedulers, pools) give back their
    per-thread stream, device buffer and pinned buffers (engine.cpp
    Staging::release): 160 short-lived threads each run a decode (gather
    staging) + encode of an 8 MiB object; device memory must not drift by
    their buffers (~19 MB each would be ~3 GB)."""
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


def _capi_case(le, oracle, cls, k, m, w, size, seed):
    """Inputs and oracle answers for one object, as numpy buffers for the C ABI."""
    data = np.frombuffer(rand_bytes(size, seed), dtype=np.uint8).copy()
    ref = oracle.encode(cls, k, m, w, data.tobytes())
    bs, filled = le.layout(cls, (k, m, w), size)
    return {"cls": cls, "cid": le._lib.CODING_IDS[cls], "p": (k, m, w), "size": size, "bs": bs,
            "filled": filled, "data": data, "ref": ref,
            "blocks": [np.frombuffer(b, dtype=np.uint8).copy() for b in ref]}


def _capi_roundtrip(le, c, t):
    """encode + decode (m blocks lost) + repair (2 blocks) through the C ABI;
    returns an error string or None."""
    import ctypes
    L = le.lib
    k, m, w = c["p"]
    bs, filled, size = c["bs"], c["filled"], c["size"]
    out = np.empty(max((k + m - filled) * bs, 1), dtype=np.uint8)
    rc = L.leoec_encode(c["cid"], k, m, w, c["data"].ctypes.data, size, out.ctypes.data, out.size)
    if rc or b"".join(c["ref"][filled:]) != out[:(k + m - filled) * bs].tobytes():
        return f"encode {c['cls']}{c['p']} size {size} rc {rc}"
    lost = sorted({(t * 7 + j * 3) % (k + m) for j in range(m)})
    ids = [b for b in range(k + m) if b not in lost][::-1]
    ptrs = (ctypes.c_void_p * len(ids))(*[c["blocks"][b].ctypes.data for b in ids])
    idv = (ctypes.c_int * len(ids))(*ids)
    dec = np.empty(max(size, 1), dtype=np.uint8)
    rc = L.leoec_decode(c["cid"], k, m, w, ptrs, idv, len(ids), bs, size, dec.ctypes.data)
    if rc or not np.array_equal(dec[:size], c["data"]):
        return f"decode {c['cls']}{c['p']} lost {lost} rc {rc}"
    rep = sorted({t % (k + m), (t + 5) % (k + m)})
    avail = [b for b in range(k + m) if b not in rep]
    ptrs = (ctypes.c_void_p * len(avail))(*[c["blocks"][b].ctypes.data for b in avail])
    idv = (ctypes.c_int * len(avail))(*avail)
    repv = (ctypes.c_int * len(rep))(*rep)
    ro = np.empty(len(rep) * bs, dtype=np.uint8)
    rc = L.leoec_repair(c["cid"], k, m, w, ptrs, idv, len(avail), bs, repv, len(rep),
                        ro.ctypes.data)
    if rc or ro.tobytes() != b"".join(c["ref"][b] for b in rep):
        return f"repair {c['cls']}{c['p']} {rep} rc {rc}"
    return None


@pytest.mark.parametrize("form", ["product", "always-batch", "per-thread", "lanes4",
                                  "lanes4-always-batch", "fail-one", "zc-batch"])
def test_host_batching_mixed_callers(gpu, le, oracle, form, request):
    """Cross-call batching (hostq.cpp): 24 threads call the C ABI at once with
    mixed classes, widths, sizes (ragged, and 9 MiB objects above the batch
    cap, which take the per-thread path) and erasure patterns, so one batch
    holds several different maps (several launches) and identical maps are
    merged into one launch.  Every result equals the oracle's.  The
    measurement build forces every call through the queue (always-batch) or
    none (per-thread) and reports how calls were batched; "lanes4" runs the
    node dispatcher with 4 lanes (queues) mapped onto the box's device(s),
    every lane carrying jobs; "fail-one" makes the batched launches of one
    spec report a HIP error: exactly those calls fail, every other call in
    the same batches succeeds bit-exact."""
    import concurrent.futures as cf
    stats = lane_jobs = None
    fail_bs = None
    if form != "product":
        ms = request.getfixturevalue("measure")
        if form in ("always-batch", "lanes4-always-batch", "fail-one", "zc-batch"):
            ms.setenv("LEOEC_HOSTQ_DIRECT", "0")
            ms.setenv("LEOEC_HOSTQ_DIRECT_MAP", "0")
        if form == "per-thread":
            ms.setenv("LEOEC_HOST_BATCH", "0")
        if form.startswith("lanes4"):
            ms.setenv("LEOEC_HOSTQ_LANES", "4")
            assert len(le._lib.host_lanes()) == 4
        if form == "zc-batch":
            ms.setenv("LEOEC_HOSTQ_ZC", "1")
        if form == "fail-one":
            fail_bs = 1296  # cauchyrs(4,2,3) on 5000 B: bs = ceil16(5000 / 12) * 3
            ms.setenv("LEOEC_HOSTQ_FAIL_BS", str(fail_bs))
        stats = le._lib._current.leoec_measure_hostq_stats
        lane_jobs = le._lib._current.leoec_measure_hostq_lane_jobs
    specs = [("vandrs", 10, 4, 8, 1048576), ("vandrs", 10, 4, 8, 1048576),
             ("vandrs", 10, 4, 8, 300001), ("cauchyrs", 10, 4, 8, 1048576 + 77),
             ("isars", 10, 4, 8, 65536 + 7), ("liberation", 4, 2, 7, 777777),
             ("vandrs", 4, 2, 16, 123457), ("vandrs", 6, 3, 32, 99999),
             ("vandrs", 10, 4, 8, 9 << 20), ("cauchyrs", 4, 2, 3, 5000),
             ("vandrs", 20, 6, 8, 2000003)]
    cases = [_capi_case(le, oracle, *sp, seed=100 + i) for i, sp in enumerate(specs)]
    import ctypes
    buf = (ctypes.c_double * 14)()
    lanes = (ctypes.c_double * 64)()
    if stats:
        stats(buf)
        lane_jobs(lanes)

    def worker(t):
        failed = 0
        for r in range(8):
            c = cases[(t + r) % len(cases)]
            e = _capi_roundtrip(le, c, t + r)
            if fail_bs is not None and c["bs"] == fail_bs:
                # the injected failure: the encode reports the HIP error
                if not (e and e.startswith("encode") and e.endswith(f"rc {le._lib.E_HIP}")):
                    return f"thread {t}: expected an injected failure, got {e}"
                failed += 1
                continue
            if e:
                return f"thread {t}: {e}"
        return None

    with cf.ThreadPoolExecutor(24) as ex:
        errs = [e for e in ex.map(worker, range(24)) if e]
    assert not errs, errs
    if stats:
        stats(buf)
        lane_jobs(lanes)
        batches, jobs, launches = buf[0], buf[1], buf[2]
        if form in ("always-batch", "lanes4-always-batch", "zc-batch"):
            # 24 x 8 x 3 calls, minus the 9 MiB ones (per-thread path)
            assert jobs >= 24 * 8 * 3 * 0.8 and batches < jobs and launches > batches, list(buf)
        elif form == "per-thread":
            assert batches == 0, list(buf)
        if form.startswith("lanes4"):
            assert sum(1 for x in lanes[:4] if x > 0) >= (4 if "always" in form else 2), \
                list(lanes[:4])
            assert sum(lanes[4:]) == 0
