"""Measurement-build form tests: every A/B kernel form and staging / queue
policy of libleoec_measure.so against the CPU oracle (bit-exact).

They run in a process of their own that loads only the measurement library
(LEOEC_LIBRARY=measure), started by
test_gpu_parity.py::test_measurement_forms_in_own_process, so the product
tests' process never holds two HIP libraries; knobs are set through the
library's setter (leoec_measure_set_knob), never through the environment.
Run directly: LEOEC_LIBRARY=measure python -m pytest tests/test_measure_forms.py -m measure_gpu
"""
import numpy as np
import pytest

from gpu_helpers import batch as _batch
from gpu_helpers import mixed_callers, rand_bytes

pytestmark = [pytest.mark.gpu, pytest.mark.measure_gpu]



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
    _liberation_roundtrips(le, oracle)


@pytest.mark.parametrize("env", [{}, {"LEOEC_LIB_LA": "4"}, {"LEOEC_LIB_LA": "8"},
                                 {"LEOEC_LIB_WG": "256"}, {"LEOEC_LIB_WG": "256", "LEOEC_LIB_LA": "4"},
                                 {"LEOEC_LIB_DEC_WG": "64"}, {"LEOEC_LIB_DEC_LA": "4"},
                                 {"LEOEC_LIB_DEC_LA": "8", "LEOEC_LIB_DEC_WG": "64"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()) or "shipped")
def test_liberation_buffer_load_forms(gpu, le, oracle, env, measure):
    """libb_apply / libb_dec_apply (LEOEC_LIB_BUF=1: branch-free raw buffer
    loads, the block count compiled in, one instance per (w, k)): every w, k
    from 1 to w, ragged sizes (tiles that cross a block's valid length clear
    the straddling chunk's tail where it is consumed), the look-ahead and
    lane-count forms built for the A/B configurations, against the oracle."""
    measure.setenv("LEOEC_LIB_BUF", "1")
    for k, v in env.items():
        measure.setenv(k, v)
    _liberation_roundtrips(le, oracle)


def _liberation_roundtrips(le, oracle):
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
            # syndrome repair of coding blocks (round 5): {data, P}, {data, Q},
            # P alone, Q alone, from every other block
            for want in ([0, k], [k - 1, k + 1], [k], [k + 1]):
                ids = [i for i in range(k + 2) if i not in want]
                st, rep = le.nif_repair("liberation", (k, 2, w), [blocks[i] for i in ids], ids, want)
                assert st == "ok" and rep == [blocks[i] for i in want], (k, w, want)


@pytest.mark.parametrize("k,w,size", [(7, 7, 300007), (4, 7, 1048576), (10, 11, 1048573)])
def test_liberation_device_batch_forms(gpu, le, oracle, measure, k, w, size):
    """Device-resident batch (37 objects, bytes past each object's size
    random) through every liberation encode form — lib_apply, libb_apply
    (LEOEC_LIB_BUF=1) and the generic masked kernel — and the two syndrome
    decode forms: identical outputs, equal to the oracle."""
    m = 2
    n = 37
    bs, _ = le.layout("liberation", (k, m, w), size)
    stride = max(k * bs, size + 9 - (size + 9) % 16 + 16)
    host, objs = _batch(gpu, n, size, stride, 21 + k)
    outs = []
    for form, buf in (("1", "0"), ("1", "1"), ("0", "0")):
        measure.setenv("LEOEC_LIB_FORM", form)
        measure.setenv("LEOEC_LIB_BUF", buf)
        parity = gpu.full((n, m * bs), 0x5A, dtype=gpu.uint8, device="cuda")
        le.device.encode("liberation", (k, m, w), objs, size, parity)
        gpu.cuda.synchronize()
        outs.append(parity.cpu().numpy())
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[0], outs[2])
    for o in range(0, n, 6):
        ref = oracle.encode("liberation", k, m, w, host[o, :size].tobytes())
        assert outs[0][o].tobytes() == b"".join(ref[k:]), f"object {o}"
    # decode of two lost data blocks (syndromes through P and Q) in place
    measure.setenv("LEOEC_LIB_FORM", "1")
    parity = gpu.from_numpy(outs[0]).cuda()
    lost = [0, k - 1]
    for buf in ("0", "1"):
        measure.setenv("LEOEC_LIB_BUF", buf)
        dec = objs.clone()
        for j in lost:
            lo, hi = j * bs, min((j + 1) * bs, size)
            dec[:, lo:hi] = 0xA5
        le.device.decode("liberation", (k, m, w), dec, size, parity, lost)
        gpu.cuda.synchronize()
        assert gpu.equal(dec[:, :size], objs[:, :size]), f"decode LIB_BUF={buf}"


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


@pytest.mark.parametrize("form", ["1", "2", "3", "4", "5", "6", "7", "8", "9"])
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


@pytest.mark.parametrize("form,env", [
    ("3", {}), ("3", {"LEOEC_GFBIT_WG": "256"}), ("3", {"LEOEC_GFBIT_PF": "2"}),
    ("3", {"LEOEC_GFBIT_PF": "3"}), ("3", {"LEOEC_GFBIT_PF": "4"}), ("3", {"LEOEC_GFBIT_PF": "5"}),
    ("5", {}), ("5", {"LEOEC_GFBIT_PF": "2"}), ("5", {"LEOEC_GFBIT_PF": "3"}),
    ("5", {"LEOEC_GFBIT_WG": "64"}), ("5", {"LEOEC_GFBIT_WG": "64", "LEOEC_GFBIT_PF": "3"}),
    ("5", {"LEOEC_GFBIT_WG": "256"}), ("5", {"LEOEC_GFBIT_WAVES": "2", "LEOEC_GFBIT_PF": "2"})],
    ids=lambda e: e if isinstance(e, str) else (",".join(f"{k}={v}" for k, v in e.items()) or "default"))
def test_cauchy_16B_forms_batches(gpu, le, oracle, measure, form, env):
    """cauchyrs through the 16-byte-access forms gfba_apply
    (LEOEC_GFBIT_FORM=3: line-aligned 16-byte copies into per-wave LDS slots,
    read back at each packet's phase; round 4's gfbs_apply, form 4, ran here
    too before it was removed, code at cd96abc) and gfbk_apply (FORM=5: K = 10
    compiled in, 16-byte lanes, one wave per SIMD, blocks of loads in flight;
    the other k fall back to the shipped kernel).  Object rows at every
    16-byte phase mod 128 (row stride = k*bs + 48), sizes whose blocks are
    full, short (last block 103,936 of 104,960 B), one packet of 16 B, and
    empty (size 1,040: block 9 holds nothing); encode parity equal to the
    shipped kernel's and to the oracle's, decode and repair of erased data
    and parity blocks in place."""
    measure.setenv("LEOEC_GFBIT_FORM", form)
    for key, v in env.items():
        measure.setenv(key, v)
    sizes = [(10, 4, 1048576), (10, 4, 1048576 - 16 * 21), (10, 4, 77776),
             (10, 4, 1040), (6, 3, 300000), (4, 2, 262144 + 4096)]
    for k, m, size in sizes:
        w, n = 8, 11
        bs, _ = le.layout("cauchyrs", (k, m, w), size)
        stride = max(k, m) * bs + 48
        host, objs = _batch(gpu, n, size, stride, 91 + size % 89)
        ref = objs.clone()
        outs = []
        for f in ("0", form):
            measure.setenv("LEOEC_GFBIT_FORM", f)
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
        assert st == "ok" and rep == [ref[b] for b in lost], (cls, k, m, w, size,
                                                              rep if st != "ok" else "")


@pytest.mark.parametrize("chunks", ["2", "3", "8"])
def test_host_zero_copy_chunks(gpu, le, oracle, chunks, measure):
    """The measurement build's chunked zero-copy form (LEOEC_ZC_CHUNKS,
    engine.cpp zc_chunked): a lone caller's GF(2^w) map in column chunks,
    packing chunk c + 1 while chunk c runs and unpacking each as its launch
    completes.  Encode / decode / repair through the per-thread path (the
    queue never batches: LEOEC_HOST_BATCH=0), bit-exact with the oracle, over
    ragged sizes and chunk edges inside and past the valid bytes; bitmatrix
    classes fall back to one piece."""
    measure.setenv("LEOEC_ZC_CHUNKS", chunks)
    measure.setenv("LEOEC_HOST_BATCH", "0")
    cases = [("vandrs", 10, 4, 8, 1 << 20), ("vandrs", 10, 4, 8, (1 << 20) - 4095),
             ("isars", 10, 4, 8, 3 * (1 << 20) + 17), ("vandrs", 4, 2, 8, 40000),
             ("vandrs", 6, 3, 16, 777777), ("vandrs", 5, 3, 32, 1 << 20),
             ("vandrs", 20, 6, 8, 2000003), ("cauchyrs", 10, 4, 8, 1 << 20),
             ("liberation", 7, 2, 7, 1 << 20)]
    for cls, k, m, w, size in cases:
        data = rand_bytes(size, size + 31 * k)
        ref = oracle.encode(cls, k, m, w, data)
        st, blocks = le.nif_encode(cls, (k, m, w), data, size)
        assert st == "ok" and blocks == ref, (cls, k, m, w, size)
        ids = list(range(m, k + m))[::-1]
        st, out = le.nif_decode(cls, (k, m, w), [ref[b] for b in ids], ids, size)
        assert st == "ok" and out == data, (cls, k, m, w, size)
        lost = [0, k + m - 1]
        avail = [b for b in range(k + m) if b not in lost]
        st, rep = le.nif_repair(cls, (k, m, w), [ref[b] for b in avail], avail, lost)
        assert st == "ok" and rep == [ref[b] for b in lost], (cls, k, m, w, size)


@pytest.mark.parametrize("form", ["always-batch", "per-thread", "lanes4",
                                  "lanes4-always-batch", "fail-one", "zc-batch",
                                  "always-batch-slot-stream", "fail-one-slot-stream",
                                  "always-batch-eager", "fail-one-eager"])
def test_host_batching_mixed_callers(gpu, le, oracle, form, measure):
    """gpu_helpers.mixed_callers under the measurement build's queue
    policies: every call through the queue (always-batch) or none
    (per-thread), with the batching counters checked; "lanes4" runs the node
    dispatcher with 4 lanes (queues) mapped onto the box's device(s), every
    lane carrying jobs; "zc-batch" batches without DMA copies; "fail-one"
    makes the batched launches of one spec (cauchyrs(4,2,3) on 5000 B, bs
    1296) report a HIP error: its encodes, repairs and data-rebuilding
    decodes fail with LEOEC_E_HIP, every other call of the same batches
    succeeds bit-exact.  The queue's copies run on its two copy streams
    (shipped) except in the "-slot-stream" forms (LEOEC_HOSTQ_STREAMS=0: a
    batch's copies and launches all on its slot's stream), and the "-eager"
    forms hand a complete batch to the worker as its last job reserves
    (LEOEC_HOSTQ_EAGER)."""
    import ctypes
    fail_bs = None
    if form.endswith("-eager"):  # complete batches handed over early (LEOEC_HOSTQ_EAGER)
        measure.setenv("LEOEC_HOSTQ_EAGER", "1")
        form = form[:-len("-eager")]
    if form.endswith("-slot-stream"):
        measure.setenv("LEOEC_HOSTQ_STREAMS", "0")
        form = form[:-len("-slot-stream")]
    if form in ("always-batch", "lanes4-always-batch", "fail-one", "zc-batch"):
        measure.setenv("LEOEC_HOSTQ_DIRECT", "0")
        measure.setenv("LEOEC_HOSTQ_DIRECT_MAP", "0")
    if form == "per-thread":
        measure.setenv("LEOEC_HOST_BATCH", "0")
    if form.startswith("lanes4"):
        measure.setenv("LEOEC_HOSTQ_LANES", "4")
        assert len(le._lib.host_lanes()) == 4
        if form == "lanes4":  # some calls per-thread, enough batched to reach every lane
            measure.setenv("LEOEC_HOSTQ_DIRECT", "4")
            measure.setenv("LEOEC_HOSTQ_DIRECT_MAP", "2")
    if form == "zc-batch":
        measure.setenv("LEOEC_HOSTQ_ZC", "1")
    if form == "fail-one":
        fail_bs = 1296  # cauchyrs(4,2,3) on 5000 B: bs = ceil16(5000 / 12) * 3
        measure.setenv("LEOEC_HOSTQ_FAIL_BS", str(fail_bs))
    stats = le._lib._current.leoec_measure_hostq_stats
    lane_jobs = le._lib._current.leoec_measure_hostq_lane_jobs
    buf = (ctypes.c_double * 14)()
    lanes = (ctypes.c_double * 64)()
    stats(buf)
    lane_jobs(lanes)
    errs, injected = mixed_callers(le, oracle, fail_bs=fail_bs)
    assert not errs, errs
    if fail_bs is not None:
        assert injected > 0
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


def test_pattern_kernels_do_what_they_claim(gpu, le):
    """bench.py's pattern-ceiling kernels (measurement library,
    csrc/xor_pattern.hip) on a ragged batch: xor_pattern writes every parity
    block as the XOR of the 10 data blocks (zero past the object); the
    read half writes nothing; the write half writes its documented pattern
    and reads nothing."""
    import ctypes

    import torch

    from leo_erasure_amd import _lib
    mlib = _lib.measure_library()
    # the last data block is short (29,280 of 30,080 B); the object ends on a
    # 16-byte boundary: a 16-byte buffer load across the range's end reads
    # zeros at the hardware's granularity, which bytes of a straddling chunk
    # is not what this checks
    n, size = 12, 300000
    bs = ((size + 79) // 80 + 15) // 16 * 16 * 8
    stride = (size + 15) // 16 * 16 + 64
    g = torch.Generator(device="cuda").manual_seed(7)
    objs = torch.randint(0, 256, (n, stride), dtype=torch.uint8, device="cuda", generator=g)
    parity = torch.full((n, 4 * bs), 0xAB, dtype=torch.uint8, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    args = (objs.data_ptr(), stride, size, n, parity.data_ptr(), 4 * bs, st)

    assert mlib.leoec_measure_stream_half_dev(0, *args) == 0
    torch.cuda.synchronize()
    assert bool((parity == 0xAB).all()), "the read half wrote"

    assert mlib.leoec_measure_xor_pattern_dev(*args) == 0
    torch.cuda.synchronize()
    host = objs.cpu().numpy()
    data = np.zeros((n, 10 * bs), dtype=np.uint8)
    data[:, :size] = host[:, :size]
    want = np.bitwise_xor.reduce(data.reshape(n, 10, bs), axis=1)
    got = parity.cpu().numpy().reshape(n, 4, bs)
    for r in range(4):
        assert np.array_equal(got[:, r], want), f"xor_pattern parity block {r}"

    assert mlib.leoec_measure_stream_half_dev(1, *args) == 0
    torch.cuda.synchronize()
    got = parity.cpu().numpy().reshape(n, 4, bs // 16, 4 * 4).view(np.uint32).reshape(n, 4, bs // 16, 4)
    off = np.arange(bs // 16, dtype=np.uint32) * 16
    for o in (0, 5, n - 1):
        for r in range(4):
            exp = np.stack([(off // 16) % 64, np.full_like(off, o), off, np.full_like(off, r)], axis=1)
            assert np.array_equal(got[o, r], exp), f"write half object {o} block {r}"
    assert mlib.leoec_measure_stream_half_dev(2, *args) == -1
