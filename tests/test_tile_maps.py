"""The workgroup-id remaps of the GPU kernels (leo_erasure_amd/csrc/
tile_maps.hpp), compiled for the CPU: every map the launchers use is a
permutation of [0, n) — no tile skipped or done twice — including batches
that are not whole rounds of 8 groups, and each XCD's share is what the map
promises (whole objects for tile map 3, runs of consecutive tiles for tile
map 4)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def maps(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("tm") / "libtile_maps_test.so")
    subprocess.run(["g++", "-std=c++17", "-O2", "-fPIC", "-shared", "-Wall", "-Werror",
                    os.path.join(HERE, "tile_maps_test.cpp"), "-o", so], check=True)
    L = ctypes.CDLL(so)
    L.tile_map_image.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
    L.packet_lane_check.argtypes = [ctypes.c_uint32] * 6
    return L


def image(maps, kind, n, tiles=1):
    out = np.zeros(n, dtype=np.uint32)
    rc = maps.tile_map_image(kind, n, tiles, out.ctypes.data)
    assert rc == 0, f"map {kind} n={n} tiles={tiles}: id {rc - 1} collides"
    return out


@pytest.mark.parametrize("n", [1, 7, 8, 9, 1000, 2048 * 26, 13 * 26 + 5])
def test_xcd_group_is_a_permutation(maps, n):
    m = image(maps, 0, n)
    # XCD x (ids b = x mod 8) covers one contiguous range of tiles
    for x in range(min(8, n)):
        r = np.sort(m[x::8])
        assert np.all(np.diff(r.astype(np.int64)) == 1)


# (objects, tiles per object) of the shipped launches: 1 MiB RS(10,4,8) at 26
# tiles (256 lanes), cauchyrs 7 tiles, ragged batches; tile map 4 over runs of
# 128 (and the parity tests' 5) tiles of 32 / 64 MiB objects (3,277 / 6,554
# 1 KiB tiles per block), batches of 1-64 objects
@pytest.mark.parametrize("nobj,tiles,run", [
    (2048, 26, 26), (1024, 7, 7), (13, 26, 26), (7, 64, 64), (1, 26, 26),
    (64, 6554, 128), (3, 6554, 128), (128, 3277, 128), (7, 308, 5), (7, 308, 128), (1, 6554, 128)])
def test_xcd_obj_map_is_a_permutation(maps, nobj, tiles, run):
    n = nobj * tiles
    m = image(maps, 1, n, run)
    full = (n // run // 8) * 8 * run
    # inside whole rounds, XCD x's i-th workgroup takes tile i % run of group
    # (i // run) * 8 + x: runs of `run` consecutive tiles, in order
    for x in range(8):
        ids = np.arange(x, full, 8)
        got = m[ids].astype(np.int64)
        i = ids // 8
        assert np.array_equal(got, ((i // run) * 8 + x) * run + i % run)
    assert np.array_equal(m[full:], np.arange(full, n))
    if run == tiles:  # tile map 3: every object entirely on one XCD
        xcd_of = np.empty(n, dtype=np.int64)
        xcd_of[m] = np.arange(n) % 8
        per_obj = xcd_of[: (full // tiles) * tiles].reshape(-1, tiles)
        assert np.all(per_obj == per_obj[:, :1])


def _bs(size, k, w):
    """leo_erasure's block size: ceil16(ceil(size / (k w))) w (common.cpp:24)."""
    return -(-(-(-size // (k * w))) // 16) * 16 * w


# (WG lanes, bytes per lane) of every gfbit_apply / gfb2_apply launch form:
# shipped 256 x 8 (w <= 11) and 256 x 4 (w >= 12); measurement forms 256 x 16,
# 128 x 16 (both look-ahead settings, including the one that aborted in round
# 2), 64 x 8
PACKET_FORMS = [(256, 8), (256, 4), (256, 16), (128, 16), (64, 8)]


@pytest.mark.parametrize("wg,lb", PACKET_FORMS)
def test_packet_lane_geometry(maps, wg, lb):
    """Every packet-kernel launch shape of the parity tests and the BASELINE
    configs: cauchyrs(10,4,8) at 1 MiB (ps 13,120, packets start mid line) and
    100,003 B (the round-2 abort's first call), (6,3,4), (4,2,3), every w of
    gfbit (2..16) on ragged sizes; data blocks full, partial (the tail block)
    and empty, output blocks full and clipped."""
    cases = [(1048576, 10, 8), (100003, 10, 8), (100003, 6, 4), (100003, 4, 3),
             (1054720, 10, 8), (1, 10, 8), (4097, 4, 3)]
    cases += [(150001, 5, w) for w in range(2, 17)]
    for size, k, w in cases:
        bs = _bs(size, k, w)
        tail = size - (k - 1) * bs if size > (k - 1) * bs else 0
        for vin in sorted({bs, max(tail, 0), 0, 1, bs - 1, bs // 2 + 3}):
            for vout in sorted({bs, vin}):
                if vin > bs or vout > bs:
                    continue
                rc = maps.packet_lane_check(bs, w, wg, lb, vin, vout)
                assert rc == 0, (size, k, w, bs, vin, vout, rc)
