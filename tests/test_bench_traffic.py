"""bench.py's roofline.traffic comes from a committed PMC measurement
(profiles/pmc_traffic*.json) only while the loaded library holds the code
object that measurement ran on: a stamp mismatch, a missing stamp or another
batch shape yields null, never a stale figure (CPU only: reads files)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from leo_erasure_amd import _lib, codeobj  # noqa: E402

LIB = _lib.LIB_PATH


def _write(tmp_path, name, sha, objects=2048, size=1048576, traffic=3007585843):
    rec = {"objects": objects, "object_bytes": size, "encode_bytes_per_launch": traffic}
    if sha is not None:
        rec["code_object"] = {"kernel": "gf8_apply<10, 4>", "sha256": sha}
    p = tmp_path / name
    p.write_text(json.dumps(rec))
    return str(p)


def test_library_defines_the_headline_kernel_once():
    hits = [b for b in codeobj.bundles(LIB) if codeobj.GF8_10_4 in b]
    assert len(hits) == 1
    sha = codeobj.kernel_code_object_sha256(LIB)
    assert sha and len(sha) == 64 and sha == codeobj.kernel_code_object_sha256(LIB)


def test_matching_stamp_gives_the_figure(tmp_path):
    p = _write(tmp_path, "t.json", codeobj.kernel_code_object_sha256(LIB))
    traffic, src = bench.read_traffic(p, 2048, 1048576, LIB)
    assert traffic == 3007585843 and "code object" in src


@pytest.mark.parametrize("sha", ["0" * 64, None])
def test_mismatched_or_missing_stamp_gives_null(tmp_path, sha):
    p = _write(tmp_path, "t.json", sha)
    traffic, src = bench.read_traffic(p, 2048, 1048576, LIB)
    assert traffic is None and src


def test_other_batch_shape_gives_null(tmp_path):
    p = _write(tmp_path, "t.json", codeobj.kernel_code_object_sha256(LIB), objects=1024)
    assert bench.read_traffic(p, 2048, 1048576, LIB)[0] is None


def test_first_matching_shape_is_used(tmp_path):
    sha = codeobj.kernel_code_object_sha256(LIB)
    a = _write(tmp_path, "a.json", sha, objects=64, size=67108864, traffic=6013199104)
    b = _write(tmp_path, "b.json", sha)
    assert bench.read_traffic(f"{a},{b}", 64, 67108864, LIB)[0] == 6013199104
    assert bench.read_traffic(f"{a},{b}", 2048, 1048576, LIB)[0] == 3007585843


def test_unknown_library_gives_null(tmp_path):
    p = _write(tmp_path, "t.json", codeobj.kernel_code_object_sha256(LIB))
    assert bench.read_traffic(p, 2048, 1048576, None)[0] is None
