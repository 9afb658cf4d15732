"""NIF-surface argument handling of the Python mirror (no GPU needed): the
checks that run before any block arithmetic (c_src/leo_erasure_nif.cpp)."""
import pytest


def test_encode_argument_errors(le):
    assert le.nif_encode("vandrs", (10, 4, 8), 12345, 0) == ("error", "Expected Input Bin")
    assert le.nif_encode(42, (10, 4, 8), b"abc", 3) == ("error", "Expect coding")
    assert le.nif_encode("vandrs", [10, 4, 8], b"abc", 3) == \
        ("error", "Expect tuple for coding parameters")
    assert le.nif_encode("vandrs", ("a", 4, 8), b"abc", 3) == ("error", "Invalid K")
    assert le.nif_encode("vandrs", (10, None, 8), b"abc", 3) == ("error", "Invalid M")
    assert le.nif_encode("vandrs", (10, 4), b"abc", 3) == ("error", "Invalid W")
    assert le.nif_encode("bogus", (10, 4, 8), b"abc", 3) == ("error", "Invalid Coding")
    assert le.nif_encode("vandrs", (4, 2, 7), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (w = 8/16/32)")
    assert le.nif_encode("vandrs", (0, 2, 8), b"abc", 3) == ("error", "Invalid Coding Parameters")
    assert le.nif_encode("cauchyrs", (10, 4, 3), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (larger w)")
    assert le.nif_encode("liberation", (4, 3, 7), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (m = 2)")
    assert le.nif_encode("liberation", (8, 2, 7), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (k <= w)")
    assert le.nif_encode("liberation", (4, 2, 9), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (w is prime)")
    assert le.nif_encode("isars", (4, 2, 16), b"abc", 3) == \
        ("error", "Invalid Coding Parameters (w = 8)")


def test_decode_argument_errors(le):
    b = [b"\0" * 16] * 6
    assert le.nif_decode("vandrs", (4, 2, 8), b, [0, 1, 2], 10) == \
        ("error", "Block List and ID List does not match (different Len)")
    assert le.nif_decode("vandrs", (4, 2, 8), "x", [0], 10) == ("error", "Block List Needed")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:1], "x", 10) == ("error", "ID List Needed")
    assert le.nif_decode("vandrs", (4, 2, 8), [7], [0], 10) == ("error", "Invalid Block")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:1], ["a"], 10) == ("error", "Invalid ID")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:1], [0], -1) == ("error", "Expect data size")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:3], [0, 1, 2], 10) == \
        ("error", "Not Enough Blocks")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:5], [0, 1, 2, 3, 3], 10) == \
        ("error", "Blocks should be unique")
    assert le.nif_decode("vandrs", (4, 2, 8), b[:4], [0, 1, 2, 9], 10) == \
        ("error", "Invalid Block ID")
    assert le.nif_decode("nope", (4, 2, 8), b[:4], [0, 1, 2, 3], 10) == ("error", "Invalid Coding")


def test_decode_fast_path_is_host_copy(le):
    """All data blocks present: the reference concatenates (rscoding.cpp:112-123);
    no GPU is involved, so it works here, and handles pure-padding tails."""
    data = bytes(range(256)) * 4 + b"xyz"
    bs = 128  # vandrs {10,4,8}: 1027 B -> bs 128, block 8 has 3 bytes, block 9 none
    assert le.layout("vandrs", (10, 4, 8), len(data)) == (bs, 8)
    blocks = [data[i * bs:(i + 1) * bs].ljust(bs, b"\0") for i in range(10)]
    ids = list(range(10))[::-1]
    assert le.nif_decode("vandrs", (10, 4, 8), blocks[::-1], ids, len(data)) == ("ok", data)


def test_repair_argument_errors(le):
    b = [b"\0" * 16] * 6
    ids = list(range(6))
    assert le.nif_repair("vandrs", (4, 2, 8), b, ids, "x") == ("error", "Repair ID List Needed")
    assert le.nif_repair("vandrs", (4, 2, 8), b, ids, ["z"]) == ("error", "Invalid Repair ID")
    assert le.nif_repair("vandrs", (4, 2, 8), b, ids, [6]) == ("error", "Invalid Block ID")
    # a listed block asked for is returned as staged (Jerasure classes), host-side
    assert le.nif_repair("vandrs", (4, 2, 8), b, ids, [1, 5]) == ("ok", [b[1], b[5]])


def test_erlang_wrappers_fill_defaults(le):
    assert le.env_default_coder() == "vandrs"
    le.set_default_coder("isars")
    try:
        assert le.env_default_coder() == "isars"
    finally:
        le.set_default_coder(None)
    with pytest.raises(TypeError):
        le.encode(1)
