"""Our NIF shim (leo_erasure_amd/csrc/nif/leo_erasure_nif.cpp), compiled against
the test-double erl_nif.h in tests/nif_harness/ and driven term by term.

Erlang/OTP is not installed here, so the shim is linked with a small term
store instead of the VM (tests/nif_harness/harness.cpp).  The CPU tests pin
the NIF table and every argument-error branch against the reference's order
and strings (reference c_src/leo_erasure_nif.cpp:130-353), cross-checked with
the Python mirror (leo_erasure_amd/api.py); the GPU tests run encode / decode
/ repair through the shim into libleoec.so and compare with the oracle,
including the zero-copy sub-binary layout of encode's result.
"""
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

from nif_harness.term import Atom, Harness, Raw, Sub, build, text  # noqa: E402

ok, error = Atom("ok"), Atom("error")
VANDRS = Atom("vandrs")


@pytest.fixture(scope="module")
def nif(tmp_path_factory, le):
    so = build(str(tmp_path_factory.mktemp("nif")))
    h = Harness(so)
    yield h
    h.L.h_reset()


@pytest.fixture(scope="module")
def nif_ref(tmp_path_factory, le):
    """The shim built with -DLEOEC_NIF_REF_ERRORS (the reference's error terms)."""
    so = build(str(tmp_path_factory.mktemp("nif_ref")), ("LEOEC_NIF_REF_ERRORS",))
    h = Harness(so)
    yield h
    h.L.h_reset()


@pytest.fixture(autouse=True)
def _fresh(request):
    hs = [request.getfixturevalue(n) for n in ("nif", "nif_ref") if n in request.fixturenames]
    for h in hs:
        h.L.h_reset()
    yield
    for h in hs:
        # every enif_alloc_binary was either handed to the VM or released, and
        # no term was made from a buffer the NIF does not own
        assert h.L.h_live_allocs() == 0
        assert h.L.h_violations() == 0


def err(r):
    assert isinstance(r, tuple) and len(r) == 2 and r[0] == error, r
    return text(r[1])


def test_nif_table(nif):
    # reference c_src/leo_erasure_nif.cpp:346-351: same names and arities;
    # ours run on dirty IO schedulers (a GPU round trip per call).
    assert nif.funcs() == [("gf_init", 0, 2), ("encode", 4, 2), ("decode", 5, 2),
                           ("repair", 5, 2)]


def test_gf_init_reports(nif, le):
    r = nif.call("gf_init")
    if r == ok:
        assert le.gf_init() == "ok"
    else:  # no gfx950 device here: an error tuple with the engine's text, never a CPU fallback
        assert err(r) == le.gf_init()[1]


PARAMS = (10, 4, 8)
DATA = bytes(range(256)) * 5

# (args, reason) for encode/4 — reference nif.cpp:130-166 check order
ENCODE_ERRORS = [
    ((VANDRS, PARAMS, Atom("x"), 0), "Expected Input Bin"),
    ((Atom("nope"), Atom("p"), 7, 0), "Expected Input Bin"),       # data checked first
    ((VANDRS, PARAMS, [b"a", (1,)], 0), "Expected Input Bin"),     # tuple is not an iolist
    ((VANDRS, PARAMS, [b"a", 256], 0), "Expected Input Bin"),      # byte out of range
    ((b"vandrs", PARAMS, DATA, 0), "Expect coding"),
    ((VANDRS, [10, 4, 8], DATA, 0), "Expect tuple for coding parameters"),
    ((Atom("nope"), [10, 4, 8], DATA, 0), "Expect tuple for coding parameters"),
    ((VANDRS, (Atom("k"), 4, 8), DATA, 0), "Invalid K"),
    ((VANDRS, (1 << 31, 4, 8), DATA, 0), "Invalid K"),             # not a C int
    ((VANDRS, (10, b"4", 8), DATA, 0), "Invalid M"),
    ((VANDRS, (10, 4), DATA, 0), "Invalid W"),
    ((VANDRS, (), DATA, 0), "Invalid K"),
    ((Atom("nope"), PARAMS, DATA, 0), "Invalid Coding"),
    ((Atom("nope"), (Atom("k"), 4, 8), DATA, 0), "Invalid K"),     # params before class
]


@pytest.mark.parametrize("args,reason", ENCODE_ERRORS, ids=[r for _, r in ENCODE_ERRORS])
def test_encode_argument_errors(nif, args, reason):
    assert err(nif.call("encode", *args)) == reason


@pytest.mark.parametrize("cls,params", [("vandrs", (10, 4, 7)), ("vandrs", (0, 4, 8)),
                                        ("cauchyrs", (4, 2, 1)), ("liberation", (4, 2, 8)),
                                        ("liberation", (8, 2, 7)), ("liberation", (4, 3, 7)),
                                        ("isars", (10, 4, 16)), ("vandrs", (200, 100, 8))])
def test_encode_parameter_errors(nif, le, oracle, cls, params):
    # coder constructor errors: the engine's text, which is the reference's
    # coder message (e.g. rscoding.cpp:30-37), same as the Python mirror
    r = err(nif.call("encode", Atom(cls), params, DATA, len(DATA)))
    assert r == le.strerror(oracle.check_params(cls, *params))
    assert ("error", r) == le.nif_encode(cls, params, DATA, len(DATA))


def _ok_blocks(n=3, size=8):
    return [bytes([i]) * size for i in range(n)]


DECODE_ERRORS = [
    ((VANDRS, PARAMS, b"x", [0], 10), "Block List Needed"),
    ((VANDRS, PARAMS, [b"x"], 0, 10), "ID List Needed"),
    ((VANDRS, PARAMS, [b"x", b"y"], [0], 10), "Block List and ID List does not match (different Len)"),
    ((VANDRS, PARAMS, [b"x", Atom("y")], [0, 1], 10), "Invalid Block"),
    ((VANDRS, PARAMS, [b"x", b"y"], [0, Atom("a")], 10), "Invalid ID"),
    ((VANDRS, PARAMS, [b"x", b"y"], [0, 1 << 40], 10), "Invalid ID"),
    ((VANDRS, PARAMS, [b"x"], [0], -1), "Expect data size"),
    ((VANDRS, PARAMS, [b"x"], [0], Atom("s")), "Expect data size"),
    ((Atom("nope"), Atom("p"), [b"x"], [0], -1), "Expect data size"),  # size before coding
    ((b"c", PARAMS, [b"x"], [0], 10), "Expect coding"),
    ((VANDRS, 5, [b"x"], [0], 10), "Expect tuple for coding parameters"),
    ((VANDRS, (10, 4, Atom("w")), [b"x"], [0], 10), "Invalid W"),
    ((Atom("nope"), PARAMS, [b"x"], [0], 10), "Invalid Coding"),
]


@pytest.mark.parametrize("args,reason", DECODE_ERRORS, ids=[r for _, r in DECODE_ERRORS])
def test_decode_argument_errors(nif, args, reason):
    assert err(nif.call("decode", *args)) == reason


REPAIR_ERRORS = [
    ((VANDRS, PARAMS, Atom("b"), [0], [1]), "Block List Needed"),
    ((VANDRS, PARAMS, [b"x"], [Atom("i")], [1]), "Invalid ID"),
    ((VANDRS, PARAMS, [b"x"], [0], 1), "Repair ID List Needed"),
    ((VANDRS, PARAMS, [b"x"], [0], [1, b"2"]), "Invalid Repair ID"),
    ((Atom("nope"), Atom("p"), [b"x"], [0], 1), "Repair ID List Needed"),
    ((1, PARAMS, [b"x"], [0], [1]), "Expect coding"),
    ((VANDRS, [1], [b"x"], [0], [1]), "Expect tuple for coding parameters"),
    ((Atom("nope"), PARAMS, [b"x"], [0], [1]), "Invalid Coding"),
]


@pytest.mark.parametrize("args,reason", REPAIR_ERRORS, ids=[r for _, r in REPAIR_ERRORS])
def test_repair_argument_errors(nif, args, reason):
    assert err(nif.call("repair", *args)) == reason


def _py(v):
    """The same arguments in the Python mirror's vocabulary (atoms -> str)."""
    if isinstance(v, Atom):
        return str(v)
    if isinstance(v, tuple):
        return tuple(_py(x) for x in v)
    if isinstance(v, list):
        return [_py(x) for x in v]
    return v


@pytest.mark.parametrize("fn,table", [("nif_encode", ENCODE_ERRORS), ("nif_decode", DECODE_ERRORS),
                                      ("nif_repair", REPAIR_ERRORS)])
def test_python_mirror_agrees(le, fn, table):
    # The mirror takes str for atoms; every case above keeps its meaning.
    for args, reason in table:
        assert getattr(le, fn)(*_py(args)) == ("error", reason), (fn, args)


@pytest.mark.parametrize("args,reason", ENCODE_ERRORS, ids=[r for _, r in ENCODE_ERRORS])
def test_ref_errors_build_keeps_argument_errors(nif_ref, args, reason):
    """-DLEOEC_NIF_REF_ERRORS changes only coder errors: argument errors and
    "Invalid Coding" (thrown outside the coder, nif.cpp:71,158-161) keep
    their text."""
    assert err(nif_ref.call("encode", *args)) == reason


@pytest.mark.parametrize("cls,params", [("vandrs", (10, 4, 7)), ("liberation", (4, 2, 8)),
                                        ("isars", (10, 4, 16))])
def test_ref_errors_build_slices_coder_errors(nif_ref, nif, cls, params):
    """Coder exceptions rethrown by value read "std::exception" in the
    reference (nif.cpp:80-83); the default build keeps the coder's text."""
    assert err(nif_ref.call("encode", Atom(cls), params, DATA, len(DATA))) == "std::exception"
    assert err(nif.call("encode", Atom(cls), params, DATA, len(DATA))) != "std::exception"
    r = nif_ref.call("decode", Atom(cls), params, [b"abcd", b"abc"], [0, 1], 7)
    assert err(r) == "std::exception"
    r = nif_ref.call("repair", Atom(cls), params, [b"abcd", b"abc"], [0, 1], [2])
    assert err(r) == "std::exception"


def test_ref_errors_build_gf_init(nif_ref, le):
    r = nif_ref.call("gf_init")
    if le.gf_init() == "ok":
        assert r == ok
    else:  # nif.cpp:124
        assert err(r) == "Galois Initialization Failed! w=8"


def test_iolist_input_is_copied_into_an_owned_binary(nif, le):
    """An iolist encode input is flattened into a binary the NIF allocates
    (enif_make_binary on the flattened view is no term in ERTS); the harness
    counts a violation otherwise.  Without a GPU the call then fails in the
    engine, after the copy."""
    r = nif.call("encode", VANDRS, PARAMS, [b"ab", [99, b"def"], b""], 6)
    if le.gf_init() == "ok":
        assert r[0] == ok and b"".join(bytes(b) for b in r[1][:1])[:6] == b"abcdef"
    else:
        assert err(r) == le.strerror(-16)
    r = nif.call("encode", VANDRS, PARAMS, [], 0)  # empty iolist
    assert r[0] == ok and len(r[1]) == 14 and all(len(b) == 0 for b in r[1])


def test_mismatched_block_sizes(nif, le):
    r = nif.call("decode", VANDRS, PARAMS, [b"abcd", b"abc"], [0, 1], 7)
    assert err(r) == le.strerror(-13)
    r = nif.call("repair", VANDRS, PARAMS, [b"abcd", b"abc"], [0, 1], [2])
    assert err(r) == le.strerror(-13)


def test_no_cpu_fallback(nif, le):
    """Well-formed calls reach the engine; without a GPU they fail with its text."""
    if le.gf_init() == "ok":
        pytest.skip("GPU present: covered by the -m gpu tests")
    r = nif.call("encode", VANDRS, PARAMS, DATA, len(DATA))
    assert err(r) == le.strerror(-16)
    r = nif.call("encode", VANDRS, PARAMS, [b"ab", [99, b"def"], b""], 6)  # iolist input
    assert err(r) == le.strerror(-16)
    bs, _ = le.layout("vandrs", PARAMS, 1000)
    blocks = _ok_blocks(14, bs)
    # a data block missing: GF(2^8) reconstruction is needed (an intact
    # stripe is only a concatenation, as in the reference, and succeeds)
    r = nif.call("decode", VANDRS, PARAMS, blocks[1:], list(range(1, 14)), 1000)
    assert err(r) == le.strerror(-16)


# ---------------------------------------------------------------------------
# GPU: the shim end to end
CASES = [("vandrs", (10, 4, 8)), ("cauchyrs", (4, 2, 3)), ("liberation", (4, 2, 7)),
         ("isars", (10, 4, 8)), ("vandrs", (6, 3, 16)), ("cauchyrs", (5, 3, 8))]


def _bs(le, cls, params, size):
    return le.layout(cls, params, size)


@pytest.mark.gpu
@pytest.mark.parametrize("cls,params", CASES, ids=[f"{c}{p}" for c, p in CASES])
@pytest.mark.parametrize("size", [1, 1000, 65543, 300001])
def test_gpu_encode_matches_oracle(nif, gpu, oracle, le, cls, params, size):
    data = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8).tobytes()
    r = nif.call("encode", Atom(cls), params, data, size)
    assert r[0] == ok, r
    blocks = r[1]
    k, m, w = params
    bs, filled = _bs(le, cls, params, size)
    assert len(blocks) == k + m and all(len(b) == bs for b in blocks)
    assert [bytes(b) for b in blocks] == oracle.encode(cls, k, m, w, data)
    # zero-copy: whole data blocks alias the input binary, the rest one fresh binary
    src_owner = blocks[0].owner if filled else None
    for i, b in enumerate(blocks[:filled]):
        assert b.owner == src_owner and b.off == i * bs
    fresh = {b.owner for b in blocks[filled:]}
    assert len(fresh) == 1 and src_owner not in fresh
    assert [b.off for b in blocks[filled:]] == [i * bs for i in range(k + m - filled)]


@pytest.mark.gpu
def test_gpu_encode_iolist_equals_binary(nif, gpu):
    parts = [b"hello ", [119, 111, [b"rld"]], b"", bytes(range(200)) * 50]
    flat = b"hello world" + bytes(range(200)) * 50
    r1 = nif.call("encode", VANDRS, PARAMS, parts, len(flat))
    r2 = nif.call("encode", VANDRS, PARAMS, flat, len(flat))
    assert r1[0] == ok and r2[0] == ok
    assert [bytes(b) for b in r1[1]] == [bytes(b) for b in r2[1]]


@pytest.mark.gpu
@pytest.mark.parametrize("cls,params", CASES, ids=[f"{c}{p}" for c, p in CASES])
def test_gpu_decode_repair_roundtrip(nif, gpu, oracle, cls, params):
    k, m, w = params
    size = 123457
    data = np.random.default_rng(k * 31 + m).integers(0, 256, size, dtype=np.uint8).tobytes()
    r = nif.call("encode", Atom(cls), params, data, size)
    assert r[0] == ok
    handles = [b.handle for b in r[1]]
    blocks = [bytes(b) for b in r[1]]
    rng = np.random.default_rng(7)
    for _ in range(6):
        lost = sorted(rng.choice(k + m, size=m, replace=False).tolist())
        keep = [i for i in range(k + m) if i not in lost]
        rng.shuffle(keep)
        # pass the encode result's own sub-binaries back in (no copies)
        args = [Raw(handles[i]) for i in keep]
        d = nif.call("decode", Atom(cls), params, args, keep, size)
        assert d[0] == ok and bytes(d[1]) == data
        assert bytes(d[1]) == oracle.decode(cls, k, m, w, [blocks[i] for i in keep], keep, size)
        rp = nif.call("repair", Atom(cls), params, args, keep, lost)
        assert rp[0] == ok
        assert [bytes(b) for b in rp[1]] == [blocks[i] for i in lost]
        assert len({b.owner for b in rp[1]}) == 1  # one binary, sub-binaries per block


@pytest.mark.gpu
def test_gpu_engine_errors_through_shim(nif, gpu, le):
    r = nif.call("encode", VANDRS, PARAMS, DATA, len(DATA))
    blocks = [Raw(b.handle) for b in r[1]]
    # fewer than k blocks
    assert err(nif.call("decode", VANDRS, PARAMS, blocks[:9], list(range(9)), len(DATA))) == \
        le.strerror(-9)
    # duplicate ids: fewer than k distinct -> not enough; k distinct + a repeat -> not unique
    ids = list(range(9)) + [0]
    assert err(nif.call("decode", VANDRS, PARAMS, blocks[:10], ids, len(DATA))) == le.strerror(-9)
    ids = list(range(10)) + [0]
    assert err(nif.call("decode", VANDRS, PARAMS, blocks[:11], ids, len(DATA))) == le.strerror(-10)
    # id out of range
    ids = list(range(9)) + [14]
    assert err(nif.call("decode", VANDRS, PARAMS, blocks[:10], ids, len(DATA))) == \
        le.nif_decode("vandrs", PARAMS, [bytes(b) for b in r[1][:10]], ids, len(DATA))[1]
    # sub-binary of an encode block as a (wrongly sized) block
    sub = Sub(r[1][0].handle, 0, 3)
    assert err(nif.call("decode", VANDRS, PARAMS, [sub] + blocks[1:10], list(range(10)),
                        len(DATA))) == le.strerror(-13)


def _load_with(nif, spec):
    import subprocess
    import sys
    code = ("import sys; sys.path[:0] = [%r, %r]\n"
            "import leo_erasure_amd\n"
            "from nif_harness.term import Harness\n"
            "print(Harness(%r).L.h_load())\n") % (ROOT, HERE, nif.path)
    env = {k: v for k, v in os.environ.items() if k != "LEOEC_HOST_DEVICES"}
    if spec is not None:
        env["LEOEC_HOST_DEVICES"] = spec
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                         timeout=120, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    return int(out.stdout.strip().splitlines()[-1]), out.stderr


@pytest.mark.parametrize("spec,rc", [(None, 0), ("", 0), ("current", 0), ("all", 0), ("0", 0),
                                     ("0,1,7", 0), ("0,x", 1), (",", 1), ("1,", 1), ("-1", 1),
                                     ("gpu0", 1), ("Current", 1)])
def test_load_host_devices(nif, spec, rc):
    """The shim's load callback (the reference registers none): host calls
    spread over every gfx950 device by default (unset = "all"),
    LEOEC_HOST_DEVICES picks a set or "current" / "" for none; it is parsed
    at load, a malformed value fails the load, a well-formed one that the
    runtime cannot serve (no GPU here) is left to the data calls.  Run in a
    child process: the test never writes its own environment."""
    if spec not in ("", "current", "0,x", ",", "1,", "-1", "gpu0", "Current"):
        import leo_erasure_amd as le
        if le.lib.leoec_host_lanes(None, 0) > 0:
            pytest.skip("a GPU is present: test_load_host_devices_on_gpu")
    assert _load_with(nif, spec)[0] == rc


@pytest.mark.gpu
@pytest.mark.parametrize("spec,rc", [(None, 0), ("all", 0), ("current", 0), ("0", 0),
                                     ("0,63", 2), ("63", 2)])
def test_load_host_devices_on_gpu(nif, spec, rc):
    """With a GPU present, a well-formed LEOEC_HOST_DEVICES naming a device
    the process cannot use fails the load (exit status 2, message on stderr)
    instead of silently leaving every call on the scheduler thread's current
    device (round-4 advisor)."""
    got, err = _load_with(nif, spec)
    assert got == rc, err[-2000:]
    if rc:
        assert "LEOEC_HOST_DEVICES" in err
