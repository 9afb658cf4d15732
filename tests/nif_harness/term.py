"""ctypes driver for the NIF-shim test double (erl_nif.h + harness.cpp here).

Compiles leo_erasure_amd/csrc/nif/leo_erasure_nif.cpp against the test-double
erl_nif.h with the term store in harness.cpp, and converts Python values to
terms and back:

    Atom("ok")  <-> atom        int   <-> integer
    bytes       <-> binary      tuple <-> tuple       list <-> list

Erlang strings come back as lists of ints (see ``text``).  libleoec.so is
promoted to RTLD_GLOBAL so the shim's leoec_* references resolve to the very
library the package loaded (no second copy, no torch/HIP soname clash).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
SHIM = os.path.join(ROOT, "leo_erasure_amd", "csrc", "nif", "leo_erasure_nif.cpp")

T = ctypes.c_size_t  # ERL_NIF_TERM


class Atom(str):
    def __repr__(self):
        return f"Atom({str(self)!r})"


def build(outdir, defines=()):
    """defines: extra -D flags for the shim, e.g. ("LEOEC_NIF_REF_ERRORS",)."""
    so = os.path.join(outdir, "libnif_harness%s.so" % "".join("_" + d.lower() for d in defines))
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fPIC", "-shared", "-Wall", "-Werror",
           "-DHAVE_ERL_NIF", "-I", HERE, "-I", os.path.join(ROOT, "include")]
    cmd += ["-D" + d for d in defines]
    cmd += [os.path.join(HERE, "harness.cpp"), SHIM, "-o", so]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return so


class Harness:
    def __init__(self, so):
        from leo_erasure_amd import _lib
        self.path = so
        ctypes.CDLL(_lib.LIB_PATH, mode=ctypes.RTLD_GLOBAL | os.RTLD_NOLOAD)
        L = ctypes.CDLL(so)
        for name, res, args in [
            ("h_reset", None, []), ("h_live_allocs", ctypes.c_long, []),
            ("h_load", ctypes.c_int, []),
            ("h_violations", ctypes.c_long, []),
            ("h_atom", T, [ctypes.c_char_p]), ("h_int", T, [ctypes.c_longlong]),
            ("h_bin", T, [ctypes.c_char_p, ctypes.c_size_t]),
            ("h_sub", T, [T, ctypes.c_size_t, ctypes.c_size_t]),
            ("h_tuple", T, [ctypes.POINTER(T), ctypes.c_uint]),
            ("h_list", T, [ctypes.POINTER(T), ctypes.c_uint]),
            ("h_kind", ctypes.c_int, [T]), ("h_intval", ctypes.c_longlong, [T]),
            ("h_atomname", ctypes.c_char_p, [T]), ("h_len", ctypes.c_uint, [T]),
            ("h_elem", T, [T, ctypes.c_uint]), ("h_bindata", ctypes.c_void_p, [T]),
            ("h_binowner", ctypes.c_long, [T]), ("h_binoff", ctypes.c_size_t, [T]),
            ("h_call", T, [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(T),
                           ctypes.POINTER(ctypes.c_uint)]),
            ("h_nfuncs", ctypes.c_uint, []),
            ("h_func", ctypes.c_char_p, [ctypes.c_uint, ctypes.POINTER(ctypes.c_uint),
                                         ctypes.POINTER(ctypes.c_uint)]),
        ]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        self.L = L

    # ---- Python -> term
    def term(self, v):
        L = self.L
        if isinstance(v, Atom):
            return L.h_atom(str(v).encode("latin-1"))
        if isinstance(v, bool):
            raise TypeError("no booleans in this term model; use Atom('true')")
        if isinstance(v, int):
            return L.h_int(v)
        if isinstance(v, (bytes, bytearray)):
            return L.h_bin(bytes(v), len(v))
        if isinstance(v, Sub):
            return L.h_sub(v.parent, v.pos, v.size)
        if isinstance(v, Raw):
            return v.t
        if isinstance(v, (tuple, list)):
            hs = [self.term(x) for x in v]
            arr = (T * max(len(hs), 1))(*hs)
            return (L.h_tuple if isinstance(v, tuple) else L.h_list)(arr, len(hs))
        raise TypeError(type(v))

    # ---- term -> Python (binaries as Bin, keeping identity information)
    def value(self, t):
        L = self.L
        k = L.h_kind(t)
        if k == 0:
            return Atom(L.h_atomname(t).decode("latin-1"))
        if k == 1:
            return L.h_intval(t)
        if k == 2:
            n = L.h_len(t)
            data = ctypes.string_at(L.h_bindata(t), n) if n else b""
            return Bin(data, L.h_binowner(t), L.h_binoff(t), t)
        if k in (3, 4):
            xs = [self.value(L.h_elem(t, i)) for i in range(L.h_len(t))]
            return tuple(xs) if k == 3 else xs
        raise ValueError(f"bad term handle {t}")

    def call(self, name, *args):
        hs = [self.term(a) for a in args]
        arr = (T * max(len(hs), 1))(*hs)
        flags = ctypes.c_uint()
        r = self.L.h_call(name.encode(), len(hs), arr, ctypes.byref(flags))
        assert r, f"no NIF {name}/{len(hs)}"
        return self.value(r)

    def funcs(self):
        out = []
        for i in range(self.L.h_nfuncs()):
            a, f = ctypes.c_uint(), ctypes.c_uint()
            name = self.L.h_func(i, ctypes.byref(a), ctypes.byref(f)).decode()
            out.append((name, a.value, f.value))
        return out


class Bin(bytes):
    """A binary term's bytes plus which owner buffer / offset it views."""

    def __new__(cls, data, owner, off, handle):
        b = super().__new__(cls, data)
        b.owner, b.off, b.handle = owner, off, handle
        return b


class Sub:
    """enif_make_sub_binary(parent, pos, size) as an argument."""

    def __init__(self, parent, pos, size):
        self.parent, self.pos, self.size = parent, pos, size


class Raw:
    """An existing term handle passed through unchanged."""

    def __init__(self, t):
        self.t = t


def text(v):
    """An Erlang string (list of char codes) as str."""
    assert isinstance(v, list) and all(isinstance(c, int) for c in v), v
    return bytes(v).decode("latin-1")
