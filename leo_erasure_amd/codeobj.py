"""Identify the device code a measurement was taken on.

The engine's kernels live in the `.hip_fatbin` section of libleoec.so: one
clang offload bundle per translation unit, each holding that unit's gfx950
code object.  `kernel_code_object_sha256` hashes the bundle that defines a
given kernel, so a measurement file (the PMC traffic of `gf8_apply<10,4>`,
profiles/pmc_traffic*.json) can carry the hash of the code it was measured
on, and bench.py can refuse to print a stale figure after the kernel changes
(host-only changes and other kernels leave the hash alone).
"""
import hashlib
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

# the shipped headline kernel: gf8_apply<K=10, R=4, ...> (mangled prefix)
GF8_10_4 = b"_ZN5leoec6detail9gf8_applyILi10ELi4E"


def _section(data, name):
    """(offset, size) of ELF64 section `name`, or None."""
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError("not an ELF64 file")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    str_off, = struct.unpack_from("<Q", data, shoff + shstrndx * shentsize + 0x18)
    for i in range(shnum):
        h = shoff + i * shentsize
        name_off, = struct.unpack_from("<I", data, h)
        end = data.index(b"\0", str_off + name_off)
        if data[str_off + name_off:end].decode() == name:
            off, size = struct.unpack_from("<QQ", data, h + 0x18)
            return off, size
    return None


def bundles(lib_path):
    """The offload bundles of a HIP shared library, as bytes objects."""
    with open(lib_path, "rb") as fh:
        data = fh.read()
    sec = _section(data, ".hip_fatbin")
    if sec is None:
        return []
    base, size = sec
    out = []
    pos = data.find(_MAGIC, base, base + size)
    while pos >= 0:
        n, = struct.unpack_from("<Q", data, pos + len(_MAGIC))
        h = pos + len(_MAGIC) + 8
        end = pos
        for _ in range(n):
            off, sz, tsz = struct.unpack_from("<QQQ", data, h)
            h += 24 + tsz
            end = max(end, pos + off + sz)
        out.append(data[pos:end])
        pos = data.find(_MAGIC, end, base + size)
    return out


def kernel_code_object_sha256(lib_path, symbol=GF8_10_4):
    """sha256 of the offload bundle of `lib_path` whose code object defines
    `symbol` (a mangled-name prefix), or None if no bundle does."""
    for b in bundles(lib_path):
        if symbol in b:
            return hashlib.sha256(b).hexdigest()
    return None
