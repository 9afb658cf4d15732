"""The product library's gfx950 kernels keep their scratch small (CPU test,
on the objects build() leaves in leo_erasure_amd/csrc/_build).

A kernel whose registers spill reads and writes scratch memory in its hot
loop, and its first launch makes the runtime back the whole device's scratch
(round 6: a measurement-only form compiled into the w = 13 syndrome decode
spilled 1,800+ VGPRs, 3.5 KB per lane, and the warm-up's first w = 13 launch
took 2 GiB of device memory: test_host_spread_warms_its_devices caught the
memory, this test names the kernel).  Reads each object's offload bundle
with the ROCm LLVM tools (clang-offload-bundler, llvm-readelf) and checks
every kernel's metadata: at most kMaxScratch bytes of private segment per
lane.  (Some gf8_apply instances for K >= 9 spill 2-30 VGPRs, up to 267 in
the branchy variants no launch selects (kGf8Default.branchy = 0): 8-192
bytes; the BASELINE kernels spill nothing: checked by name below.)"""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "leo_erasure_amd", "csrc", "_build")
LLVM = "/opt/rocm/lib/llvm/bin"
kMaxScratch = 256  # bytes of private segment per lane
# mangled-name prefixes of the BASELINE configs' kernels: gf8_apply<10,4> and
# <10,3>/<10,2>/<10,1> (vandrs / isars RS(10,4,8) encode and decode),
# gfbit_apply<8,4,...> and gfbk_apply (cauchyrs(10,4,8))
HOT = {"gf8_apply<10,4> encode": "_ZN5leoec6detail9gf8_applyILi10ELi4ELb0ELi1ELb1ELb0ELb0ELb0ELb1ELi5ELi256ELi0ELb0ELb0ELb0E",
       "gfbk_apply<10,3,64>": "_ZN5leoec12gfbit_detail10gfbk_applyILi10ELi3ELi64ELb0ELi1E",
       "gfbit_apply<8,4>": "_ZN5leoec6detail11gfbit_applyILi8ELi4E"}


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def kernel_notes(obj, tmp):
    """[(kernel name, {metadata key: value})] of the gfx950 code object in obj."""
    fat = os.path.join(tmp, os.path.basename(obj) + ".fatbin")
    subprocess.run([_tool("llvm-objcopy"), "--dump-section", f".hip_fatbin={fat}", obj, os.devnull],
                   check=True, capture_output=True)
    targets = subprocess.run([_tool("clang-offload-bundler"), "--list", "--type=o", f"--input={fat}"],
                             check=True, capture_output=True, text=True).stdout.split()
    tgt = [t for t in targets if "gfx950" in t]
    assert tgt, (obj, targets)
    co = fat + ".co"
    subprocess.run([_tool("clang-offload-bundler"), "--type=o", f"--targets={tgt[0]}",
                    f"--input={fat}", f"--output={co}", "--unbundle"], check=True, capture_output=True)
    notes = subprocess.run([_tool("llvm-readelf"), "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    kernels, cur = [], None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = {}
            kernels.append((m.group(1), cur))
            continue
        m = re.match(r"\s+\.(\w+):\s+(\S+)", line)
        if m and cur is not None:
            cur[m.group(1)] = m.group(2)
    return kernels


@pytest.mark.skipif(not glob.glob(os.path.join(BUILD, "*.o")), reason="product objects not built")
@pytest.mark.skipif(not (_tool("clang-offload-bundler") and _tool("llvm-readelf") and _tool("llvm-objcopy")),
                    reason="ROCm LLVM tools absent")
def test_product_kernels_scratch(tmp_path):
    objs = sorted(glob.glob(os.path.join(BUILD, "*.o")))
    seen, bad, hot = 0, [], {}
    for o in objs:
        try:
            ks = kernel_notes(o, str(tmp_path))
        except (AssertionError, subprocess.CalledProcessError):
            continue  # (an object with no device code)
        for name, md in ks:
            if "vgpr_spill_count" not in md:
                continue
            seen += 1
            scratch = int(md.get("private_segment_fixed_size", "0"))
            if scratch > kMaxScratch:
                bad.append((os.path.basename(o), name[:90], scratch, md["vgpr_spill_count"]))
            for key, frag in HOT.items():
                if name.startswith(frag):
                    hot[key] = (int(md["vgpr_spill_count"]), scratch)
    assert seen > 100, seen  # every TU's kernels were read
    assert not bad, bad[:10]
    # the BASELINE configs' kernels: found, and no spill at all
    assert set(hot) == set(HOT), set(HOT) - set(hot)
    assert all(v == (0, 0) for v in hot.values()), hot
