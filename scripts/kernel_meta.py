"""Kernel metadata of the built library (diagnostic, and the CPU test's scratch guard):
the gfx950 code object is cut out of libtdstep.so's .hip_fatbin bundle and its AMDGPU
metadata notes are read with llvm-readelf.

  python scripts/kernel_meta.py [libtdstep.so]   -> name, sgpr, vgpr, scratch, lds per kernel
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(HERE, "gym-td_amd", "lib", "libtdstep.so")


def kernels(lib=LIB):
    """{kernel symbol: {"sgpr", "vgpr", "scratch", "lds"}} from the library's gfx950 code
    objects (one offload bundle per translation unit in .hip_fatbin)."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    notes = ""
    with tempfile.TemporaryDirectory() as d:
        fat = os.path.join(d, "fat.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section=.hip_fatbin=" + fat, lib,
                               os.path.join(d, "copy.so")])
        blob = open(fat, "rb").read()
        starts = [i for i in range(len(blob)) if blob.startswith(magic, i)]
        for k, a in enumerate(starts):
            part, co = os.path.join(d, "b%d.bin" % k), os.path.join(d, "b%d.co" % k)
            open(part, "wb").write(blob[a:starts[k + 1] if k + 1 < len(starts) else len(blob)])
            subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--input=" + part,
                                   "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co, "--unbundle"])
            notes += subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co]).decode() + "\n"
    out, cur = {}, None
    keys = {".sgpr_count": "sgpr", ".vgpr_count": "vgpr", ".private_segment_fixed_size": "scratch",
            ".group_segment_fixed_size": "lds"}
    for line in notes.split("\n"):
        if re.match(r"^  - \.", line):  # a kernel's map starts (amdhsa.kernels list item)
            cur = {}
        m = re.match(r"^  (?:- |  )(\.[a-z_]+):\s+(\S+)", line)
        if not m or cur is None:
            continue
        k, v = m.group(1), m.group(2)
        if k == ".name":
            out[v] = cur
        elif k in keys:
            cur[keys[k]] = int(v)
    return out


if __name__ == "__main__":
    for name, r in sorted(kernels(sys.argv[1] if len(sys.argv) > 1 else LIB).items()):
        print("%-70s %s" % (name, r))
