"""Kernel descriptors of the gfx950 code objects inside a HIP shared library.

hipcc embeds one clang offload bundle per translation unit in the library's
`.hip_fatbin` section. This reads every bundle, extracts its gfx950 code
object and parses the AMDGPU metadata note (`llvm-readelf --notes`) into one
dict per kernel: name, .private_segment_fixed_size, .uses_dynamic_stack,
.vgpr_count, .sgpr_count, .vgpr_spill_count.

Used by tests/test_kernel_stack.py (the guard against a dynamic stack coming
back into the Kryo encoder kernels) and usable by hand:
    python tools/kernel_notes.py corda_amd/libcordahip.so
"""
import os
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = b"hipv4-amdgcn-amd-amdhsa--gfx950"


def fatbin_section(lib):
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fat.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "-O", "binary", "--only-section=.hip_fatbin",
                               lib, out])
        with open(out, "rb") as f:
            return f.read()


def code_objects(fat):
    """gfx950 code objects of every bundle in a .hip_fatbin section"""
    objs = []
    pos = fat.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen]
            p += 24 + tlen
            if triple == TARGET and size:
                objs.append(fat[pos + off:pos + off + size])
        pos = fat.find(MAGIC, pos + 32)
    return objs


FIELDS = {
    ".private_segment_fixed_size": int,
    ".uses_dynamic_stack": lambda v: v.strip() == "true",
    ".vgpr_count": int,
    ".sgpr_count": int,
    ".vgpr_spill_count": int,
    ".sgpr_spill_count": int,
}


def kernels_of(co):
    """kernel descriptors (dicts) of one code object, from its metadata note"""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(co)
        f.flush()
        text = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", f.name], text=True)
    ks, cur = [], None
    for line in text.splitlines():
        s = line.strip()
        if s.startswith("- .agpr_count:") or s.startswith("- .args:"):
            cur = {}
            ks.append(cur)
        if cur is None or ":" not in s:
            continue
        key, _, val = s.lstrip("- ").partition(":")
        key = key.strip()
        if key == ".name" and "name" not in cur:
            cur["name"] = val.strip()
        elif key in FIELDS:
            cur[key] = FIELDS[key](val)
    # the kernel list's entries all carry a .symbol; arg entries do not
    return [k for k in ks if "name" in k and ".uses_dynamic_stack" in k]


def library_kernels(lib):
    out = []
    for co in code_objects(fatbin_section(lib)):
        out.extend(kernels_of(co))
    return out


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "corda_amd",
                                                              "libcordahip.so")
    for k in library_kernels(lib):
        print("%-90s stack %5d dyn %-5s vgpr %3s spill %s" % (k["name"][:90], k[".private_segment_fixed_size"],
                                                           k[".uses_dynamic_stack"], k.get(".vgpr_count"),
                                                           k.get(".vgpr_spill_count")))


if __name__ == "__main__":
    main()
