"""List the GPU kernels a HIP shared library carries (test/measurement tool).

Reads the host ELF's .hip_fatbin section, finds every embedded amdgcn code
object (ELF64, EM_AMDGPU) and returns the kernel-descriptor symbols ("*.kd")
of each, demangled with c++filt when it is on PATH.  Pure Python apart from
the optional c++filt: no GPU and no ROCm tools needed.

usage: python tools/code_objects.py blockframe-rs_amd/libbfrs.so
"""
import shutil
import struct
import subprocess
import sys

EM_AMDGPU = 224


def _sections(elf: bytes):
    """{name: (offset, size)} of an ELF64 little-endian image."""
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        o = shoff + i * shentsize
        name, typ, _flags, _addr, off, size, link = struct.unpack_from("<IIQQQQI", elf, o)
        hdrs.append((name, typ, off, size, link))
    stroff = hdrs[shstrndx][2]
    out = {}
    for name, typ, off, size, link in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, typ, link)
    return out, hdrs


def _elf_end(elf: bytes, at: int) -> int:
    shoff, = struct.unpack_from("<Q", elf, at + 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, at + 0x3A)
    return at + shoff + shentsize * shnum


def device_code_objects(path: str):
    """The amdgcn code objects embedded in a host shared library."""
    data = open(path, "rb").read()
    secs, _ = _sections(data)
    if ".hip_fatbin" not in secs:
        return []
    off, size = secs[".hip_fatbin"][:2]
    fb = data[off:off + size]
    objs, pos = [], 0
    while True:
        i = fb.find(b"\x7fELF", pos)
        if i < 0:
            break
        machine, = struct.unpack_from("<H", fb, i + 0x12)
        if fb[i + 4] == 2 and machine == EM_AMDGPU:  # ELFCLASS64, amdgcn
            end = _elf_end(fb, i)
            objs.append(fb[i:end])
            pos = end
        else:
            pos = i + 4
    return objs


def kernel_symbols(code_object: bytes):
    """Kernel names (mangled) of one code object: its "*.kd" symbols."""
    secs, hdrs = _sections(code_object)
    names = []
    for name, (off, size, typ, link) in secs.items():
        if typ != 2:  # SHT_SYMTAB
            continue
        stroff = hdrs[link][2]
        for o in range(off, off + size, 24):
            st_name, = struct.unpack_from("<I", code_object, o)
            end = code_object.index(b"\0", stroff + st_name)
            s = code_object[stroff + st_name:end].decode()
            if s.endswith(".kd"):
                names.append(s[:-3])
    return sorted(set(names))


def demangle(names):
    tool = shutil.which("c++filt") or shutil.which("llvm-cxxfilt")
    if not tool or not names:
        return list(names)
    r = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True)
    return r.stdout.splitlines()


def kernels(path: str):
    """Demangled kernel names of every code object in the library."""
    out = []
    for co in device_code_objects(path):
        out.extend(kernel_symbols(co))
    return demangle(sorted(set(out)))


if __name__ == "__main__":
    for k in kernels(sys.argv[1]):
        print(k)
