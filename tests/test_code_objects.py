"""The gfx950 code objects inside the shipped libraries keep what the HIP runtime resolves kernels by.

Round 5 linked the device code with ``--strip-all`` once: the first launch then crashed inside the
runtime (profiles/r05c_gpu_tests_strip_all_crash.txt), because that flag drops each code object's
``.symtab``, where the runtime looks kernels up; the kernel descriptors (``<kernel>.kd``) survive only in
``.dynsym``. The Makefile went back to ``--discard-all`` (local symbols only). These CPU tests read the
offload bundles out of the built ``.so`` files and check, for every kernel listed in each code object's
AMDGPU metadata note, that ``.symtab`` holds both the kernel's symbol and its ``.kd`` descriptor; and they
build a one-kernel object both ways to show the check tells the two links apart.
"""
import os
import shutil
import struct
import subprocess

import msgpack
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nex-nccl_amd")
HIPCC = "/opt/rocm/bin/hipcc"

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def gfx950_code_objects(blob):
    """Every gfx950 ELF in the clang offload bundles of a host binary (uncompressed bundles: magic,
    u64 entry count, then per entry u64 offset, u64 size, u64 triple length, triple)."""
    out = []
    i = blob.find(_MAGIC)
    while i >= 0:
        (n,) = struct.unpack_from("<Q", blob, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if triple.endswith("gfx950"):
                out.append(blob[i + off:i + off + size])
        i = blob.find(_MAGIC, i + len(_MAGIC))
    return out


def elf_tables(co):
    """(symbol-table name -> set of symbol names, [AMDGPU metadata maps]) of an ELF64 code object."""
    assert co[:4] == b"\x7fELF" and co[4] == 2, "not an ELF64 object"
    (shoff,) = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", co, 0x3A)
    secs = [struct.unpack_from("<IIQQQQIIQQ", co, shoff + k * shentsize) for k in range(shnum)]

    def cstr(sec, o):
        start = sec[4] + o
        return co[start:co.index(b"\0", start)].decode()

    tables, notes = {}, []
    for sec in secs:
        name, typ, _flags, _addr, off, size, link = sec[:7]
        if typ in (2, 11):  # SHT_SYMTAB, SHT_DYNSYM
            strtab = secs[link]
            names = set()
            for j in range(size // 24):
                (st_name,) = struct.unpack_from("<I", co, off + j * 24)
                if st_name:
                    names.add(cstr(strtab, st_name))
            tables[cstr(secs[shstrndx], name)] = names
        elif typ == 7:  # SHT_NOTE
            p = off
            while p < off + size:
                namesz, descsz, ntype = struct.unpack_from("<III", co, p)
                p += 12 + ((namesz + 3) & ~3)
                desc = co[p:p + descsz]
                p += (descsz + 3) & ~3
                if ntype == 32:  # NT_AMDGPU_METADATA
                    notes.append(msgpack.unpackb(desc, raw=False))
    return tables, notes


def missing_kernel_symbols(co):
    """Kernels of one code object whose symbol or .kd descriptor is not in .symtab (a list of names);
    raises if the object lists no kernels at all."""
    tables, notes = elf_tables(co)
    kernels = [k for n in notes for k in n.get("amdhsa.kernels", [])]
    assert kernels, "code object lists no kernels"
    symtab = tables.get(".symtab", set())
    missing = []
    for k in kernels:
        for sym in (k[".name"], k[".symbol"]):
            if sym not in symtab:
                missing.append(sym)
    return missing


def _read(path):
    with open(path, "rb") as f:
        return f.read()


@pytest.mark.parametrize("lib", ["libnexr.so"])
def test_shipped_code_objects_keep_kernel_symbols(lib):
    path = os.path.join(PKG, lib)
    if not os.path.exists(path):
        pytest.skip(f"{lib} not built")
    cos = gfx950_code_objects(_read(path))
    # one object per datatype (10) and the LL / LL128 object
    assert len(cos) == 11, len(cos)
    total = 0
    for co in cos:
        assert missing_kernel_symbols(co) == []
        _tables, notes = elf_tables(co)
        names = [k[".name"] for n in notes for k in n["amdhsa.kernels"]]
        assert all(n.endswith(".kd") is False for n in names)
        total += len(names)
    assert total > 0


def test_the_check_catches_a_strip_all_link(tmp_path):
    """A one-kernel object linked with --discard-all passes; the same with --strip-all fails."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = tmp_path / "k.hip"
    src.write_text(
        "#include <hip/hip_runtime.h>\n"
        "__global__ void probe_kernel(unsigned* p) { p[threadIdx.x] += 1u; }\n")
    verdicts = {}
    for flag in ("--discard-all", "--strip-all"):
        obj = tmp_path / f"k{flag.replace('-', '_')}.o"
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-fPIC", "-Xoffload-linker", flag, "-c", str(src), "-o",
                        str(obj)], check=True, capture_output=True, timeout=300)
        cos = gfx950_code_objects(_read(obj))
        assert len(cos) == 1
        verdicts[flag] = missing_kernel_symbols(cos[0])
    assert verdicts["--discard-all"] == []
    assert sorted(verdicts["--strip-all"]) == sorted(["_Z12probe_kernelPj", "_Z12probe_kernelPj.kd"])


def test_makefile_links_device_code_with_discard_all():
    mk = _read(os.path.join(PKG, "csrc", "Makefile")).decode()
    kflags = [l for l in mk.splitlines() if l.startswith("KFLAGS")]
    assert kflags and "--discard-all" in kflags[0] and "--strip-all" not in kflags[0]
    assert shutil.which("make") is not None
