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
import re
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


# ---- which reduce-copy kernels are compiled (round 6: routing instead of every combination) ----------
SUM, PROD, MINMAX, PREMULSUM, SUMPOSTDIV = range(5)
INT8, UINT8, INT32, UINT32, INT64, UINT64, F16, F32, F64, BF16 = range(10)
_SIGNED = {INT8, INT32, INT64}
_INTS = {INT8, UINT8, INT32, UINT32, INT64, UINT64}


def expected_kernels():
    """(batch, dt, op, K, policy, isMin) of every kernel the routing (nexr_api.cpp routeKernel,
    nexr_internal.h kernel_compiled) can launch: K = 1 without arithmetic runs the uint8 Sum copy,
    signed integers run only Min / Max (Sum, Prod, PreMulSum, SumPostDiv on the unsigned kernels), batch
    launches run the plain and nt-load policies only."""
    out = set()
    for dt in range(10):
        for op in range(5):
            if op == SUMPOSTDIV and dt not in _INTS:
                continue
            for k in range(1, 9):
                if k == 1:
                    ok = (op == SUM and dt == UINT8) or (dt not in _SIGNED and op in (PREMULSUM, SUMPOSTDIV))
                else:
                    ok = dt not in _SIGNED or op == MINMAX
                if not ok:
                    continue
                for batch, pols in ((0, (0, 1, 3)), (1, (0, 1))):
                    for pol in pols:
                        for is_min in ((0, 1) if op == MINMAX else (0,)):
                            out.add((batch, dt, op, k, pol, is_min))
    return out


_KNAME = re.compile(r"_ZN4nexr(18reduce_copy_kernel|24reduce_copy_batch_kernel)ILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])")


def test_compiled_reduce_copy_kernels_are_exactly_the_routed_set():
    path = os.path.join(PKG, "libnexr.so")
    if not os.path.exists(path):
        pytest.skip("libnexr.so not built")
    got = set()
    for co in gfx950_code_objects(_read(path)):
        _tables, notes = elf_tables(co)
        for k in (k for n in notes for k in n["amdhsa.kernels"]):
            m = _KNAME.match(k[".name"])
            if m:
                key = (int("batch" in m.group(1)), int(m.group(2)), int(m.group(3)), int(m.group(4)),
                       int(m.group(5)), int(m.group(6)))
                assert key not in got, key
                got.add(key)
    want = expected_kernels()
    assert got == want, (sorted(got - want)[:5], sorted(want - got)[:5])
    assert len(want) == 1595  # 2,688 before round 6 (every dt x op x K x policy x {single, batch})
