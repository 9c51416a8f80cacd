"""nexrReduceCopyHost on host memory the caller registered with hipHostRegister (include/nexr.h: "when
every buffer is pinned host memory (hipHostMalloc / hipHostRegister / torch pin_memory) the kernel
reads and writes it in place"). The fork's transport allocates its staging buffers once
(src/include/device.h:753-771), so registering them once is how a caller gets the zero-copy path on
memory it did not allocate with the HIP runtime.

Every pointer here lies INSIDE one registered mapping, at offsets that are not page-aligned, so the
library's device address for each must be the mapping's device base plus the offset; a wrong
translation would read or write the wrong bytes and the exact check would fail. fp32 a + b is one
IEEE add, so numpy's float32 sum is the oracle's value bit for bit."""
import ctypes
import importlib
import mmap
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HIP_HOST_REGISTER_MAPPED = 2  # hipHostRegisterMapped


@pytest.fixture(scope="module")
def hip():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU tests need an MI355X")
    torch.cuda.init()
    L = ctypes.CDLL("libamdhip64.so")
    L.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    L.hipHostRegister.restype = ctypes.c_int
    L.hipHostUnregister.argtypes = [ctypes.c_void_p]
    L.hipHostUnregister.restype = ctypes.c_int
    return L


class Region:
    """One anonymous mapping (page-aligned), registered with hipHostRegister for its lifetime."""

    def __init__(self, hip, nbytes: int, register: bool = True):
        self.hip, self.m = hip, mmap.mmap(-1, nbytes)
        self.buf = np.frombuffer(self.m, dtype=np.uint8)
        self.base = self.buf.ctypes.data
        self.registered = False
        if register:
            rc = hip.hipHostRegister(self.base, nbytes, HIP_HOST_REGISTER_MAPPED)
            assert rc == 0, f"hipHostRegister = {rc}"
            self.registered = True

    def f32(self, offset: int, n: int) -> np.ndarray:
        return self.buf[offset:offset + 4 * n].view(np.float32)

    def close(self):
        """Unregisters; the mapping itself goes when the last numpy view of it does."""
        if self.registered:
            self.registered = False
            assert self.hip.hipHostUnregister(self.base) == 0


def _fill(rng, v: np.ndarray):
    v[:] = rng.random(v.size, dtype=np.float32) * 2 - 1


@pytest.mark.parametrize("n", [1, 4099, 1_000_003, 16 << 20])
def test_registered_interior_pointers_zero_copy(hip, n):
    nexr = importlib.import_module("nex-nccl_amd")
    rng = np.random.default_rng(n)
    gap = 4096 * 3 + 48  # offsets inside the mapping that are not page- (or even 64 B-) aligned
    offs = [gap + 16, 2 * gap + 4 * n + 4, 3 * gap + 8 * n + 12]
    reg = Region(hip, offs[-1] + 4 * n + gap)
    try:
        a, b, out = (reg.f32(o, n) for o in offs)
        _fill(rng, a)
        _fill(rng, b)
        out[:] = np.nan
        guard_before = reg.buf[offs[2] - 64:offs[2]].copy()
        guard_after = reg.buf[offs[2] + 4 * n:offs[2] + 4 * n + 64].copy()
        nexr.host_path_stats(reset=True)
        nexr.reduce_copy_ptrs([reg.base + offs[0], reg.base + offs[1]], [reg.base + offs[2]], n, 7, 0, host=True)
        st = nexr.host_path_stats()
        # which path ran: one zero-copy call, every buffer classified by the runtime's pointer query
        # (the caller registered it, not the library), no staging copies
        assert (st["calls"], st["zeroCopyCalls"], st["pointerQueries"], st["registeredHits"]) == (1, 1, 3, 0), st
        assert st["copyNs"] == 0, st
        assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
        assert np.array_equal(reg.buf[offs[2] - 64:offs[2]], guard_before)
        assert np.array_equal(reg.buf[offs[2] + 4 * n:offs[2] + 4 * n + 64], guard_after)
    finally:
        reg.close()


def test_registered_sources_pageable_destination(hip):
    """A mix: the sources in a registered mapping, the destination in plain pageable memory (the
    library reads the registered ones in place and stages only the destination)."""
    nexr = importlib.import_module("nex-nccl_amd")
    n = 3_000_017
    rng = np.random.default_rng(7)
    reg = Region(hip, 8 * n + 8192)
    try:
        a, b = reg.f32(4096 + 4, n), reg.f32(4096 + 4 + 4 * n, n)
        _fill(rng, a)
        _fill(rng, b)
        out = np.full(n, np.nan, dtype=np.float32)
        nexr.reduce_copy_ptrs([a.ctypes.data, b.ctypes.data], [out.ctypes.data], n, 7, 0, host=True)
        assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
    finally:
        reg.close()


def test_registered_rate_beside_pageable(hip):
    """C2's mix (2 x 256 MiB in, 1 out) on one registered mapping against the same bytes unregistered:
    both exact; the registered call takes the zero-copy path, so it is not slower than the pageable
    one (both rates printed; the bench's h2d_inclusive line carries the measured figures)."""
    nexr = importlib.import_module("nex-nccl_amd")
    n = 64 << 20
    rng = np.random.default_rng(11)
    secs = {}
    for register in (True, False):
        reg = Region(hip, 12 * n + 3 * 4096, register=register)
        try:
            a, b, out = reg.f32(0, n), reg.f32(4 * n + 4096, n), reg.f32(8 * n + 8192, n)
            _fill(rng, a)
            _fill(rng, b)
            ptrs = ([reg.base, reg.base + 4 * n + 4096], [reg.base + 8 * n + 8192])
            nexr.reduce_copy_ptrs(*ptrs, n, 7, 0, host=True)  # warm-up (staging rings, code objects)
            t = []
            for _ in range(3):
                t0 = time.perf_counter()
                nexr.reduce_copy_ptrs(*ptrs, n, 7, 0, host=True)
                t.append(time.perf_counter() - t0)
            assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
            secs[register] = min(t)
        finally:
            reg.close()
    gbs = {k: 12 * n / v / 1e9 for k, v in secs.items()}
    print(f"registered {gbs[True]:.1f} GB/s, pageable {gbs[False]:.1f} GB/s")
    assert secs[True] <= secs[False] * 1.10, gbs


HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, HIP_POINTER_ATTRIBUTE_RANGE_SIZE = 11, 12


def test_runtime_reports_the_registered_range(hip):
    """nexrReduceCopyHost reads a caller-registered buffer in place only when the range the runtime
    reports for it (hipPointerGetAttribute RANGE_START_ADDR / RANGE_SIZE) covers the whole buffer.
    This pins that the runtime answers those queries for an interior pointer of a hipHostRegister-ed
    mapping, so the check is live (profiles/r05*_host_register_gpu_tests.txt records the values)."""
    hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    hip.hipPointerGetAttribute.restype = ctypes.c_int
    reg = Region(hip, 1 << 20)
    try:
        beg, size = ctypes.c_uint64(0), ctypes.c_uint64(0)
        p = reg.base + 12345
        rc1 = hip.hipPointerGetAttribute(ctypes.byref(beg), HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, p)
        rc2 = hip.hipPointerGetAttribute(ctypes.byref(size), HIP_POINTER_ATTRIBUTE_RANGE_SIZE, p)
        print(f"rc {rc1} {rc2}: start {beg.value:#x} (mapping {reg.base:#x}), size {size.value} (mapping {1 << 20})")
        assert rc1 == 0 and rc2 == 0
        assert beg.value <= p and beg.value + size.value >= reg.base + (1 << 20)
    finally:
        reg.close()


def test_library_registration_is_read_in_place_without_queries(hip):
    """nexrHostRegister (ncclCommRegister's counterpart): the library records the range, so a call on
    buffers inside it is classified from the cache with no runtime query and runs zero-copy; a range
    inside it shares the entry; a partly overlapping one is refused; after the last deregistration
    the same call stages the (now pageable) bytes and is still exact."""
    nexr = importlib.import_module("nex-nccl_amd")
    n = 1_000_003
    gap = 4096 + 48
    offs = [gap, 2 * gap + 4 * n, 3 * gap + 8 * n]
    reg = Region(hip, offs[-1] + 4 * n + gap, register=False)
    rng = np.random.default_rng(5)
    a, b, out = (reg.f32(o, n) for o in offs)
    _fill(rng, a)
    _fill(rng, b)
    ptrs = ([reg.base + offs[0], reg.base + offs[1]], [reg.base + offs[2]])
    h = nexr.host_register(reg.base, reg.buf.size)
    try:
        inner = nexr.host_register(reg.base + 8192, 4096)  # inside: the same entry, one more reference
        assert inner == h
        nexr.host_deregister(inner)
        with pytest.raises(nexr.NexrError) as e:  # straddles the entry's end
            nexr.host_register(reg.base + reg.buf.size - 4096, 8192)
        assert e.value.code == 5
        out[:] = np.nan
        nexr.host_path_stats(reset=True)
        nexr.reduce_copy_ptrs(*ptrs, n, 7, 0, host=True)
        st = nexr.host_path_stats()
        assert (st["calls"], st["zeroCopyCalls"], st["registeredHits"], st["pointerQueries"]) == (1, 1, 3, 0), st
        assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
    finally:
        nexr.host_deregister(h)
    out[:] = np.nan
    nexr.host_path_stats(reset=True)
    nexr.reduce_copy_ptrs(*ptrs, n, 7, 0, host=True)
    st = nexr.host_path_stats()
    assert (st["zeroCopyCalls"], st["registeredHits"], st["pointerQueries"]) == (0, 0, 3), st
    assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))


def test_buffer_past_a_registered_range_is_staged(hip):
    """A buffer that starts inside a registered range but runs past its end must not be read in place
    (the device mapping covers only the range): the cache lookup misses, the runtime reports the
    range, and the call stages the buffer instead (exact, zero-copy count 0)."""
    nexr = importlib.import_module("nex-nccl_amd")
    n = 1 << 20
    reg = Region(hip, 4 * n * 4, register=False)
    rng = np.random.default_rng(9)
    a, b, out = reg.f32(0, n), reg.f32(4 * n, n), reg.f32(8 * n, n)
    _fill(rng, a)
    _fill(rng, b)
    h = nexr.host_register(reg.base, 8 * n + 4 * n // 2)  # covers a, b and half of out
    try:
        out[:] = np.nan
        nexr.host_path_stats(reset=True)
        nexr.reduce_copy_ptrs([reg.base, reg.base + 4 * n], [reg.base + 8 * n], n, 7, 0, host=True)
        st = nexr.host_path_stats()
        assert (st["zeroCopyCalls"], st["registeredHits"], st["pointerQueries"]) == (0, 2, 1), st
        assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
    finally:
        nexr.host_deregister(h)


def test_register_inside_an_allocation_then_free(hip):
    """Advisor r5 (medium): memory from nexrHostMemAlloc may be registered (the reference's
    ncclMemAlloc-then-ncclCommRegister pattern). The registration is one more reference on the
    allocation's entry that nexrHostDeregister drops; nexrHostMemFree refuses while it is live; a
    handle whose entry is gone stays invalid, even after a new allocation lands at the same address
    (handles are ids, not addresses)."""
    nexr = importlib.import_module("nex-nccl_amd")
    n = 4099
    p = nexr.host_mem_alloc(3 * 4 * n + 64)
    h = nexr.host_register(p + 16, 2 * 4 * n)
    h2 = nexr.host_register(p + 32, 64)  # the same entry: one more reference
    assert h == h2 and h not in (0, p)
    with pytest.raises(nexr.NexrError) as e:
        nexr.host_mem_free(p)  # registrations inside it remain
    assert e.value.code == 5
    a = np.ctypeslib.as_array((ctypes.c_float * n).from_address(p + 16))
    b = np.ctypeslib.as_array((ctypes.c_float * n).from_address(p + 16 + 4 * n))
    out = np.ctypeslib.as_array((ctypes.c_float * n).from_address(p + 16 + 8 * n))
    rng = np.random.default_rng(21)
    _fill(rng, a)
    _fill(rng, b)
    out[:] = np.nan
    nexr.host_path_stats(reset=True)
    nexr.reduce_copy_ptrs([p + 16, p + 16 + 4 * n], [p + 16 + 8 * n], n, 7, 0, host=True)
    st = nexr.host_path_stats()
    assert (st["zeroCopyCalls"], st["registeredHits"], st["pointerQueries"]) == (1, 3, 0), st
    assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32))
    nexr.host_deregister(h)
    nexr.host_deregister(h2)
    with pytest.raises(nexr.NexrError) as e:
        nexr.host_deregister(h)  # no reference left
    assert e.value.code == 5
    nexr.host_mem_free(p)
    q = nexr.host_mem_alloc(3 * 4 * n + 64)  # possibly at p again
    try:
        with pytest.raises(nexr.NexrError) as e:
            nexr.host_deregister(h)  # the old handle names nothing, whatever q's address
        assert e.value.code == 5
        hq = nexr.host_register(q, 64)
        assert hq != h
        nexr.host_deregister(hq)
    finally:
        nexr.host_mem_free(q)
    with pytest.raises(nexr.NexrError) as e:
        nexr.host_deregister(12345678)  # never issued
    assert e.value.code == 5


def test_sub_page_neighbours_register_separately(hip):
    """Advisor r5 (low): hipHostRegister pins whole pages, so two disjoint buffers in one page (adjacent
    heap blocks, as the C1 bench's numpy arrays are) both touch the same page. On this ROCm the runtime
    maps each registration separately: two entries, two handles, each buffer read in place from the
    cache, and deregistering one leaves the other's mapping working. A range that overlaps an entry's
    bytes is refused with nexrInvalidUsage."""
    nexr = importlib.import_module("nex-nccl_amd")
    reg = Region(hip, 4 * 4096, register=False)
    n = 100
    a_off, out_off = 4096 + 2048, 4096 + 16  # a and b share page 1 with out
    try:
        hs = nexr.host_register(reg.base + a_off, 8 * n)      # a and b: one range
        ho = nexr.host_register(reg.base + out_off, 4 * n)    # out: same page, disjoint bytes
        assert hs != ho
        with pytest.raises(nexr.NexrError) as e:  # overlaps out's bytes
            nexr.host_register(reg.base + out_off + 8, 4 * n)
        assert e.value.code == 5
        a = reg.f32(a_off, n)
        b = reg.f32(a_off + 4 * n, n)
        out = reg.f32(out_off, n)
        rng = np.random.default_rng(22)
        ptrs = ([reg.base + a_off, reg.base + a_off + 4 * n], [reg.base + out_off])
        for drop in (None, "sources", "output"):
            _fill(rng, a)
            _fill(rng, b)
            out[:] = np.nan
            nexr.host_path_stats(reset=True)
            nexr.reduce_copy_ptrs(*ptrs, n, 7, 0, host=True)
            st = nexr.host_path_stats()
            assert np.array_equal(out.view(np.uint32), (a + b).view(np.uint32)), drop
            if drop is None:
                assert (st["zeroCopyCalls"], st["registeredHits"], st["pointerQueries"]) == (1, 3, 0), st
                nexr.host_deregister(hs)
            elif drop == "sources":  # out still registered and read in place; a, b found by the runtime
                assert st["registeredHits"] == 1, st
                nexr.host_deregister(ho)
            else:
                assert st["registeredHits"] == 0, st
    finally:
        reg.close()
