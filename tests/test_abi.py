"""CPU tests of the drop-in boundary (include/nexr.h, nex-nccl_amd/libnexr.so) — no GPU calls.

The library must load, export exactly the symbols the header declares, keep every enum numerically
identical to the reference, reject bad arguments with ncclInvalidArgument (4) before touching the
device, and encode ops exactly as hostToDevRedOp does (src/enqueue.cc:2185-2278).
"""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

import make_golden as mg

HEADER = os.path.join(ROOT, "include", "nexr.h")


def _declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"NEXR_API\s+[\w\s\*]+?\b(nexr\w+)\s*\(", text)))


def test_header_declares_the_abi(nexr):
    assert _declared_symbols() == sorted(nexr.ABI_SYMBOLS)


def test_library_exports_every_declared_symbol(nexr):
    L = nexr.lib()
    for name in _declared_symbols():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", nexr.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    ours = {s for s in exported if s.startswith("nexr")}
    assert ours == set(_declared_symbols()), "only the ABI may be exported"


def test_enums_match_reference(nexr):
    # src/nccl.h.in:40-48 (ncclResult_t), :259-270 (ncclRedOp_t), :278-290 (ncclDataType_t),
    # src/include/device.h:683-687 (ncclDevRedOp_t)
    assert [int(r) for r in nexr.Result] == list(range(8))
    assert (nexr.RedOp.Sum, nexr.RedOp.Prod, nexr.RedOp.Max, nexr.RedOp.Min, nexr.RedOp.Avg) == (0, 1, 2, 3, 4)
    assert [int(d) for d in nexr.DataType] == list(range(12))
    assert (nexr.DataType.Float16, nexr.DataType.Float32, nexr.DataType.Bfloat16) == (6, 7, 9)
    assert [int(o) for o in nexr.DevRedOp] == [0, 1, 2, 3, 4]
    text = open(HEADER).read()
    for name, val in (("nexrInvalidArgument", 4), ("nexrFloat8e5m2", 11), ("nexrDevSumPostDiv", 4),
                      ("NEXR_MAX_SRCS", 8), ("NEXR_MAX_DSTS", 8)):
        assert re.search(rf"\b{name}\s*=?\s*{val}\b", text), name


def test_type_size_and_strings(nexr):
    L = nexr.lib()
    for dt, sz in nexr.TYPE_SIZE.items():
        assert L.nexrTypeSize(int(dt)) == sz
    assert L.nexrTypeSize(12) == 0
    assert L.nexrGetErrorString(4) == b"invalid argument"
    assert nexr.version() == 300


def _call(nexr, nsrcs=2, ndsts=1, n=16, dt=7, op=0, arg=0, pre=None, srcs=None, dsts=None):
    L = nexr.lib()
    s = srcs if srcs is not None else [0x1000 * (i + 1) for i in range(nsrcs)]
    d = dsts if dsts is not None else [0x100000 * (i + 1) for i in range(ndsts)]
    sa = (ctypes.c_void_p * 16)(*s)
    da = (ctypes.c_void_p * 16)(*d)
    pre = pre or []
    pa = (ctypes.c_uint64 * 16)(*pre) if pre else None
    return L.nexrReduceCopy(nsrcs, sa, ndsts, da, n, dt, op, arg, len(pre), pa, 0, None)


def test_invalid_arguments_fail_before_the_device(nexr):
    assert _call(nexr, nsrcs=0) == 4
    assert _call(nexr, nsrcs=9) == 4
    assert _call(nexr, ndsts=9) == 4
    assert _call(nexr, dt=12) == 4
    assert _call(nexr, dt=10) == 4                     # fp8: the fork compiles the path out
    assert _call(nexr, op=5) == 4
    assert _call(nexr, op=4, dt=7) == 4                # SumPostDiv only for integers
    assert _call(nexr, op=4, dt=0, arg=(256 << 1) | 1) == 4  # divisor truncates to (int8)0
    assert _call(nexr, srcs=[0x1000, 0]) == 4          # null source
    assert _call(nexr, dsts=[0]) == 4                  # null destination
    L = nexr.lib()
    sa = (ctypes.c_void_p * 2)(0x1000, 0x2000)
    da = (ctypes.c_void_p * 1)(0x3000)
    assert L.nexrReduceCopy(2, sa, 1, da, 16, 7, 0, 0, 3, None, 0, None) == 4  # nPreOp > nSrcs
    assert L.nexrReduceCopy(2, sa, 1, da, 16, 7, 0, 0, 1, None, 0, None) == 4  # preOpArgs NULL


def test_host_registration_validates_before_the_device(nexr):
    """nexrHostRegister / Deregister / MemAlloc / MemFree / GetHostPathStats reject bad arguments and
    accept the NULL no-ops (ncclCommDeregister and ncclMemFree take NULL, register.cc:147, allocator.cc)
    with no HIP call; the stats read and reset without a device."""
    L = nexr.lib()
    h = ctypes.c_void_p()
    assert L.nexrHostRegister(None, 4096, ctypes.byref(h)) == 4
    assert L.nexrHostRegister(ctypes.c_void_p(0x10000), 0, ctypes.byref(h)) == 4
    assert L.nexrHostRegister(ctypes.c_void_p(0x10000), 4096, None) == 4
    assert L.nexrHostDeregister(None) == 0
    assert L.nexrHostDeregister(ctypes.c_void_p(0x1234)) == 5  # not a handle of this library
    p = ctypes.c_void_p()
    assert L.nexrHostMemAlloc(None, 4096) == 4
    assert L.nexrHostMemAlloc(ctypes.byref(p), 0) == 4
    assert L.nexrHostMemFree(None) == 0
    assert L.nexrHostMemFree(ctypes.c_void_p(0x1234)) == 4   # not from nexrHostMemAlloc
    assert L.nexrGetHostPathStats(None, 0) == 4
    st = nexr.HostPathStats()
    assert L.nexrGetHostPathStats(ctypes.byref(st), 1) == 0
    assert nexr.host_path_stats()["calls"] == 0


# Restatement of the reference struct (src/include/device.h:682-693, src/nccl.h.in:259-270), compiled
# beside include/nexr.h as C11 and as C++17 (the reference's host code is C++): the two layouts must be
# identical, field by field.
_REF_STRUCT = r"""
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif
#include "nexr.h"
typedef enum { ncclSum, ncclProd, ncclMax, ncclMin, ncclAvg, ncclNumOps, ncclMaxRedOp = 0x7fffffff } ncclRedOp_t;
enum ncclDevRedOp_t { ncclDevSum, ncclDevProd, ncclDevMinMax, ncclDevPreMulSum, ncclDevSumPostDiv, ncclNumDevRedOps };
struct ncclDevRedOpFull {
  enum ncclDevRedOp_t op;
  ncclRedOp_t proxyOp;
  bool scalarArgIsPtr;
  uint64_t scalarArg;
};
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(struct ncclDevRedOpFull), offsetof(struct ncclDevRedOpFull, op),
         offsetof(struct ncclDevRedOpFull, proxyOp), offsetof(struct ncclDevRedOpFull, scalarArgIsPtr),
         offsetof(struct ncclDevRedOpFull, scalarArg));
  printf("%zu %zu %zu %zu %zu\n", sizeof(nexrDevRedOpFull), offsetof(nexrDevRedOpFull, op),
         offsetof(nexrDevRedOpFull, proxyOp), offsetof(nexrDevRedOpFull, scalarArgIsPtr),
         offsetof(nexrDevRedOpFull, scalarArg));
  printf("%zu %zu\n", sizeof(((struct ncclDevRedOpFull*)0)->scalarArgIsPtr),
         sizeof(((nexrDevRedOpFull*)0)->scalarArgIsPtr));
  return 0;
}
"""


@pytest.mark.parametrize("compiler,std,suffix", [("gcc", "-std=c11", ".c"), ("g++", "-std=c++17", ".cc")])
def test_dev_red_op_full_is_byte_exact_with_reference(nexr, tmp_path, compiler, std, suffix):
    src = tmp_path / ("layout" + suffix)
    src.write_text(_REF_STRUCT)
    exe = tmp_path / "layout"
    subprocess.run([compiler, std, "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True, capture_output=True, text=True, timeout=120)
    ref, ours, bools = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines()
    assert ref == ours == "24 0 4 8 16"
    assert bools == "1 1"
    # The Python mirror has the same layout.
    F = nexr.DevRedOpFull
    assert ctypes.sizeof(F) == 24
    assert (F.op.offset, F.proxyOp.offset, F.scalarArgIsPtr.offset, F.scalarArg.offset) == (0, 4, 8, 16)
    assert F.scalarArgIsPtr.size == 1


def test_dev_red_op_full_padding_is_never_read(nexr):
    """A caller's struct whose padding bytes 9-15 are 0xFF still reads scalarArgIsPtr = false: the flag
    is the single byte at offset 8 (with an int-sized flag, as in round 1, the same bytes read as a
    non-zero int and the scalar would be dereferenced as a pointer)."""
    raw = bytearray(24)
    raw[0:4] = (3).to_bytes(4, "little")        # ncclDevPreMulSum
    raw[4:8] = (0).to_bytes(4, "little")
    raw[8] = 0
    raw[9:16] = b"\xff" * 7
    raw[16:24] = (0x3F800000).to_bytes(8, "little")
    f = nexr.DevRedOpFull.from_buffer_copy(bytes(raw))
    assert f.scalarArgIsPtr is False and f.op == 3 and f.scalarArg == 0x3F800000
    # The C ABI receives exactly these 24 bytes by value (same layout as checked above).
    assert bytes(f)[9:16] == b"\xff" * 7


def test_query_launch_grid_respects_the_work_item_limit(nexr):
    """Advisor r1: the grid cap must keep grid x block <= 2^32 - 1 (HIP's limit); a call that needs
    more workgroups is capped and grid-strides instead of failing. Pointers with mixed 16-B phases
    take the packed path too (unaligned 16-B accesses), never an element-per-work-item path."""
    # int8, K=2, mixed phases: packed, unaligned; 1 TiB per buffer needs 2^32 workgroups of 256
    info = nexr.query_launch([0x1000, 0x2001], [0x3000], 1 << 40, 0)
    assert (info.unaligned, info.block, info.packsPerLane) == (1, 256, 4)
    assert info.grid * info.block <= 0xFFFFFFFF
    assert info.grid == 0xFFFFFFFF // 256
    info = nexr.query_launch([0x1000, 0x2001], [0x3000], 1 << 32, 0)
    assert info.unaligned == 1 and info.grid == (1 << 32) // 16 // 4 // 256
    # fp16 K=8 under the nt-store policy (block 512): a 16 GiB body needs 2^21 workgroups -> under the
    # 2^23 cap
    srcs = [0x10000 * (i + 1) for i in range(8)]
    info = nexr.query_launch(srcs, [0x100000], 8 << 30, 6)
    assert info.block == 512 and info.packsPerLane == 1
    assert info.grid == (8 << 30) * 2 // 16 // 512 and info.grid * info.block <= 0xFFFFFFFF
    # fp16 K=8 with mixed phases at 2^33 elements: packed like the aligned call above
    info = nexr.query_launch([0x10000 * (i + 1) + (i & 1) * 2 for i in range(8)], [0x100000], 1 << 33, 6)
    assert info.unaligned == 1 and info.grid == (1 << 34) // 16 // 512
    # C2 geometry: 256 MiB fp32 K=2, U=4 packs per lane, one 16 KiB trip per workgroup, nt loads
    info = nexr.query_launch([0x10000000, 0x20000000], [0x30000000], 64 << 20, 7)
    assert (info.grid, info.block, info.packsPerLane, info.policy) == (16384, 256, 4, 3)
    # K = 4: the geometry follows the cache policy (nexr_internal.h shape_for): C4 (64 MiB per
    # buffer, 320 MiB streamed: nt loads) runs 2 packs x 512 lanes for 1-, 2- and 8-byte types and the
    # default 4 x 256 for 4-byte ones; >= 512 MiB streamed (nt loads and stores) 1 x 1024, except fp16
    # (4 x 256) and bf16 (1 x 512, two per CU: round 6);
    # below 64 MiB streamed the default 4 x 256.
    k4 = [0x10000000 * (i + 1) for i in range(4)]
    for dt, n, want in ((2, 16 << 20, (4096, 256, 4, 1)), (0, 64 << 20, (4096, 512, 2, 1)),
                        (9, 32 << 20, (4096, 512, 2, 1)), (7, 16 << 20, (4096, 256, 4, 1)),
                        (2, 64 << 20, (16384, 1024, 1, 3)), (9, 128 << 20, (32768, 512, 1, 3)),
                        (6, 128 << 20, (16384, 256, 4, 3)), (2, 1 << 20, (256, 256, 4, 0))):
        info = nexr.query_launch(k4, [0x60000000], n, dt)
        assert (info.grid, info.block, info.packsPerLane, info.policy) == want, (dt, n)
    # K = 3 and K = 5: the default below the nt-store policy; under it K = 5 runs 1 x 1024 at one
    # workgroup per CU like K = 4 (round 5, fp16 excepted) and K = 3 keeps the default
    for k in (3, 5):
        srcs_k = k4[:3] + [0x50000000, 0x58000000][:k - 3]
        info = nexr.query_launch(srcs_k, [0x60000000], 16 << 20, 7)
        assert (info.block, info.packsPerLane, info.policy) == (256, 4, 1), k
        info = nexr.query_launch(srcs_k, [0x60000000], 64 << 20, 7)
        assert (info.block, info.packsPerLane, info.policy) == ((1024, 1, 3) if k == 5 else (256, 4, 3)), k
        info = nexr.query_launch(srcs_k, [0x60000000], 128 << 20, 6)
        assert (info.block, info.packsPerLane, info.policy) == (256, 4, 3), k
    # K >= 6 under the nt-store policy (>= 512 MiB streamed): 1 x 512 for every type (bf16 too since
    # round 6's hardware RNE); below it the default, except 16-bit K = 8, which is 1 x 1024 at every size
    k8 = [0x10000000 * (i + 1) for i in range(8)]
    for k, dt, n, want in ((6, 7, 64 << 20, (32768, 512, 1, 3)), (8, 2, 64 << 20, (32768, 512, 1, 3)),
                           (7, 8, 32 << 20, (32768, 512, 1, 3)), (8, 9, 128 << 20, (32768, 512, 1, 3)),
                           (6, 9, 128 << 20, (32768, 512, 1, 3)), (8, 6, 128 << 20, (32768, 512, 1, 3)),
                           (8, 7, 4 << 20, (1024, 256, 4, 1)), (6, 0, 1 << 20, (64, 256, 4, 0)),
                           (8, 9, 1 << 20, (128, 1024, 1, 0)), (8, 6, 8 << 20, (1024, 1024, 1, 1))):
        info = nexr.query_launch(k8[:k], [0x90000000], n, dt)
        assert (info.grid, info.block, info.packsPerLane, info.policy) == want, (k, dt, n)
    # K = 1 with M = 1-4, K = 2 with M = 1-7 and K = 3 with M = 2-7 take nt stores from 96 MiB streamed
    # (rounds 5-6); K = 3 with one destination, K = 1 with M >= 5, K = 2-3 with M = 8, K >= 4 the general
    # rule (nt loads from 64 MiB, nt stores from 512)
    d2, d3 = [0x90000000, 0xa0000000], [0x90000000, 0xa0000000, 0xb0000000]
    d5 = [0x90000000 + 0x10000000 * i for i in range(5)]
    for srcs_, dsts_, mib, want_pol in ((k8[:2], [0x90000000], 8, 0), (k8[:2], [0x90000000], 32, 3),
                                         (k8[:2], d2, 32, 3), (k8[:2], d2, 20, 1), (k8[:3], [0x90000000], 32, 1),
                                         (k8[:2], [0x90000000], 16, 0), (k8[:1], [0x90000000], 48, 3),
                                         (k8[:1], [0x90000000], 32, 1), (k8[:1], d2, 32, 3), (k8[:2], d3, 32, 3),
                                         (k8[:1], d5[:4], 20, 3), (k8[:3], d2, 20, 3), (k8[:3], d3, 16, 3),
                                         (k8[:4], d2, 16, 1), (k8[:2], d5, 16, 3), (k8[:1], d5, 20, 1),
                                         (k8[:3], d5, 12, 3), (k8[:2], d5 + d2, 12, 3), (k8[:3], d5 + d2[:1], 12, 3),
                                         (k8[:3], d5 + d2, 12, 3), (k8[:2], d5 + d3, 12, 1), (k8[:3], d5 + d3, 12, 1)):
        info = nexr.query_launch(srcs_, dsts_, (mib << 20) // 4, 7)
        assert info.policy == want_pol, (len(srcs_), len(dsts_), mib)
    # head/body/tail split for a shared 4-B phase: the head brings dst0 to its next 128-B boundary
    # (31 fp32 elements), then 17 packs, then 1 tail element
    info = nexr.query_launch([0x1004, 0x2004], [0x3004], 100, 7)
    assert (info.unaligned, info.headElts, info.bodyPacks) == (0, 31, 17)
    # mixed phases, dst0 already on a 128-B boundary: no head, 6 unaligned packs, 4 tail bytes
    info = nexr.query_launch([0x1000, 0x2001], [0x3080], 100, 0)
    assert (info.unaligned, info.headElts, info.bodyPacks) == (1, 0, 6)
    # dst0 not on an element boundary (fp32 at an odd address): no head, all 16-B accesses unaligned
    info = nexr.query_launch([0x1000, 0x2000], [0x3001], 100, 7)
    assert (info.unaligned, info.headElts, info.bodyPacks) == (1, 0, 25)
    # the diagnostics struct of ABI 0.2 (round 1's always-zero `generic` field dropped)
    import ctypes
    L = nexr.LaunchInfo
    assert ctypes.sizeof(L) == 40 and L.policy.offset == 12 and L.unaligned.offset == 16
    assert not hasattr(L, "generic")
    assert L.headElts.offset == 24 and L.bodyPacks.offset == 32
    # validation as nexrReduceCopy; empty calls launch nothing
    with pytest.raises(nexr.NexrError):
        nexr.query_launch([0x1000, 0], [0x3000], 16, 7)
    assert nexr.query_launch([0x1000], [0x3000], 0, 7).grid == 0


def test_nt_store_table_at_its_threshold(nexr):
    """pickPolicy's (K, M) table (nexr_api.cpp, round 5): every K = 1..8 x M = 1..8 just at and just
    below 96 MiB streamed. Inside the table (K = 1 with M = 1-4, K = 2 with M = 1-7, K = 3 with M = 2-7)
    the call takes nt loads + stores (3) from 96 MiB; everywhere else, and below 96 MiB, the general
    rule's nt loads (1) between 64 and 512 MiB."""
    table = {1: range(1, 5), 2: range(1, 8), 3: range(2, 8)}
    mib96 = 96 << 20
    for k in range(1, 9):
        for m in range(1, 9):
            n = -(-mib96 // (k + m))  # the first size streaming >= 96 MiB (uint8: 1 byte per element)
            srcs = [0x100000000 * (i + 1) for i in range(k)]
            dsts = [0x1000000000 + 0x100000000 * d for d in range(m)]
            at = nexr.query_launch(srcs, dsts, n, 1).policy
            below = nexr.query_launch(srcs, dsts, n - 1, 1).policy
            assert at == (3 if m in table.get(k, ()) else 1), (k, m)
            assert below == 1, (k, m)


def test_empty_calls_are_noops(nexr):
    # nElts == 0 and nDsts == 0 return success without launching (common_kernel.h:288-289).
    assert _call(nexr, n=0) == 0
    assert _call(nexr, ndsts=0) == 0


def test_batch_work_layout_matches_header(nexr):
    # nexrReduceCopyWork: int, int, 8 src ptrs, 8 dst ptrs, size_t, u64, int, int, 8 u64.
    W = nexr.ReduceCopyWork
    assert ctypes.sizeof(W) == 8 + 64 + 64 + 8 + 8 + 8 + 64
    assert (W.srcs.offset, W.dsts.offset, W.nElts.offset, W.preOpArgs.offset) == (8, 72, 136, 160)
    assert re.search(r"#define\s+NEXR_MAX_BATCH_WORKS\s+(\d+)", open(HEADER).read()).group(1) == str(
        nexr.MAX_BATCH_WORKS)


_LL_STEPS_LAYOUT = r"""
#include <stddef.h>
#include <stdio.h>
#include "nexr.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(nexrLLStep), offsetof(nexrLLStep, srcIx),
         offsetof(nexrLLStep, dstIx), offsetof(nexrLLStep, nElts), offsetof(nexrLLStep, recv),
         offsetof(nexrLLStep, send), offsetof(nexrLLStep, srcBuf), offsetof(nexrLLStep, dstBuf),
         offsetof(nexrLLStep, postOp));
  printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(nexrLLConnSet), offsetof(nexrLLConnSet, nRecv),
         offsetof(nexrLLConnSet, recvFifo), offsetof(nexrLLConnSet, recvHead), offsetof(nexrLLConnSet, recvStep),
         offsetof(nexrLLConnSet, sendFifo), offsetof(nexrLLConnSet, sendHead), offsetof(nexrLLConnSet, sendStep),
         offsetof(nexrLLConnSet, slotBytes), offsetof(nexrLLConnSet, nSlots), offsetof(nexrLLConnSet, pad));
  return 0;
}
"""


def test_ll_steps_structs_match_header(nexr, tmp_path):
    """nexrLLStep / nexrLLConnSet (ABI 0.3): the C layout (compiled from include/nexr.h) and the ctypes
    mirror agree field by field; a step is 32 bytes (kLLStepsMax of them fit one launch's 4 KiB)."""
    src = tmp_path / "ll_steps_layout.c"
    src.write_text(_LL_STEPS_LAYOUT)
    exe = tmp_path / "ll_steps_layout"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), str(src), "-o",
                    str(exe)], check=True, capture_output=True, text=True, timeout=120)
    step, conns = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines()
    S, C = nexr.LLStep, nexr.LLConnSet
    assert step.split() == [str(v) for v in (ctypes.sizeof(S), S.srcIx.offset, S.dstIx.offset, S.nElts.offset,
                                               S.recv.offset, S.send.offset, S.srcBuf.offset, S.dstBuf.offset,
                                               S.postOp.offset)]
    assert ctypes.sizeof(S) == 32
    assert conns.split() == [str(v) for v in (ctypes.sizeof(C), C.nRecv.offset, C.recvFifo.offset, C.recvHead.offset,
                                                C.recvStep.offset, C.sendFifo.offset, C.sendHead.offset,
                                                C.sendStep.offset, C.slotBytes.offset, C.nSlots.offset,
                                                C.pad.offset)]
    hdr = open(HEADER).read()
    assert re.search(r"#define\s+NEXR_LL_STEPS_MAX_PEERS\s+(\d+)", hdr).group(1) == str(nexr.LL_STEPS_MAX_PEERS)
    assert re.search(r"#define\s+NEXR_LL_HEAD_BYTES\s+(\d+)", hdr).group(1) == str(nexr.LL_HEAD_BYTES)


def test_ll_steps_validate_before_the_device(nexr):
    """nexrReduceCopyLLSteps rejects a bad connection set or step before anything is launched."""
    L = nexr.lib()
    fifo, head, slot = 0x100000, 0x200000, 1 << 16

    def call(conns, steps, dt=7, op=0):
        arr = (nexr.LLStep * max(1, len(steps)))(*steps)
        return L.nexrReduceCopyLLSteps(ctypes.byref(conns) if conns is not None else None, arr, len(steps), dt, op,
                                       0, None, 0, None)

    def conns(n_recv=1, n_send=1, slot_bytes=slot, n_slots=8, inp=0x10000, out=0x20000):
        c = nexr.LLConnSet()
        c.input, c.output, c.nRecv, c.nSend = inp, out, n_recv, n_send
        for i in range(min(n_recv, 3)):
            c.recvFifo[i], c.recvHead[i] = fifo, head
        for i in range(min(n_send, 3)):
            c.sendFifo[i], c.sendHead[i] = fifo + slot * 8, head + 4096
        c.slotBytes, c.nSlots = slot_bytes, n_slots
        return c

    ok = nexr.ll_step(0, 0, 1, 0, 100, recv=True, send=True)
    assert call(conns(), []) == 0                                    # nothing to run
    assert call(None, [ok]) == 4
    assert call(conns(n_recv=4), [ok]) == 4                          # > NEXR_LL_STEPS_MAX_PEERS
    assert call(conns(slot_bytes=1000), [ok]) == 4                   # not a 16-B multiple
    assert call(conns(n_slots=0), [ok]) == 4
    assert call(conns(), [ok], dt=10) == 4                           # fp8
    assert call(conns(), [ok], dt=7, op=4) == 4                      # SumPostDiv on a float
    bad_fifo = conns()
    bad_fifo.recvFifo[0] = fifo + 8                                  # FIFO not 16-B aligned
    assert call(bad_fifo, [ok]) == 4
    bad_head = conns()
    bad_head.sendHead[0] = 0
    assert call(bad_head, [ok]) == 4
    assert call(conns(n_recv=0), [ok]) == 4                          # a recv step without receive connections
    assert call(conns(), [nexr.ll_step(0, 0, 1, 0, slot // 2 // 4 + 1, recv=True)]) == 4  # more than a slot's data
    assert call(conns(), [nexr.ll_step(-1, 0, 1, 0, 100)]) == 4      # no source and no receive
    assert call(conns(), [nexr.ll_step(0, 0, 2, 0, 100)]) == 4       # dstBuf out of range
    assert call(conns(out=0), [nexr.ll_step(0, 0, 1, 0, 100)]) == 4  # output buffer missing
    assert call(conns(), [ok, nexr.ll_step(0, -1, 1, 0, 100)]) == 4  # a later bad step: nothing runs


def test_batch_validates_every_work_before_launching(nexr):
    L = nexr.lib()
    good = nexr.make_work([0x1000, 0x2000], [0x3000], 16)
    bad_null = nexr.make_work([0x1000, 0], [0x3000], 16)
    bad_pre = nexr.make_work([0x1000], [0x3000], 16, pre_op_args=[1])
    bad_pre.nPreOpSrcs = 2  # > nSrcs
    for bad in (bad_null, bad_pre):
        arr = (nexr.ReduceCopyWork * 3)(good, bad, good)
        assert L.nexrReduceCopyBatch(arr, 3, 7, 0, None) == 4
    arr = (nexr.ReduceCopyWork * 1)(good)
    assert L.nexrReduceCopyBatch(arr, 1, 10, 0, None) == 4  # fp8
    assert L.nexrReduceCopyBatch(arr, 1, 7, 4, None) == 4   # SumPostDiv on a float
    assert L.nexrReduceCopyBatch(arr, -1, 7, 0, None) == 4
    assert L.nexrReduceCopyBatch(None, 2, 7, 0, None) == 4
    # Empty batches and works with nothing to store never reach the device.
    assert L.nexrReduceCopyBatch(None, 0, 7, 0, None) == 0
    empty = nexr.make_work([0x1000, 0x2000], [0x3000], 0)
    nodst = nexr.make_work([0x1000, 0x2000], [], 16)
    arr = (nexr.ReduceCopyWork * 2)(empty, nodst)
    assert L.nexrReduceCopyBatch(arr, 2, 7, 0, None) == 0
    with pytest.raises(nexr.NexrError):
        nexr.make_work([1] * 9, [2], 4)


def test_multi_device_validates_before_any_thread(nexr):
    L = nexr.lib()
    good = nexr.make_work([0x1000, 0x2000], [0x3000], 16)
    bad = nexr.make_work([0x1000, 0], [0x3000], 16)
    dev = (ctypes.c_int * 3)(0, 0, 0)
    secs = ctypes.c_double(-1.0)
    arr = (nexr.ReduceCopyWork * 3)(good, bad, good)
    assert L.nexrReduceCopyMultiDevice(arr, dev, 3, 7, 0, 1, ctypes.byref(secs)) == 4
    arr = (nexr.ReduceCopyWork * 1)(good)
    assert L.nexrReduceCopyMultiDevice(arr, dev, 1, 7, 0, 0, None) == 4     # reps < 1
    assert L.nexrReduceCopyMultiDevice(arr, None, 1, 7, 0, 1, None) == 4    # no device list
    assert L.nexrReduceCopyMultiDevice(arr, dev, 1, 11, 0, 1, None) == 4    # fp8
    assert L.nexrReduceCopyMultiDevice(arr, dev, 65, 7, 0, 1, None) == 4    # > NEXR_MAX_MULTI_DEVICE_WORKS
    assert L.nexrReduceCopyMultiDevice(None, None, 0, 7, 0, 1, ctypes.byref(secs)) == 0
    assert secs.value == 0.0
    with pytest.raises(nexr.NexrError):
        nexr.reduce_copy_multi_device([good], [0, 1], 7, 0)


def test_multi_device_sets_validates_every_set_before_any_thread(nexr):
    """nexrReduceCopyMultiDeviceSets: every work of every set is validated first (a bad work in the
    last set of the last device fails the call with nothing run); nSets outside [1, 8] is rejected."""
    L = nexr.lib()
    good = nexr.make_work([0x1000, 0x2000], [0x3000], 16)
    bad = nexr.make_work([0x1000, 0], [0x3000], 16)
    dev = (ctypes.c_int * 2)(0, 0)
    arr = (nexr.ReduceCopyWork * 6)(good, good, good, good, good, bad)
    assert L.nexrReduceCopyMultiDeviceSets(arr, dev, 2, 3, 7, 0, 1, None) == 4
    arr = (nexr.ReduceCopyWork * 1)(good)
    assert L.nexrReduceCopyMultiDeviceSets(arr, dev, 1, 0, 7, 0, 1, None) == 4   # nSets < 1
    assert L.nexrReduceCopyMultiDeviceSets(arr, dev, 1, 9, 7, 0, 1, None) == 4   # > NEXR_MAX_MULTI_DEVICE_SETS
    assert L.nexrReduceCopyMultiDeviceSets(arr, dev, 1, 1, 7, 0, 0, None) == 4   # reps < 1
    assert L.nexrReduceCopyMultiDeviceSets(None, None, 0, 3, 7, 0, 1, None) == 0
    with pytest.raises(nexr.NexrError):
        nexr.reduce_copy_multi_device_sets([[good, good], [good]], [0, 0], 7, 0)


@pytest.mark.parametrize("dt", sorted(mg.DT_NAMES) + [10, 11])
@pytest.mark.parametrize("op,nranks", [(0, 2), (1, 2), (2, 4), (3, 4), (4, 1), (4, 3), (4, 8), (5, 2)])
def test_host_to_dev_red_op_matches_oracle(nexr, oracle, dt, op, nranks):
    L = nexr.lib()
    out = nexr.DevRedOpFull()
    rc = L.nexrHostToDevRedOp(ctypes.byref(out), op, dt, nranks)
    if op == 5 or (op == 4 and dt in (10, 11)):
        assert rc == 4
        return
    assert rc == 0
    if dt in (10, 11):  # oracle has no fp8 arithmetic; encoding only
        bits = 8
        all_bits = (1 << bits) - 1
        exp = {0: (0, 0), 1: (1, 0), 2: (2, all_bits), 3: (2, 0)}[op]
    else:
        exp = oracle.host_to_dev_red_op(op, dt, nranks)
    assert (out.op, out.scalarArg) == exp
    assert out.proxyOp == op and out.scalarArgIsPtr is False


def _declared(header: str):
    text = open(os.path.join(ROOT, "include", header)).read()
    return sorted(set(re.findall(r"NEXR_API\s+[\w\s\*]+?\b(nexr\w+)\s*\(", text)))


def _exported(path: str):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line and "nexr" in line}


def test_ring_library_exports_its_header():
    """libnexr_ring.so (the default build) exports exactly include/nexr_ring.h: none of the opt-in
    extras (include/nexr_extras.h) and no PAT."""
    import importlib
    ring = importlib.import_module("nex-nccl_amd.ring")
    declared = _declared("nexr_ring.h")
    assert declared == sorted(ring.RING_ABI_SYMBOLS)
    L = ring.ring_lib()
    assert _exported(ring.RING_LIB_PATH) == set(declared)
    for name in declared:
        assert hasattr(L, name)
    assert not any("Pat" in name for name in declared + _declared("nexr_extras.h"))


def test_extras_library_exports_both_headers():
    """libnexr_extras.so (make EXTRAS=1) is a superset: nexr_ring.h's entry points plus nexr_extras.h's."""
    import importlib
    ring = importlib.import_module("nex-nccl_amd.ring")
    extras = _declared("nexr_extras.h")
    assert extras == sorted(ring.EXTRAS_ABI_SYMBOLS)
    assert not set(extras) & set(_declared("nexr_ring.h"))
    if not ring.extras_available():
        pytest.skip("libnexr_extras.so not built (make -C nex-nccl_amd/csrc EXTRAS=1)")
    assert _exported(ring.EXTRAS_LIB_PATH) == set(extras) | set(_declared("nexr_ring.h"))


def test_extras_calls_need_an_extras_communicator(oracle):
    """Send/recv and the resident collectives on a communicator of the default library fail with the
    library's InvalidUsage, never with a missing-symbol error."""
    import importlib
    import numpy as np
    nexr_pkg = importlib.import_module("nex-nccl_amd")
    ring = importlib.import_module("nex-nccl_amd.ring")
    fn = ctypes.cast(oracle.lib().oracle_reduce_copy_fn, ctypes.c_void_p).value
    x = [np.zeros(8, np.float32) for _ in range(2)]
    with ring.RingComm(2, ring.HOST_MEMORY, 8 * 1024, fn) as comm:
        for call in (lambda: comm.all_reduce_resident([a.ctypes.data for a in x], [a.ctypes.data for a in x], 8, 7, 0),
                     lambda: comm.send_recv([a.ctypes.data for a in x], [1, 0], [a.ctypes.data for a in x], [1, 0], 4)):
            with pytest.raises(nexr_pkg.NexrError) as e:
                call()
            assert e.value.code == nexr_pkg.Result.InvalidUsage


def test_package_fails_loudly_without_library(nexr, monkeypatch, tmp_path):
    monkeypatch.setattr(nexr, "_lib", None)
    monkeypatch.setattr(nexr, "LIB_PATH", str(tmp_path / "missing.so"))
    with pytest.raises(nexr.NexrError):
        nexr.lib()


@pytest.mark.parametrize("order", ["lib_first", "torch_first"])
def test_one_hip_runtime_per_process(order):
    """libnexr and torch must share ONE libamdhip64: with two, torch's streams are foreign handles to
    libnexr and the first launch fails (hipError 100 — what bench.py hit when it loaded the library
    before importing torch). Checked in a fresh interpreter, whichever is loaded first."""
    body = ("p.lib(); import torch" if order == "lib_first" else "import torch; p.lib()")
    code = ("import importlib, sys; sys.path.insert(0, %r); p = importlib.import_module('nex-nccl_amd'); %s; "
            "print(len({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}))" % (ROOT, body))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, check=True, timeout=300)
    assert out.stdout.strip().splitlines()[-1] == "1", out.stdout + out.stderr


def test_peer_ring_rejects_bad_configs_before_the_device():
    import importlib
    ring = importlib.import_module("nex-nccl_amd.ring")
    L = ring.ring_lib()
    h = ctypes.c_void_p()
    cases = [dict(nRanks=0), dict(rank=2), dict(rank=-1), dict(shmName=b"noslash"), dict(shmName=b"/a/b"),
             dict(shmName=None), dict(protocol=3), dict(buffBytes=1000), dict(protocol=2, buffBytes=8 * 16 * 100)]
    for bad in cases:
        f = dict(nRanks=2, rank=0, device=0, buffBytes=0, protocol=0, timeoutMs=10, shmName=b"/nexr_abi_test")
        f.update(bad)
        cfg = ring.PeerRingConfig(**f)
        assert L.nexrPeerRingCommCreate(ctypes.byref(h), ctypes.byref(cfg)) == 4, bad
    assert L.nexrPeerRingAllReduce(None, None, None, 0, 7, 0) == 4


def test_c_example_builds_with_plain_c(tmp_path):
    """include/nexr.h and include/nexr_ring.h are plain C: the example host program (the fork's C
    host code's view of the boundary) compiles and links with gcc -std=c11 -Wall -Wextra -Werror."""
    import subprocess
    out = tmp_path / "reduce_copy_c"
    lib = os.path.join(ROOT, "nex-nccl_amd")
    subprocess.run(["gcc", "-std=c11", "-O2", "-Wall", "-Wextra", "-Werror", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "reduce_copy_c.c"), "-L" + lib, "-lnexr_ring", "-lnexr",
                    "-Wl,-rpath," + lib, "-o", str(out)], check=True, capture_output=True, text=True, timeout=120)
    assert out.exists()


def test_multi_device_c_example_builds(monkeypatch):
    """examples/multi_device_c.c (C5 from plain C through nexrReduceCopyMultiDevice, device memory from
    the HIP runtime's C API) compiles and links with gcc -std=c11 -Wall -Wextra -Werror."""
    import __graft_entry__
    exe = __graft_entry__.build_c_multi_device()
    assert os.path.exists(exe) and os.access(exe, os.X_OK)


def test_ll_steps_c_example_builds():
    """examples/ll_steps_c.c (a run of LL steps with device credits from plain C through
    nexrReduceCopyLLSteps, streams from hipExtStreamCreateWithCUMask) compiles and links with gcc
    -std=c11 -Wall -Wextra -Werror."""
    import __graft_entry__
    exe = __graft_entry__.build_c_ll_steps()
    assert os.path.exists(exe) and os.access(exe, os.X_OK)


def test_hip_runtime_is_the_one_libnexr_uses(nexr):
    """nexr.hip_runtime() hands back the single mapped libamdhip64 (harness calls such as
    hipDeviceEnablePeerAccess must reach the runtime the kernels launch on)."""
    h = nexr.hip_runtime()
    mapped = {ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln and "/" in ln}
    assert mapped == {h._name}
    assert hasattr(h, "hipDeviceEnablePeerAccess")
