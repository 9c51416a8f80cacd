// nexr_ll.hip — the LL-protocol reduce-copy for gfx950.
//
// What it computes is LLGenericOp<RECV, SEND, SrcBuf, DstBuf> (reference src/device/prims_ll.h:
// 218-283) for one FIFO step whose slot pointers and flags the caller resolved:
//   per 8-byte data line l:  d = src[l] (applyPreOp with redOpArg when the source is the user input)
//                            d = RECV ? (SRC ? op(peer0[l], d) : peer0[l]) : d
//                            d = op(peer_i[l], d) for i = 1..nRecv-1      (peer is the FIRST operand)
//                            d = postOp ? applyPostOp(d) : d
//                            send_i[l] = {lo32(d), flag_i, hi32(d), flag_i}   (storeLL :152-158)
//                            dst[l] = d (only the line's valid elements, storeData :202-216)
// A recv line is valid when both its flags equal the expected step flag (readLL :91-109); the
// kernel polls them with system-scope relaxed 64-bit loads, bounded in time, and reports a
// timeout through the optional status word instead of hanging (checkAbort, primitives.h:142-156).
//
// MI355X mapping: one lane handles TWO consecutive lines, i.e. one 16-byte data pack, so the LL
// path reuses the SIMPLE path's per-datatype pack arithmetic (nexr_types.hpp) unchanged; the two
// 16-byte wire lines of a lane are one 32-byte contiguous read per peer.
#include "nexr_types.hpp"

namespace nexr {

typedef __attribute__((address_space(1))) uint64_t g_u64;

__device__ __forceinline__ uint64_t ld_sys(const char* p) {
  return __hip_atomic_load((const g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(char* p, uint64_t v) {
  __hip_atomic_store((g_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait for the two lines at p (32 bytes) to carry `flag` in all four flag words; returns the 16
// data bytes as a pack, or false after the timeout. `nLines` (1 or 2) lines are real.
__device__ __forceinline__ bool read_lines(const char* p, int nLines, uint32_t flag, const LLParams& a,
                                           u32x4* out) {
  uint64_t w[4] = {0, 0, 0, 0};
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (j < 2 * nLines) {
        w[j] = ld_sys(p + 8 * j);
        ok &= (uint32_t)(w[j] >> 32) == flag;
      }
    }
    if (ok) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > a.timeoutTicks) {
      if (a.status) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  *out = (u32x4){(uint32_t)w[0], (uint32_t)w[1], (uint32_t)w[2], (uint32_t)w[3]};
  return true;
}

template <int D, int OP, bool IsMin>
__device__ __forceinline__ void ll_pair(const LLParams& a, uint64_t pair) {
  using T = Ty<D>;
  using V = typename T::V;
  constexpr int esz = 16 / T::EPP;
  const uint64_t nBytes = a.nElts * esz;
  const uint64_t b0 = pair * 16;                               // first data byte of the pair
  const uint64_t nLinesTotal = (nBytes + 7) / 8;
  const int nLines = (pair * 2 + 1 < nLinesTotal) ? 2 : 1;     // the last pair may hold one line
  const uint64_t valid = nBytes - b0 < 16 ? nBytes - b0 : 16;  // valid data bytes of this pair

  u32x4 d = (u32x4)0u;
  if (a.src) {
    if (valid == 16 && (((uintptr_t)(a.src + b0)) & 15) == 0) d = *(const g_cu32x4*)(a.src + b0);
    else __builtin_memcpy(&d, a.src + b0, valid);
    if constexpr (OP == nexrDevPreMulSum) {
      if (a.srcIsInput) d = bc<u32x4>(T::mul(bc<V>(d), T::splat(a.redArg)));  // applyPreOp(redOp, ·)
    }
  }
  for (int i = 0; i < NEXR_MAX_SRCS; i++) {
    if (i >= a.nRecv) break;
    u32x4 peer;
    if (!read_lines(a.recv[i] + pair * 32, nLines, a.recvFlag[i], a, &peer)) return;
    if ((i == 0 && !a.src) || a.firstWins) d = peer;  // SKIP_COMP: applyReduce returns the peer
    else d = bc<u32x4>(reduce_step<D, OP, IsMin>(bc<V>(peer), bc<V>(d)));  // applyReduce(redOp, peer, d)
  }
  if constexpr (OP == nexrDevSumPostDiv) {
    if (a.postOp) d = bc<u32x4>(T::divide(bc<V>(d), a.redArg));
  }
  if constexpr (D == nexrFloat16) {
    // ncclFromFloat canonicalises NaN whenever arithmetic ran on the pack
    const bool arith = !a.firstWins && ((a.nRecv >= 1 && a.src) || a.nRecv >= 2 ||
                                        (OP == nexrDevPreMulSum && a.src && a.srcIsInput));
    if (arith) d = bc<u32x4>(T::canon(bc<V>(d)));
  }
  for (int i = 0; i < NEXR_MAX_DSTS; i++) {
    if (i >= a.nSend) break;
    char* q = a.send[i] + pair * 32;
    const uint64_t f = (uint64_t)a.sendFlag[i] << 32;
    st_sys(q + 0, f | d.x);
    st_sys(q + 8, f | d.y);
    if (nLines == 2) {
      st_sys(q + 16, f | d.z);
      st_sys(q + 24, f | d.w);
    }
  }
  if (a.dst) {
    if (valid == 16 && (((uintptr_t)(a.dst + b0)) & 15) == 0) *(g_u32x4*)(a.dst + b0) = d;
    else __builtin_memcpy(a.dst + b0, &d, valid);
  }
}

template <int D, int OP>
__global__ __launch_bounds__(kBlock) void reduce_copy_ll_kernel(LLParams a) {
  const uint64_t nPairs = (a.nElts * (16 / Ty<D>::EPP) + 15) / 16;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t p = (uint64_t)blockIdx.x * kBlock + threadIdx.x; p < nPairs; p += stride) {
    if constexpr (OP == nexrDevMinMax) {
      if ((a.redArg & 1) == 0) ll_pair<D, OP, true>(a, p);
      else ll_pair<D, OP, false>(a, p);
    } else {
      ll_pair<D, OP, false>(a, p);
    }
  }
}

template <int D>
static hipError_t launch_ll_dt(const LLParams& a, int op, int grid, hipStream_t s) {
  const void* fn = nullptr;
  switch (op) {
    case nexrDevSum: fn = (const void*)&reduce_copy_ll_kernel<D, nexrDevSum>; break;
    case nexrDevProd: fn = (const void*)&reduce_copy_ll_kernel<D, nexrDevProd>; break;
    case nexrDevMinMax: fn = (const void*)&reduce_copy_ll_kernel<D, nexrDevMinMax>; break;
    case nexrDevPreMulSum: fn = (const void*)&reduce_copy_ll_kernel<D, nexrDevPreMulSum>; break;
    case nexrDevSumPostDiv:
      if constexpr (Ty<D>::kIsInt) fn = (const void*)&reduce_copy_ll_kernel<D, nexrDevSumPostDiv>;
      break;
  }
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<LLParams*>(&a)};
  return hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args, 0, s);
}

hipError_t launch_ll(int dt, const LLParams& a, int op, int grid, hipStream_t s) {
  switch (dt) {
    case nexrInt8: return launch_ll_dt<nexrInt8>(a, op, grid, s);
    case nexrUint8: return launch_ll_dt<nexrUint8>(a, op, grid, s);
    case nexrInt32: return launch_ll_dt<nexrInt32>(a, op, grid, s);
    case nexrUint32: return launch_ll_dt<nexrUint32>(a, op, grid, s);
    case nexrInt64: return launch_ll_dt<nexrInt64>(a, op, grid, s);
    case nexrUint64: return launch_ll_dt<nexrUint64>(a, op, grid, s);
    case nexrFloat16: return launch_ll_dt<nexrFloat16>(a, op, grid, s);
    case nexrFloat32: return launch_ll_dt<nexrFloat32>(a, op, grid, s);
    case nexrFloat64: return launch_ll_dt<nexrFloat64>(a, op, grid, s);
    case nexrBfloat16: return launch_ll_dt<nexrBfloat16>(a, op, grid, s);
  }
  return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------------------------
// LL128 (reference src/device/prims_ll128.h:86-331). The reference moves a 2 KiB wire slice per
// warp-32: lane wid holds regs[2g..2g+1] = user 16-B chunk ix(g, wid) = g*32 - 4*(g/2) + wid -
// (g%2)*(wid/8) and sends them as wire words 64g + 2wid (+1); lanes wid%8 == 7 carry the line flag
// in their odd word and therefore only half a chunk per g (the other half moved to g+1 by
// loadRegsFinish). Here one lane owns one 16-byte wire UNIT q = 32g + wid of a slice and derives
// which user bytes it carries from that same map, so the wire is byte-identical to the reference's
// while the kernel itself is laid out for 64-wide waves (any number of slices per workgroup).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ bool wait_flag64(const char* p, uint64_t flag, uint64_t timeoutTicks, uint32_t* status) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (ld_sys(p) != flag) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > timeoutTicks) {
      if (status) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

template <int D, int OP, bool IsMin>
__device__ __forceinline__ void ll128_unit(const LL128Params& a, uint64_t unit) {
  using T = Ty<D>;
  using V = typename T::V;
  constexpr int esz = 16 / T::EPP;
  const uint64_t slice = unit >> 7;
  const int q = (int)(unit & 127);
  const int g = q >> 5, wid = q & 31;
  const bool flagLane = (wid & 7) == 7;
  const uint64_t nBytes = a.nElts * esz;
  const uint64_t dBase = slice * kLL128SliceData;
  const uint64_t eltBytes = nBytes - dBase < kLL128SliceData ? nBytes - dBase : kLL128SliceData;
  uint64_t off, len;
  if (!flagLane) {
    off = (uint64_t)(g * 32 - 4 * (g / 2) + wid - (g % 2) * (wid / 8)) * 16;
    len = 16;
  } else {
    const int ge = g & ~1;  // the chunk loaded at the even g; odd g carries its second half
    off = (uint64_t)(ge * 32 - 4 * (ge / 2) + wid) * 16 + (g & 1) * 8;
    len = 8;
  }
  const uint64_t valid = off < eltBytes ? (eltBytes - off < len ? eltBytes - off : len) : 0;
  const uint64_t wireOff = slice * kLL128SliceBytes + (uint64_t)q * 16;
  const uint64_t flagOff = slice * kLL128SliceBytes + (uint64_t)(4 * g + wid / 8) * 128 + 120;

  u32x4 d = (u32x4)0u;
  if (a.src) {
    if (valid == 16 && (((uintptr_t)(a.src + dBase + off)) & 15) == 0) d = *(const g_cu32x4*)(a.src + dBase + off);
    else if (valid) __builtin_memcpy(&d, a.src + dBase + off, valid);
    if constexpr (OP == nexrDevPreMulSum) {
      if (a.srcIsInput) d = bc<u32x4>(T::mul(bc<V>(d), T::splat(a.redArg)));
    }
  }
  for (int i = 0; i < NEXR_MAX_SRCS; i++) {
    if (i >= a.nRecv) break;
    if (!wait_flag64(a.recv[i] + flagOff, a.recvFlag[i], a.timeoutTicks, a.status)) return;
    const uint64_t lo = ld_sys(a.recv[i] + wireOff), hi = ld_sys(a.recv[i] + wireOff + 8);
    const u32x4 peer = (u32x4){(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    if ((i == 0 && !a.src) || a.firstWins) d = peer;
    else d = bc<u32x4>(reduce_step<D, OP, IsMin>(bc<V>(peer), bc<V>(d)));
  }
  if constexpr (OP == nexrDevSumPostDiv) {
    if (a.postOp) d = bc<u32x4>(T::divide(bc<V>(d), a.redArg));
  }
  if constexpr (D == nexrFloat16) {
    const bool arith = !a.firstWins && ((a.nRecv >= 1 && a.src) || a.nRecv >= 2 ||
                                        (OP == nexrDevPreMulSum && a.src && a.srcIsInput));
    if (arith) d = bc<u32x4>(T::canon(bc<V>(d)));
  }
  const uint64_t lo = ((uint64_t)d.y << 32) | d.x, hi = ((uint64_t)d.w << 32) | d.z;
  for (int i = 0; i < NEXR_MAX_DSTS; i++) {
    if (i >= a.nSend) break;
    st_sys(a.send[i] + wireOff, lo);
    st_sys(a.send[i] + wireOff + 8, flagLane ? a.sendFlag[i] : hi);
  }
  if (a.dst && valid) {
    if (valid == 16 && (((uintptr_t)(a.dst + dBase + off)) & 15) == 0) *(g_u32x4*)(a.dst + dBase + off) = d;
    else __builtin_memcpy(a.dst + dBase + off, &d, valid);
  }
}

template <int D, int OP>
__global__ __launch_bounds__(kBlock) void reduce_copy_ll128_kernel(LL128Params a) {
  const uint64_t nSlices = (a.nElts * (16 / Ty<D>::EPP) + kLL128SliceData - 1) / kLL128SliceData;
  const uint64_t nUnits = nSlices * 128;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  for (uint64_t u = (uint64_t)blockIdx.x * kBlock + threadIdx.x; u < nUnits; u += stride) {
    if constexpr (OP == nexrDevMinMax) {
      if ((a.redArg & 1) == 0) ll128_unit<D, OP, true>(a, u);
      else ll128_unit<D, OP, false>(a, u);
    } else {
      ll128_unit<D, OP, false>(a, u);
    }
  }
}

template <int D>
static hipError_t launch_ll128_dt(const LL128Params& a, int op, int grid, hipStream_t s) {
  const void* fn = nullptr;
  switch (op) {
    case nexrDevSum: fn = (const void*)&reduce_copy_ll128_kernel<D, nexrDevSum>; break;
    case nexrDevProd: fn = (const void*)&reduce_copy_ll128_kernel<D, nexrDevProd>; break;
    case nexrDevMinMax: fn = (const void*)&reduce_copy_ll128_kernel<D, nexrDevMinMax>; break;
    case nexrDevPreMulSum: fn = (const void*)&reduce_copy_ll128_kernel<D, nexrDevPreMulSum>; break;
    case nexrDevSumPostDiv:
      if constexpr (Ty<D>::kIsInt) fn = (const void*)&reduce_copy_ll128_kernel<D, nexrDevSumPostDiv>;
      break;
  }
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<LL128Params*>(&a)};
  return hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args, 0, s);
}

hipError_t launch_ll128(int dt, const LL128Params& a, int op, int grid, hipStream_t s) {
  switch (dt) {
    case nexrInt8: return launch_ll128_dt<nexrInt8>(a, op, grid, s);
    case nexrUint8: return launch_ll128_dt<nexrUint8>(a, op, grid, s);
    case nexrInt32: return launch_ll128_dt<nexrInt32>(a, op, grid, s);
    case nexrUint32: return launch_ll128_dt<nexrUint32>(a, op, grid, s);
    case nexrInt64: return launch_ll128_dt<nexrInt64>(a, op, grid, s);
    case nexrUint64: return launch_ll128_dt<nexrUint64>(a, op, grid, s);
    case nexrFloat16: return launch_ll128_dt<nexrFloat16>(a, op, grid, s);
    case nexrFloat32: return launch_ll128_dt<nexrFloat32>(a, op, grid, s);
    case nexrFloat64: return launch_ll128_dt<nexrFloat64>(a, op, grid, s);
    case nexrBfloat16: return launch_ll128_dt<nexrBfloat16>(a, op, grid, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace nexr
