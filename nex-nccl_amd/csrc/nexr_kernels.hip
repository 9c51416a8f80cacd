// nexr_kernels.hip — the reduce-copy kernel for gfx950, compiled once per datatype with
// -DNEXR_DT=<nexrDataType_t value> (see Makefile) so the 10 objects build in parallel.
//
// What it computes is the reference's reduceCopy (src/device/common_kernel.h:269-349 →
// reduceCopyPacks :141-253) with the real per-type arithmetic of src/device/reduce_kernel.h
// (:238-539, SKIP_COMP at :432 removed). How it computes it is MI355X-first:
//   - one 16-B load per lane per source per pack (global_load_dwordx4), 64-lane waves; each
//     workgroup owns one 16 KiB trip of every buffer (U packs per lane x B lanes = 1024 packs,
//     by default U = 4 with 4 waves; unroll_for/block_for in nexr_internal.h), a "one-shot" grid of
//     nPacks/1024 workgroups (a grid-stride loop only beyond (2^32-1)/B workgroups, HIP's
//     work-item limit), so every lane has U*K independent loads in flight;
//   - every address is a workgroup-uniform base (SGPRs) plus the lane's 32-bit offset, so the
//     accesses use the scalar-base form of global_load/store and no lane holds a 64-bit pointer per
//     buffer (this keeps the 16-bit K = 8 kernels at two workgroups per CU);
//   - all K source loads of a trip are issued before the first reduce step;
//   - cache policy by working-set size: non-temporal loads once a call streams more than
//     64 MiB, non-temporal loads AND stores beyond 512 MiB (2x the Infinity Cache);
//   - no LDS and no cross-lane traffic: every output element depends only on the same index of
//     the inputs, so the reference's warp-32 hunk layout (common_kernel.h:94-113) is irrelevant
//     to the result and is not reproduced.
// The element arithmetic keeps the reference's left-fold order (acc is the first operand,
// reduce_kernel.h:152-168) and rounds to T after every step. MinMax is compiled as two kernels,
// min and max, picked on the host from redOpArg bit 0 (isMin = (arg & 1) == 0, reduce_kernel.h:64).
#include "nexr_fold.hpp"

#include <atomic>

#ifndef NEXR_DT
#error "compile with -DNEXR_DT=<datatype>"
#endif

namespace nexr {

// One element through the same pack arithmetic (lanes other than 0 hold zeros and are dropped).
// Byte-wise accesses in rolled loops: the ABI allows pointers that are not even element-aligned,
// and these are at most 128/esz + 16/esz elements per call, so their code is kept small.
template <int D, int OP, int K, bool IsMin>
__device__ __forceinline__ void do_element(const RCParams& p, const Fold<D, OP, K, IsMin>& f, uint64_t i) {
  constexpr int esz = 16 / Ty<D>::EPP;
  u32x4 in[K];
#pragma unroll
  for (int s = 0; s < K; s++) {
    const unsigned char* q = (const unsigned char*)p.src[s] + i * esz;
    uint64_t v = 0;
#pragma unroll 1
    for (int b = esz - 1; b >= 0; b--) v = (v << 8) | q[b];
    in[s] = (u32x4){(uint32_t)v, (uint32_t)(v >> 32), 0u, 0u};
  }
  const u32x4 out = f.run(in);
  const uint64_t o = (uint64_t)out[0] | ((uint64_t)out[1] << 32);
#pragma unroll 1
  for (int d = 0; d < p.nDsts; d++) {
    unsigned char* q = (unsigned char*)p.dst[d] + i * esz;
#pragma unroll 1
    for (int b = 0; b < esz; b++) q[b] = (unsigned char)(o >> (8 * b));
  }
}

// A workgroup-uniform value pinned to SGPRs. Without it the compiler turns every buffer's trip
// address into a per-lane 64-bit induction variable (two VGPRs per buffer, no scalar-base form).
__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// `bid`/`nblk`: this workgroup's index among the `nblk` workgroups working on `p` (the whole grid
// for a single launch; a slice of it for a batch launch).
template <int D, int OP, int K, int POL, bool IsMin, int U, int B>
__device__ __forceinline__ void body(const RCParams& p, uint64_t bid, uint64_t nblk) {
  using T = Ty<D>;
  constexpr int esz = 16 / T::EPP;
  Fold<D, OP, K, IsMin> f(p);
  if constexpr (OP == nexrDevPreMulSum) {
    if (p.prePtr) {  // scalarArgIsPtr (onerank.cc:32-42): the scalar lives in device memory
      uint64_t raw = 0;
      __builtin_memcpy(&raw, p.prePtr, esz);
      f.factor[0] = T::splat(raw);
    }
  }
  // Every pointer the first trip needs, fetched from the kernel arguments in the same batch of scalar
  // loads as the sizes (otherwise the compiler sinks them past the trip-count check: a second
  // round trip to the argument segment before the first load, ~0.6 us on a 16 MiB launch).
#pragma unroll
  for (int s = 0; s < K; s++) asm volatile("" ::"s"(p.src[s]));
  asm volatile("" ::"s"(p.dst[0]));
  const int nDsts = p.nDsts;
  const uint64_t gid = bid * B + threadIdx.x;
  const uint64_t nthreads = nblk * B;

  const uint64_t head = p.head;

  // Packed body, starting past the head edge (the edge elements follow it, below, so that the
  // body's first loads wait for nothing but their pointers). Pointers without the common 16-B phase are read /
  // written with unaligned 16-B accesses (ld16 / st16 assume only byte alignment).
  const uint64_t bodyOff = head * esz;
  const uint64_t nPacks = p.nPacks;
  const uint64_t nFull = nPacks / (B * U);  // trips of B*U packs
  constexpr uint64_t kTrip = (uint64_t)B * U * 16;
  const uint32_t lane = threadIdx.x * 16u;
  // Full trips: K*U 16-B loads in flight per lane (every source's pack u = 0, then u = 1, ...), then
  // the fold, then U stores per destination. The trip base is uniform: it stays in SGPRs.
  for (uint64_t g = bid; g < nFull; g += nblk) {
    const uint64_t tb = bodyOff + g * kTrip;
    u32x4 in[U][K];
#pragma unroll
    for (int s = 0; s < K; s++) {
      const char* base = (const char*)uniform64((uint64_t)(p.src[s] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) in[u][s] = ld16<POL>(base + (uint32_t)(lane + u * B * 16));
    }
    u32x4 out[U];
#pragma unroll
    for (int u = 0; u < U; u++) out[u] = f.run(in[u]);
    {
      char* base = (char*)uniform64((uint64_t)(p.dst[0] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) st16<POL>(base + (uint32_t)(lane + u * B * 16), out[u]);
    }
    // A second destination (a ring step's recvReduceCopySend: user buffer + next peer) unrolled
    // as well; any further ones in a rolled loop whose pointer is read from the kernel arguments with
    // a scalar load (a rolled second store cost a 16 MiB M = 2 step 1-4 %, profiles/r05a_body_ab.txt).
    if (nDsts > 1) {
      char* base = (char*)uniform64((uint64_t)(p.dst[1] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) st16<POL>(base + (uint32_t)(lane + u * B * 16), out[u]);
    }
#pragma unroll 1
    for (int d = 2; d < nDsts; d++) {
      char* base = (char*)uniform64((uint64_t)(p.dst[d] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) st16<POL>(base + (uint32_t)(lane + u * B * 16), out[u]);
    }
  }
  // Remaining packs (< B*U): one pack per thread.
  for (uint64_t j = nFull * (B * U) + gid; j < nPacks; j += nthreads) {
    const uint64_t off = bodyOff + j * 16;
    u32x4 in[K];
#pragma unroll
    for (int s = 0; s < K; s++) in[s] = ld16<POL>(p.src[s] + off);
    const u32x4 out = f.run(in);
#pragma unroll 1
    for (int d = 0; d < nDsts; d++) st16<POL>(p.dst[d] + off, out);
  }
  // Edge elements before/after the packed body: fewer than 128/esz + 16/esz of them.
  const uint64_t bodyElts = nPacks * T::EPP;
  const uint64_t tail = p.nElts - head - bodyElts;
  if (gid < head + tail) {
    const uint64_t e = gid < head ? gid : head + bodyElts + (gid - head);
    do_element<D, OP, K, IsMin>(p, f, e);
  }
}

template <int D, int OP, int K, int POL, bool IsMin = false, int U = unroll_for(D, K, POL),
          int B = block_for(D, K, POL)>
__global__ __launch_bounds__(B) void reduce_copy_kernel(RCParams p) {
  body<D, OP, K, POL, IsMin, U, B>(p, blockIdx.x, gridDim.x);
}

// Batch launch (the analogue of a kernel running a ncclDevWorkBatch: src/device/common.h:307-342):
// up to kMaxBatch independent reduce-copies with the same (datatype, op, K, and for MinMax the same
// isMin) in one launch; work i owns workgroups [start[i], start[i+1]). The work index is
// wave-uniform, so the descriptor is read straight from the kernel-argument segment with scalar loads.
template <int D, int OP, int K, int POL, bool IsMin = false>
__global__ __launch_bounds__(block_for(D, K, POL)) void reduce_copy_batch_kernel(BatchParams b) {
  int i = 0;
  while (i + 1 < b.nWorks && blockIdx.x >= b.start[i + 1]) i++;
  body<D, OP, K, POL, IsMin, unroll_for(D, K, POL), block_for(D, K, POL)>(b.w[i], blockIdx.x - b.start[i],
                                                                         b.start[i + 1] - b.start[i]);
}

// A kernel launched with more than 64 KiB of dynamic LDS must be allowed it first, once per device.
// The attribute applies to the function on the CURRENT device, while the launch runs on the stream's:
// so it is set on the stream's device (switching to it for the call when the caller's current device
// differs) and recorded per that device.
static hipError_t allow_lds(const void* fn, int lds, std::atomic<uint64_t>& allowed, hipStream_t s) {
  if (lds <= 64 * 1024) return hipSuccess;
  int dev = 0;
  hipError_t e = hipStreamGetDevice(s, &dev);
  if (e != hipSuccess) return e;
  const uint64_t bit = dev < 64 ? 1ull << dev : 0;
  if (bit && (allowed.load(std::memory_order_acquire) & bit)) return hipSuccess;
  int cur = 0;
  e = hipGetDevice(&cur);
  if (e != hipSuccess) return e;
  if (cur != dev && (e = hipSetDevice(dev)) != hipSuccess) return e;
  e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  if (cur != dev) {
    const hipError_t back = hipSetDevice(cur);
    if (e == hipSuccess) e = back;
  }
  if (e == hipSuccess && bit) allowed.fetch_or(bit, std::memory_order_acq_rel);
  return e;
}

template <int D, int OP, int K, bool IsMin>
static const void* kernel_for(int pol) {
  return pol == kPolNt       ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNt, IsMin>
         : pol == kPolNtLoad ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNtLoad, IsMin>
                             : (const void*)&reduce_copy_kernel<D, OP, K, kPolPlain, IsMin>;
}

template <int D, int OP, int K>
static hipError_t launch_k(const RCParams& p, const Geometry& g, hipStream_t s) {
  const void* fn = kernel_for<D, OP, K, false>(g.pol);
  if constexpr (OP == nexrDevMinMax) {
    if ((p.redArg & 1) == 0) fn = kernel_for<D, OP, K, true>(g.pol);
  }
  const int lds = lds_for(D, K, g.pol);
  if (lds > 64 * 1024) {
    static std::atomic<uint64_t> allowed[2][4];  // [isMin][policy]: devices the attribute is set on
    const hipError_t e = allow_lds(fn, lds, allowed[fn == kernel_for<D, OP, K, false>(g.pol) ? 0 : 1][g.pol & 3], s);
    if (e != hipSuccess) return e;
  }
  void* args[] = {const_cast<RCParams*>(&p)};
  return hipLaunchKernel(fn, dim3(g.grid), dim3(block_for(D, K, g.pol)), args, lds, s);
}

// Only the kernels kernel_compiled() names are instantiated (the host routes every other call onto
// one of them, nexr_internal.h); asking for another is an invalid launch, never a silent fallback.
#define NEXR_K_CASE(K, CALL) \
  case K:                    \
    if constexpr (kernel_compiled(D, OP, K)) return CALL; \
    break;

template <int D, int OP>
static hipError_t launch_op(const RCParams& p, int nSrcs, const Geometry& g, hipStream_t s) {
  switch (nSrcs) {
    NEXR_K_CASE(1, (launch_k<D, OP, 1>(p, g, s)))
    NEXR_K_CASE(2, (launch_k<D, OP, 2>(p, g, s)))
    NEXR_K_CASE(3, (launch_k<D, OP, 3>(p, g, s)))
    NEXR_K_CASE(4, (launch_k<D, OP, 4>(p, g, s)))
    NEXR_K_CASE(5, (launch_k<D, OP, 5>(p, g, s)))
    NEXR_K_CASE(6, (launch_k<D, OP, 6>(p, g, s)))
    NEXR_K_CASE(7, (launch_k<D, OP, 7>(p, g, s)))
    NEXR_K_CASE(8, (launch_k<D, OP, 8>(p, g, s)))
  }
  return hipErrorInvalidValue;
}

// Batches run the plain and non-temporal-load policies only (kBatchPolicies; a batch that would stream
// enough for non-temporal stores is run as single launches by the host), whose shapes never reserve LDS.
template <int D, int OP, int K, bool IsMin>
static const void* batch_kernel_for(int pol) {
  static_assert(lds_for(D, K, kPolPlain) == 0 && lds_for(D, K, kPolNtLoad) == 0, "batch shapes reserve no LDS");
  return pol == kPolNtLoad ? (const void*)&reduce_copy_batch_kernel<D, OP, K, kPolNtLoad, IsMin>
                           : (const void*)&reduce_copy_batch_kernel<D, OP, K, kPolPlain, IsMin>;
}

// Every work of a MinMax batch has the same isMin (reduceCopyBatch groups them so).
template <int D, int OP, int K>
static hipError_t launch_batch_k(const BatchParams& b, int pol, int grid, hipStream_t s) {
  if (pol != kPolPlain && pol != kPolNtLoad) return hipErrorInvalidValue;
  const void* fn = batch_kernel_for<D, OP, K, false>(pol);
  if constexpr (OP == nexrDevMinMax) {
    if ((b.w[0].redArg & 1) == 0) fn = batch_kernel_for<D, OP, K, true>(pol);
  }
  void* args[] = {const_cast<BatchParams*>(&b)};
  return hipLaunchKernel(fn, dim3(grid), dim3(block_for(D, K, pol)), args, 0, s);
}

template <int D, int OP>
static hipError_t launch_batch_op(const BatchParams& b, int nSrcs, int pol, int grid, hipStream_t s) {
  switch (nSrcs) {
    NEXR_K_CASE(1, (launch_batch_k<D, OP, 1>(b, pol, grid, s)))
    NEXR_K_CASE(2, (launch_batch_k<D, OP, 2>(b, pol, grid, s)))
    NEXR_K_CASE(3, (launch_batch_k<D, OP, 3>(b, pol, grid, s)))
    NEXR_K_CASE(4, (launch_batch_k<D, OP, 4>(b, pol, grid, s)))
    NEXR_K_CASE(5, (launch_batch_k<D, OP, 5>(b, pol, grid, s)))
    NEXR_K_CASE(6, (launch_batch_k<D, OP, 6>(b, pol, grid, s)))
    NEXR_K_CASE(7, (launch_batch_k<D, OP, 7>(b, pol, grid, s)))
    NEXR_K_CASE(8, (launch_batch_k<D, OP, 8>(b, pol, grid, s)))
  }
  return hipErrorInvalidValue;
}

#define NEXR_CAT2(a, b) a##b
#define NEXR_CAT(a, b) NEXR_CAT2(a, b)

hipError_t NEXR_CAT(launch_dt, NEXR_DT)(const RCParams& p, int op, int nSrcs, const Geometry& g, hipStream_t s) {
  constexpr int D = NEXR_DT;
  switch (op) {
    case nexrDevSum: return launch_op<D, nexrDevSum>(p, nSrcs, g, s);
    case nexrDevProd: return launch_op<D, nexrDevProd>(p, nSrcs, g, s);
    case nexrDevMinMax: return launch_op<D, nexrDevMinMax>(p, nSrcs, g, s);
    case nexrDevPreMulSum: return launch_op<D, nexrDevPreMulSum>(p, nSrcs, g, s);
    case nexrDevSumPostDiv:
      if constexpr (Ty<D>::kIsInt) return launch_op<D, nexrDevSumPostDiv>(p, nSrcs, g, s);
      break;
  }
  return hipErrorInvalidValue;
}

hipError_t NEXR_CAT(launch_batch_dt, NEXR_DT)(const BatchParams& b, int op, int nSrcs, int pol, int grid,
                                              hipStream_t s) {
  constexpr int D = NEXR_DT;
  switch (op) {
    case nexrDevSum: return launch_batch_op<D, nexrDevSum>(b, nSrcs, pol, grid, s);
    case nexrDevProd: return launch_batch_op<D, nexrDevProd>(b, nSrcs, pol, grid, s);
    case nexrDevMinMax: return launch_batch_op<D, nexrDevMinMax>(b, nSrcs, pol, grid, s);
    case nexrDevPreMulSum: return launch_batch_op<D, nexrDevPreMulSum>(b, nSrcs, pol, grid, s);
    case nexrDevSumPostDiv:
      if constexpr (Ty<D>::kIsInt) return launch_batch_op<D, nexrDevSumPostDiv>(b, nSrcs, pol, grid, s);
      break;
  }
  return hipErrorInvalidValue;
}

}  // namespace nexr
