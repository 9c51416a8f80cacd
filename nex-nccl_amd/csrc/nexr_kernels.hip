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
//   - all K source loads of a trip are issued before the first reduce step;
//   - cache policy by working-set size: non-temporal loads once a call streams more than
//     64 MiB, non-temporal loads AND stores beyond 512 MiB (2x the Infinity Cache) —
//     steady-state sweeps in tools/tune_kernel.hip / tools/hbm_ceiling.hip, DESIGN.md §Kernel;
//   - no LDS and no cross-lane traffic: every output element depends only on the same index of
//     the inputs, so the reference's warp-32 hunk layout (common_kernel.h:94-113) is irrelevant
//     to the result and is not reproduced.
// The element arithmetic keeps the reference's left-fold order (acc is the first operand,
// reduce_kernel.h:152-168) and rounds to T after every step.
#include "nexr_fold.hpp"

#ifndef NEXR_DT
#error "compile with -DNEXR_DT=<datatype>"
#endif

namespace nexr {

// One element through the same pack arithmetic (lanes other than 0 hold zeros and are dropped).
// Byte-wise copies: the ABI allows pointers that are not even element-aligned.
template <int D, int OP, int K, bool IsMin>
__device__ __forceinline__ void do_element(const char* const (&src)[K], char* const (&dst)[NEXR_MAX_DSTS], int nDsts,
                                           const Fold<D, OP, K, IsMin>& f, uint64_t i) {
  constexpr int esz = 16 / Ty<D>::EPP;
  u32x4 in[K];
#pragma unroll
  for (int s = 0; s < K; s++) {
    in[s] = (u32x4)0u;
    __builtin_memcpy(&in[s], src[s] + i * esz, esz);
  }
  u32x4 out = f.run(in);
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++)
    if (d < nDsts) __builtin_memcpy(dst[d] + i * esz, &out, esz);
}

// `bid`/`nblk`: this workgroup's index among the `nblk` workgroups working on `p` (the whole grid
// for a single launch; a slice of it for a batch launch).
template <int D, int OP, int K, int POL, bool IsMin, int U, int B, bool PM>
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
  const char* src[K];
#pragma unroll
  for (int s = 0; s < K; s++) src[s] = p.src[s];
  char* dst[NEXR_MAX_DSTS];
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++) dst[d] = p.dst[d];
  const int nDsts = p.nDsts;
  const uint64_t gid = bid * B + threadIdx.x;
  const uint64_t nthreads = nblk * B;

  // Edge elements before/after the packed body: fewer than 128/esz + 16/esz of them.
  const uint64_t bodyElts = p.nPacks * T::EPP;
  const uint64_t head = p.head;
  const uint64_t tail = p.nElts - head - bodyElts;
  if (gid < head + tail) {
    const uint64_t e = gid < head ? gid : head + bodyElts + (gid - head);
    do_element<D, OP, K, IsMin>(src, dst, nDsts, f, e);
  }

  // Packed body: base pointers advanced past the head edge. Pointers without the common 16-B phase
  // are read / written with unaligned 16-B accesses (ld16 / st16 assume only byte alignment).
#pragma unroll
  for (int s = 0; s < K; s++) src[s] += head * esz;
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++) dst[d] += head * esz;
  const uint64_t nPacks = p.nPacks;
  const uint64_t nFull = nPacks / (B * U);  // groups of B*U packs
  uint64_t g = bid;
  // Full groups: K*U 16-B loads in flight per lane, then the fold, then M*U stores. PM (pack-major)
  // issues the loads pack by pack (pack u of every source before pack u + 1 of any) and stores each
  // pack right after its fold, so pack 0 folds and leaves while pack 1's loads are still arriving;
  // otherwise source by source, and every pack is stored after the last fold.
  for (; g < nFull; g += nblk) {
    const uint64_t off = (g * (B * U) + threadIdx.x) * 16;
    u32x4 in[U][K];
    if constexpr (PM) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int s = 0; s < K; s++) in[u][s] = ld16<POL>(src[s] + off + u * B * 16);
#pragma unroll
      for (int u = 0; u < U; u++) {
        const u32x4 out = f.run(in[u]);
#pragma unroll
        for (int d = 0; d < NEXR_MAX_DSTS; d++)
          if (d < nDsts) st16<POL>(dst[d] + off + u * B * 16, out);
      }
    } else {
#pragma unroll
      for (int s = 0; s < K; s++)
#pragma unroll
        for (int u = 0; u < U; u++) in[u][s] = ld16<POL>(src[s] + off + u * B * 16);
      u32x4 out[U];
#pragma unroll
      for (int u = 0; u < U; u++) out[u] = f.run(in[u]);
#pragma unroll
      for (int d = 0; d < NEXR_MAX_DSTS; d++) {
        if (d < nDsts) {
#pragma unroll
          for (int u = 0; u < U; u++) st16<POL>(dst[d] + off + u * B * 16, out[u]);
        }
      }
    }
  }
  // Remaining packs (< B*U): one pack per thread.
  for (uint64_t j = nFull * (B * U) + gid; j < nPacks; j += nthreads) {
    u32x4 in[K];
#pragma unroll
    for (int s = 0; s < K; s++) in[s] = ld16<POL>(src[s] + j * 16);
    u32x4 out = f.run(in);
#pragma unroll
    for (int d = 0; d < NEXR_MAX_DSTS; d++)
      if (d < nDsts) st16<POL>(dst[d] + j * 16, out);
  }
}

template <int D, int OP, int K, int POL, int U, int B, bool PM = pack_major_for(D, K, POL)>
__device__ __forceinline__ void dispatch_minmax(const RCParams& p, uint64_t bid, uint64_t nblk) {
  if constexpr (OP == nexrDevMinMax) {
    if ((p.redArg & 1) == 0) body<D, OP, K, POL, true, U, B, PM>(p, bid, nblk);  // isMin = (arg&1)==0, reduce_kernel.h:64
    else body<D, OP, K, POL, false, U, B, PM>(p, bid, nblk);
  } else {
    body<D, OP, K, POL, false, U, B, PM>(p, bid, nblk);
  }
}

template <int D, int OP, int K, int POL, int U = unroll_for(D, K, POL), int B = block_for(D, K, POL),
          bool PM = pack_major_for(D, K, POL)>
__global__ __launch_bounds__(B) void reduce_copy_kernel(RCParams p) {
  dispatch_minmax<D, OP, K, POL, U, B, PM>(p, blockIdx.x, gridDim.x);
}

// Batch launch (the analogue of a kernel running a ncclDevWorkBatch: src/device/common.h:307-342):
// up to kMaxBatch independent reduce-copies with the same (datatype, op, K) in one launch; work i
// owns workgroups [start[i], start[i+1]). The work index is wave-uniform, so the descriptor is read
// straight from the kernel-argument segment with scalar loads.
template <int D, int OP, int K, int POL>
__global__ __launch_bounds__(block_for(D, K, POL)) void reduce_copy_batch_kernel(BatchParams b) {
  int i = 0;
  while (i + 1 < b.nWorks && blockIdx.x >= b.start[i + 1]) i++;
  dispatch_minmax<D, OP, K, POL, unroll_for(D, K, POL), block_for(D, K, POL)>(b.w[i], blockIdx.x - b.start[i],
                                                                                b.start[i + 1] - b.start[i]);
}

template <int D, int OP, int K>
static hipError_t launch_k(const RCParams& p, const Geometry& g, hipStream_t s) {
  const void* fn = g.pol == kPolNt       ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNt>
                   : g.pol == kPolNtLoad ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNtLoad>
                                         : (const void*)&reduce_copy_kernel<D, OP, K, kPolPlain>;
  void* args[] = {const_cast<RCParams*>(&p)};
  return hipLaunchKernel(fn, dim3(g.grid), dim3(block_for(D, K, g.pol)), args, 0, s);
}

template <int D, int OP>
static hipError_t launch_op(const RCParams& p, int nSrcs, const Geometry& g, hipStream_t s) {
  switch (nSrcs) {
    case 1: return launch_k<D, OP, 1>(p, g, s);
    case 2: return launch_k<D, OP, 2>(p, g, s);
    case 3: return launch_k<D, OP, 3>(p, g, s);
    case 4: return launch_k<D, OP, 4>(p, g, s);
    case 5: return launch_k<D, OP, 5>(p, g, s);
    case 6: return launch_k<D, OP, 6>(p, g, s);
    case 7: return launch_k<D, OP, 7>(p, g, s);
    case 8: return launch_k<D, OP, 8>(p, g, s);
  }
  return hipErrorInvalidValue;
}

template <int D, int OP, int K>
static hipError_t launch_batch_k(const BatchParams& b, int pol, int grid, hipStream_t s) {
  const void* fn = pol == kPolNt       ? (const void*)&reduce_copy_batch_kernel<D, OP, K, kPolNt>
                   : pol == kPolNtLoad ? (const void*)&reduce_copy_batch_kernel<D, OP, K, kPolNtLoad>
                                       : (const void*)&reduce_copy_batch_kernel<D, OP, K, kPolPlain>;
  void* args[] = {const_cast<BatchParams*>(&b)};
  return hipLaunchKernel(fn, dim3(grid), dim3(block_for(D, K, pol)), args, 0, s);
}

template <int D, int OP>
static hipError_t launch_batch_op(const BatchParams& b, int nSrcs, int pol, int grid, hipStream_t s) {
  switch (nSrcs) {
    case 1: return launch_batch_k<D, OP, 1>(b, pol, grid, s);
    case 2: return launch_batch_k<D, OP, 2>(b, pol, grid, s);
    case 3: return launch_batch_k<D, OP, 3>(b, pol, grid, s);
    case 4: return launch_batch_k<D, OP, 4>(b, pol, grid, s);
    case 5: return launch_batch_k<D, OP, 5>(b, pol, grid, s);
    case 6: return launch_batch_k<D, OP, 6>(b, pol, grid, s);
    case 7: return launch_batch_k<D, OP, 7>(b, pol, grid, s);
    case 8: return launch_batch_k<D, OP, 8>(b, pol, grid, s);
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

}  // namespace nexr

namespace nexr {
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
