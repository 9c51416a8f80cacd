// nexr_fold.hpp — the per-position fold of K loaded 16-byte packs (reduceCopyPacks' inner step,
// reference src/device/common_kernel.h:145-212, with applyPreOp / applyPostOp of
// src/device/reduce_kernel.h:498-539): shared by the reduce-copy kernel (nexr_kernels.hip) and the
// resident ring (nexr_resident.hip).
#pragma once
#include "nexr_types.hpp"

namespace nexr {

template <int D, int OP, int K, bool IsMin>
struct Fold {
  using T = Ty<D>;
  using V = typename T::V;
  V factor[K];  // PreMulSum scalars, broadcast
  int nPreOp;
  bool post, canon;
  uint64_t redArg;

  __device__ Fold(const RCParams& p) {
    nPreOp = p.nPreOp;
    post = (OP == nexrDevSumPostDiv) && p.postOp;
    redArg = p.redArg;
    // ncclFromFloat runs whenever any arithmetic step ran (K>=2, or a pre-op on src0).
    canon = (K >= 2) || (OP == nexrDevPreMulSum && p.nPreOp > 0);
    if constexpr (OP == nexrDevPreMulSum) {
#pragma unroll
      for (int s = 0; s < K; s++) factor[s] = T::splat(p.pre[s]);
    }
  }
  // One pre-op scalar for source 0 only (a Primitives' redOpArgs[0] with PreOpSrcs <= 1), without an
  // RCParams in memory: the resident ring's form.
  __device__ Fold(uint64_t pre0, int nPre, bool postOp, uint64_t arg) {
    nPreOp = nPre;
    post = (OP == nexrDevSumPostDiv) && postOp;
    redArg = arg;
    canon = (K >= 2) || (OP == nexrDevPreMulSum && nPre > 0);
    if constexpr (OP == nexrDevPreMulSum) {
#pragma unroll
      for (int s = 0; s < K; s++) factor[s] = T::splat(pre0);
    }
  }
  __device__ __forceinline__ V pre(V x, int s) const {
    if constexpr (OP == nexrDevPreMulSum) {
      if (s < nPreOp) return T::mul(x, factor[s]);  // Apply_PreOp<FuncPreMulSum> :498-518
    }
    return x;
  }
  // in[s] = the K loaded packs of one position
  __device__ __forceinline__ u32x4 run(const u32x4 (&in)[K]) const {
    if constexpr ((D == nexrInt8 || D == nexrUint8) && K >= 2 &&
                  (OP == nexrDevSum || OP == nexrDevProd || OP == nexrDevMinMax)) {
      using F = Fold8<OP, D == nexrInt8, IsMin>;  // two bytes per packed 16-bit instruction
      u16x8 ae, ao;
      F::split(in[0], ae, ao);
#pragma unroll
      for (int s = 1; s < K; s++) {
        u16x8 e, o;
        F::split(in[s], e, o);
        ae = F::step(ae, e);
        ao = F::step(ao, o);
      }
      return F::join(ae, ao);
    }
    V acc = pre(bc<V>(in[0]), 0);
#pragma unroll
    for (int s = 1; s < K; s++) acc = reduce_step<D, OP, IsMin>(acc, pre(bc<V>(in[s]), s));
    if constexpr (OP == nexrDevSumPostDiv) {
      if (post) acc = T::divide(acc, redArg);  // Apply_PostOp<FuncSumPostDiv> :520-539
    }
    if constexpr (T::kCanon) {  // float16 / bfloat16: NaN -> 0x7fff once, after the fold
      if (canon) acc = T::canon(acc);
    }
    return bc<u32x4>(acc);
  }
};

}  // namespace nexr
