// nexr_kernels.hip — the reduce-copy kernel for gfx950, compiled once per datatype with
// -DNEXR_DT=<nexrDataType_t value> (see Makefile) so the 10 objects build in parallel.
//
// What it computes is the reference's reduceCopy (src/device/common_kernel.h:269-349 →
// reduceCopyPacks :141-253) with the real per-type arithmetic of src/device/reduce_kernel.h
// (:238-539, SKIP_COMP at :432 removed). How it computes it is MI355X-first:
//   - one 16-B load per lane per source per pack (global_load_dwordx4), 64-lane waves,
//     4 waves per workgroup; each workgroup owns one 16 KiB trip of every buffer (U = 4 packs
//     per lane, "one-shot" grid of nPacks/(256*4) workgroups; a grid-stride loop only beyond
//     2^24 workgroups), so every lane has 4*K independent loads in flight;
//   - all K source loads of a trip are issued before the first reduce step;
//   - cache policy by working-set size: non-temporal loads once a call streams more than
//     64 MiB, non-temporal loads AND stores beyond 512 MiB (2x the Infinity Cache) —
//     steady-state sweeps in tools/tune_kernel.hip / tools/hbm_ceiling.hip, DESIGN.md §Kernel;
//   - no LDS and no cross-lane traffic: every output element depends only on the same index of
//     the inputs, so the reference's warp-32 hunk layout (common_kernel.h:94-113) is irrelevant
//     to the result and is not reproduced.
// The element arithmetic keeps the reference's left-fold order (acc is the first operand,
// reduce_kernel.h:152-168) and rounds to T after every step.
#include "nexr_internal.h"

#ifndef NEXR_DT
#error "compile with -DNEXR_DT=<datatype>"
#endif

// Bit-exact float semantics need separate rounding of every multiply and add (a PreMulSum
// step must not become an fma): the Makefile passes -ffp-contract=off as well.
#pragma clang fp contract(off)

namespace nexr {

typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));
typedef int8_t i8x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef int16_t i16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));
typedef int32_t i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));
typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

template <typename To, typename From>
__device__ __forceinline__ To bc(From x) {
  static_assert(sizeof(To) == sizeof(From), "bitcast size");
  return __builtin_bit_cast(To, x);
}

// ---------------------------------------------------------------------------------------------
// Per-datatype 16-byte pack arithmetic. V is the pack as the op sees it.
//   add/mul  : ncclAdd / ncclMultiply          (reduce_kernel.h:238-248, :317-368)
//   min/max  : isMin ? (v<c?v:c) : (v>c?v:c)   (reduce_kernel.h:455-478), c = acc, v = new operand
//   splat    : ncclDecodeScalar<T>(raw)        (reduce_kernel.h:218-236, :317-345) broadcast
//   canon    : float16 only — ncclFromFloat maps every NaN to 0x7fff (CUDA __float2half host path)
//   divide   : FuncSumPostDiv::divide          (reduce_kernel.h:83-97), integers only
// ---------------------------------------------------------------------------------------------
template <int D> struct Ty;

// Integer packs: sum/prod in the unsigned representation (generate.py:128-136 folds signed
// sum/prod onto the unsigned kernel; wraps modulo 2^bits), min/max at the signedness of the
// user's datatype.
template <typename UV, typename SV, typename CV, typename US, typename SS, bool Signed, int N>
struct IntTy {
  using V = UV;
  static constexpr int EPP = N;
  static constexpr bool kIsInt = true;
  __device__ static V add(V a, V b) { return a + b; }
  __device__ static V mul(V a, V b) { return a * b; }
  __device__ static V vmin(V c, V v) {
    if constexpr (Signed) return bc<V>(__builtin_elementwise_min(bc<SV>(c), bc<SV>(v)));
    else return __builtin_elementwise_min(c, v);
  }
  __device__ static V vmax(V c, V v) {
    if constexpr (Signed) return bc<V>(__builtin_elementwise_max(bc<SV>(c), bc<SV>(v)));
    else return __builtin_elementwise_max(c, v);
  }
  __device__ static V splat(uint64_t raw) { return (V)((US)raw); }
  __device__ static V canon(V x) { return x; }
  // divisor = redArg>>1 (0 -> 1), isSigned = redArg&1 (reduce_kernel.h:79-82); the signed path
  // divides at the signed type after C++ promotion (8-bit operands promote to int), and the
  // one quotient C leaves undefined, MIN / -1, wraps to MIN.
  __device__ static V divide(V x, uint64_t redArg) {
    uint32_t divisor = (uint32_t)(redArg >> 1);
    if (divisor == 0) divisor = 1;
    const bool isSigned = (redArg & 1) != 0;
    V out;
#pragma unroll
    for (int e = 0; e < N; e++) {
      US u = x[e];
      if (!isSigned) {
        if constexpr (sizeof(US) < 4) out[e] = (US)((uint32_t)u / divisor);
        else if constexpr (sizeof(US) == 4) out[e] = (US)(u / divisor);
        else out[e] = (US)(u / (uint64_t)divisor);
      } else {
        SS s = (SS)u;
        SS d = (SS)divisor;
        if constexpr (sizeof(SS) < 4) {
          out[e] = (US)(SS)((int32_t)s / (int32_t)d);
        } else {
          SS q = (d == (SS)-1) ? (SS)(0 - (US)s) : (SS)(s / d);
          out[e] = (US)q;
        }
      }
    }
    return out;
  }
};

template <> struct Ty<nexrInt8> : IntTy<u8x16, i8x16, i8x16, uint8_t, int8_t, true, 16> {};
template <> struct Ty<nexrUint8> : IntTy<u8x16, i8x16, i8x16, uint8_t, int8_t, false, 16> {};
template <> struct Ty<nexrInt32> : IntTy<u32x4, i32x4, i32x4, uint32_t, int32_t, true, 4> {};
template <> struct Ty<nexrUint32> : IntTy<u32x4, i32x4, i32x4, uint32_t, int32_t, false, 4> {};
template <> struct Ty<nexrInt64> : IntTy<u64x2, i64x2, i64x2, uint64_t, int64_t, true, 2> {};
template <> struct Ty<nexrUint64> : IntTy<u64x2, i64x2, i64x2, uint64_t, int64_t, false, 2> {};

template <> struct Ty<nexrFloat32> {
  using V = f32x4;
  static constexpr int EPP = 4;
  static constexpr bool kIsInt = false;
  __device__ static V add(V a, V b) { return a + b; }
  __device__ static V mul(V a, V b) { return a * b; }
  __device__ static V vmin(V c, V v) { return v < c ? v : c; }
  __device__ static V vmax(V c, V v) { return v > c ? v : c; }
  __device__ static V splat(uint64_t raw) { return (V)(bc<float>((uint32_t)raw)); }
  __device__ static V canon(V x) { return x; }
  __device__ static V divide(V x, uint64_t) { return x; }
};

template <> struct Ty<nexrFloat64> {
  using V = f64x2;
  static constexpr int EPP = 2;
  static constexpr bool kIsInt = false;
  __device__ static V add(V a, V b) { return a + b; }
  __device__ static V mul(V a, V b) { return a * b; }
  __device__ static V vmin(V c, V v) { return v < c ? v : c; }
  __device__ static V vmax(V c, V v) { return v > c ? v : c; }
  __device__ static V splat(uint64_t raw) { return (V)(bc<double>(raw)); }
  __device__ static V canon(V x) { return x; }
  __device__ static V divide(V x, uint64_t) { return x; }
};

// float16: the reference computes half(float(a) op float(b)) with RNE (reduce_kernel.h:329-337).
// A native f16 add/mul is the same value: the f32 result of two halves rounded once more to
// half is innocuous double rounding (24 >= 2*11+2), and the f32 product of two halves is exact.
// Only NaN differs (hardware keeps a payload, the reference writes 0x7fff): canon() fixes it
// once at the end, which is equivalent because a NaN accumulator stays NaN through every op.
template <> struct Ty<nexrFloat16> {
  using V = f16x8;
  static constexpr int EPP = 8;
  static constexpr bool kIsInt = false;
  __device__ static V add(V a, V b) { return a + b; }
  __device__ static V mul(V a, V b) { return a * b; }
  __device__ static V vmin(V c, V v) { return v < c ? v : c; }
  __device__ static V vmax(V c, V v) { return v > c ? v : c; }
  __device__ static V splat(uint64_t raw) { return (V)(bc<_Float16>((uint16_t)raw)); }
  __device__ static V canon(V x) {
    i16x8 isnan = x != x;
    return bc<V>(isnan ? (u16x8)(uint16_t)0x7fff : bc<u16x8>(x));
  }
  __device__ static V divide(V x, uint64_t) { return x; }
};

// bfloat16: computed in f32 and rounded back to bf16 after every step with round-to-nearest-even,
// every NaN to 0x7fff (CUDA __float2bfloat16_rn host path, reduce_kernel.h:352-367).
template <> struct Ty<nexrBfloat16> {
  using V = u16x8;
  static constexpr int EPP = 8;
  static constexpr bool kIsInt = false;
  __device__ static f32x8 widen(V x) { return bc<f32x8>(__builtin_convertvector(x, u32x8) << 16); }
  __device__ static V narrow(f32x8 f) {
    u32x8 u = bc<u32x8>(f);
    u32x8 r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    i32x8 isnan = (u & 0x7fffffffu) > 0x7f800000u;
    r = isnan ? (u32x8)0x7fffu : r;
    return __builtin_convertvector(r, V);
  }
  __device__ static V add(V a, V b) { return narrow(widen(a) + widen(b)); }
  __device__ static V mul(V a, V b) { return narrow(widen(a) * widen(b)); }
  __device__ static V vmin(V c, V v) {
    f32x8 fc = widen(c), fv = widen(v);
    return narrow(fv < fc ? fv : fc);
  }
  __device__ static V vmax(V c, V v) {
    f32x8 fc = widen(c), fv = widen(v);
    return narrow(fv > fc ? fv : fc);
  }
  __device__ static V splat(uint64_t raw) { return (V)((uint16_t)raw); }
  __device__ static V canon(V x) { return x; }
  __device__ static V divide(V x, uint64_t) { return x; }
};

// ---------------------------------------------------------------------------------------------
// Memory access: explicit global (address_space 1) pointers so every access is a global_load /
// global_store with a 64-bit VGPR address (never flat, never via scratch).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

// Cache policy POL: bit 0 = non-temporal loads, bit 1 = non-temporal stores.
enum { kPolPlain = 0, kPolNtLoad = 1, kPolNtStore = 2, kPolNt = 3 };
template <int POL>
__device__ __forceinline__ u32x4 ld16(const char* p) {
  g_cu32x4* q = (g_cu32x4*)(p);
  if constexpr (POL & kPolNtLoad) return __builtin_nontemporal_load(q);
  else return *q;
}
template <int POL>
__device__ __forceinline__ void st16(char* p, u32x4 v) {
  g_u32x4* q = (g_u32x4*)(p);
  if constexpr (POL & kPolNtStore) __builtin_nontemporal_store(v, q);
  else *q = v;
}

// ---------------------------------------------------------------------------------------------
// The fold (reduceCopyPacks :145-212): acc = pre0(src0); acc = red(acc, pre_s(src_s)); post.
// ---------------------------------------------------------------------------------------------
template <int D, int OP, bool IsMin>
__device__ __forceinline__ typename Ty<D>::V reduce_step(typename Ty<D>::V acc, typename Ty<D>::V v) {
  using T = Ty<D>;
  if constexpr (OP == nexrDevProd) return T::mul(acc, v);
  else if constexpr (OP == nexrDevMinMax) return IsMin ? T::vmin(acc, v) : T::vmax(acc, v);
  else return T::add(acc, v);  // Sum, PreMulSum, SumPostDiv all reduce with ncclAdd (:437-496)
}

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
  __device__ __forceinline__ V pre(V x, int s) const {
    if constexpr (OP == nexrDevPreMulSum) {
      if (s < nPreOp) return T::mul(x, factor[s]);  // Apply_PreOp<FuncPreMulSum> :498-518
    }
    return x;
  }
  // in[s] = the K loaded packs of one position
  __device__ __forceinline__ u32x4 run(const u32x4 (&in)[K]) const {
    V acc = pre(bc<V>(in[0]), 0);
#pragma unroll
    for (int s = 1; s < K; s++) acc = reduce_step<D, OP, IsMin>(acc, pre(bc<V>(in[s]), s));
    if constexpr (OP == nexrDevSumPostDiv) {
      if (post) acc = T::divide(acc, redArg);  // Apply_PostOp<FuncSumPostDiv> :520-539
    }
    if constexpr (D == nexrFloat16) {
      if (canon) acc = T::canon(acc);
    }
    return bc<u32x4>(acc);
  }
};

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

template <int D, int OP, int K, int POL, bool IsMin, int U, int B>
__device__ __forceinline__ void body(const RCParams& p) {
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
  const uint64_t gid = (uint64_t)blockIdx.x * B + threadIdx.x;
  const uint64_t nthreads = (uint64_t)gridDim.x * B;

  if (p.generic) {  // pointers share no 16-B phase: every element on the scalar path
    for (uint64_t i = gid; i < p.nElts; i += nthreads) do_element<D, OP, K, IsMin>(src, dst, nDsts, f, i);
    return;
  }
  // Edge elements before/after the aligned body: at most 2*(16/esz - 1) of them.
  const uint64_t bodyElts = p.nPacks * T::EPP;
  const uint64_t head = p.head;
  const uint64_t tail = p.nElts - head - bodyElts;
  if (gid < head + tail) {
    const uint64_t e = gid < head ? gid : head + bodyElts + (gid - head);
    do_element<D, OP, K, IsMin>(src, dst, nDsts, f, e);
  }

  // Aligned body: base pointers advanced past the head edge.
#pragma unroll
  for (int s = 0; s < K; s++) src[s] += head * esz;
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++) dst[d] += head * esz;
  const uint64_t nPacks = p.nPacks;
  const uint64_t nFull = nPacks / (B * U);  // groups of B*U packs
  uint64_t g = blockIdx.x;
  // Full groups: K*U 16-B loads in flight per lane, then the fold, then M*U stores.
  for (; g < nFull; g += gridDim.x) {
    const uint64_t off = (g * (B * U) + threadIdx.x) * 16;
    u32x4 in[U][K];
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

template <int D, int OP, int K, int POL, int U = unroll_for(K), int B = kBlock>
__global__ __launch_bounds__(B) void reduce_copy_kernel(RCParams p) {
  if constexpr (OP == nexrDevMinMax) {
    if ((p.redArg & 1) == 0) body<D, OP, K, POL, true, U, B>(p);  // isMin = (arg&1)==0, reduce_kernel.h:64
    else body<D, OP, K, POL, false, U, B>(p);
  } else {
    body<D, OP, K, POL, false, U, B>(p);
  }
}

template <int D, int OP, int K>
static hipError_t launch_k(const RCParams& p, const Geometry& g, hipStream_t s) {
  const void* fn = g.pol == kPolNt       ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNt>
                   : g.pol == kPolNtLoad ? (const void*)&reduce_copy_kernel<D, OP, K, kPolNtLoad>
                                         : (const void*)&reduce_copy_kernel<D, OP, K, kPolPlain>;
  void* args[] = {const_cast<RCParams*>(&p)};
  return hipLaunchKernel(fn, dim3(g.grid), dim3(kBlock), args, 0, s);
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
