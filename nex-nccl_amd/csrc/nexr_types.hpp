// nexr_types.hpp — device-side building blocks shared by the reduce-copy kernels
// (nexr_kernels.hip: SIMPLE-protocol packs, nexr_ll.hip: LL-protocol lines): the per-datatype
// 16-byte pack arithmetic (reference src/device/reduce_kernel.h:238-539) and the memory-access
// helpers. Included by exactly one .hip translation unit per object.
#pragma once
#include "nexr_internal.h"

// Bit-exact float semantics need separate rounding of every multiply and add (a PreMulSum
// step must not become an fma): the Makefile passes -ffp-contract=off as well.
#pragma clang fp contract(off)

namespace nexr {

typedef uint8_t u8x16 __attribute__((ext_vector_type(16)));
typedef int8_t i8x16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef int16_t i16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
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
//   canon    : float16 / bfloat16 (kCanon) — ncclFromFloat maps every NaN to 0x7fff (CUDA
//              __float2half / __float2bfloat16_rn host path), applied once after the fold
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
  static constexpr bool kCanon = false;
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
  static constexpr bool kCanon = false;
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
  static constexpr bool kCanon = false;
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
  static constexpr bool kCanon = true;
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
// every NaN to 0x7fff (CUDA __float2bfloat16_rn host path, reduce_kernel.h:352-367). The rounding is
// gfx950's v_cvt_pk_bf16_f32 (RNE, two elements per instruction; f32 denormals are kept, so bf16
// subnormals round as IEEE says). It keeps a NaN's payload where the reference writes 0x7fff: canon()
// fixes that once after the fold, which gives the same bytes because a NaN accumulator stays NaN
// through every op (add, mul, and the ternary min/max, which keeps the accumulator when either side is
// NaN and drops a NaN operand whatever its bits). Round 5's integer RNE with a NaN select after every
// step cost 4 VALU per element per step.
template <> struct Ty<nexrBfloat16> {
  using V = u16x8;
  static constexpr int EPP = 8;
  static constexpr bool kIsInt = false;
  static constexpr bool kCanon = true;
  __device__ static f32x8 widen(V x) { return bc<f32x8>(__builtin_convertvector(x, u32x8) << 16); }
  __device__ static V narrow(f32x8 f) { return bc<V>(__builtin_convertvector(f, bf16x8)); }
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
  __device__ static V canon(V x) {
    const i16x8 isnan = (x & (uint16_t)0x7fff) > (uint16_t)0x7f80;
    return isnan ? (V)(uint16_t)0x7fff : x;
  }
  __device__ static V divide(V x, uint64_t) { return x; }
};

// ---------------------------------------------------------------------------------------------
// Memory access: explicit global (address_space 1) pointers so every access is a global_load /
// global_store with a 64-bit VGPR address (never flat, never via scratch).
// ---------------------------------------------------------------------------------------------
typedef __attribute__((address_space(1))) const u32x4 g_cu32x4;
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
// The reduce-copy's 16-B accesses assume byte alignment only: for 16-B aligned addresses the
// instruction is the same global_load/store_dwordx4 (identical ISA), and for the rest gfx950 runs the
// unaligned dwordx4 itself, at near the aligned rate (tools/misalign_rate.py).
typedef u32x4 __attribute__((aligned(1))) u32x4_a1;
typedef __attribute__((address_space(1))) const u32x4_a1 g_cu32x4_a1;
typedef __attribute__((address_space(1))) u32x4_a1 g_u32x4_a1;

// Cache policy POL: bit 0 = non-temporal loads, bit 1 = non-temporal stores.
enum { kPolPlain = 0, kPolNtLoad = 1, kPolNtStore = 2, kPolNt = 3 };
template <int POL>
__device__ __forceinline__ u32x4 ld16(const char* p) {
  g_cu32x4_a1* q = (g_cu32x4_a1*)(p);
  if constexpr (POL & kPolNtLoad) return __builtin_nontemporal_load(q);
  else return *q;
}
template <int POL>
__device__ __forceinline__ void st16(char* p, u32x4 v) {
  g_u32x4_a1* q = (g_u32x4_a1*)(p);
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

// 8-bit packs, two bytes per 16-bit lane, so that one packed 16-bit instruction
// (v_pk_{add,mul_lo}_u16, v_pk_{min,max}_{i16,u16}) folds two bytes; the fold stays in this form
// across all K sources and is packed back once. Bit-identical to the byte-wise fold:
//   Sum/Prod: even bytes in the LOW byte of each lane with the odd byte above it as don't-care, odd
//     bytes shifted down: the low byte of a 16-bit sum or product depends only on the operands' low
//     bytes, which is ncclAdd / ncclMultiply on the unsigned byte (wrap mod 2^8).
//   Min/Max: every byte in the HIGH byte of a lane over a zero low byte: 16-bit order (signed for
//     int8, unsigned for uint8) is then exactly the byte's order, with no sign extension.
template <int OP, bool Signed, bool IsMin>
struct Fold8 {
  static constexpr bool kHigh = OP == nexrDevMinMax;
  __device__ static __forceinline__ void split(u32x4 x, u16x8& ev, u16x8& od) {
    const u16x8 h = bc<u16x8>(x);
    if constexpr (kHigh) {
      // Min/Max fold each byte in the HIGH half of a 16-bit lane. The odd bytes already sit there;
      // the even byte below them needs no masking: a 16-bit compare is decided by the high byte
      // whenever the high bytes differ, and when they are equal either operand carries the same high
      // byte, so the high byte of min/max(a, b) is min/max of the high bytes whatever the low bytes
      // hold (signed or unsigned). Only the high bytes reach the result (join).
      ev = h << 8;
      od = h;
    } else {
      ev = h;
      od = h >> 8;
    }
  }
  __device__ static __forceinline__ u16x8 step(u16x8 c, u16x8 v) {
    if constexpr (OP == nexrDevProd) {
      return c * v;
    } else if constexpr (OP == nexrDevMinMax && Signed) {
      return bc<u16x8>(IsMin ? __builtin_elementwise_min(bc<i16x8>(c), bc<i16x8>(v))
                             : __builtin_elementwise_max(bc<i16x8>(c), bc<i16x8>(v)));
    } else if constexpr (OP == nexrDevMinMax) {
      return IsMin ? __builtin_elementwise_min(c, v) : __builtin_elementwise_max(c, v);
    } else {
      return c + v;
    }
  }
  // result byte 2i from the even lane i, byte 2i+1 from the odd lane i (v_perm_b32: bytes 0-3 select
  // from the second operand, 4-7 from the first)
  __device__ static __forceinline__ u32x4 join(u16x8 ev, u16x8 od) {
    const u32x4 e = bc<u32x4>(ev), o = bc<u32x4>(od);
    constexpr uint32_t sel = kHigh ? 0x07030501u : 0x06020400u;
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; i++) r[i] = __builtin_amdgcn_perm(o[i], e[i], sel);
    return r;
  }
};

}  // namespace nexr
