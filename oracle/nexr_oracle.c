/*
 * nexr_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded (or pthread-sliced) CPU restatement of the reference reduce-copy,
 * used as the CHECKER for the HIP path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product (nex-nccl_amd/libnexr.so) never links or calls it.
 *
 * What it restates (reference = MJChku/nex-nccl, paths relative to /root/reference):
 *   - the element loop of reduceCopyPacks, src/device/common_kernel.h:141-237:
 *       acc = ld(src0)            (+ applyPreOp when 0 < PreOpSrcs, :145-157)
 *       for s in 1..nSrcs-1: acc = applyReduce(fn, acc, preOp_s?(ld(src_s)))   (:160-206)
 *       if postOp: acc = applyPostOp(fn, acc)                                   (:208-212)
 *       st(dst_d, acc) for every d                                               (:214-237)
 *     with the pack-level ops reduced to their per-element definition
 *     (Apply_Reduce, src/device/reduce_kernel.h:152-168: acc is the FIRST argument);
 *   - the scalar arithmetic of src/device/reduce_kernel.h with SKIP_COMP (:432) removed:
 *       ncclReduceScalar :434-496, ncclAdd/ncclMultiply :238-248 (generic), :329-337 (half),
 *       :357-367 (bfloat16), ncclDecodeScalar :218-236, :317-321, :340-345,
 *       FuncMinMax :59-65 (isMin = (arg&1)==0), FuncSumPostDiv::divide :74-98,
 *       Apply_PreOp<FuncPreMulSum> :498-518, Apply_PostOp<FuncSumPostDiv> :520-539;
 *   - datatype folding of src/device/generate.py:128-136 (signed sum/prod run on the unsigned
 *     type; min/max are compared at the user's signedness — upstream-NCCL semantics, which the
 *     fork's xormask-free FuncMinMax reproduces when instantiated at the signed type; see
 *     DESIGN.md "Deviations");
 *   - hostToDevRedOp, src/enqueue.cc:2185-2278 (built-in ops).
 *
 * Third-party arithmetic (not in /root/reference): the half/bfloat16 conversions are CUDA 12.8's
 * host paths of __half2float/__float2half and __bfloat162float/__float2bfloat16_rn
 * (cuda_fp16.hpp __internal_float2half, cuda_bf16.hpp __internal_float2bfloat16): IEEE-754
 * round-to-nearest-even, overflow to infinity, subnormals kept, every NaN -> 0x7fff.
 * They are restated below from that published algorithm.
 *
 * Parity pinning: see DESIGN.md §Oracle. The reference cannot be compiled here (its headers need
 * CUDA's <nv/target>, absent from the image, and the absent NEX runtime), so this file is pinned
 * by SURVEY.md §8(c)'s known answers from the compiled reference and by independent IEEE
 * implementations (tests/golden/make_golden.py: numpy float16, torch bfloat16).
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>

/* enum values identical to include/nexr.h (= ncclDataType_t / ncclDevRedOp_t) */
enum { DT_I8 = 0, DT_U8 = 1, DT_I32 = 2, DT_U32 = 3, DT_I64 = 4, DT_U64 = 5, DT_F16 = 6, DT_F32 = 7,
       DT_F64 = 8, DT_BF16 = 9, DT_F8E4M3 = 10, DT_F8E5M2 = 11, DT_NUM = 12 };
enum { OP_SUM = 0, OP_PROD = 1, OP_MINMAX = 2, OP_PREMULSUM = 3, OP_SUMPOSTDIV = 4, OP_NUM = 5 };
enum { R_OK = 0, R_INVALID = 4 };

size_t oracle_type_size(int dt) {
  switch (dt) {
    case DT_I8: case DT_U8: case DT_F8E4M3: case DT_F8E5M2: return 1;
    case DT_F16: case DT_BF16: return 2;
    case DT_I32: case DT_U32: case DT_F32: return 4;
    case DT_I64: case DT_U64: case DT_F64: return 8;
  }
  return 0;
}

/* ---- bit casts --------------------------------------------------------------------------- */
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline double u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

/* ---- half <-> float (CUDA host path restated) -------------------------------------------- */
float oracle_half_to_float(uint16_t h) {
  uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu;
  uint32_t man = h & 0x3ffu;
  if (exp == 0x1f) return u2f(sign | 0x7f800000u | (man << 13)); /* inf / NaN */
  if (exp == 0) {
    if (man == 0) return u2f(sign);
    /* subnormal: value = man * 2^-24, exact in float */
    float v = (float)man * u2f(0x33800000u); /* 2^-24 */
    return sign ? -v : v;
  }
  return u2f(sign | ((exp + 112u) << 23) | (man << 13));
}

uint16_t oracle_float_to_half(float f) {
  uint32_t x = f2u(f);
  uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t a = x & 0x7fffffffu;
  if (a > 0x7f800000u) return 0x7fffu;                       /* NaN -> canonical 0x7fff */
  if (a == 0x7f800000u) return (uint16_t)(sign | 0x7c00u);   /* inf */
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);   /* >= 65520 rounds to inf */
  if (a < 0x33000001u) return (uint16_t)sign;                /* <= 2^-25 rounds to 0 */
  uint32_t mant, shift;
  if (a >= 0x38800000u) { mant = a - 0x38000000u; shift = 13; }            /* normal half */
  else { mant = (a & 0x7fffffu) | 0x800000u; shift = 126u - (a >> 23); }    /* subnormal */
  uint32_t q = mant >> shift;
  uint32_t rem = mant & ((1u << shift) - 1u);
  uint32_t halfway = 1u << (shift - 1u);
  if (rem > halfway || (rem == halfway && (q & 1u))) q++;
  return (uint16_t)(sign | q);
}

/* ---- bfloat16 <-> float ------------------------------------------------------------------ */
float oracle_bf16_to_float(uint16_t b) { return u2f((uint32_t)b << 16); }
uint16_t oracle_float_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fffu;
  uint32_t rem = u << 16, q = u >> 16;
  if (rem > 0x80000000u || (rem == 0x80000000u && (q & 1u))) q++;
  return (uint16_t)q;
}

/* ---- one reduce step per type: ncclReduceScalar(fn, current, value) ---------------------- */
typedef struct {
  int op;
  int isMin;              /* FuncMinMax: (arg & 1) == 0 */
  uint32_t divisor;       /* FuncSumPostDiv: arg >> 1, 0 -> 1 */
  int isSigned;           /* FuncSumPostDiv: arg & 1 */
} Fn;

static inline void make_fn(Fn* fn, int op, uint64_t arg) {
  fn->op = op;
  fn->isMin = (arg & 1) == 0;
  fn->divisor = (uint32_t)(arg >> 1);
  if (fn->divisor == 0) fn->divisor = 1;
  fn->isSigned = (arg & 1) != 0;
}

/* ---- reduction semantics (include/nexr.h nexrSemantics_t), process-wide like the library's ------
 * 0 nccl:    real arithmetic, min/max at the user's signedness (the default);
 * 1 fork:    real arithmetic under the fork's dispatch — signed min/max run on the unsigned kernel
 *            (generate.py:128-136), whose FuncMinMax ignores the sign xormask (reduce_kernel.h:59-65);
 * 2 shipped: SKIP_COMP (reduce_kernel.h:432) — ncclReduceScalar returns its first operand, the
 *            PreMulSum pre-op and SumPostDiv post-op return their input (:434-539). */
static int g_semantics = 0;
int oracle_set_semantics(int s) {
  if (s < 0 || s > 2) return 4;
  g_semantics = s;
  return 0;
}
int oracle_get_semantics(void) { return g_semantics; }
static int fork_dispatch_type(int dt, int op) {
  if (op != 2 /* OP_MINMAX */) return dt;
  return dt == 0 ? 1 : dt == 2 ? 3 : dt == 4 ? 5 : dt; /* i8 -> u8, i32 -> u32, i64 -> u64 */
}
/* A SIMPLE reduceCopy call as the semantics run it: shipped = a K = 1 copy of srcs[0]. */
static void semantics_shape(int* dt, int* op, int* nSrcs, int* nPreOp, int* postOp) {
  if (g_semantics == 1) *dt = fork_dispatch_type(*dt, *op);
  if (g_semantics == 2) { *op = 0; *nSrcs = 1; *nPreOp = 0; *postOp = 0; }
}

#define MINMAX(isMin, c, v) ((isMin) ? ((v) < (c) ? (v) : (c)) : ((v) > (c) ? (v) : (c)))

/* unsigned-representation integer ops (sum/prod wrap), signed compare where the type is signed */
#define INT_REDUCE(UT, ST, SIGNED)                                                          \
  static inline UT red_##UT##_##SIGNED(const Fn* fn, UT c, UT v) {                          \
    switch (fn->op) {                                                                       \
      case OP_PROD: return (UT)(c * v);                                                     \
      case OP_MINMAX:                                                                       \
        if (SIGNED) { ST sc = (ST)c, sv = (ST)v; return (UT)MINMAX(fn->isMin, sc, sv); }     \
        return MINMAX(fn->isMin, c, v);                                                     \
      default: return (UT)(c + v); /* Sum, PreMulSum, SumPostDiv */                         \
    }                                                                                       \
  }
INT_REDUCE(uint8_t, int8_t, 0)
INT_REDUCE(uint8_t, int8_t, 1)
INT_REDUCE(uint32_t, int32_t, 0)
INT_REDUCE(uint32_t, int32_t, 1)
INT_REDUCE(uint64_t, int64_t, 0)
INT_REDUCE(uint64_t, int64_t, 1)

/* FuncSumPostDiv::divide (reduce_kernel.h:83-97) */
static inline uint8_t div_u8(const Fn* fn, uint8_t u) {
  if (!fn->isSigned) return (uint8_t)((uint32_t)u / fn->divisor);
  int8_t s = (int8_t)u, d = (int8_t)fn->divisor; /* d != 0: rejected by the callers */
  return (uint8_t)(int8_t)((int)s / (int)d);
}
static inline uint32_t div_u32(const Fn* fn, uint32_t u) {
  if (!fn->isSigned) return u / fn->divisor;
  int32_t s = (int32_t)u, d = (int32_t)fn->divisor;
  if (d == -1) return (uint32_t)0 - u; /* MIN/-1 is undefined in C: wraps, as the GPU does */
  return (uint32_t)(s / d);
}
static inline uint64_t div_u64(const Fn* fn, uint64_t u) {
  if (!fn->isSigned) return u / (uint64_t)fn->divisor;
  int64_t s = (int64_t)u, d = (int64_t)fn->divisor;
  return (uint64_t)(s / d);
}

static inline float red_f32(const Fn* fn, float c, float v) {
  switch (fn->op) {
    case OP_PROD: return c * v;
    case OP_MINMAX: return MINMAX(fn->isMin, c, v);
    default: return c + v;
  }
}
static inline double red_f64(const Fn* fn, double c, double v) {
  switch (fn->op) {
    case OP_PROD: return c * v;
    case OP_MINMAX: return MINMAX(fn->isMin, c, v);
    default: return c + v;
  }
}
/* half / bfloat16: compute in float, convert back after every step (reduce_kernel.h:329-367,
 * :470-473) */
static inline uint16_t red_f16(const Fn* fn, uint16_t c, uint16_t v) {
  float fc = oracle_half_to_float(c), fv = oracle_half_to_float(v), r;
  switch (fn->op) {
    case OP_PROD: r = fc * fv; break;
    case OP_MINMAX: r = MINMAX(fn->isMin, fc, fv); break;
    default: r = fc + fv;
  }
  return oracle_float_to_half(r);
}
static inline uint16_t red_bf16(const Fn* fn, uint16_t c, uint16_t v) {
  float fc = oracle_bf16_to_float(c), fv = oracle_bf16_to_float(v), r;
  switch (fn->op) {
    case OP_PROD: r = fc * fv; break;
    case OP_MINMAX: r = MINMAX(fn->isMin, fc, fv); break;
    default: r = fc + fv;
  }
  return oracle_float_to_bf16(r);
}

/* ---- the element loop --------------------------------------------------------------------- */
typedef struct {
  int nSrcs, nDsts, dt, op, nPreOp, postOp;
  const void* const* srcs;
  void* const* dsts;
  const uint64_t* pre;
  uint64_t arg;
  size_t begin, end;
} Job;

/* LOOP(T, LOAD-REDUCE-...): shared skeleton of common_kernel.h:141-237 per element */
#define ELEMENT_LOOP(T, PREOP, REDUCE, POSTOP)                                               \
  do {                                                                                       \
    const T* const* S = (const T* const*)j->srcs;                                            \
    T* const* D = (T* const*)j->dsts;                                                        \
    for (size_t i = j->begin; i < j->end; i++) {                                             \
      T acc = S[0][i];                                                                       \
      if (isPreMul && 0 < j->nPreOp) acc = PREOP(acc, 0);                                    \
      for (int s = 1; s < j->nSrcs; s++) {                                                   \
        T v = S[s][i];                                                                       \
        if (isPreMul && s < j->nPreOp) v = PREOP(v, s);                                      \
        acc = REDUCE(&fn, acc, v);                                                           \
      }                                                                                      \
      if (isPostDiv && j->postOp) acc = POSTOP(&fn, acc);                                    \
      for (int d = 0; d < j->nDsts; d++) D[d][i] = acc;                                      \
    }                                                                                        \
  } while (0)

#define NOPOST(fn, x) (x)

static void run_job(const Job* j) {
  Fn fn;
  make_fn(&fn, j->op, j->arg);
  const int isPreMul = j->op == OP_PREMULSUM;
  const int isPostDiv = j->op == OP_SUMPOSTDIV;
  /* Apply_PreOp<FuncPreMulSum>: v * ncclDecodeScalar<T>(preOpArgs[s]) */
#define PRE_U8(x, s) ((uint8_t)((x) * (uint8_t)j->pre[s]))
#define PRE_U32(x, s) ((uint32_t)((x) * (uint32_t)j->pre[s]))
#define PRE_U64(x, s) ((uint64_t)((x) * (uint64_t)j->pre[s]))
#define PRE_F32(x, s) ((x) * u2f((uint32_t)j->pre[s]))
#define PRE_F64(x, s) ((x) * u2d(j->pre[s]))
#define PRE_F16(x, s) oracle_float_to_half(oracle_half_to_float(x) * oracle_half_to_float((uint16_t)j->pre[s]))
#define PRE_BF16(x, s) oracle_float_to_bf16(oracle_bf16_to_float(x) * oracle_bf16_to_float((uint16_t)j->pre[s]))
  switch (j->dt) {
    case DT_I8: ELEMENT_LOOP(uint8_t, PRE_U8, red_uint8_t_1, div_u8); break;
    case DT_U8: ELEMENT_LOOP(uint8_t, PRE_U8, red_uint8_t_0, div_u8); break;
    case DT_I32: ELEMENT_LOOP(uint32_t, PRE_U32, red_uint32_t_1, div_u32); break;
    case DT_U32: ELEMENT_LOOP(uint32_t, PRE_U32, red_uint32_t_0, div_u32); break;
    case DT_I64: ELEMENT_LOOP(uint64_t, PRE_U64, red_uint64_t_1, div_u64); break;
    case DT_U64: ELEMENT_LOOP(uint64_t, PRE_U64, red_uint64_t_0, div_u64); break;
    case DT_F32: ELEMENT_LOOP(float, PRE_F32, red_f32, NOPOST); break;
    case DT_F64: ELEMENT_LOOP(double, PRE_F64, red_f64, NOPOST); break;
    case DT_F16: ELEMENT_LOOP(uint16_t, PRE_F16, red_f16, NOPOST); break;
    case DT_BF16: ELEMENT_LOOP(uint16_t, PRE_BF16, red_bf16, NOPOST); break;
  }
}

static int check(int nSrcs, int nDsts, int dt, int op, uint64_t arg, int nPreOp, const uint64_t* pre) {
  if (nSrcs < 1 || nSrcs > 8 || nDsts < 0 || nDsts > 8) return R_INVALID;
  if (dt < 0 || dt >= DT_NUM || dt == DT_F8E4M3 || dt == DT_F8E5M2) return R_INVALID;
  if (op < 0 || op >= OP_NUM) return R_INVALID;
  if (op == OP_SUMPOSTDIV && dt > DT_U64) return R_INVALID;
  if (op == OP_SUMPOSTDIV && dt == DT_I8) {
    uint32_t d = (uint32_t)(arg >> 1);
    if (d == 0) d = 1;
    if ((int8_t)d == 0) return R_INVALID;
  }
  if (nPreOp < 0 || nPreOp > nSrcs || (nPreOp > 0 && !pre)) return R_INVALID;
  return R_OK;
}

int oracle_reduce_copy(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                       int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                       const uint64_t* preOpArgs, int postOp) {
  int r = check(nSrcs, nDsts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != R_OK) return r;
  semantics_shape(&datatype, &devRedOp, &nSrcs, &nPreOpSrcs, &postOp);
  Job j = {nSrcs, nDsts, datatype, devRedOp, nPreOpSrcs, postOp, srcs, dsts, preOpArgs, redOpArg, 0, nElts};
  run_job(&j);
  return R_OK;
}

/* The same computation with the nexrReduceCopyFn signature (include/nexr_ring.h), so tests can run
 * the ring schedule on CPU with the oracle underneath (the stream argument is ignored). */
int oracle_reduce_copy_fn(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                          int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                          const uint64_t* preOpArgs, int postOp, void* stream) {
  (void)stream;
  return oracle_reduce_copy(nSrcs, srcs, nDsts, dsts, nElts, datatype, devRedOp, redOpArg, nPreOpSrcs,
                            preOpArgs, postOp);
}

static void* thread_main(void* a) { run_job((const Job*)a); return NULL; }

/* Same computation sliced over nThreads pthreads (contiguous slices) — the "all cores" CPU
 * baseline. */
int oracle_reduce_copy_mt(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                          int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                          const uint64_t* preOpArgs, int postOp, int nThreads) {
  int r = check(nSrcs, nDsts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != R_OK) return r;
  semantics_shape(&datatype, &devRedOp, &nSrcs, &nPreOpSrcs, &postOp);
  if (nThreads < 1) nThreads = 1;
  if (nThreads > 256) nThreads = 256;
  pthread_t th[256];
  int live[256];
  Job jobs[256];
  size_t per = (nElts + (size_t)nThreads - 1) / (size_t)nThreads;
  per = (per + 63) & ~(size_t)63;
  for (int t = 0; t < nThreads; t++) {
    size_t b = per * (size_t)t, e = b + per;
    live[t] = 0;
    if (b >= nElts) continue;
    if (e > nElts) e = nElts;
    Job j = {nSrcs, nDsts, datatype, devRedOp, nPreOpSrcs, postOp, srcs, dsts, preOpArgs, redOpArg, b, e};
    jobs[t] = j;
    if (pthread_create(&th[t], NULL, thread_main, &jobs[t]) == 0) live[t] = 1;
    else run_job(&jobs[t]);
  }
  for (int t = 0; t < nThreads; t++)
    if (live[t]) pthread_join(th[t], NULL);
  return R_OK;
}

/* ---- the reference's CPU execution of reduceCopy: cooperative threads run one after another ----
 *
 * The fork runs a kernel launch's threads as fibers of ONE pthread (cuda_emulator.hh:342-382), and
 * reduceCopy has no barrier, so every emulated thread runs its whole reduceCopy before the next one
 * starts. oracle_reduce_copy_emulated restates that execution, not just the element arithmetic:
 * nThreads threads of 32-lane warps, each running reduceCopy's pass sequence (common_kernel.h:
 * 288-328: 16-B packs with Unroll, then Unroll = 1, when every pointer is 16-B aligned; then
 * sizeof(T) packs with Unroll*(16/sizeof(T))/2, then Unroll = 1) over reduceCopyPacks' hunk layout
 * (:92-113: thread start warp*Unroll*32*BPP + lane*BPP, stride nWarps hunks, partial hunks only
 * at Unroll = 1, the warp rotation at the end of every pass :255-265), with every pack moved by a
 * BPP-byte memcpy (the fork's global_memcpy, op128.h:165-179) into a register pack and folded
 * element by element. The result equals the element loop's; the cost is the reference's (strided
 * 16-B accesses, each 64-B line visited by four emulated threads a whole sweep apart). bench.py
 * times it as the reference CPU path. */
typedef struct {
  int nSrcs, nDsts, dt, nPreOp, postOp, nThreads, unroll;
  const char* const* srcs;
  char* const* dsts;
  const uint64_t* pre;
  Fn fn;
} EJob;

/* One reduceCopyPacks pass of one emulated thread (common_kernel.h:87-266). */
#define EMU_PASS(NAME, T, BPP, PREOP, REDUCE, POSTOP)                                              \
  static void NAME(const EJob* j, int Unroll, int* thread, int64_t* nBehind, int64_t* nAhead) {     \
    const Fn fn = j->fn;                                                                            \
    const int isPreMul = fn.op == OP_PREMULSUM, isPostDiv = fn.op == OP_SUMPOSTDIV;                \
    const int64_t hunk = (int64_t)Unroll * 32 * BPP;                                                \
    const int nWarps = j->nThreads / 32, warp = *thread / 32, lane = *thread % 32;                  \
    int64_t tBehind = *nBehind + warp * hunk + lane * BPP;                                         \
    int64_t tAhead = *nAhead - (warp * hunk + lane * BPP);                                         \
    int64_t nHunks = *nAhead / hunk;                                                                \
    *nBehind += nHunks * hunk;                                                                      \
    *nAhead -= nHunks * hunk;                                                                       \
    if (Unroll == 1 && BPP <= *nAhead) {                                                            \
      nHunks += 1;                                                                                  \
      *nBehind += *nAhead - *nAhead % BPP;                                                          \
      *nAhead = *nAhead % BPP;                                                                      \
    }                                                                                               \
    nHunks -= warp;                                                                                 \
    const int epp = BPP / (int)sizeof(T);                                                           \
    while (Unroll == 1 ? (BPP <= tAhead) : (0 < nHunks)) {                                          \
      T acc[128], tmp[16 / sizeof(T)]; /* Unroll packs of epp elements: at most 8 x 16 B */         \
      for (int u = 0; u < Unroll; u++) {                                                            \
        memcpy(&acc[u * epp], j->srcs[0] + tBehind + (int64_t)u * 32 * BPP, (size_t)BPP);           \
        if (isPreMul && 0 < j->nPreOp)                                                              \
          for (int e = 0; e < epp; e++) acc[u * epp + e] = PREOP(acc[u * epp + e], 0);              \
      }                                                                                             \
      for (int s = 1; s < j->nSrcs; s++)                                                            \
        for (int u = 0; u < Unroll; u++) {                                                          \
          memcpy(tmp, j->srcs[s] + tBehind + (int64_t)u * 32 * BPP, (size_t)BPP);                   \
          for (int e = 0; e < epp; e++) {                                                           \
            T v = tmp[e];                                                                           \
            if (isPreMul && s < j->nPreOp) v = PREOP(v, s);                                         \
            acc[u * epp + e] = REDUCE(&fn, acc[u * epp + e], v);                                    \
          }                                                                                         \
        }                                                                                           \
      if (isPostDiv && j->postOp)                                                                   \
        for (int u = 0; u < Unroll; u++)                                                            \
          for (int e = 0; e < epp; e++) acc[u * epp + e] = POSTOP(&fn, acc[u * epp + e]);           \
      for (int d = 0; d < j->nDsts; d++)                                                            \
        for (int u = 0; u < Unroll; u++)                                                            \
          memcpy(j->dsts[d] + tBehind + (int64_t)u * 32 * BPP, &acc[u * epp], (size_t)BPP);         \
      tBehind += nWarps * hunk;                                                                     \
      tAhead -= nWarps * hunk;                                                                      \
      nHunks -= nWarps;                                                                             \
    }                                                                                               \
    if (Unroll == 1 && nHunks > 0) nHunks -= nWarps;                                                \
    *thread = (int)(-nHunks) * 32 + lane; /* warp rotation, :262-265 */                            \
  }

/* (PRE_* are run_job's pre-op macros above). Pack sizes are compile-time, as in the reference's
 * templates: BytePack<16> and BytePack<sizeof(T)>. */
#define EMU_TYPE(SFX, T, PREOP, REDUCE, POSTOP)                       \
  EMU_PASS(emu_pass16_##SFX, T, 16, PREOP, REDUCE, POSTOP)            \
  EMU_PASS(emu_passT_##SFX, T, (int)sizeof(T), PREOP, REDUCE, POSTOP)
EMU_TYPE(i8, uint8_t, PRE_U8, red_uint8_t_1, div_u8)
EMU_TYPE(u8, uint8_t, PRE_U8, red_uint8_t_0, div_u8)
EMU_TYPE(i32, uint32_t, PRE_U32, red_uint32_t_1, div_u32)
EMU_TYPE(u32, uint32_t, PRE_U32, red_uint32_t_0, div_u32)
EMU_TYPE(i64, uint64_t, PRE_U64, red_uint64_t_1, div_u64)
EMU_TYPE(u64, uint64_t, PRE_U64, red_uint64_t_0, div_u64)
EMU_TYPE(f32, float, PRE_F32, red_f32, NOPOST)
EMU_TYPE(f64, double, PRE_F64, red_f64, NOPOST)
EMU_TYPE(f16, uint16_t, PRE_F16, red_f16, NOPOST)
EMU_TYPE(bf16, uint16_t, PRE_BF16, red_bf16, NOPOST)

typedef void (*EmuPassFn)(const EJob*, int, int*, int64_t*, int64_t*);

/* reduceCopy for one emulated thread (common_kernel.h:273-329). */
static void emu_thread(const EJob* j, EmuPassFn pass16, EmuPassFn passT, int tid, int64_t nBytes, int aligned16) {
  const int esz = (int)oracle_type_size(j->dt);
  int thread = tid;
  int64_t nBehind = 0, nAhead = nBytes;
  if (16 > esz && aligned16) {
    pass16(j, j->unroll, &thread, &nBehind, &nAhead);
    if (nAhead == 0) return;
    pass16(j, 1, &thread, &nBehind, &nAhead);
    if (nAhead == 0) return;
  }
  passT(j, j->unroll * (16 / esz) / 2, &thread, &nBehind, &nAhead);
  if (nAhead == 0) return;
  passT(j, 1, &thread, &nBehind, &nAhead);
}

/* nThreads (a multiple of 32, at most 1024) emulated threads with reduceCopy's Unroll (the fork's
 * ring steps: 512 threads, COLL_UNROLL 4), run one after another on the calling thread. */
int oracle_reduce_copy_emulated(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                                int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                                const uint64_t* preOpArgs, int postOp, int nThreads, int unroll) {
  int r = check(nSrcs, nDsts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != R_OK) return r;
  if (nThreads < 32 || nThreads > 1024 || nThreads % 32 || unroll < 1 || unroll > 8) return R_INVALID;
  if (nDsts == 0 || nElts == 0) return R_OK; /* :288-289 */
  semantics_shape(&datatype, &devRedOp, &nSrcs, &nPreOpSrcs, &postOp);
  EJob j = {nSrcs, nDsts, datatype, nPreOpSrcs, postOp, nThreads, unroll, (const char* const*)srcs,
            (char* const*)dsts, preOpArgs, {0, 0, 0, 0}};
  make_fn(&j.fn, devRedOp, redOpArg);
  static const EmuPassFn p16[DT_NUM] = {emu_pass16_i8, emu_pass16_u8, emu_pass16_i32, emu_pass16_u32,
                                       emu_pass16_i64, emu_pass16_u64, emu_pass16_f16, emu_pass16_f32,
                                       emu_pass16_f64, emu_pass16_bf16, NULL, NULL};
  static const EmuPassFn pT[DT_NUM] = {emu_passT_i8, emu_passT_u8, emu_passT_i32, emu_passT_u32,
                                      emu_passT_i64, emu_passT_u64, emu_passT_f16, emu_passT_f32,
                                      emu_passT_f64, emu_passT_bf16, NULL, NULL};
  int aligned = 1; /* the __all_sync vote over every src and dst pointer, :299-303 */
  for (int s = 0; s < nSrcs; s++) aligned &= ((uintptr_t)srcs[s] % 16) == 0;
  for (int d = 0; d < nDsts; d++) aligned &= ((uintptr_t)dsts[d] % 16) == 0;
  const int64_t nBytes = (int64_t)(nElts * oracle_type_size(datatype));
  for (int t = 0; t < nThreads; t++) emu_thread(&j, p16[datatype], pT[datatype], t, nBytes, aligned);
  return R_OK;
}

/* The reference's geometry for a ring step's reduceCopy in the fork's g++ build: NCCL_CUDA_ARCH is
 * 0 without nvcc, so Unroll = ncclCollUnroll() = 4 (device.h:652-655, :1131-1134), and a SIMPLE
 * step of NCCL_SIMPLE_MAX_NTHREADS = 512 threads with a send peer gives nworkers = 512 - 32 = 480
 * (prims_simple.h:614, device.h:715-716). With the nexrReduceCopyFn signature (include/nexr_ring.h),
 * so the emulated collectives can run every step the reference's way on a host core. */
enum { REF_RING_WORKERS = 480, REF_COLL_UNROLL = 4 };
int oracle_reduce_copy_emulated_fn(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                                   int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                                   const uint64_t* preOpArgs, int postOp, void* stream) {
  (void)stream;
  return oracle_reduce_copy_emulated(nSrcs, srcs, nDsts, dsts, nElts, datatype, devRedOp, redOpArg, nPreOpSrcs,
                                     preOpArgs, postOp, REF_RING_WORKERS, REF_COLL_UNROLL);
}

typedef struct {
  int nSrcs, nDsts, dt, op, nPreOp, postOp, nThreads, unroll, ret;
  const void* srcs[8];
  void* dsts[8];
  const uint64_t* pre;
  uint64_t arg;
  size_t nElts;
} EmuSlice;

static void* emu_slice_main(void* a) {
  EmuSlice* s = (EmuSlice*)a;
  s->ret = oracle_reduce_copy_emulated(s->nSrcs, s->srcs, s->nDsts, s->dsts, s->nElts, s->dt, s->op, s->arg,
                                       s->nPreOp, s->pre, s->postOp, s->nThreads, s->unroll);
  return NULL;
}

/* The same over nPthreads contiguous slices, one emulated launch per pthread (as separate blocks
 * of a launch would run on separate host threads) — the "all cores" reference CPU path. Slices
 * start at 4 KiB multiples, so each keeps the call's pointer alignment. */
int oracle_reduce_copy_emulated_mt(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                                   int datatype, int devRedOp, uint64_t redOpArg, int nPreOpSrcs,
                                   const uint64_t* preOpArgs, int postOp, int nThreads, int unroll, int nPthreads) {
  int r = check(nSrcs, nDsts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != R_OK) return r;
  if (nPthreads < 1) nPthreads = 1;
  if (nPthreads > 256) nPthreads = 256;
  const size_t esz = oracle_type_size(datatype);
  size_t per = (nElts + (size_t)nPthreads - 1) / (size_t)nPthreads;
  per = (per + 4096 / esz - 1) / (4096 / esz) * (4096 / esz);
  pthread_t th[256];
  int live[256];
  EmuSlice sl[256];
  for (int t = 0; t < nPthreads; t++) {
    size_t b = per * (size_t)t, e = b + per;
    live[t] = 0;
    if (b >= nElts) continue;
    if (e > nElts) e = nElts;
    EmuSlice* s = &sl[t];
    s->nSrcs = nSrcs; s->nDsts = nDsts; s->dt = datatype; s->op = devRedOp; s->nPreOp = nPreOpSrcs;
    s->postOp = postOp; s->nThreads = nThreads; s->unroll = unroll; s->pre = preOpArgs; s->arg = redOpArg;
    s->nElts = e - b; s->ret = R_OK;
    for (int k = 0; k < nSrcs; k++) s->srcs[k] = (const char*)srcs[k] + b * esz;
    for (int d = 0; d < nDsts; d++) s->dsts[d] = (char*)dsts[d] + b * esz;
    if (pthread_create(&th[t], NULL, emu_slice_main, s) == 0) live[t] = 1;
    else emu_slice_main(s);
  }
  for (int t = 0; t < nPthreads; t++)
    if (live[t]) pthread_join(th[t], NULL);
  for (int t = 0; t < nPthreads; t++)
    if ((size_t)t * per < nElts && sl[t].ret != R_OK) return sl[t].ret;
  return R_OK;
}

/* ---- LL protocol step (reference src/device/prims_ll.h:218-283) ------------------------------ */
/* One element through one reduce step with the PEER as the first operand: out = op(c, v). */
static void elem_reduce(int dt, const Fn* fn, const uint8_t* c, const uint8_t* v, uint8_t* out) {
  switch (dt) {
    case DT_I8: case DT_U8: { uint8_t a = *c, b = *v, r = dt == DT_I8 ? red_uint8_t_1(fn, a, b) : red_uint8_t_0(fn, a, b); *out = r; break; }
    case DT_I32: case DT_U32: { uint32_t a, b, r; memcpy(&a, c, 4); memcpy(&b, v, 4);
      r = dt == DT_I32 ? red_uint32_t_1(fn, a, b) : red_uint32_t_0(fn, a, b); memcpy(out, &r, 4); break; }
    case DT_I64: case DT_U64: { uint64_t a, b, r; memcpy(&a, c, 8); memcpy(&b, v, 8);
      r = dt == DT_I64 ? red_uint64_t_1(fn, a, b) : red_uint64_t_0(fn, a, b); memcpy(out, &r, 8); break; }
    case DT_F32: { float a, b, r; memcpy(&a, c, 4); memcpy(&b, v, 4); r = red_f32(fn, a, b); memcpy(out, &r, 4); break; }
    case DT_F64: { double a, b, r; memcpy(&a, c, 8); memcpy(&b, v, 8); r = red_f64(fn, a, b); memcpy(out, &r, 8); break; }
    case DT_F16: { uint16_t a, b, r; memcpy(&a, c, 2); memcpy(&b, v, 2); r = red_f16(fn, a, b); memcpy(out, &r, 2); break; }
    case DT_BF16: { uint16_t a, b, r; memcpy(&a, c, 2); memcpy(&b, v, 2); r = red_bf16(fn, a, b); memcpy(out, &r, 2); break; }
  }
}
/* applyPreOp(FuncPreMulSum(raw), x) */
static void elem_premul(int dt, uint64_t raw, uint8_t* x) {
  switch (dt) {
    case DT_I8: case DT_U8: *x = (uint8_t)(*x * (uint8_t)raw); break;
    case DT_I32: case DT_U32: { uint32_t a; memcpy(&a, x, 4); a = a * (uint32_t)raw; memcpy(x, &a, 4); break; }
    case DT_I64: case DT_U64: { uint64_t a; memcpy(&a, x, 8); a = a * raw; memcpy(x, &a, 8); break; }
    case DT_F32: { float a; memcpy(&a, x, 4); a = a * u2f((uint32_t)raw); memcpy(x, &a, 4); break; }
    case DT_F64: { double a; memcpy(&a, x, 8); a = a * u2d(raw); memcpy(x, &a, 8); break; }
    case DT_F16: { uint16_t a; memcpy(&a, x, 2);
      a = oracle_float_to_half(oracle_half_to_float(a) * oracle_half_to_float((uint16_t)raw)); memcpy(x, &a, 2); break; }
    case DT_BF16: { uint16_t a; memcpy(&a, x, 2);
      a = oracle_float_to_bf16(oracle_bf16_to_float(a) * oracle_bf16_to_float((uint16_t)raw)); memcpy(x, &a, 2); break; }
  }
}
static void elem_postdiv(int dt, const Fn* fn, uint8_t* x) {
  switch (dt) {
    case DT_I8: case DT_U8: *x = div_u8(fn, *x); break;
    case DT_I32: case DT_U32: { uint32_t a; memcpy(&a, x, 4); a = div_u32(fn, a); memcpy(x, &a, 4); break; }
    case DT_I64: case DT_U64: { uint64_t a; memcpy(&a, x, 8); a = div_u64(fn, a); memcpy(x, &a, 8); break; }
  }
}

/* Lines are 16 bytes {data1, flag1, data2, flag2} (union ncclLLFifoLine). Returns 0, 4 (bad
 * arguments) or 3 when a recv line does not carry the expected flags (the device would wait). */
int oracle_reduce_copy_ll(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                          const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                          const uint32_t* sendFlags, size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                          int postOp) {
  int r = check(1, 0, datatype, devRedOp, redOpArg, 0, NULL);
  if (r != R_OK) return r;
  if (nRecv < 0 || nRecv > 8 || nSend < 0 || nSend > 8 || (!src && !nRecv) || (!dst && !nSend)) return R_INVALID;
  const int firstWins = g_semantics == 2; /* SKIP_COMP: applyReduce(redOp, peer, d) returns the peer */
  if (g_semantics == 1) datatype = fork_dispatch_type(datatype, devRedOp);
  if (firstWins) { srcIsInput = 0; postOp = 0; }
  Fn fn;
  make_fn(&fn, devRedOp, redOpArg);
  const size_t esz = oracle_type_size(datatype);
  const size_t epl = 8 / esz;
  const size_t nLines = (nElts * esz + 7) / 8;
  for (size_t l = 0; l < nLines; l++) {
    size_t eltN = nElts - l * epl < epl ? nElts - l * epl : epl;
    uint8_t d[8] = {0};
    if (src) {
      memcpy(d, (const uint8_t*)src + l * 8, eltN * esz);
      if (devRedOp == OP_PREMULSUM && srcIsInput)
        for (size_t e = 0; e < epl; e++) elem_premul(datatype, redOpArg, d + e * esz);
    }
    for (int i = 0; i < nRecv; i++) {
      const uint8_t* line = (const uint8_t*)recvLines[i] + l * 16;
      uint32_t f1, f2;
      memcpy(&f1, line + 4, 4);
      memcpy(&f2, line + 12, 4);
      if (f1 != recvFlags[i] || f2 != recvFlags[i]) return 3;
      uint8_t peer[8];
      memcpy(peer, line, 4);
      memcpy(peer + 4, line + 8, 4);
      if ((i == 0 && !src) || firstWins) memcpy(d, peer, 8);
      else
        for (size_t e = 0; e < epl; e++) elem_reduce(datatype, &fn, peer + e * esz, d + e * esz, d + e * esz);
    }
    if (devRedOp == OP_SUMPOSTDIV && postOp)
      for (size_t e = 0; e < epl; e++) elem_postdiv(datatype, &fn, d + e * esz);
    for (int i = 0; i < nSend; i++) {
      uint8_t* line = (uint8_t*)sendLines[i] + l * 16;
      memcpy(line, d, 4);
      memcpy(line + 4, &sendFlags[i], 4);
      memcpy(line + 8, d + 4, 4);
      memcpy(line + 12, &sendFlags[i], 4);
    }
    if (dst) memcpy((uint8_t*)dst + l * 8, d, eltN * esz);
  }
  return R_OK;
}

/* ---- LL128 protocol step (reference src/device/prims_ll128.h:86-331) --------------------------- */
/* Restated literally from the warp-32 register flow: per 2 KiB wire slice (WireWordPerSlice = 32
 * lanes x 8 u64), 1920 data bytes (DataEltPerSlice); lane `wid` holds regs[0..7]; user 16-B chunk
 * ix = g*32 - 4*(g/2) + wid - (g%2)*(wid/8) goes to regs[2g..2g+1] (loadRegsBegin :86-131); flag
 * lanes (wid%8 == 7) load only even g and move regs[2g-1] -> regs[2g] (loadRegsFinish :133-140);
 * regs[u], regs[u+1] travel as wire words u*32 + 2*wid (+1), the flag lane's odd word carrying the
 * flag (recvReduceSendCopy :184-292); storeRegs (:142-174) reverses the permutation. */
static void ll128_words(int dt, const Fn* fn, int op, uint64_t* w, int n, const uint8_t* peerW, int mode) {
  /* mode 0: w = peer; 1: w = op(peer, w); applied per element of each u64 */
  (void)op;
  const size_t esz = oracle_type_size(dt);
  for (int k = 0; k < n; k++) {
    if (mode == 0) { memcpy(&w[k], peerW + 8 * k, 8); continue; }
    uint8_t* x = (uint8_t*)&w[k];
    for (size_t e = 0; e < 8 / esz; e++) elem_reduce(dt, fn, peerW + 8 * k + e * esz, x + e * esz, x + e * esz);
  }
}

int oracle_reduce_copy_ll128(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                             const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                             const uint64_t* sendFlags, size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                             int postOp) {
  int r = check(1, 0, datatype, devRedOp, redOpArg, 0, NULL);
  if (r != R_OK) return r;
  if (nRecv < 0 || nRecv > 8 || nSend < 0 || nSend > 8 || (!src && !nRecv) || (!dst && !nSend)) return R_INVALID;
  const int firstWins = g_semantics == 2; /* SKIP_COMP: every applyReduce returns the peer's words */
  if (g_semantics == 1) datatype = fork_dispatch_type(datatype, devRedOp);
  if (firstWins) { srcIsInput = 0; postOp = 0; }
  Fn fn;
  make_fn(&fn, devRedOp, redOpArg);
  const size_t esz = oracle_type_size(datatype);
  const size_t nBytes = nElts * esz;
  const size_t nSlices = (nBytes + 1919) / 1920;
  for (size_t sl = 0; sl < nSlices; sl++) {
    const size_t dBase = sl * 1920, wBase = sl * 256;                 /* bytes / u64 words */
    const size_t eltBytes = nBytes - dBase < 1920 ? nBytes - dBase : 1920;
    /* 1. every lane waits for its lines' flags (needReload over all u, :193-206) */
    for (int i = 0; i < nRecv; i++)
      for (int wid = 7; wid < 32; wid += 8)
        for (int u = 0; u < 8; u += 2) {
          uint64_t f;
          memcpy(&f, (const uint8_t*)recvWire[i] + 8 * (wBase + u * 32 + 2 * wid + 1), 8);
          if (f != recvFlags[i]) return 3;
        }
    for (int wid = 0; wid < 32; wid++) {
      const int flagThread = (wid % 8) == 7;
      uint64_t v[8] = {0};
      if (src) {
        for (int g = 0; g < 4; g++) {
          int ix = g * 32 - 4 * (g / 2) + wid - (g % 2) * (wid / 8);
          if ((!flagThread || g % 2 == 0) && (size_t)ix * 16 < eltBytes) {
            size_t nb = eltBytes - (size_t)ix * 16 < 16 ? eltBytes - (size_t)ix * 16 : 16;
            memcpy(&v[2 * g], (const uint8_t*)src + dBase + (size_t)ix * 16, nb);
          }
        }
        for (int g = 1; g < 4; g += 2)
          if (flagThread) v[2 * g] = v[2 * g - 1];
        if (devRedOp == OP_PREMULSUM && srcIsInput)
          for (int u = 0; u < 8; u += 2) {
            for (size_t e = 0; e < 8 / esz; e++) elem_premul(datatype, redOpArg, (uint8_t*)&v[u] + e * esz);
            if (!flagThread)
              for (size_t e = 0; e < 8 / esz; e++) elem_premul(datatype, redOpArg, (uint8_t*)&v[u + 1] + e * esz);
          }
      }
      for (int i = 0; i < nRecv; i++) {
        for (int u = 0; u < 8; u += 2) {
          const uint8_t* wp = (const uint8_t*)recvWire[i] + 8 * (wBase + u * 32 + 2 * wid);
          ll128_words(datatype, &fn, devRedOp, &v[u], 2, wp, ((i == 0 && !src) || firstWins) ? 0 : 1);
        }
      }
      if (devRedOp == OP_SUMPOSTDIV && postOp)
        for (int u = 0; u < 8; u++)
          for (size_t e = 0; e < 8 / esz; e++) elem_postdiv(datatype, &fn, (uint8_t*)&v[u] + e * esz);
      for (int i = 0; i < nSend; i++)
        for (int u = 0; u < 8; u += 2) {
          uint8_t* wp = (uint8_t*)sendWire[i] + 8 * (wBase + u * 32 + 2 * wid);
          uint64_t hi = flagThread ? sendFlags[i] : v[u + 1];
          memcpy(wp, &v[u], 8);
          memcpy(wp + 8, &hi, 8);
        }
      if (dst) {
        uint64_t w[8];
        memcpy(w, v, sizeof(w));
        for (int g = 1; g < 4; g += 2)
          if (flagThread) w[2 * g - 1] = w[2 * g];
        for (int g = 0; g < 4; g++) {
          int ix = g * 32 - 4 * (g / 2) + wid - (g % 2) * (wid / 8);
          if ((!flagThread || g % 2 == 0) && (size_t)ix * 16 < eltBytes) {
            size_t nb = eltBytes - (size_t)ix * 16 < 16 ? eltBytes - (size_t)ix * 16 : 16;
            memcpy((uint8_t*)dst + dBase + (size_t)ix * 16, &w[2 * g], nb);
          }
        }
      }
    }
  }
  return R_OK;
}

/* The LL step with the nexrReduceCopyLLFn signature (include/nexr_ring.h): lets tests run the LL
 * ring schedule on CPU. A not-ready line (flag mismatch) reports through *status like the kernel. */
int oracle_reduce_copy_ll_fn(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                             const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                             const uint32_t* sendFlags, size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                             int postOp, uint32_t* status, uint32_t timeoutUs, void* stream) {
  (void)timeoutUs;
  (void)stream;
  int r = oracle_reduce_copy_ll(src, srcIsInput, nRecv, recvLines, recvFlags, dst, nSend, sendLines, sendFlags, nElts,
                                datatype, devRedOp, redOpArg, postOp);
  if (r == 3) {
    if (status) *status = 1;
    return R_OK;
  }
  return r;
}

int oracle_reduce_copy_ll128_fn(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                                const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                                const uint64_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs, void* stream) {
  (void)timeoutUs;
  (void)stream;
  int r = oracle_reduce_copy_ll128(src, srcIsInput, nRecv, recvWire, recvFlags, dst, nSend, sendWire, sendFlags, nElts,
                                   datatype, devRedOp, redOpArg, postOp);
  if (r == 3) {
    if (status) *status = 1;
    return R_OK;
  }
  return r;
}

/* hostToDevRedOp restated (reference src/enqueue.cc:2185-2278), built-in ops only.
 * out[0] = devRedOp, out[1] = scalarArg. Returns 0 or 4. */
int oracle_host_to_dev_redop(int op, int datatype, int nRanks, uint64_t* out) {
  size_t sz = oracle_type_size(datatype);
  if (sz == 0) return R_INVALID;
  int nbits = 8 * (int)sz;
  uint64_t allBits = ~(uint64_t)0 >> (64 - nbits);
  uint64_t signBit = allBits ^ (allBits >> 1);
  int isSigned = datatype == DT_I8 || datatype == DT_I32 || datatype == DT_I64;
  uint64_t arg = 0;
  int dop;
  switch (op) {
    case 0: dop = OP_SUM; break;
    case 1: dop = OP_PROD; break;
    case 2: case 3:
      dop = OP_MINMAX;
      if (isSigned) arg ^= signBit;
      arg ^= (op == 2) ? allBits : 0; /* ncclMax = 2 */
      break;
    case 4:
      if (nRanks < 1) return R_INVALID;
      if (datatype <= DT_U64) { dop = OP_SUMPOSTDIV; arg = ((uint64_t)nRanks << 1) | (uint64_t)isSigned; }
      else if (datatype == DT_F16) { dop = OP_PREMULSUM; arg = oracle_float_to_half((float)(1.0 / nRanks)); }
      else if (datatype == DT_BF16) { dop = OP_PREMULSUM; arg = oracle_float_to_bf16((float)(1.0 / nRanks)); }
      else if (datatype == DT_F32) { dop = OP_PREMULSUM; arg = f2u((float)(1.0 / nRanks)); }
      else if (datatype == DT_F64) { double d = 1.0 / nRanks; dop = OP_PREMULSUM; memcpy(&arg, &d, 8); }
      else return R_INVALID;
      break;
    default: return R_INVALID;
  }
  out[0] = (uint64_t)dop;
  out[1] = arg;
  return R_OK;
}

/* Coverage of the reference's single-rank PreMulSum kernel (onerank.cc:23-30,:77-78): block b of
 * bn = min(32, divUp(nElts*esz, 16 KiB)) handles [b*alignUp(nElts/bn, 16/esz), (b+1)*...) clipped
 * to nElts. Returns how many leading elements the reference writes (DESIGN.md "Deviations"). */
size_t oracle_onerank_reference_coverage(size_t nElts, int datatype) {
  size_t esz = oracle_type_size(datatype);
  if (esz == 0 || nElts == 0) return 0;
  size_t bytes = nElts * esz;
  size_t bn = (bytes + (16u << 10) - 1) / (16u << 10);
  if (bn > 32) bn = 32;
  size_t epp = 16 / esz;
  size_t seg = ((nElts / bn) + epp - 1) / epp * epp;
  size_t cov = bn * seg;
  return cov < nElts ? cov : nElts;
}
