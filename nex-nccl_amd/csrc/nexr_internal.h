// nexr_internal.h — shared between the C-ABI host code (nexr_api.cpp) and the per-datatype
// kernel objects (nexr_kernels.hip). Not installed; not part of the ABI.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <hip/hip_runtime.h>
#include "../../include/nexr.h"

namespace nexr {

constexpr int kBlock = 256;  // 4 waves of 64 lanes per workgroup

// Launch parameters of one reduce-copy, passed by value as the kernel argument.
//
// Element range layout (host computes it, see planLayout in nexr_api.cpp):
//   [0, head)                    edge elements before dst[0]'s next 128-B boundary (scalar path)
//   [head, head + nPacks*EPP)    the packed body: pack i = 16 contiguous bytes of every buffer
//   [.., nElts)                  tail edge elements (scalar path)
// When the pointers share a 16-B phase every body access is 16-B aligned; otherwise (`unaligned`)
// the others are unaligned 16-B accesses.
struct RCParams {
  const char* src[NEXR_MAX_SRCS];
  char* dst[NEXR_MAX_DSTS];
  uint64_t pre[NEXR_MAX_SRCS];  // raw pre-op scalar bits per src (PreMulSum), reduce_kernel.h:145,:166
  const void* prePtr;           // if non-null, pre[0] is loaded from this device address (onerank.cc:32-42)
  uint64_t redArg;              // op argument (MinMax bit 0, SumPostDiv divisor<<1|signed)
  uint64_t nElts;
  uint64_t head;                // edge elements before the body
  uint64_t nPacks;              // 16-B packs in the body
  int nDsts;
  int nPreOp;                   // pre-op applies to srcs[s] for s < nPreOp
  int postOp;
  int unaligned;  // no common 16-B phase: body packs use unaligned 16-B accesses (diagnostics)
};

// Launch parameters of one LL-protocol step (nexr_ll.hip; reference src/device/prims_ll.h:218-283).
struct LLParams {
  const char* src;                  // user buffer (nullable)
  const char* recv[NEXR_MAX_SRCS];  // peer LL lines of this step
  uint32_t recvFlag[NEXR_MAX_SRCS];
  char* dst;                        // user buffer (nullable)
  char* send[NEXR_MAX_DSTS];
  uint32_t sendFlag[NEXR_MAX_DSTS];
  uint64_t nElts;
  uint64_t redArg;
  uint32_t* status;                 // set to 1 when a recv flag never arrived (nullable)
  uint64_t timeoutTicks;            // s_memrealtime ticks (100 MHz) before giving up
  int nRecv, nSend, srcIsInput, postOp;
  int firstWins;                    // nexrSemanticsShipped: every reduce returns its first operand
};
hipError_t launch_ll(int dt, const LLParams& a, int op, int grid, hipStream_t s);

// A run of LL steps of one Primitives in one launch (nexrReduceCopyLLSteps; nexr_ll.hip). Workgroup w
// owns line tiles t = w, w + grid, ... of every step and its wave v the same lines of each tile, on both
// ends of a connection, so the credit of a slot is per wave: head word (w, v) of a connection holds the
// steps the receiver's wave v of workgroup w has read.
constexpr int kLLStepsMax = 96;        // steps per launch: the parameter block stays under 4 KiB
constexpr int kLLHeadStride = 16;      // bytes between a connection's head words (one per wave)
constexpr int kLLStepsMaxGrid = NEXR_LL_HEAD_BYTES / (kLLHeadStride * (kBlock / 64));
struct LLStepsParams {
  const char* input;
  char* output;
  const char* recvFifo[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t* recvHead[NEXR_LL_STEPS_MAX_PEERS];
  char* sendFifo[NEXR_LL_STEPS_MAX_PEERS];
  const uint64_t* sendHead[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t recvStep[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t sendStep[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t slotBytes;
  uint64_t redArg;
  uint32_t* status;
  uint64_t timeoutTicks;
  int nRecv, nSend, nSlots, nSteps;
  int firstWins;
#ifdef NEXR_LL_STEPS_TRACE
  uint64_t* trace;  // tuning harness only (tools/ll_steps_trace.hip)
#endif
  nexrLLStep step[kLLStepsMax];
};
static_assert(sizeof(LLStepsParams) <= 4096, "kernel argument block");
hipError_t launch_ll_steps(int dt, const LLStepsParams& a, int op, int grid, hipStream_t s);

// Launch parameters of one LL128-protocol step (nexr_ll.hip; reference src/device/prims_ll128.h).
// Wire: 2 KiB slices of 16 x 128-B lines carrying 1920 data bytes; word 15 of every line is the flag.
constexpr int kLL128SliceBytes = 2048;
constexpr int kLL128SliceData = 1920;
// Work per workgroup iteration (nexr_ll.hip): LL, kLLU sub-tiles of 2 * kBlock lines (8 data bytes
// each); LL128, kLL128U sub-tiles of kBlock 16-byte wire units. One sub-tile (4 KiB of data or wire
// per workgroup) is fastest at the protocols' step sizes, 32 KiB-4 MiB, by up to 1.8x over four, and
// for LL at 64 MiB as well; four gain <= 10 % only for LL128 at 64 MiB (tools/ll_bits.hip,
// profiles/r02s5_ll_bits.txt).
#ifndef NEXR_LL_U  // overridable only by tuning harnesses (tools/ll_bits.hip)
#define NEXR_LL_U 1
#endif
constexpr int kLLU = NEXR_LL_U;
constexpr int kLLSubLines = 2 * kBlock;
constexpr int kLLTileLines = kLLU * kLLSubLines;
constexpr int kLL128U = NEXR_LL_U;
constexpr int kLL128TileUnits = kLL128U * kBlock;
struct LL128Params {
  const char* src;
  const char* recv[NEXR_MAX_SRCS];
  uint64_t recvFlag[NEXR_MAX_SRCS];
  char* dst;
  char* send[NEXR_MAX_DSTS];
  uint64_t sendFlag[NEXR_MAX_DSTS];
  uint64_t nElts;
  uint64_t redArg;
  uint32_t* status;
  uint64_t timeoutTicks;
  int nRecv, nSend, srcIsInput, postOp;
  int firstWins;  // as LLParams
};
hipError_t launch_ll128(int dt, const LL128Params& a, int op, int grid, hipStream_t s);

// A batch of independent reduce-copies with the same (datatype, op, K) in one launch.
constexpr int kMaxBatch = 14;  // keeps the parameter block under the 4 KiB kernel-argument limit
struct BatchParams {
  int nWorks;
  uint32_t start[kMaxBatch + 1];  // work i owns workgroups [start[i], start[i+1])
  RCParams w[kMaxBatch];
};
static_assert(sizeof(BatchParams) <= 4000, "batch parameters must fit the kernel-argument segment");
static_assert(kMaxBatch == NEXR_MAX_BATCH_WORKS, "public batch limit must match the kernel's");

// Launch geometry chosen by the host.
struct Geometry {
  int grid;
  int pol;  // cache policy: 0 plain, 1 non-temporal loads, 3 non-temporal loads and stores
};

// One entry point per datatype, defined in the kernel object compiled with -DNEXR_DT=<dt>.
// Returns hipSuccess or the launch error.
#define NEXR_DECLARE_LAUNCH(dt) \
  hipError_t launch_dt##dt(const RCParams& p, int op, int nSrcs, const Geometry& g, hipStream_t s);
NEXR_DECLARE_LAUNCH(0) NEXR_DECLARE_LAUNCH(1) NEXR_DECLARE_LAUNCH(2) NEXR_DECLARE_LAUNCH(3)
NEXR_DECLARE_LAUNCH(4) NEXR_DECLARE_LAUNCH(5) NEXR_DECLARE_LAUNCH(6) NEXR_DECLARE_LAUNCH(7)
NEXR_DECLARE_LAUNCH(8) NEXR_DECLARE_LAUNCH(9)
#undef NEXR_DECLARE_LAUNCH
#define NEXR_DECLARE_BATCH(dt) \
  hipError_t launch_batch_dt##dt(const BatchParams& b, int op, int nSrcs, int pol, int grid, hipStream_t s);
NEXR_DECLARE_BATCH(0) NEXR_DECLARE_BATCH(1) NEXR_DECLARE_BATCH(2) NEXR_DECLARE_BATCH(3)
NEXR_DECLARE_BATCH(4) NEXR_DECLARE_BATCH(5) NEXR_DECLARE_BATCH(6) NEXR_DECLARE_BATCH(7)
NEXR_DECLARE_BATCH(8) NEXR_DECLARE_BATCH(9)
#undef NEXR_DECLARE_BATCH

// Workgroup geometry per (datatype, fan-in, cache policy): U packs per lane x B lanes per workgroup,
// and how many workgroups per CU the launch admits (lds_for; 0: as the registers allow). A workgroup owns one trip
// of U x B packs of every buffer, so the one-shot grid is nPacks / (U x B). U = 4, B = 256 is the default
// (round-1 steady-state sweeps over U in {1,2,4,8} x B in {256,512,1024} x occupancy caps for K = 2, 4, 8:
// profiles/r01_tune_*.log, r01_skew.log, r01s2_geom_*.log). The exceptions, each measured in one process
// against the alternatives on several boxes with byte-identical outputs:
//   - K = 4 with non-temporal loads and cached stores (64-512 MiB streamed, C4's regime), 1-, 2- and
//     8-byte types: U = 2, B = 512 — +0.9 % on average over 9 datatypes x {sum, min} on four boxes in
//     round 2 (profiles/r02_geom_sweep_*.log); with the round-5 body +0.9-3.6 % for int8, fp16 and bf16,
//     equal for uint64, and at one or two workgroups per CU 1-18 % slower; 4-byte types keep 4 x 256,
//     0.7-3.0 % faster with the round-5 body (int32 min at 16-100 MiB, int32 prod, fp32 sum;
//     profiles/r05s_occupancy_c4sizes.txt, r05t_occupancy_c4types.txt, r05l_occupancy_k8lanes.txt);
//   - the nt-store policy (>= 512 MiB streamed), where a CU's loads in flight are the lever (round 5,
//     tools/occupancy_ab.hip, profiles/r05b_occupancy_ab.txt, r05i_occupancy_wide.txt,
//     r05k_occupancy_k8shape.txt, r05l_occupancy_k8lanes.txt): the fastest point is about 64 KiB of
//     loads in flight per CU, i.e. 4096 / K lanes with one pack each, at ONE workgroup per CU
//       K = 4-5 (every type but fp16, mixed there at K = 4): U = 1, B = 1024 — at K = 4 4.2 % faster than
//         the two workgroups per CU its registers allow and +0.5-4 % over 4 x 256
//         (profiles/r02_geom_sweep_*); at K = 5 3.3-3.4 % over 4 x 256 (fp32, bf16, 1.5 GiB streamed;
//         profiles/r05zp_occupancy_k35.txt). bf16 alone takes two 512-lane workgroups per CU instead (round
//         6, with its hardware-RNE fold): 1.4-3.2 % faster at K = 4 and 2.8 % at K = 5 on two boxes, where
//         fp32, fp64, int32 and int8 lose 1.0-3.5 % that way (profiles/r06a_bf16cvt.txt, r06b_k45.txt).
//         K = 3 keeps 4 x 256: 1 x 1024 gained 2.9 % at 1 GiB with one
//         destination but lost 1.2-5.8 % at 96-300 MiB with 2-5 (profiles/r05zr_occupancy_k3m.txt), where
//         the nt-store table of pickPolicy (nexr_api.cpp) puts those calls under this policy;
//       K >= 6: U = 1, B = 512 — fp16 K = 8 2.5-2.7 % and fp32 K = 8 3.6 % faster than 1 x 1024, fp32
//         K = 6 1.3 %; 256 lanes are 10-20 % slower, 384 or 640 lanes 2 % slower. bf16 too since round 6:
//         with the hardware RNE (v_cvt_pk_bf16_f32, nexr_types.hpp) its fold no longer needs 1024 lanes
//         to hide it, and 1 x 512 is 1.6 % faster than the round-5 fold at 1 x 1024 and level with fp16
//         and a bare uint32 stream of the same bytes (profiles/r06a_bf16cvt.txt);
//   - 16-bit floats, K >= 8, below the nt-store policy: U = 1, B = 1024 as the registers admit (two per
//     CU): rounds 1 and 5 chose 1 x 1024 over 4 x 256 (profiles/r01s3_*_geometry_ab.txt); held to one
//     workgroup per CU it is 3.2-9.3 % slower under nt loads (64-512 MiB streamed) and equal under plain
//     (profiles/r05zm_occupancy_k8mid.txt) — the reservation pays only under nt stores (above).
// K = 2 keeps the default everywhere (U = 1 loses 10-13 %, U = 2 loses 1-5 %; 2 to 8 workgroups per CU
// are flat, profiles/r05b_occupancy_ab.txt).
constexpr int kTripPacks = 1024;  // the default trip (4 x 256)
struct Shape {
  int u, b;
  int wgsPerCu;  // 0: as the registers allow; 1 or 2: held there by an LDS reservation (lds_for)
};
__host__ __device__ constexpr Shape shape_for(int dt, int k, int pol) {
  const bool half = dt == nexrFloat16 || dt == nexrBfloat16;
  const bool four = dt == nexrInt32 || dt == nexrUint32 || dt == nexrFloat32;
  return (pol == 3 && k >= 6)                       ? Shape{1, 512, 1}
         : (half && k >= 8)                         ? Shape{1, 1024, 0}
         : (k == 4 && pol == 1 && !four)            ? Shape{2, 512, 0}
         : (k >= 4 && k <= 5 && pol == 3 && dt == nexrBfloat16) ? Shape{1, 512, 2}
         : (k >= 4 && k <= 5 && pol == 3 && dt != nexrFloat16) ? Shape{1, 1024, 1}
                                                    : Shape{4, 256, 0};
}
__host__ __device__ constexpr int unroll_for(int dt, int k, int pol) { return shape_for(dt, k, pol).u; }
__host__ __device__ constexpr int block_for(int dt, int k, int pol) { return shape_for(dt, k, pol).b; }
// n workgroups per CU: the launch reserves this many bytes of dynamic LDS (the kernel never touches
// it), so that only n fit in a CU's 160 KiB whatever the kernel's registers would admit.
constexpr int kLdsOneWorkgroupPerCu = 120 * 1024;  // one per CU (160 / 2 < 120 <= 160)
constexpr int kLdsTwoWorkgroupsPerCu = 66 * 1024;  // two per CU (160 / 3 < 66 <= 160 / 2)
__host__ __device__ constexpr int lds_for(int dt, int k, int pol) {
  return shape_for(dt, k, pol).wgsPerCu == 1   ? kLdsOneWorkgroupPerCu
         : shape_for(dt, k, pol).wgsPerCu == 2 ? kLdsTwoWorkgroupsPerCu
                                              : 0;
}

// The reduce-copy kernels that are compiled (round 6). Every other (datatype, op, K) is routed by the
// host onto one of them with the same bytes (routeKernel, nexr_api.cpp), so it is never launched:
//   - K = 1 without arithmetic (no pre-op scalar, no post-op divide) is a byte copy: uint8 Sum;
//   - signed integers' Sum, Prod, PreMulSum and SumPostDiv run the unsigned type's kernels (wrapping
//     two's-complement arithmetic, the reference's own equivalent_primary, generate.py:128-136; the
//     divide reads its signedness from redOpArg), so the signed objects hold Min / Max only;
//   - PreMulSum without pre-op sources and SumPostDiv without the divide are Sum.
// Batch launches are compiled for the plain and non-temporal-load policies only: a batch that would
// stream enough for non-temporal stores (>= 512 MiB) runs its works as single launches, where one launch
// per work costs nothing measurable against the work itself.
__host__ __device__ constexpr bool is_signed_int(int dt) { return dt == nexrInt8 || dt == nexrInt32 || dt == nexrInt64; }
__host__ __device__ constexpr bool kernel_compiled(int dt, int op, int k) {
  return k == 1 ? (op == nexrDevSum && dt == nexrUint8) ||
                      (!is_signed_int(dt) && (op == nexrDevPreMulSum || op == nexrDevSumPostDiv))
                : !is_signed_int(dt) || op == nexrDevMinMax;
}
constexpr int kBatchPolicies = 2;  // plain (0) and non-temporal loads (1)

}  // namespace nexr
