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
// the others are unaligned 16-B accesses. `generic` (every element on the scalar path) is no longer
// used and stays 0.
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
  int generic;
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
// always one trip of kTripPacks 16-B packs (16 KiB) per buffer, so the grid is nPacks / kTripPacks
// whatever the geometry. U = 4, B = 256 is the default (round-1 steady-state sweeps over U in
// {1,2,4,8} x B in {256,512,1024} x occupancy caps for K = 2, 4, 8: profiles/r01_tune_*.log,
// r01_skew.log, r01s2_geom_*.log). Three exceptions, each measured in one process against the default
// on several boxes with byte-identical outputs:
//   - 16-bit floats, K >= 8 (any size): U = 1, B = 1024 — fp16 399.9 vs 407.9 us, bf16 394.9 vs
//     402.0 us at C3 in same-box A/Bs alternated six times (profiles/r01s3_*_geometry_ab.txt);
//   - K = 4 with non-temporal loads and cached stores (64-512 MiB streamed, C4's regime): U = 2,
//     B = 512 — +0.9 % on average over 9 datatypes x {sum, min} on four boxes, never below -0.7 %
//     (tools/geom_sweep.hip, profiles/r02_geom_sweep_*.log; int8 min/max/prod +1-2 %);
//   - K = 4 with non-temporal loads and stores (>= 512 MiB streamed), every type but fp16: U = 1,
//     B = 1024 — +0.5-4 % (+2 % on average) on the same boxes; fp16 alone is mixed there;
//   - K >= 6 with non-temporal loads and stores, every type (round 5): U = 1, B = 1024 at one
//     workgroup per CU (lds_for) — 1.3-2.8 % faster than U = 4, B = 256 for fp32 / uint32 / fp64 /
//     int8 at K = 8 and fp32 / fp16 at K = 6, byte-identical; at 32 MiB per buffer (nt loads only)
//     3.8 % slower, so only under the nt-store policy (tools/occupancy_ab.hip wide,
//     profiles/r05i_occupancy_wide.txt).
// K = 2 keeps the default everywhere (U = 1 loses 10-13 %, U = 2 loses 1-5 %).
constexpr int kTripPacks = 1024;
__host__ __device__ constexpr int unroll_for(int dt, int k, int pol) {
  return ((dt == nexrFloat16 || dt == nexrBfloat16) && k >= 8) ? 1
         : (k >= 6 && pol == 3)                                 ? 1
         : (k == 4 && pol == 1)                                 ? 2
         : (k == 4 && pol == 3 && dt != nexrFloat16)            ? 1
                                                                : 4;
}
__host__ __device__ constexpr int block_for(int dt, int k, int pol) { return kTripPacks / unroll_for(dt, k, pol); }
// Workgroups per CU: the registers of the round-5 kernels admit two 1024-lane workgroups of the K >= 6
// geometry per CU (2 x K x 16 KiB of loads in flight per CU); one is 1.4-3.0 % faster on four boxes, for
// fp16 and bf16 alike at K = 8 (tools/body_ab.hip, tools/occupancy_ab.hip, tools/data_ab.hip;
// profiles/r05a_body_ab.txt, r05b_occupancy_ab.txt, r05c_data_ab.txt), and the K >= 6 geometry above
// was measured at one. The launch reserves this many bytes of dynamic LDS (the kernel never touches
// it) so that only one fits in a CU's 160 KiB. Every other geometry runs as its registers allow: C2
// is flat from 2 to 8 workgroups per CU, C4 from 2 to 4.
constexpr int kLdsOneWorkgroupPerCu = 120 * 1024;
__host__ __device__ constexpr int lds_for(int dt, int k, int pol) {
  return unroll_for(dt, k, pol) == 1 && block_for(dt, k, pol) == 1024 && k >= 6 ? kLdsOneWorkgroupPerCu : 0;
}

}  // namespace nexr
