// nexr_resident.hip — the ring and tree collectives as ONE device-resident launch per GPU
// (beyond SURVEY §8: the opt-in extras library, libnexr_extras.so).
//
// What it runs is the reference's device kernel for ncclAllReduce with NCCL_ALGO_RING /
// NCCL_PROTO_SIMPLE — runRing (src/device/all_reduce.h:12-84), and likewise ReduceScatter
// (reduce_scatter.h:12-52), AllGather (all_gather.h:12-66), Reduce (reduce.h:12-50), Broadcast
// (broadcast.h:12-58) and the tree all-reduce's runTreeSplit (all_reduce.h:150-230) — over
// Primitives::genericOp (src/device/prims_simple.h:190-330) with the FIFO credit protocol of
// waitPeer / postPeer (:111-188): NCCL_STEPS = 8 slots of stepBytes per connection, a slice spans StepPerSlice steps, the
// receiver waits for tail >= step + StepPerSlice, the sender for head + NCCL_STEPS >= step +
// StepPerSlice, and each side posts its step once the slice is done. The host-sequenced ring in
// nexr_ring.cpp (the default product) runs the same schedule with one reduce-copy launch per slice; this file runs every
// rank's whole schedule inside one launch, each rank's blocks waiting on the step counters in HBM
// instead of the host waiting on streams.
//
// MI355X mapping:
//   - a (rank, channel) is a TEAM of `team` workgroups, not one block: every FIFO slot's bytes are
//     cut into `team` fixed runs of whole 16-byte packs, and workgroup g of a team moves the
//     elements of every slice of its rank that fall in run g. Member g of rank r only ever consumes
//     what member g of rank r-1 produced, into bytes only they touch, so each member runs the credit
//     protocol on its own (tail, head) record and a team needs no barrier across workgroups: the
//     reference's one-block-per-channel FIFO, replicated `team` times over disjoint byte ranges of
//     each slot. What every element goes through (which rank reduces it at which step, operand
//     order, rounding) is the reference's, so results equal the host-sequenced schedules'.
//   - FIFO data moves with system-coherent 16-byte buffer accesses (sc0 sc1, as the LL steps'
//     wire accesses, nexr_ll.hip): the consumer may sit on another XCD or another GPU, whose caches
//     do not snoop the producer's writes; with every wave's accesses drained before the one-lane
//     counter store, no L2 write-back or invalidate is needed per slice. User buffers use ordinary
//     16-byte accesses.
//   - step counters are 64-bit words, one record per member in its own 128-byte lines, written by
//     one workgroup and polled by one other; every wait is bounded in time (s_memrealtime) and a
//     timeout is reported in the device's status word, never a hang.
// Compiled once per datatype with -DNEXR_DT=<nexrDataType_t value> (see Makefile), like the
// reduce-copy kernels, so the objects build in parallel.
#include "nexr_fold.hpp"
#include "nexr_resident.h"

#ifndef NEXR_DT
#error "compile with -DNEXR_DT=<datatype>"
#endif

namespace nexr {

constexpr int kResU = 4;  // packs per lane per pass (the SIMPLE kernel's default unroll)
constexpr int kResBits = 17;  // raw_buffer aux bits: sc0 (bit 0) | sc1 (bit 4), system coherence

__device__ __forceinline__ __amdgpu_buffer_rsrc_t res_rsrc(const char* base, uint64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 fifo_ld(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return bc<u32x4>(__builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kResBits));
}
__device__ __forceinline__ void fifo_st(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kResBits);
}
typedef __attribute__((address_space(1))) uint64_t g_u64;
__device__ __forceinline__ uint64_t ctr_ld(const char* p) {
  return __hip_atomic_load((const g_u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void ctr_st(char* p, uint64_t v) {
  __hip_atomic_store((g_u64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Every vector memory access of this wave complete (stores acknowledged, loads returned). Inline asm,
// so that no compiler pass can drop it (MI355X_MICROARCH.md, "Compiler hazard").
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ int64_t imin(int64_t x, int64_t y) { return x < y ? x : y; }
__device__ __forceinline__ int64_t imax(int64_t x, int64_t y) { return x > y ? x : y; }
__device__ __forceinline__ int64_t divUp64(int64_t x, int64_t y) { return (x + y - 1) / y; }

// The call-wide scalars every workgroup needs, copied out of the kernel argument.
struct ResScalars {
  int64_t chunkCount, stepElems, count;
  uint64_t stepBytes, redArg, timeoutTicks;
  uint32_t* status;
  int stepPerSlice, slicePerChunk, team, nRanks, root;
};

struct ResShared {
  uint64_t recvStep[3], sendStep[3];
  int ok;
};

// The first n (< 16) bytes at p as a zero-padded pack, and the reverse.
__device__ __forceinline__ u32x4 ld_bytes(const char* p, uint32_t n) {
  uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 16; k++)
    if ((uint32_t)k < n) w[k >> 2] |= (uint32_t)(uint8_t)p[k] << (8 * (k & 3));
  return (u32x4){w[0], w[1], w[2], w[3]};
}
__device__ __forceinline__ void st_bytes(char* p, uint32_t n, u32x4 v) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 16; k++)
    if ((uint32_t)k < n) p[k] = (char)(w[k >> 2] >> (8 * (k & 3)));
}

// One workgroup's piece of a slice: srcs = [user src if US] + NR recv FIFOs, dsts = [user dst if UD]
// + NS send FIFOs (genericOp's order, prims_simple.h:131-132, :238-242), `bytes` bytes. FIFO pieces
// start 16-byte aligned and own their slot up to the next 16 bytes, so a partial last pack moves
// whole there; user buffers get exactly their bytes.
template <int N> using PtrArr = const char* [N > 0 ? N : 1];
template <int D, int OP, bool IsMin, bool US, int NR, bool UD, int NS>
__device__ __forceinline__ void piece(const char* usrc, const PtrArr<NR>& rfifo, char* udst, const PtrArr<NS>& sfifo,
                                      uint64_t bytes, const Fold<D, OP, (int)US + NR, IsMin>& f) {
  constexpr int K = (int)US + NR;
  const uint64_t rbytes = (bytes + 15) & ~15ull;
  __amdgpu_buffer_rsrc_t rr[NR > 0 ? NR : 1], sr[NS > 0 ? NS : 1];
#pragma unroll
  for (int i = 0; i < NR; i++) rr[i] = res_rsrc(rfifo[i], rbytes);
#pragma unroll
  for (int i = 0; i < NS; i++) sr[i] = res_rsrc(sfifo[i], rbytes);
  const uint64_t nFull = bytes / 16;
  constexpr uint64_t kPass = (uint64_t)kBlock * kResU;
  uint64_t base = 0;
  for (; base + kPass <= nFull; base += kPass) {
    u32x4 in[kResU][K];
#pragma unroll
    for (int u = 0; u < kResU; u++) {
      const uint64_t j = base + u * kBlock + threadIdx.x;
      if constexpr (US) in[u][0] = ld16<kPolPlain>(usrc + j * 16);
#pragma unroll
      for (int i = 0; i < NR; i++) in[u][(int)US + i] = fifo_ld(rr[i], (uint32_t)(j * 16));
    }
#pragma unroll
    for (int u = 0; u < kResU; u++) {
      const uint64_t j = base + u * kBlock + threadIdx.x;
      const u32x4 out = f.run(in[u]);
      if constexpr (UD) st16<kPolPlain>(udst + j * 16, out);
#pragma unroll
      for (int i = 0; i < NS; i++) fifo_st(sr[i], (uint32_t)(j * 16), out);
    }
  }
  const uint64_t nPacks = (bytes + 15) / 16;
  for (uint64_t j = base + threadIdx.x; j < nPacks; j += kBlock) {
    const uint32_t valid = j < nFull ? 16u : (uint32_t)(bytes - nFull * 16);
    u32x4 in[K];
    if constexpr (US) in[0] = valid == 16 ? ld16<kPolPlain>(usrc + j * 16) : ld_bytes(usrc + j * 16, valid);
#pragma unroll
    for (int i = 0; i < NR; i++) in[(int)US + i] = fifo_ld(rr[i], (uint32_t)(j * 16));
    const u32x4 out = f.run(in);
    if constexpr (UD) {
      if (valid == 16) st16<kPolPlain>(udst + j * 16, out);
      else st_bytes(udst + j * 16, valid, out);
    }
#pragma unroll
    for (int i = 0; i < NS; i++) fifo_st(sr[i], (uint32_t)(j * 16), out);
  }
}

// One rank's Primitives for one (channel, team member): up to MR recv and MS send connections (the
// ring has one of each; the tree's FanAsymmetric / FanSymmetric up to NCCL_MAX_TREE_ARITY = 3),
// their step counters, and the user buffers.
template <int D, int OP, bool IsMin, int MR, int MS>
struct ResPrims {
  static constexpr int esz = 16 / Ty<D>::EPP;
  ResScalars a;  // by value: a reference to the kernel argument would copy it to scratch
  const char* input;
  char* output;
  int member;
  int nRecv, nSend;
  const char* recvFifo[MR];
  char* recvTail[MR];  // this member's records of the connections into this rank
  char* recvHead[MR];
  const char* sendFifo[MS];
  char* sendTail[MS];  // this member's records of the connections out of it (on the peers' GPUs)
  char* sendHead[MS];
  uint64_t recvStep[MR], sendStep[MS];
  ResShared* sh;  // the wait's outcome and the attached steps, broadcast from thread 0

  // waitPeer's spin (prims_simple.h:116-123), thread 0 only, bounded like checkAbort
  // (primitives.h:142-156): false after a timeout (status 1) or once the status word is non-zero:
  // another workgroup's timeout, or the host's relay of the communicator's abort word (2), which a
  // workgroup that gives up on it turns into 3, so that the host can tell a kernel that stopped
  // mid-protocol from one that finished before the relay arrived.
  __device__ __forceinline__ bool wait_ge(const char* p, uint64_t target) const {
    uint64_t t0 = 0;
    for (uint32_t spins = 0;; spins++) {
      if (ctr_ld(p) >= target) return true;
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (!t0) t0 = now;
      if ((spins & 255) == 255) {
        const uint32_t st = __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (st != 0) {
          if (st == 2) __hip_atomic_store(a.status, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          return false;
        }
      }
      if (now - t0 > a.timeoutTicks) {
        __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }

  // loadRecvConn / loadSendConn (prims_simple.h:512-517, :557-558): steps resume from the previous
  // collective's, rounded up to SlicePerChunk * StepPerSlice, the receiver publishing its rounded step.
  __device__ __forceinline__ void attach() {
    if (threadIdx.x == 0) {
      const uint64_t cs = (uint64_t)(a.stepPerSlice * a.slicePerChunk);
#pragma unroll
      for (int i = 0; i < MR; i++) {  // static indices: a private array indexed at run time spills
        if (i < nRecv) {
          const uint64_t rs = (ctr_ld(recvHead[i]) + cs - 1) / cs * cs;
          ctr_st(recvHead[i], rs);
          sh->recvStep[i] = rs;
        }
      }
#pragma unroll
      for (int i = 0; i < MS; i++)
        if (i < nSend) sh->sendStep[i] = (ctr_ld(sendTail[i]) + cs - 1) / cs * cs;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MR; i++) recvStep[i] = i < nRecv ? sh->recvStep[i] : 0;
#pragma unroll
    for (int i = 0; i < MS; i++) sendStep[i] = i < nSend ? sh->sendStep[i] : 0;
    __syncthreads();
  }

  // genericOp<0, 0, Recv, Send, SrcBuf, DstBuf> (prims_simple.h:190-330) for this member's pieces:
  // Recv = every recv connection, Send = every send connection. The run-time fan-in and fan-out
  // pick a compile-time instance; only reachable ones are built (R / S imply at least one
  // connection, and Sym — the tree root's recvReduceCopySend — has as many sends as receives).
  template <bool US, bool R, bool UD, bool S, bool Sym = false>
  __device__ __forceinline__ bool op(int64_t srcIx, int64_t dstIx, int64_t nelem, bool postOp) {
    if constexpr (!R) {
      return opS<US, 0, UD, S>(srcIx, dstIx, nelem, postOp);
    } else {
      if constexpr (MR >= 2) {
        if (nRecv == 2) return Sym ? opN<US, 2, UD, (S ? 2 : 0)>(srcIx, dstIx, nelem, postOp)
                                   : opS<US, 2, UD, S>(srcIx, dstIx, nelem, postOp);
      }
      if constexpr (MR >= 3) {
        if (nRecv == 3) return Sym ? opN<US, 3, UD, (S ? 3 : 0)>(srcIx, dstIx, nelem, postOp)
                                   : opS<US, 3, UD, S>(srcIx, dstIx, nelem, postOp);
      }
      return Sym ? opN<US, 1, UD, (S ? 1 : 0)>(srcIx, dstIx, nelem, postOp) : opS<US, 1, UD, S>(srcIx, dstIx, nelem, postOp);
    }
  }
  template <bool US, int NR, bool UD, bool S>
  __device__ __forceinline__ bool opS(int64_t srcIx, int64_t dstIx, int64_t nelem, bool postOp) {
    if constexpr (!S) {
      return opN<US, NR, UD, 0>(srcIx, dstIx, nelem, postOp);
    } else {
      if constexpr (MS >= 2) {
        if (nSend == 2) return opN<US, NR, UD, 2>(srcIx, dstIx, nelem, postOp);
      }
      if constexpr (MS >= 3) {
        if (nSend == 3) return opN<US, NR, UD, 3>(srcIx, dstIx, nelem, postOp);
      }
      return opN<US, NR, UD, 1>(srcIx, dstIx, nelem, postOp);
    }
  }
  template <bool US, int NR, bool UD, int NS>
  __device__ __forceinline__ bool opN(int64_t srcIx, int64_t dstIx, int64_t nelem, bool postOp) {
    constexpr int K = (int)US + NR;
    nelem = nelem < 0 ? 0 : nelem;
    int64_t sliceSize = a.stepElems * a.stepPerSlice;
    sliceSize = imax(divUp64(nelem, 16 * (int64_t)a.slicePerChunk) * 16, sliceSize / 32);
    int64_t offset = 0;
    for (int slice = 0; slice < a.slicePerChunk; slice++) {
      sliceSize = imin(sliceSize, nelem - offset);
      if (sliceSize < 0) sliceSize = 0;
      if (threadIdx.x == 0) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NR; i++) ok = ok && wait_ge(recvTail[i], recvStep[i] + a.stepPerSlice);
#pragma unroll
        for (int i = 0; i < NS; i++)
          if (ok && sendStep[i] + a.stepPerSlice > 8) ok = wait_ge(sendHead[i], sendStep[i] + a.stepPerSlice - 8);
        sh->ok = ok ? 1 : 0;
      }
      __syncthreads();  // the other waves load the handed-off bytes only behind the poll
      if (!sh->ok) return false;
      // This member's piece of the slice. Pieces sit on a grid fixed for the call — the largest
      // slice (StepPerSlice steps) cut into `team` runs of whole 16-byte packs — so that member g
      // always owns the same bytes of every FIFO slot: its credits then cover exactly the bytes it
      // writes, whatever size the slice that last used the slot had. A smaller slice leaves the
      // high members idle.
      constexpr int64_t epp = 16 / esz;
      const int64_t per = divUp64(divUp64(a.stepElems * a.stepPerSlice, a.team), epp) * epp;
      const int64_t lo = imin(sliceSize, per * member), hi = imin(sliceSize, lo + per);
      if constexpr (K > 0 && ((int)UD + NS) > 0) {  // else no data moves (genericOp's k > 0 && m > 0)
        if (hi > lo) {
        // PreOpSrcs = SrcBuf == Input (prims_simple.h:279-280), preOpArgs = redOpArgs
        const Fold<D, OP, K, IsMin> f(a.redArg, US ? 1 : 0, postOp, a.redArg);
        const uint64_t slotOff = (uint64_t)lo * esz;
        const char* rf[NR > 0 ? NR : 1];
        const char* sf[NS > 0 ? NS : 1];
#pragma unroll
        for (int i = 0; i < NR; i++) rf[i] = recvFifo[i] + (recvStep[i] % 8) * a.stepBytes + slotOff;
#pragma unroll
        for (int i = 0; i < NS; i++) sf[i] = sendFifo[i] + (sendStep[i] % 8) * a.stepBytes + slotOff;
        piece<D, OP, IsMin, US, NR, UD, NS>(US ? input + (srcIx + offset + lo) * esz : nullptr, rf,
                                            UD ? output + (dstIx + offset + lo) * esz : nullptr, sf,
                                            (uint64_t)(hi - lo) * esz, f);
        }
      }
      // postPeer (prims_simple.h:177-188): every wave's FIFO stores acknowledged and FIFO loads
      // returned, then one lane posts for the workgroup. FIFO bytes are written and read only with
      // system-coherent accesses, so no cache write-back or invalidate is needed (the hand-off form
      // "sc1 stores and loads both sides" of MI355X_MICROARCH.md, Guideline 16).
      drain();
      __syncthreads();
#pragma unroll
      for (int i = 0; i < NR; i++) recvStep[i] += a.stepPerSlice;
#pragma unroll
      for (int i = 0; i < NS; i++) sendStep[i] += a.stepPerSlice;
      if (threadIdx.x == 0) {
#pragma unroll
        for (int i = 0; i < NR; i++) ctr_st(recvHead[i], recvStep[i]);
#pragma unroll
        for (int i = 0; i < NS; i++) ctr_st(sendTail[i], sendStep[i]);
      }
      offset += sliceSize;
    }
    return true;
  }
};

template <int D, int OP, bool IsMin>
using RingPrims = ResPrims<D, OP, IsMin, 1, 1>;

// runRing for ncclAllReduce (all_reduce.h:12-84), one rank's view of one channel part. Primitive
// shapes op<user src, recv, user dst, send>: sendInput <1,0,0,1>, recvReduceSend <1,1,0,1>,
// recvReduceCopySend <1,1,1,1>, recvCopySend <0,1,1,1>, recvOutput <0,1,1,0>, recvReduceCopy <1,1,1,0>,
// copySend <1,0,1,1> (prims_simple.h:897-976).
template <int D, int OP, bool IsMin>
__device__ __forceinline__ void run_all_reduce(RingPrims<D, OP, IsMin>& p, int rank, int64_t partOffset, int64_t partCount) {
  const int nranks = p.a.nRanks;
  int64_t chunkCount = p.a.chunkCount;
  const int64_t loopCount = nranks * chunkCount;
  constexpr int64_t epp = 16 / RingPrims<D, OP, IsMin>::esz;
  auto modRanks = [&](int r) { return r - (r >= nranks ? nranks : 0); };
  for (int64_t elemOffset = 0; elemOffset < partCount; elemOffset += loopCount) {
    const int64_t remCount = partCount - elemOffset;
    if (remCount < loopCount) chunkCount = ((remCount + nranks - 1) / nranks + epp - 1) / epp * epp;
    auto at = [&](int chunk, int64_t* offset) {
      const int64_t chunkOffset = chunk * chunkCount;
      *offset = partOffset + elemOffset + chunkOffset;
      return imin(chunkCount, remCount - chunkOffset);
    };
    int64_t offset, nelem;
    nelem = at(modRanks(rank + nranks - 1), &offset);  // step 0: push data to the next rank
    if (!p.template op<true, false, false, true>(offset, -1, nelem, false)) return;
    for (int j = 2; j < nranks; ++j) {  // k-2 steps: reduce and copy to the next rank
      nelem = at(modRanks(rank + nranks - j), &offset);
      if (!p.template op<true, true, false, true>(offset, -1, nelem, false)) return;
    }
    nelem = at(rank, &offset);  // step k-1: reduce this chunk -> final result, stored and pushed
    if (!p.template op<true, true, true, true>(offset, offset, nelem, true)) return;
    for (int j = 1; j < nranks - 1; ++j) {  // k-2 steps: copy to the next rank
      nelem = at(modRanks(rank + nranks - j), &offset);
      if (!p.template op<false, true, true, true>(-1, offset, nelem, false)) return;
    }
    nelem = at(modRanks(rank + 1), &offset);  // final copy from the FIFO to the output
    if (!p.template op<false, true, true, false>(-1, offset, nelem, false)) return;
  }
}

// runRing for ncclReduceScatter (reduce_scatter.h:12-52): a.count is the per-rank recvcount; rank
// d's segment starts at d * count in every sendbuff.
template <int D, int OP, bool IsMin>
__device__ __forceinline__ void run_reduce_scatter(RingPrims<D, OP, IsMin>& p, int r, int64_t partOffset, int64_t partCount) {
  const int nranks = p.a.nRanks;
  const int64_t count = p.a.count, chunkCount = p.a.chunkCount;
  for (int64_t elemOffset = 0; elemOffset < partCount; elemOffset += chunkCount) {
    const int64_t nelem = imin(chunkCount, partCount - elemOffset);
    const int64_t dataOffset = partOffset + elemOffset;
    int rankDest = (r + nranks - 1) % nranks;
    if (!p.template op<true, false, false, true>(dataOffset + rankDest * count, -1, nelem, false)) return;
    for (int j = 2; j < nranks; ++j) {
      rankDest = (r + nranks - j) % nranks;
      if (!p.template op<true, true, false, true>(dataOffset + rankDest * count, -1, nelem, false)) return;
    }
    if (!p.template op<true, true, true, false>(dataOffset + (int64_t)r * count, dataOffset, nelem, true)) return;
  }
}

// runRing for ncclAllGather (all_gather.h:12-66): a.count is the per-rank sendcount; in place when
// the input chunk already sits at its place in the output (:52-56).
template <int D, int OP, bool IsMin>
__device__ __forceinline__ void run_all_gather(RingPrims<D, OP, IsMin>& p, int r, int64_t partOffset, int64_t partCount) {
  constexpr int esz = RingPrims<D, OP, IsMin>::esz;
  const int nranks = p.a.nRanks;
  const int64_t count = p.a.count, chunkCount = p.a.chunkCount;
  for (int64_t elemOffset = 0; elemOffset < partCount; elemOffset += chunkCount) {
    const int64_t nelem = imin(chunkCount, partCount - elemOffset);
    const int64_t dataOffset = partOffset + elemOffset;
    int64_t offset = dataOffset + (int64_t)r * count;
    const bool inPlace = p.input + dataOffset * esz == p.output + offset * esz;
    if (!(inPlace ? p.template op<true, false, false, true>(dataOffset, -1, nelem, false)
                  : p.template op<true, false, true, true>(dataOffset, offset, nelem, false)))
      return;
    for (int j = 1; j < nranks - 1; ++j) {
      offset = dataOffset + (int64_t)((r + nranks - j) % nranks) * count;
      if (!p.template op<false, true, true, true>(-1, offset, nelem, false)) return;
    }
    offset = dataOffset + (int64_t)((r + 1) % nranks) * count;
    if (!p.template op<false, true, true, false>(-1, offset, nelem, false)) return;
  }
}

// runRing for ncclReduce (reduce.h:12-50) and ncclBroadcast (broadcast.h:12-58), ProtoSimple<1,1>.
template <int D, int OP, bool IsMin>
__device__ __forceinline__ void run_reduce(RingPrims<D, OP, IsMin>& p, int r, int64_t partOffset, int64_t partCount) {
  const int nranks = p.a.nRanks, root = p.a.root, prevRank = (r + nranks - 1) % nranks;
  for (int64_t elemOffset = 0; elemOffset < partCount; elemOffset += p.a.chunkCount) {
    const int64_t offset = partOffset + elemOffset;
    const int64_t nelem = imin(p.a.chunkCount, partCount - elemOffset);
    bool ok;
    if (prevRank == root) ok = p.template op<true, false, false, true>(offset, -1, nelem, false);
    else if (r == root) ok = p.template op<true, true, true, false>(offset, offset, nelem, true);
    else ok = p.template op<true, true, false, true>(offset, -1, nelem, false);
    if (!ok) return;
  }
}
template <int D, int OP, bool IsMin>
__device__ __forceinline__ void run_broadcast(RingPrims<D, OP, IsMin>& p, int r, int64_t partOffset, int64_t partCount) {
  const int nranks = p.a.nRanks, root = p.a.root, nextRank = (r + 1) % nranks;
  for (int64_t elemOffset = 0; elemOffset < partCount; elemOffset += p.a.chunkCount) {
    const int64_t offset = partOffset + elemOffset;
    const int64_t nelem = imin(p.a.chunkCount, partCount - elemOffset);
    bool ok;
    if (r == root)
      ok = p.input == p.output ? p.template op<true, false, false, true>(offset, -1, nelem, false)
                               : p.template op<true, false, true, true>(offset, offset, nelem, false);
    else if (nextRank == root) ok = p.template op<false, true, true, false>(-1, offset, nelem, false);
    else ok = p.template op<false, true, true, true>(-1, offset, nelem, false);
    if (!ok) return;
  }
}

template <int D, int OP, bool IsMin>
__device__ __forceinline__ ResScalars scalars_of(const ResParams& a) {
  return {a.chunkCount, a.stepElems, a.count, a.stepBytes, a.redArg, a.timeoutTicks, a.status,
          a.stepPerSlice, a.slicePerChunk, a.team, a.nRanks, a.root};
}

template <int D, int OP, bool IsMin>
__global__ __launch_bounds__(kBlock) void ring_resident(ResParams a) {
  __shared__ ResShared sh;
  const int member = blockIdx.x % a.team;
  const int part = (blockIdx.x / a.team) % a.nParts;
  const int rank = a.rankOf[blockIdx.x / (a.team * a.nParts)];
  const ResConn& c = a.conns[a.partChannel[part] * a.nRanks + rank];
  RingPrims<D, OP, IsMin> p{scalars_of<D, OP, IsMin>(a)};
  p.input = a.input[rank];
  p.output = a.output[rank];
  p.member = member;
  p.nRecv = p.nSend = 1;
  p.recvFifo[0] = c.recvFifo;
  p.sendFifo[0] = c.sendFifo;
  p.recvTail[0] = c.recvCtr + (size_t)member * kResCtrBytes;
  p.recvHead[0] = p.recvTail[0] + kResHeadOff;
  p.sendTail[0] = c.sendCtr + (size_t)member * kResCtrBytes;
  p.sendHead[0] = p.sendTail[0] + kResHeadOff;
  p.sh = &sh;
  p.attach();
  const int64_t off = a.partOffset[part], cnt = a.partCount[part];
  switch (a.coll) {
    case kResAllReduce: run_all_reduce(p, rank, off, cnt); break;
    case kResReduceScatter: run_reduce_scatter(p, rank, off, cnt); break;
    case kResAllGather: run_all_gather(p, rank, off, cnt); break;
    case kResReduce: run_reduce(p, rank, off, cnt); break;
    case kResBroadcast: run_broadcast(p, rank, off, cnt); break;
  }
}

// runTreeSplit for ncclAllReduce (all_reduce.h:150-230), ProtoSimple<1,1>. Each (rank, channel) has
// two teams, as the reference splits a block's threads: role 0 reduces up (recv from the children,
// send to the parent: FanAsymmetric<3,1>), role 1 broadcasts down (recv from the parent, send to the
// children: FanAsymmetric<1,3>). The root's role 0 does both in one recvReduceCopySend over its
// children (FanSymmetric<3>); its role 1 has nothing to do.
template <int D, int OP, bool IsMin, int MR, int MS>
__device__ __forceinline__ void tree_role(const ResParams& a, ResShared* sh, const ResTreeConn& t, int rank, int role,
                                          int member, int64_t off, int64_t cnt) {
  ResPrims<D, OP, IsMin, MR, MS> p{scalars_of<D, OP, IsMin>(a)};
  p.input = a.input[rank];
  p.output = a.output[rank];
  p.member = member;
  p.sh = sh;
  const size_t m = (size_t)member * kResCtrBytes;
  const bool up = role == 0;
  p.nRecv = up ? t.nDown : 1;
  p.nSend = up ? (t.root ? t.nDown : 1) : t.nDown;
#pragma unroll
  for (int i = 0; i < MR; i++) {  // unused entries are never dereferenced (nRecv / nSend bound every use)
    p.recvFifo[i] = up ? t.upRecvFifo[i] : t.downRecvFifo;
    p.recvTail[i] = (up ? t.upRecvCtr[i] : t.downRecvCtr) + m;
    p.recvHead[i] = p.recvTail[i] + kResHeadOff;
  }
#pragma unroll
  for (int i = 0; i < MS; i++) {
    p.sendFifo[i] = up && !t.root ? t.upSendFifo : t.downSendFifo[i];
    p.sendTail[i] = (up && !t.root ? t.upSendCtr : t.downSendCtr[i]) + m;
    p.sendHead[i] = p.sendTail[i] + kResHeadOff;
  }
  p.attach();
  const bool leaf = t.nDown == 0;
  for (int64_t elemOffset = 0; elemOffset < cnt; elemOffset += a.chunkCount) {
    const int64_t offset = off + elemOffset;
    const int64_t nelem = imin(a.chunkCount, cnt - elemOffset);
    bool ok;
    if (t.root) ok = p.template op<true, true, true, true, /*Sym=*/true>(offset, offset, nelem, true);
    else if (up) ok = leaf ? p.template op<true, false, false, true>(offset, -1, nelem, false)
                           : p.template op<true, true, false, true>(offset, -1, nelem, false);
    else ok = leaf ? p.template op<false, true, true, false>(-1, offset, nelem, false)
                   : p.template op<false, true, true, true>(-1, offset, nelem, false);
    if (!ok) return;
  }
}

template <int D, int OP, bool IsMin>
__global__ __launch_bounds__(kBlock) void tree_resident(ResParams a) {
  __shared__ ResShared sh;
  const int member = blockIdx.x % a.team;
  const int role = (blockIdx.x / a.team) % 2;
  const int part = (blockIdx.x / (2 * a.team)) % a.nParts;
  const int rank = a.rankOf[blockIdx.x / (2 * a.team * a.nParts)];
  const ResTreeConn& t = a.tree[a.partChannel[part] * a.nRanks + rank];
  const int64_t off = a.partOffset[part], cnt = a.partCount[part];
  if (t.root) {
    if (role == 0) tree_role<D, OP, IsMin, 3, 3>(a, &sh, t, rank, 0, member, off, cnt);
  } else if (role == 0) {
    tree_role<D, OP, IsMin, 3, 1>(a, &sh, t, rank, 0, member, off, cnt);
  } else {
    tree_role<D, OP, IsMin, 1, 3>(a, &sh, t, rank, 1, member, off, cnt);
  }
}

template <int D, int OP>
static const void* kernel_op(uint64_t redArg, bool tree) {
  if constexpr (OP == nexrDevMinMax) {
    if ((redArg & 1) == 0)  // isMin, reduce_kernel.h:64
      return tree ? (const void*)&tree_resident<D, OP, true> : (const void*)&ring_resident<D, OP, true>;
  }
  return tree ? (const void*)&tree_resident<D, OP, false> : (const void*)&ring_resident<D, OP, false>;
}

template <int D>
static const void* kernel_for(int op, uint64_t redArg, bool tree) {
  switch (op) {
    case nexrDevSum: return kernel_op<D, nexrDevSum>(redArg, tree);
    case nexrDevProd: return kernel_op<D, nexrDevProd>(redArg, tree);
    case nexrDevMinMax: return kernel_op<D, nexrDevMinMax>(redArg, tree);
    case nexrDevPreMulSum: return kernel_op<D, nexrDevPreMulSum>(redArg, tree);
    case nexrDevSumPostDiv:
      if constexpr (Ty<D>::kIsInt) return kernel_op<D, nexrDevSumPostDiv>(redArg, tree);
      break;
  }
  return nullptr;
}

#define NEXR_CAT2(a, b) a##b
#define NEXR_CAT(a, b) NEXR_CAT2(a, b)

hipError_t NEXR_CAT(launch_resident_dt, NEXR_DT)(int op, const ResParams& p, int grid, hipStream_t s) {
  const void* fn = kernel_for<NEXR_DT>(op, p.redArg, p.coll == kResTreeAllReduce);
  if (!fn) return hipErrorInvalidValue;
  void* args[] = {const_cast<ResParams*>(&p)};
  return hipLaunchKernel(fn, dim3(grid), dim3(kBlock), args, 0, s);
}

hipError_t NEXR_CAT(resident_blocks_per_cu_dt, NEXR_DT)(int op, uint64_t redArg, int coll, int* blocks) {
  const void* fn = kernel_for<NEXR_DT>(op, redArg, coll == kResTreeAllReduce);
  if (!fn) return hipErrorInvalidValue;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, fn, kBlock, 0);
}

}  // namespace nexr
