// nexr_ring.cpp — CPU-emulated ring all-reduce (include/nexr_ring.h): the reference's own
// collective schedule, restated on host threads, calling the reduce-copy ABI at exactly the
// reduceCopy sites of Primitives::genericOp. This is the drop-in demonstration for BASELINE
// configs[0] ("fp32 sum all-reduce, 4 MiB, 2 CPU-emulated ranks"): the schedule is unchanged,
// only the primitive underneath is the MI355X kernel.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <thread>
#include <vector>

#include "../../include/nexr_ring.h"

namespace {

constexpr int kSteps = 8;                                // NCCL_STEPS (src/include/device.h:649)
constexpr int kSliceSteps = kSteps / 4;                  // ALLREDUCE_SLICESTEPS (collectives.h:17)
constexpr int kChunkSteps = kSteps / 2;                  // ALLREDUCE_CHUNKSTEPS (collectives.h:18)
constexpr int kSlicePerChunk = kChunkSteps / kSliceSteps;
constexpr size_t kDefaultBuffBytes = 4u << 20;           // NCCL_BUFFSIZE default (init.cc:620-634)
constexpr size_t kDefaultLLBuffBytes = 8 * 512 * kSteps * 16;  // DEFAULT_LL_BUFFSIZE (init.cc:618)
constexpr size_t kDefaultLL128BuffBytes = 120 * 640 * kSteps * 8;  // DEFAULT_LL128_BUFFSIZE (init.cc:619)

// One directed connection prev -> r. The FIFO belongs to the receiver (the sender writes into it,
// like a P2P/SHM transport's recv buffer, src/include/device.h:753-771).
struct Conn {
  char* fifo = nullptr;
  alignas(64) std::atomic<uint64_t> tail{0};  // steps published by the sender   (postPeer, Send)
  alignas(64) std::atomic<uint64_t> head{0};  // steps released by the receiver  (postPeer, Recv)
};

int64_t divUp(int64_t a, int64_t b) { return (a + b - 1) / b; }
int64_t alignUp(int64_t a, int64_t b) { return divUp(a, b) * b; }

}  // namespace

struct nexrRingComm {
  nexrRingConfig cfg;
  size_t stepBytes = 0;
  std::vector<Conn*> conns;          // conns[r]: connection into rank r from rank r-1
  std::vector<uint64_t> recvStep;    // per rank: next step to consume from conns[r]
  std::vector<uint64_t> sendStep;    // per rank: next step to produce into conns[(r+1)%n]
  std::vector<int> devices;
  std::vector<hipStream_t> streams;
  std::vector<uint32_t*> status;     // LL: per-rank pinned status word the kernel reports timeouts in
  bool ll = false;     // LL or LL128: one FIFO step per primitive call, data readiness in line flags
  int proto = nexrRingProtoSimple;
  bool pinnedStatus = false;  // status words from hipHostMalloc (else calloc)
  bool broken = false;
};

namespace {

struct Shared {
  std::atomic<bool> abort{false};
  std::atomic<int> firstError{0};
  void fail(nexrResult_t r) {
    int expected = 0;
    firstError.compare_exchange_strong(expected, (int)r);
    abort.store(true);
  }
};

// One rank's Primitives<T, RedOp, FanSymmetric<1>, 1, ProtoSimple> (prims_simple.h), host side.
struct Prims {
  nexrRingComm* c;
  Shared* sh;
  int rank;
  Conn* recvConn;
  Conn* sendConn;
  const char* userInput;
  char* userOutput;
  size_t esz;
  int64_t stepSize;  // elements per FIFO step (prims_simple.h:607)
  int datatype, devOp;
  uint64_t redOpArgs[1];
  nexrReduceCopyFn fn;
  nexrReduceCopyLLFn llFn;
  nexrReduceCopyLL128Fn ll128Fn;
  uint32_t* status;
  hipStream_t stream;
  bool device;

  // Spin until `a` >= target (waitPeer's connStepCache loop, prims_simple.h:116-123), bounded and
  // abortable like checkAbort (primitives.h:142-156).
  bool waitAtLeast(std::atomic<uint64_t>& a, uint64_t target) {
    if (a.load(std::memory_order_acquire) >= target) return true;
    const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 0;; spins++) {
      if (a.load(std::memory_order_acquire) >= target) return true;
      if (sh->abort.load(std::memory_order_relaxed)) return false;
      if ((spins & 1023) == 0 &&
          std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) {
        sh->fail(nexrInternalError);
        return false;
      }
      std::this_thread::yield();
    }
  }

  // genericOp<DirectRecv=0, DirectSend=0, Recv, Send, SrcBuf, DstBuf> (prims_simple.h:190-330),
  // with the non-direct FIFO pointers (waitPeer :150-164 default branch).
  bool genericOp(bool Recv, bool Send, bool Src, bool Dst, int64_t srcIx, int64_t dstIx, int64_t nelem,
                 bool postOp) {
    nelem = nelem < 0 ? 0 : nelem;
    int64_t sliceSize = stepSize * kSliceSteps;
    sliceSize = std::max(divUp(nelem, 16 * kSlicePerChunk) * 16, sliceSize / 32);
    int64_t offset = 0;
    for (int slice = 0; slice < kSlicePerChunk; slice++) {
      sliceSize = std::min(sliceSize, nelem - offset);
      if (sliceSize < 0) sliceSize = 0;
      uint64_t& rs = c->recvStep[rank];
      uint64_t& ss = c->sendStep[rank];
      const char* recvPtr = nullptr;
      char* sendPtr = nullptr;
      if (Recv) {  // wait for the peer's data: tail >= step + StepPerSlice
        if (!waitAtLeast(recvConn->tail, rs + kSliceSteps)) return false;
        recvPtr = recvConn->fifo + (rs % kSteps) * c->stepBytes;
      }
      if (Send) {  // wait for credit: head + NCCL_STEPS >= step + StepPerSlice
        if (ss + kSliceSteps > (uint64_t)kSteps && !waitAtLeast(sendConn->head, ss + kSliceSteps - kSteps))
          return false;
        sendPtr = sendConn->fifo + (ss % kSteps) * c->stepBytes;
      }
      if (sliceSize > 0) {
        // srcs: local buffer at index 0 (if Src), peers after it; dsts: user output at 0 (if Dst),
        // next peer after it (prims_simple.h:131-132, :238-242).
        const void* srcs[2];
        void* dsts[2];
        int ns = 0, nd = 0;
        if (Src) srcs[ns++] = userInput + (srcIx + offset) * esz;
        if (Recv) srcs[ns++] = recvPtr;
        if (Dst) dsts[nd++] = userOutput + (dstIx + offset) * esz;
        if (Send) dsts[nd++] = sendPtr;
        // PreOpSrcs = SrcBuf != Input ? 0 : 1 (prims_simple.h:279-280); preOpArgs = redOpArgs.
        const int nPre = Src ? 1 : 0;
        nexrResult_t r = fn(ns, srcs, nd, dsts, (size_t)sliceSize, datatype, devOp, redOpArgs[0], nPre,
                            nPre ? redOpArgs : nullptr, postOp ? 1 : 0, (nexrStream_t)stream);
        if (r == nexrSuccess && device) {
          hipError_t e = hipStreamSynchronize(stream);  // data complete before the step is posted
          if (e != hipSuccess) r = nexrUnhandledCudaError;
        }
        if (r != nexrSuccess) {
          sh->fail(r);
          return false;
        }
      }
      // postPeer (prims_simple.h:177-188): release the slot / publish the data.
      if (Recv) {
        rs += kSliceSteps;
        recvConn->head.store(rs, std::memory_order_release);
      }
      if (Send) {
        ss += kSliceSteps;
        sendConn->tail.store(ss, std::memory_order_release);
      }
      offset += sliceSize;
    }
    return true;
  }
  // LLGenericOp<RECV, SEND, SrcBuf, DstBuf> (prims_ll.h:218-283): one FIFO step per call. The
  // sender waits for a credit (waitSend :55-75); the receiver's data readiness is the line flags
  // NCCL_LL_FLAG(step+1) (:42-43). The host additionally waits for the sender's step so that the
  // kernel's flag poll succeeds at once: two emulated ranks may share one GPU, and a kernel spinning
  // on a producer that cannot be scheduled beside it must never be launched.
  bool genericOpLL(bool Recv, bool Send, bool Src, bool Dst, int64_t srcIx, int64_t dstIx, int64_t nelem,
                   bool postOp) {
    nelem = nelem < 0 ? 0 : nelem;
    uint64_t& rs = c->recvStep[rank];
    uint64_t& ss = c->sendStep[rank];
    if (Send && ss + 1 > (uint64_t)kSteps && !waitAtLeast(sendConn->head, ss + 1 - kSteps)) return false;
    if (Recv && !waitAtLeast(recvConn->tail, rs + 1)) return false;
    if (nelem > 0) {
      const void* recvLines[1] = {recvConn->fifo + (rs % kSteps) * c->stepBytes};
      void* sendLines[1] = {sendConn->fifo + (ss % kSteps) * c->stepBytes};
      const uint32_t recvFlag[1] = {(uint32_t)(rs + 1)};  // NCCL_LL_FLAG(recvStep+1)
      const uint32_t sendFlag[1] = {(uint32_t)(ss + 1)};
      if (status) *status = 0;
      const uint32_t tmo = (uint32_t)((c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 1000u);
      nexrResult_t r;
      if (c->proto == nexrRingProtoLL128) {  // 64-bit flags = step + 1 (prims_ll128.h:49-50)
        const uint64_t rf[1] = {rs + 1}, sf[1] = {ss + 1};
        r = ll128Fn(Src ? userInput + srcIx * esz : nullptr, Src ? 1 : 0, Recv ? 1 : 0, recvLines, rf,
                    Dst ? userOutput + dstIx * esz : nullptr, Send ? 1 : 0, sendLines, sf, (size_t)nelem, datatype,
                    devOp, redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      } else {
        r = llFn(Src ? userInput + srcIx * esz : nullptr, Src ? 1 : 0, Recv ? 1 : 0, recvLines, recvFlag,
                 Dst ? userOutput + dstIx * esz : nullptr, Send ? 1 : 0, sendLines, sendFlag, (size_t)nelem,
                 datatype, devOp, redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      }
      if (r == nexrSuccess && device && hipStreamSynchronize(stream) != hipSuccess) r = nexrUnhandledCudaError;
      if (r == nexrSuccess && status && __atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) r = nexrInternalError;
      if (r != nexrSuccess) {
        sh->fail(r);
        return false;
      }
    }
    if (Recv) {  // postRecv (:80-83)
      rs += 1;
      recvConn->head.store(rs, std::memory_order_release);
    }
    if (Send) {  // incSend (:85-93); the flag-wrap cleanup at NCCL_LL_CLEAN_MASK needs ~2^31 steps
      ss += 1;
      sendConn->tail.store(ss, std::memory_order_release);
    }
    return true;
  }
  bool op(bool Recv, bool Send, bool Src, bool Dst, int64_t srcIx, int64_t dstIx, int64_t n, bool postOp) {
    return c->ll ? genericOpLL(Recv, Send, Src, Dst, srcIx, dstIx, n, postOp)
                 : genericOp(Recv, Send, Src, Dst, srcIx, dstIx, n, postOp);
  }
  bool directSend(int64_t inpIx, int64_t n) { return op(false, true, true, false, inpIx, -1, n, false); }
  bool directRecvReduceDirectSend(int64_t inpIx, int64_t n) { return op(true, true, true, false, inpIx, -1, n, false); }
  bool directRecvReduceCopyDirectSend(int64_t inpIx, int64_t outIx, int64_t n, bool postOp) {
    return op(true, true, true, true, inpIx, outIx, n, postOp);
  }
  bool directRecvCopyDirectSend(int64_t outIx, int64_t n) { return op(true, true, false, true, -1, outIx, n, false); }
  bool directRecv(int64_t outIx, int64_t n) { return op(true, false, false, true, -1, outIx, n, false); }
};

// runRing<T, RedOp, ProtoSimple> (all_reduce.h:12-84) for one rank, 1 channel (gridOffset 0,
// channelCount = count, chunkCount = chunkSize / sizeof(T): enqueue.cc:1993-1996, :655-678).
void runRing(Prims& p, int nranks, int64_t count) {
  const int ringIx = p.rank;
  // SIMPLE: chunkSize = stepSize * chunkSteps; LL: stepSize / 2; LL128: stepSize / 16 * 15, aligned
  // to the 1920-B grain (enqueue.cc:1993-1999, :2062)
  int64_t chunkBytes = (int64_t)(p.c->stepBytes * kChunkSteps);
  if (p.c->proto == nexrRingProtoLL) chunkBytes = (int64_t)(p.c->stepBytes / 2);
  if (p.c->proto == nexrRingProtoLL128) chunkBytes = (int64_t)(p.c->stepBytes / 16 * 15) / 1920 * 1920;
  int64_t chunkCount = chunkBytes / (int64_t)p.esz;
  const int64_t loopCount = nranks * chunkCount;
  auto modRanks = [&](int r) { return r - (r >= nranks ? nranks : 0); };
  for (int64_t elemOffset = 0; elemOffset < count; elemOffset += loopCount) {
    const int64_t remCount = count - elemOffset;
    if (remCount < loopCount) chunkCount = alignUp(divUp(remCount, nranks), 16 / (int64_t)p.esz);
    auto at = [&](int chunk, int64_t* offset) {
      const int64_t chunkOffset = chunk * chunkCount;
      *offset = elemOffset + chunkOffset;
      return std::min(chunkCount, remCount - chunkOffset);
    };
    int64_t offset, nelem;
    // step 0: push data to next GPU
    nelem = at(modRanks(ringIx + nranks - 1), &offset);
    if (!p.directSend(offset, nelem)) return;
    // k-2 steps: reduce and copy to next GPU
    for (int j = 2; j < nranks; ++j) {
      nelem = at(modRanks(ringIx + nranks - j), &offset);
      if (!p.directRecvReduceDirectSend(offset, nelem)) return;
    }
    // step k-1: reduce this buffer and data -> final result, stored and pushed
    nelem = at(ringIx, &offset);
    if (!p.directRecvReduceCopyDirectSend(offset, offset, nelem, /*postOp=*/true)) return;
    // k-2 steps: copy to next GPU
    for (int j = 1; j < nranks - 1; ++j) {
      nelem = at(modRanks(ringIx + nranks - j), &offset);
      if (!p.directRecvCopyDirectSend(offset, nelem)) return;
    }
    // final copy from buffer to dest
    nelem = at(modRanks(ringIx + 1), &offset);
    if (!p.directRecv(offset, nelem)) return;
  }
}

nexrResult_t defaultHostFn(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t n, int dt,
                           int op, uint64_t arg, int nPre, const uint64_t* pre, int post, nexrStream_t s) {
  return nexrReduceCopyHost(nSrcs, srcs, nDsts, dsts, n, dt, op, arg, nPre, pre, post, s);
}
nexrResult_t defaultLLFn(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                         const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                         const uint32_t* sendFlags, size_t n, int dt, int op, uint64_t arg, int post, uint32_t* status,
                         uint32_t timeoutUs, nexrStream_t s) {
  return nexrReduceCopyLL(src, srcIsInput, nRecv, recvLines, recvFlags, dst, nSend, sendLines, sendFlags, n, dt, op,
                          arg, post, status, timeoutUs, s);
}
nexrResult_t defaultLL128Fn(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                            const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                            const uint64_t* sendFlags, size_t n, int dt, int op, uint64_t arg, int post,
                            uint32_t* status, uint32_t timeoutUs, nexrStream_t s) {
  return nexrReduceCopyLL128(src, srcIsInput, nRecv, recvWire, recvFlags, dst, nSend, sendWire, sendFlags, n, dt, op,
                             arg, post, status, timeoutUs, s);
}
nexrResult_t defaultDeviceFn(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t n, int dt,
                             int op, uint64_t arg, int nPre, const uint64_t* pre, int post, nexrStream_t s) {
  return nexrReduceCopy(nSrcs, srcs, nDsts, dsts, n, dt, op, arg, nPre, pre, post, s);
}

}  // namespace

extern "C" {

NEXR_API nexrResult_t nexrRingCommCreate(nexrRingComm_t* out, const nexrRingConfig* cfg) {
  if (!out || !cfg || cfg->nRanks < 1 || cfg->nRanks > 1024) return nexrInvalidArgument;
  if (cfg->memMode != nexrRingHostMemory && cfg->memMode != nexrRingDeviceMemory) return nexrInvalidArgument;
  if (cfg->protocol != nexrRingProtoSimple && cfg->protocol != nexrRingProtoLL && cfg->protocol != nexrRingProtoLL128)
    return nexrInvalidArgument;
  // The LL/LL128 kernels poll live FIFO lines: they need device-visible lines, i.e. device memory,
  // unless the caller supplies its own step implementation (e.g. a CPU checker).
  if (cfg->memMode == nexrRingHostMemory && ((cfg->protocol == nexrRingProtoLL && !cfg->llFn) ||
                                             (cfg->protocol == nexrRingProtoLL128 && !cfg->ll128Fn)))
    return nexrInvalidUsage;
  auto* c = new nexrRingComm();
  c->cfg = *cfg;
  c->proto = cfg->protocol;
  c->ll = cfg->protocol != nexrRingProtoSimple;
  if (c->cfg.buffBytes == 0)
    c->cfg.buffBytes = c->proto == nexrRingProtoLL ? kDefaultLLBuffBytes
                       : c->proto == nexrRingProtoLL128 ? kDefaultLL128BuffBytes : kDefaultBuffBytes;
  if (c->cfg.buffBytes % (kSteps * 16) != 0 ||
      (c->proto == nexrRingProtoLL128 && c->cfg.buffBytes % (kSteps * 2048) != 0)) {  // whole LL128 slices
    delete c;
    return nexrInvalidArgument;
  }
  if (!c->cfg.fn) c->cfg.fn = cfg->memMode == nexrRingDeviceMemory ? defaultDeviceFn : defaultHostFn;
  if (!c->cfg.llFn) c->cfg.llFn = defaultLLFn;
  if (!c->cfg.ll128Fn) c->cfg.ll128Fn = defaultLL128Fn;
  c->stepBytes = c->cfg.buffBytes / kSteps;
  const int n = cfg->nRanks;
  c->recvStep.assign(n, 0);
  c->sendStep.assign(n, 0);
  c->devices.assign(n, 0);
  c->streams.assign(n, nullptr);
  c->status.assign(n, nullptr);
  int nDev = 0;
  const bool needHip = cfg->memMode == nexrRingDeviceMemory || (c->proto == nexrRingProtoSimple && !cfg->fn) ||
                       (c->proto == nexrRingProtoLL && !cfg->llFn) || (c->proto == nexrRingProtoLL128 && !cfg->ll128Fn);
  c->pinnedStatus = needHip;
  if (needHip) {
    if (hipGetDeviceCount(&nDev) != hipSuccess || nDev < 1) {
      delete c;
      return nexrUnhandledCudaError;
    }
  }
  for (int r = 0; r < n; r++) {
    c->conns.push_back(new Conn());
    if (nDev > 0) {
      c->devices[r] = r % nDev;
      if (hipSetDevice(c->devices[r]) != hipSuccess || hipStreamCreate(&c->streams[r]) != hipSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
    }
    if (c->ll && needHip) {  // pinned, device-mapped status word for the LL kernel's timeout report
      if (hipHostMalloc((void**)&c->status[r], sizeof(uint32_t), hipHostMallocMapped) != hipSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
      *c->status[r] = 0;
    } else if (c->ll) {  // CPU-side LL implementation: an ordinary host word
      c->status[r] = (uint32_t*)calloc(1, sizeof(uint32_t));
      if (!c->status[r]) {
        nexrRingCommDestroy(c);
        return nexrSystemError;
      }
    }
    if (cfg->memMode == nexrRingDeviceMemory) {
      if (hipMalloc((void**)&c->conns[r]->fifo, c->cfg.buffBytes) != hipSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
    } else {
      c->conns[r]->fifo = (char*)aligned_alloc(4096, c->cfg.buffBytes);
      if (!c->conns[r]->fifo) {
        nexrRingCommDestroy(c);
        return nexrSystemError;
      }
    }
  }
  if (cfg->memMode == nexrRingDeviceMemory && nDev > 1) {  // sender writes into the receiver's FIFO
    for (int r = 0; r < n; r++) {
      int a = c->devices[r], b = c->devices[(r + 1) % n];
      if (a != b) {
        (void)hipSetDevice(a);
        hipError_t e = hipDeviceEnablePeerAccess(b, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          nexrRingCommDestroy(c);
          return nexrUnhandledCudaError;
        }
        (void)hipGetLastError();
      }
    }
  }
  *out = c;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingAllReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op) {
  if (!c || !sendbuffs || !recvbuffs) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  const int n = c->cfg.nRanks;
  const size_t esz = nexrTypeSize(datatype);
  if (esz == 0 || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2) return nexrInvalidArgument;
  nexrDevRedOpFull red;
  nexrResult_t r = nexrHostToDevRedOp(&red, op, datatype, n);
  if (r != nexrSuccess) return r;
  for (int i = 0; i < n; i++)
    if (count > 0 && (!sendbuffs[i] || !recvbuffs[i])) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  const bool device = c->cfg.memMode == nexrRingDeviceMemory;

  if (n == 1) {  // ncclLaunchOneRank (onerank.cc:48-83)
    if (device) (void)hipSetDevice(c->devices[0]);
    if (red.op == nexrDevPreMulSum) {
      uint64_t arg = red.scalarArg;
      r = c->cfg.fn(1, sendbuffs, 1, recvbuffs, count, datatype, nexrDevPreMulSum, arg, 1, &arg, 1,
                    (nexrStream_t)c->streams[0]);
      if (r == nexrSuccess && device && hipStreamSynchronize(c->streams[0]) != hipSuccess) r = nexrUnhandledCudaError;
      return r;
    }
    if (sendbuffs[0] != recvbuffs[0]) {
      if (device) {
        if (hipMemcpy(recvbuffs[0], sendbuffs[0], count * esz, hipMemcpyDeviceToDevice) != hipSuccess)
          return nexrUnhandledCudaError;
      } else {
        memcpy(recvbuffs[0], sendbuffs[0], count * esz);
      }
    }
    return nexrSuccess;
  }

  Shared sh;
  std::vector<std::thread> threads;
  for (int rank = 0; rank < n; rank++) {
    threads.emplace_back([&, rank] {
      if (device || c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
      Prims p;
      p.c = c;
      p.sh = &sh;
      p.rank = rank;
      p.recvConn = c->conns[rank];
      p.sendConn = c->conns[(rank + 1) % n];
      p.userInput = (const char*)sendbuffs[rank];
      p.userOutput = (char*)recvbuffs[rank];
      p.esz = esz;
      p.stepSize = (int64_t)(c->stepBytes / esz);
      p.datatype = datatype;
      p.devOp = red.op;
      p.redOpArgs[0] = red.scalarArg;
      p.fn = c->cfg.fn;
      p.llFn = c->cfg.llFn;
      p.ll128Fn = c->cfg.ll128Fn;
      p.status = c->status[rank];
      p.stream = c->streams[rank];
      p.device = device;
      runRing(p, n, (int64_t)count);
    });
  }
  for (auto& t : threads) t.join();
  if (sh.firstError.load() != 0) {
    c->broken = true;  // step counters are mid-protocol: the communicator cannot be reused
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingCommDestroy(nexrRingComm_t c) {
  if (!c) return nexrInvalidArgument;
  for (size_t r = 0; r < c->conns.size(); r++) {
    Conn* k = c->conns[r];
    if (k->fifo) {
      if (c->cfg.memMode == nexrRingDeviceMemory) {
        (void)hipSetDevice(c->devices[r]);
        (void)hipFree(k->fifo);
      } else {
        free(k->fifo);
      }
    }
    delete k;
  }
  for (size_t r = 0; r < c->status.size(); r++)
    if (c->status[r]) {
      if (c->pinnedStatus) (void)hipHostFree(c->status[r]);
      else free(c->status[r]);
    }
  for (size_t r = 0; r < c->streams.size(); r++)
    if (c->streams[r]) {
      (void)hipSetDevice(c->devices[r]);
      (void)hipStreamDestroy(c->streams[r]);
    }
  delete c;
  return nexrSuccess;
}

}  // extern "C"
