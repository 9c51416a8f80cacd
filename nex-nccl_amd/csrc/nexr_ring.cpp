// nexr_ring.cpp — CPU-emulated ring all-reduce (include/nexr_ring.h): the reference's own
// collective schedule, restated on host threads, calling the reduce-copy ABI at exactly the
// reduceCopy sites of Primitives::genericOp. This is the drop-in demonstration for BASELINE
// configs[0] ("fp32 sum all-reduce, 4 MiB, 2 CPU-emulated ranks"): the schedule is unchanged,
// only the primitive underneath is the MI355X kernel.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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
struct ConnState {
  alignas(64) std::atomic<uint64_t> tail{0};  // steps published by the sender   (postPeer, Send)
  alignas(64) std::atomic<uint64_t> head{0};  // steps released by the receiver  (postPeer, Recv)
};
struct Conn {
  char* fifo = nullptr;
  ConnState own;
  ConnState* st = &own;  // the counters: `own` for thread ranks, a shared-memory slot for process ranks
};

// Process ranks (nexrPeerRingCommCreate): one POSIX shared-memory segment per communicator holds
// the rendezvous, every connection's head/tail counters and a common abort word. Slot r belongs to
// rank r: its FIFO's IPC handle and the counters of the connection INTO rank r.
constexpr uint32_t kPeerMagic = 0x6e657872u;  // "nexr"
struct PeerHeader {
  std::atomic<uint32_t> initState;  // 0 fresh, 1 being configured, 2 configured
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> left;
  std::atomic<uint32_t> abort;
  uint32_t magic, nRanks, protocol, pad;
  uint64_t buffBytes;
};
struct PeerSlot {
  hipIpcMemHandle_t fifoHandle;
  alignas(64) ConnState conn;
};
size_t peerShmBytes(int n) { return sizeof(PeerHeader) + (size_t)n * sizeof(PeerSlot); }
PeerHeader* peerHeader(void* base) { return (PeerHeader*)base; }
PeerSlot* peerSlot(void* base, int r) { return (PeerSlot*)((char*)base + sizeof(PeerHeader)) + r; }

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
  // Process ranks: this process is rank `self` only.
  bool peer = false;
  int self = 0;
  void* shm = nullptr;
  size_t shmBytes = 0;
  char shmName[256] = {0};
  char* peerFifo = nullptr;  // the next rank's FIFO, IPC-mapped into this process
  bool peerFifoIpc = false;
};

namespace {

struct Shared {
  std::atomic<bool> abort{false};
  std::atomic<int> firstError{0};
  std::atomic<uint32_t>* remoteAbort = nullptr;  // process ranks: the communicator-wide abort word
  void fail(nexrResult_t r) {
    int expected = 0;
    firstError.compare_exchange_strong(expected, (int)r);
    abort.store(true);
    if (remoteAbort) remoteAbort->store(1, std::memory_order_release);
  }
  bool aborted() const {
    return abort.load(std::memory_order_relaxed) || (remoteAbort && remoteAbort->load(std::memory_order_acquire));
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
      if (sh->aborted()) {
        sh->fail(nexrRemoteError);
        return false;
      }
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
        if (!waitAtLeast(recvConn->st->tail, rs + kSliceSteps)) return false;
        recvPtr = recvConn->fifo + (rs % kSteps) * c->stepBytes;
      }
      if (Send) {  // wait for credit: head + NCCL_STEPS >= step + StepPerSlice
        if (ss + kSliceSteps > (uint64_t)kSteps && !waitAtLeast(sendConn->st->head, ss + kSliceSteps - kSteps))
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
        recvConn->st->head.store(rs, std::memory_order_release);
      }
      if (Send) {
        ss += kSliceSteps;
        sendConn->st->tail.store(ss, std::memory_order_release);
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
    if (Send && ss + 1 > (uint64_t)kSteps && !waitAtLeast(sendConn->st->head, ss + 1 - kSteps)) return false;
    if (Recv && !waitAtLeast(recvConn->st->tail, rs + 1)) return false;
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
      recvConn->st->head.store(rs, std::memory_order_release);
    }
    if (Send) {  // incSend (:85-93); the flag-wrap cleanup at NCCL_LL_CLEAN_MASK needs ~2^31 steps
      ss += 1;
      sendConn->st->tail.store(ss, std::memory_order_release);
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

Prims makePrims(nexrRingComm* c, Shared* sh, int rank, Conn* recvConn, Conn* sendConn, const void* sendbuff,
                void* recvbuff, size_t esz, int datatype, const nexrDevRedOpFull& red, bool device) {
  Prims p;
  p.c = c;
  p.sh = sh;
  p.rank = rank;
  p.recvConn = recvConn;
  p.sendConn = sendConn;
  p.userInput = (const char*)sendbuff;
  p.userOutput = (char*)recvbuff;
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
  return p;
}

// ncclLaunchOneRank (onerank.cc:48-83) for rank `r`'s buffers.
nexrResult_t oneRank(nexrRingComm* c, int r, const void* sendbuff, void* recvbuff, size_t count, int datatype,
                     const nexrDevRedOpFull& red, size_t esz) {
  const bool device = c->cfg.memMode == nexrRingDeviceMemory;
  if (device) (void)hipSetDevice(c->devices[r]);
  if (red.op == nexrDevPreMulSum) {
    uint64_t arg = red.scalarArg;
    const void* srcs[1] = {sendbuff};
    void* dsts[1] = {recvbuff};
    nexrResult_t res = c->cfg.fn(1, srcs, 1, dsts, count, datatype, nexrDevPreMulSum, arg, 1, &arg, 1,
                                 (nexrStream_t)c->streams[r]);
    if (res == nexrSuccess && device && hipStreamSynchronize(c->streams[r]) != hipSuccess)
      res = nexrUnhandledCudaError;
    return res;
  }
  if (sendbuff != recvbuff) {
    if (device) {
      if (hipMemcpy(recvbuff, sendbuff, count * esz, hipMemcpyDeviceToDevice) != hipSuccess)
        return nexrUnhandledCudaError;
    } else {
      memcpy(recvbuff, sendbuff, count * esz);
    }
  }
  return nexrSuccess;
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

  if (n == 1) return oneRank(c, 0, sendbuffs[0], recvbuffs[0], count, datatype, red, esz);

  Shared sh;
  std::vector<std::thread> threads;
  for (int rank = 0; rank < n; rank++) {
    threads.emplace_back([&, rank] {
      if (device || c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
      Prims p = makePrims(c, &sh, rank, c->conns[rank], c->conns[(rank + 1) % n], sendbuffs[rank], recvbuffs[rank],
                          esz, datatype, red, device);
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
  if (c->peer) {
    if (!c->streams.empty() && c->streams[c->self]) (void)hipStreamSynchronize(c->streams[c->self]);
    if (c->peerFifoIpc && c->peerFifo) (void)hipIpcCloseMemHandle(c->peerFifo);
    if (c->shm) {
      PeerHeader* h = peerHeader(c->shm);
      // The last rank to leave removes the segment's name (each rank still unmaps its own view).
      if (h->joined.load() > 0 && h->left.fetch_add(1) + 1 == h->nRanks) shm_unlink(c->shmName);
      munmap(c->shm, c->shmBytes);
    }
    for (size_t r = 0; r < c->conns.size(); r++) {
      c->conns[r]->st = &c->conns[r]->own;           // counters lived in the unmapped segment
      if ((int)r != c->self) c->conns[r]->fifo = nullptr;  // only this rank's FIFO is owned here
    }
  }
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

// ---- process ranks: one process per GPU, FIFOs shared over IPC (xGMI between GPUs) ----------------
// The reference's P2P transport in write mode: the receiver allocates its FIFO and exports it
// (src/transport/p2p.cc:231-240), the sender maps it with cudaIpcOpenMemHandle(…LazyEnablePeerAccess)
// (:299) and its reduce-copy writes straight into it (NCCL_P2P_WRITE, :402); send/recv head and
// tail counters pair up as in p2pSendConnect/p2pRecvConnect (:514-515, :542-543). Here the steps are
// driven by each rank's host thread, so the counters live in host shared memory.
NEXR_API nexrResult_t nexrPeerRingCommCreate(nexrRingComm_t* out, const nexrPeerRingConfig* cfg) {
  if (!out || !cfg || cfg->nRanks < 1 || cfg->nRanks > 1024 || cfg->rank < 0 || cfg->rank >= cfg->nRanks)
    return nexrInvalidArgument;
  if (!cfg->shmName || cfg->shmName[0] != '/' || strlen(cfg->shmName) >= 255 || strchr(cfg->shmName + 1, '/'))
    return nexrInvalidArgument;
  if (cfg->protocol != nexrRingProtoSimple && cfg->protocol != nexrRingProtoLL && cfg->protocol != nexrRingProtoLL128)
    return nexrInvalidArgument;
  nexrRingConfig rc;
  memset(&rc, 0, sizeof(rc));
  rc.nRanks = cfg->nRanks;
  rc.buffBytes = cfg->buffBytes;
  rc.memMode = nexrRingDeviceMemory;
  rc.timeoutMs = cfg->timeoutMs;
  rc.protocol = cfg->protocol;
  auto* c = new nexrRingComm();
  c->cfg = rc;
  c->proto = cfg->protocol;
  c->ll = cfg->protocol != nexrRingProtoSimple;
  if (c->cfg.buffBytes == 0)
    c->cfg.buffBytes = c->proto == nexrRingProtoLL ? kDefaultLLBuffBytes
                       : c->proto == nexrRingProtoLL128 ? kDefaultLL128BuffBytes : kDefaultBuffBytes;
  if (c->cfg.buffBytes % (kSteps * 16) != 0 || (c->proto == nexrRingProtoLL128 && c->cfg.buffBytes % (kSteps * 2048) != 0)) {
    delete c;
    return nexrInvalidArgument;
  }
  c->cfg.fn = defaultDeviceFn;
  c->cfg.llFn = defaultLLFn;
  c->cfg.ll128Fn = defaultLL128Fn;
  c->stepBytes = c->cfg.buffBytes / kSteps;
  c->peer = true;
  const int n = cfg->nRanks, me = cfg->rank, next = (me + 1) % n;
  c->self = me;
  c->recvStep.assign(n, 0);
  c->sendStep.assign(n, 0);
  c->devices.assign(n, cfg->device);
  c->streams.assign(n, nullptr);
  c->status.assign(n, nullptr);
  c->pinnedStatus = true;
  for (int r = 0; r < n; r++) c->conns.push_back(new Conn());
  strncpy(c->shmName, cfg->shmName, sizeof(c->shmName) - 1);
  auto fail = [&](nexrResult_t r) {
    if (c->shm) peerHeader(c->shm)->abort.store(1);
    nexrRingCommDestroy(c);
    return r;
  };
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreate(&c->streams[me]) != hipSuccess)
    return fail(nexrUnhandledCudaError);
  if (c->ll) {
    if (hipHostMalloc((void**)&c->status[me], sizeof(uint32_t), hipHostMallocMapped) != hipSuccess)
      return fail(nexrUnhandledCudaError);
    *c->status[me] = 0;
  }
  // The FIFO into this rank. Uncached device memory: it is written by another process's kernels
  // (over xGMI when that process drives another GPU) between this rank's launches.
  // NEXR_PEER_FIFO_UNCACHED=0 selects ordinary (coarse-grained) device memory instead.
  const char* unc = getenv("NEXR_PEER_FIFO_UNCACHED");
  const bool uncached = !(unc && unc[0] == '0');
  if ((uncached ? hipExtMallocWithFlags((void**)&c->conns[me]->fifo, c->cfg.buffBytes, hipDeviceMallocUncached)
                : hipMalloc((void**)&c->conns[me]->fifo, c->cfg.buffBytes)) != hipSuccess)
    return fail(nexrUnhandledCudaError);
  // Rendezvous segment.
  c->shmBytes = peerShmBytes(n);
  int fd = shm_open(c->shmName, O_CREAT | O_RDWR, 0600);
  if (fd < 0) return fail(nexrSystemError);
  struct stat sb;
  if (fstat(fd, &sb) != 0 || (sb.st_size != 0 && (size_t)sb.st_size != c->shmBytes) ||
      (sb.st_size == 0 && ftruncate(fd, (off_t)c->shmBytes) != 0)) {
    close(fd);
    return fail(sb.st_size != 0 ? nexrInvalidUsage : nexrSystemError);
  }
  c->shm = mmap(nullptr, c->shmBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (c->shm == MAP_FAILED) {
    c->shm = nullptr;
    return fail(nexrSystemError);
  }
  PeerHeader* h = peerHeader(c->shm);
  const int timeoutMs = cfg->timeoutMs > 0 ? cfg->timeoutMs : 60000;
  auto waitFor = [&](auto pred) {
    auto t0 = std::chrono::steady_clock::now();
    while (!pred()) {
      if (h->abort.load(std::memory_order_acquire)) return false;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    return true;
  };
  uint32_t fresh = 0;
  if (h->initState.compare_exchange_strong(fresh, 1)) {
    h->magic = kPeerMagic;
    h->nRanks = (uint32_t)n;
    h->protocol = (uint32_t)c->proto;
    h->buffBytes = c->cfg.buffBytes;
    h->initState.store(2, std::memory_order_release);
  } else if (!waitFor([&] { return h->initState.load(std::memory_order_acquire) == 2; })) {
    return fail(nexrRemoteError);
  }
  if (h->magic != kPeerMagic || h->nRanks != (uint32_t)n || h->protocol != (uint32_t)c->proto ||
      h->buffBytes != c->cfg.buffBytes)
    return fail(nexrInvalidUsage);  // ranks disagree on the communicator (or a stale segment)
  PeerSlot* mine = peerSlot(c->shm, me);
  if (hipIpcGetMemHandle(&mine->fifoHandle, c->conns[me]->fifo) != hipSuccess) return fail(nexrUnhandledCudaError);
  c->conns[me]->st = &mine->conn;
  h->joined.fetch_add(1, std::memory_order_acq_rel);  // publishes the handle
  if (!waitFor([&] { return h->joined.load(std::memory_order_acquire) >= (uint32_t)n; })) return fail(nexrRemoteError);
  if (next != me) {
    hipIpcMemHandle_t hd = peerSlot(c->shm, next)->fifoHandle;
    if (hipIpcOpenMemHandle((void**)&c->peerFifo, hd, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
      return fail(nexrUnhandledCudaError);
    c->peerFifoIpc = true;
    c->conns[next]->fifo = c->peerFifo;
    c->conns[next]->st = &peerSlot(c->shm, next)->conn;
  }
  *out = c;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrPeerRingAllReduce(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int op) {
  if (!c || !c->peer) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  const int n = c->cfg.nRanks, me = c->self;
  const size_t esz = nexrTypeSize(datatype);
  if (esz == 0 || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2) return nexrInvalidArgument;
  nexrDevRedOpFull red;
  nexrResult_t r = nexrHostToDevRedOp(&red, op, datatype, n);
  if (r != nexrSuccess) return r;
  if (count > 0 && (!sendbuff || !recvbuff)) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  (void)hipSetDevice(c->devices[me]);
  if (n == 1) return oneRank(c, me, sendbuff, recvbuff, count, datatype, red, esz);
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  Prims p = makePrims(c, &sh, me, c->conns[me], c->conns[(me + 1) % n], sendbuff, recvbuff, esz, datatype, red, true);
  runRing(p, n, (int64_t)count);
  if (sh.firstError.load() != 0) {
    c->broken = true;
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

}  // extern "C"
