// nexr_ring.cpp — CPU-emulated collectives (include/nexr_ring.h): the reference's own collective
// schedules, restated on host threads, calling the reduce-copy ABI at exactly the reduceCopy sites
// of Primitives::genericOp. This is the drop-in demonstration for BASELINE configs[0] ("fp32 sum
// all-reduce, 4 MiB, 2 CPU-emulated ranks") and for every other caller of the primitive: the
// schedules are unchanged, only the primitive underneath is the MI355X kernel.
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
#include <functional>
#include <thread>
#include <vector>

#include "../../include/nexr_ring.h"

namespace {

constexpr int kSteps = 8;                                // NCCL_STEPS (src/include/device.h:649)
constexpr int kMaxArity = 3;                             // NCCL_MAX_TREE_ARITY (device.h:185)
constexpr size_t kDefaultBuffBytes = 4u << 20;           // NCCL_BUFFSIZE default (init.cc:620-634)
constexpr size_t kDefaultLLBuffBytes = 8 * 512 * kSteps * 16;  // DEFAULT_LL_BUFFSIZE (init.cc:618)
constexpr size_t kDefaultLL128BuffBytes = 120 * 640 * kSteps * 8;  // DEFAULT_LL128_BUFFSIZE (init.cc:619)
constexpr size_t kMinBuffBytes = kSteps * 512;           // one SIMPLE grain per step at least

// ProtoSimple<SlicePerChunk = chunkSteps/sliceSteps, StepPerSlice = sliceSteps> of a collective
// (src/include/collectives.h:16-25); LL and LL128 move one step per primitive call.
struct Geom {
  int chunkSteps, sliceSteps;
};
constexpr Geom kGeomRing{kSteps / 2, kSteps / 4};  // ALLREDUCE/ALLGATHER/REDUCESCATTER_*STEPS
constexpr Geom kGeomPipe{1, 1};                    // BROADCAST/REDUCE_*STEPS; the tree's ProtoSimple<1,1>

// One directed connection. The FIFO belongs to the receiver (the sender writes into it, like a
// P2P/SHM transport's recv buffer, src/include/device.h:753-771).
struct ConnState {
  alignas(64) std::atomic<uint64_t> tail{0};  // steps published by the sender   (postPeer, Send)
  alignas(64) std::atomic<uint64_t> head{0};  // steps released by the receiver  (postPeer, Recv)
};
struct Conn {
  char* fifo = nullptr;
  size_t slotBytes = 0;  // bytes per FIFO step; 0 = the communicator's stepBytes (P2P links: p2pChunkSize)
  int device = 0;        // device of the FIFO (device memory mode)
  bool ownsFifo = true;  // false for a peer process's FIFO mapped over IPC
  bool pinned = false;   // host-memory FIFO from hipHostMalloc
  ConnState own;
  ConnState* st = &own;  // the counters: `own` for thread ranks, a shared-memory slot for process ranks
  // Each endpoint's step (the conn->step a Primitives loads and saves, prims_simple.h:528-560): only
  // the sending thread touches sendStep and only the receiving thread touches recvStep.
  alignas(64) uint64_t sendStep = 0;
  alignas(64) uint64_t recvStep = 0;
};

// Process ranks (nexrPeerRingCommCreate): one POSIX shared-memory segment per communicator holds
// the rendezvous, every connection's head/tail counters and a common abort word. Slot r belongs to
// rank r: its FIFO's IPC handle and the counters of the connection INTO rank r.
constexpr uint32_t kPeerMagic = 0x6e657872u;  // "nexr"
struct alignas(64) PeerHeader {
  std::atomic<uint32_t> initState;  // 0 fresh, 1 being configured, 2 configured
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> left;
  std::atomic<uint32_t> abort;
  std::atomic<uint32_t> patJoined;  // ranks that published their PAT receive FIFOs
  std::atomic<uint32_t> p2pJoined;  // ranks that published their P2P receive FIFOs
  uint32_t magic, nRanks, protocol, pad;
  uint64_t buffBytes;
};
struct PeerSlot {
  hipIpcMemHandle_t fifoHandle;
  alignas(64) ConnState conn;
};
// Links beyond the ring for PAT (r -> r +- 2^d) and P2P (any r -> q), one per ordered pair: the
// receiver's FIFO handles and the link's counters. Only for communicators of up to kPeerLinkMaxRanks.
constexpr int kPeerLinkMaxRanks = 64;
struct PeerLink {
  hipIpcMemHandle_t patFifo, p2pFifo, p2pLLFifo;
  alignas(64) ConnState pat;
  alignas(64) ConnState p2p;
  alignas(64) ConnState p2pLL;
};
size_t peerShmBytes(int n) {
  return sizeof(PeerHeader) + (size_t)n * sizeof(PeerSlot) +
         (n <= kPeerLinkMaxRanks ? (size_t)n * n * sizeof(PeerLink) : 0);
}
PeerHeader* peerHeader(void* base) { return (PeerHeader*)base; }
PeerSlot* peerSlot(void* base, int r) { return (PeerSlot*)((char*)base + sizeof(PeerHeader)) + r; }
PeerLink* peerLink(void* base, int n, int from, int to) {
  return (PeerLink*)((char*)base + sizeof(PeerHeader) + (size_t)n * sizeof(PeerSlot)) + (size_t)from * n + to;
}

int64_t divUp(int64_t a, int64_t b) { return (a + b - 1) / b; }
int64_t alignUp(int64_t a, int64_t b) { return divUp(a, b) * b; }

struct TreeLinks {
  int up = -1;
  int down[kMaxArity] = {-1, -1, -1};
  int nDown() const {
    int k = 0;
    while (k < kMaxArity && down[k] >= 0) k++;
    return k;
  }
};

// ncclGetBtree (src/graph/trees.cc:31-63): the binary tree over nranks with root 0.
void getBtree(int nranks, int rank, int* u, int* d0, int* d1) {
  int bit;
  for (bit = 1; bit < nranks; bit <<= 1)
    if (bit & rank) break;
  if (rank == 0) {
    *u = -1;
    *d0 = -1;
    *d1 = nranks > 1 ? bit >> 1 : -1;
    return;
  }
  int up = (rank ^ bit) | (bit << 1);
  if (up >= nranks) up = (rank ^ bit);
  *u = up;
  int lowbit = bit >> 1;
  *d0 = lowbit == 0 ? -1 : rank - lowbit;
  int down1 = lowbit == 0 ? -1 : rank + lowbit;
  while (down1 >= nranks) {
    down1 = lowbit == 0 ? -1 : rank + lowbit;
    lowbit >>= 1;
  }
  *d1 = down1;
}

// ncclGetDtree (trees.cc:86-109): tree 0 is the btree, tree 1 its mirror (even nranks) or shift (odd).
void getDtree(int nranks, int rank, int t, int* u, int* d0, int* d1) {
  if (t == 0) {
    getBtree(nranks, rank, u, d0, d1);
  } else if (nranks % 2 == 1) {
    int uu, a, b;
    getBtree(nranks, (rank - 1 + nranks) % nranks, &uu, &a, &b);
    *u = uu == -1 ? -1 : (uu + 1) % nranks;
    *d0 = a == -1 ? -1 : (a + 1) % nranks;
    *d1 = b == -1 ? -1 : (b + 1) % nranks;
  } else {
    int uu, a, b;
    getBtree(nranks, nranks - 1 - rank, &uu, &a, &b);
    *u = uu == -1 ? -1 : nranks - 1 - uu;
    *d0 = a == -1 ? -1 : nranks - 1 - a;
    *d1 = b == -1 ? -1 : nranks - 1 - b;
  }
}

// The tree of every rank: within a node of L ranks a chain (connect.cc:51-61: up = previous,
// down[0] = next), and between nodes the double binary tree joining the node heads
// (connectTrees, connect.cc:140-163, with the NCCL_TOPO_PATTERN_TREE head as parent and both
// children) whose children are packed after the chain child by setTreeDown (:111-121).
std::vector<TreeLinks> treeTopology(int nRanks, int L, int t) {
  std::vector<TreeLinks> links(nRanks);
  const int nNodes = nRanks / L;
  for (int r = 0; r < nRanks; r++) {
    TreeLinks& k = links[r];
    const int node = r / L, i = r % L;
    k.up = i == 0 ? -1 : r - 1;
    k.down[0] = i == L - 1 ? -1 : r + 1;
    if (i == 0) {
      int u, d0, d1;
      getDtree(nNodes, node, t, &u, &d0, &d1);
      if (u != -1) k.up = u * L;
      for (int d : {d0, d1}) {
        if (d == -1) continue;
        int x = 0;
        while (x < kMaxArity && k.down[x] >= 0) x++;
        if (x < kMaxArity) k.down[x] = d * L;
      }
    }
  }
  return links;
}

}  // namespace

struct nexrRingComm {
  nexrRingConfig cfg;
  size_t stepBytes = 0;
  std::vector<Conn*> conns;     // ring: conns[r] is the connection into rank r from rank r-1
  std::vector<TreeLinks> tree;  // tree topology (computed at creation)
  std::vector<Conn*> treeUp;    // treeUp[r]: r -> parent(r) (reduce); created by the first tree call
  std::vector<Conn*> treeDown;  // treeDown[r]: parent(r) -> r (broadcast)
  std::vector<Conn*> patConns;  // PAT: patConns[from*nRanks+to] for to = from +- 2^d (ring link excluded)
  std::vector<Conn*> p2pConns;  // ncclSend/ncclRecv: p2pConns[from*nRanks+to] (connIndex 1), made on first use
  std::vector<Conn*> p2pLLConns;  // the same links' LL buffers, for messages <= 16 KiB
  size_t p2pChunkBytes = 0;     // comm->p2pChunkSize
  std::vector<int> devices;
  std::vector<hipStream_t> streams, streams2;  // streams2: the tree's broadcast-half threads
  std::vector<uint32_t*> status, status2;      // LL: pinned status words the kernel reports timeouts in
  bool ll = false;     // LL or LL128: one FIFO step per primitive call, data readiness in line flags
  int proto = nexrRingProtoSimple;
  bool needHip = false;
  bool pinnedStatus = false;  // status words from hipHostMalloc (else calloc)
  bool broken = false;
  // Process ranks: this process is rank `self` only.
  bool peer = false;
  int self = 0;
  void* shm = nullptr;
  size_t shmBytes = 0;
  char shmName[256] = {0};
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

enum { kNone = -1, kInput = 0, kOutput = 1 };  // SrcBuf / DstBuf of genericOp

// One rank's Primitives<T, RedOp, Fan, Direct, Proto> (prims_simple.h / prims_ll.h / prims_ll128.h),
// host side: up to kMaxArity recv peers and kMaxArity send peers (FanAsymmetric of the tree).
struct Prims {
  nexrRingComm* c;
  Shared* sh;
  int rank;
  Conn* recv[kMaxArity];
  int nRecv = 0;
  Conn* send[kMaxArity];
  int nSend = 0;
  const char* userInput;
  char* userOutput;
  size_t esz;
  int64_t stepSize;  // elements per FIFO step (prims_simple.h:607)
  int stepPerSlice = 1, slicePerChunk = 1;
  int datatype, devOp;
  uint64_t redOpArgs[1];
  nexrReduceCopyFn fn;
  nexrReduceCopyLLFn llFn;
  nexrReduceCopyLL128Fn ll128Fn;
  uint32_t* status;
  hipStream_t stream;
  bool device;
  int proto = nexrRingProtoSimple;  // the communicator's, or LL for a small P2P message (sendrecv.h)

  char* buf(int which) const { return which == kInput ? const_cast<char*>(userInput) : userOutput; }
  size_t slot(const Conn* q) const { return q->slotBytes ? q->slotBytes : c->stepBytes; }

  // loadRecvConn / loadSendConn (prims_simple.h:512-513, :557-558): a SIMPLE Primitives starts each
  // connection at step roundUp(conn->step, SlicePerChunk*StepPerSlice), so a collective with 2-step
  // slices that follows one with 1-step slices (Broadcast, Reduce) never starts a slice in the last
  // FIFO slot. Both endpoints of a connection hold the same step between collectives and round alike,
  // and the receiver publishes its rounded step as head ("return credits in case we rounded up",
  // :514-517): the steps skipped by rounding were never sent, so the sender must not wait for them.
  void attach() {
    if (proto != nexrRingProtoSimple) return;
    const uint64_t cs = (uint64_t)(stepPerSlice * slicePerChunk);
    for (int i = 0; i < nRecv; i++) {
      recv[i]->recvStep = (recv[i]->recvStep + cs - 1) / cs * cs;
      recv[i]->st->head.store(recv[i]->recvStep, std::memory_order_release);
    }
    for (int i = 0; i < nSend; i++) send[i]->sendStep = (send[i]->sendStep + cs - 1) / cs * cs;
  }

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
  // with the non-direct FIFO pointers (waitPeer :150-164 default branch). srcs = [user src, recv
  // peers...], dsts = [user dst, send peers...] (:131-132, :238-242).
  bool genericOp(bool Recv, bool Send, int srcBuf, int dstBuf, int64_t srcIx, int64_t dstIx, int64_t nelem,
                 bool postOp) {
    const int nr = Recv ? nRecv : 0, ns = Send ? nSend : 0;
    nelem = nelem < 0 ? 0 : nelem;
    int64_t sliceSize = stepSize * stepPerSlice;
    sliceSize = std::max(divUp(nelem, 16 * slicePerChunk) * 16, sliceSize / 32);
    int64_t offset = 0;
    for (int slice = 0; slice < slicePerChunk; slice++) {
      sliceSize = std::min(sliceSize, nelem - offset);
      if (sliceSize < 0) sliceSize = 0;
      const void* srcs[1 + kMaxArity];
      void* dsts[1 + kMaxArity];
      int k = 0, m = 0;
      if (srcBuf != kNone) srcs[k++] = buf(srcBuf) + (srcIx + offset) * esz;
      if (dstBuf != kNone) dsts[m++] = buf(dstBuf) + (dstIx + offset) * esz;
      for (int i = 0; i < nr; i++) {  // wait for the peer's data: tail >= step + StepPerSlice
        Conn* q = recv[i];
        if (!waitAtLeast(q->st->tail, q->recvStep + stepPerSlice)) return false;
        srcs[k++] = q->fifo + (q->recvStep % kSteps) * slot(q);
      }
      for (int i = 0; i < ns; i++) {  // wait for credit: head + NCCL_STEPS >= step + StepPerSlice
        Conn* q = send[i];
        if (q->sendStep + stepPerSlice > (uint64_t)kSteps &&
            !waitAtLeast(q->st->head, q->sendStep + stepPerSlice - kSteps))
          return false;
        dsts[m++] = q->fifo + (q->sendStep % kSteps) * slot(q);
      }
      if (sliceSize > 0 && k > 0 && m > 0) {
        // PreOpSrcs = SrcBuf != Input ? 0 : 1 (prims_simple.h:279-280); preOpArgs = redOpArgs.
        const int nPre = srcBuf == kInput ? 1 : 0;
        nexrResult_t r = fn(k, srcs, m, dsts, (size_t)sliceSize, datatype, devOp, redOpArgs[0], nPre,
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
      for (int i = 0; i < nr; i++) {
        recv[i]->recvStep += stepPerSlice;
        recv[i]->st->head.store(recv[i]->recvStep, std::memory_order_release);
      }
      for (int i = 0; i < ns; i++) {
        send[i]->sendStep += stepPerSlice;
        send[i]->st->tail.store(send[i]->sendStep, std::memory_order_release);
      }
      offset += sliceSize;
    }
    return true;
  }
  // LLGenericOp<RECV, SEND, SrcBuf, DstBuf> (prims_ll.h:218-283) / GenericOp of prims_ll128.h
  // (:294-331): one FIFO step per call. The sender waits for a credit (waitSend :55-75); the
  // receiver's data readiness is the line flags (NCCL_LL_FLAG(step+1), :42-43; step+1 for LL128).
  // The host additionally waits for the sender's step so that the kernel's flag poll succeeds at
  // once: two emulated ranks may share one GPU, and a kernel spinning on a producer that cannot be
  // scheduled beside it must never be launched.
  bool genericOpLL(bool Recv, bool Send, int srcBuf, int dstBuf, int64_t srcIx, int64_t dstIx, int64_t nelem,
                   bool postOp) {
    const int nr = Recv ? nRecv : 0, ns = Send ? nSend : 0;
    nelem = nelem < 0 ? 0 : nelem;
    for (int i = 0; i < ns; i++) {
      Conn* q = send[i];
      if (q->sendStep + 1 > (uint64_t)kSteps && !waitAtLeast(q->st->head, q->sendStep + 1 - kSteps)) return false;
    }
    for (int i = 0; i < nr; i++)
      if (!waitAtLeast(recv[i]->st->tail, recv[i]->recvStep + 1)) return false;
    if (nelem > 0) {
      const void* recvLines[kMaxArity];
      void* sendLines[kMaxArity];
      uint32_t rf32[kMaxArity], sf32[kMaxArity];
      uint64_t rf64[kMaxArity], sf64[kMaxArity];
      for (int i = 0; i < nr; i++) {
        recvLines[i] = recv[i]->fifo + (recv[i]->recvStep % kSteps) * slot(recv[i]);
        rf64[i] = recv[i]->recvStep + 1;
        rf32[i] = (uint32_t)rf64[i];
      }
      for (int i = 0; i < ns; i++) {
        sendLines[i] = send[i]->fifo + (send[i]->sendStep % kSteps) * slot(send[i]);
        sf64[i] = send[i]->sendStep + 1;
        sf32[i] = (uint32_t)sf64[i];
      }
      const void* src = srcBuf != kNone ? buf(srcBuf) + srcIx * esz : nullptr;
      void* dst = dstBuf != kNone ? buf(dstBuf) + dstIx * esz : nullptr;
      const int srcIsInput = srcBuf == kInput ? 1 : 0;
      if (status) *status = 0;
      const uint32_t tmo = (uint32_t)((c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 1000u);
      nexrResult_t r;
      if (proto == nexrRingProtoLL128)
        r = ll128Fn(src, srcIsInput, nr, recvLines, rf64, dst, ns, sendLines, sf64, (size_t)nelem, datatype, devOp,
                    redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      else
        r = llFn(src, srcIsInput, nr, recvLines, rf32, dst, ns, sendLines, sf32, (size_t)nelem, datatype, devOp,
                 redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      if (r == nexrSuccess && device && hipStreamSynchronize(stream) != hipSuccess) r = nexrUnhandledCudaError;
      if (r == nexrSuccess && status && __atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) r = nexrInternalError;
      if (r != nexrSuccess) {
        sh->fail(r);
        return false;
      }
    }
    for (int i = 0; i < nr; i++) {  // postRecv (:80-83)
      recv[i]->recvStep += 1;
      recv[i]->st->head.store(recv[i]->recvStep, std::memory_order_release);
    }
    for (int i = 0; i < ns; i++) {  // incSend (:85-93); the flag-wrap cleanup at NCCL_LL_CLEAN_MASK needs ~2^31 steps
      send[i]->sendStep += 1;
      send[i]->st->tail.store(send[i]->sendStep, std::memory_order_release);
    }
    return true;
  }
  bool op(bool Recv, bool Send, int srcBuf, int dstBuf, int64_t srcIx, int64_t dstIx, int64_t n, bool postOp) {
    return proto != nexrRingProtoSimple ? genericOpLL(Recv, Send, srcBuf, dstBuf, srcIx, dstIx, n, postOp)
                 : genericOp(Recv, Send, srcBuf, dstBuf, srcIx, dstIx, n, postOp);
  }
  // The primitives the schedules use (prims_simple.h:897-976; the direct* forms reduce to these
  // without registered peer buffers).
  bool sendInput(int64_t inpIx, int64_t n) { return op(false, true, kInput, kNone, inpIx, -1, n, false); }
  bool copySend(int64_t inpIx, int64_t outIx, int64_t n) { return op(false, true, kInput, kOutput, inpIx, outIx, n, false); }
  bool sendFromOutput(int64_t outIx, int64_t n) { return op(false, true, kOutput, kNone, outIx, -1, n, false); }
  bool recvReduceSend(int64_t inpIx, int64_t n) { return op(true, true, kInput, kNone, inpIx, -1, n, false); }
  bool recvReduceCopy(int64_t inpIx, int64_t outIx, int64_t n, bool postOp) {
    return op(true, false, kInput, kOutput, inpIx, outIx, n, postOp);
  }
  bool recvReduceCopySend(int64_t inpIx, int64_t outIx, int64_t n, bool postOp) {
    return op(true, true, kInput, kOutput, inpIx, outIx, n, postOp);
  }
  bool recvCopySend(int64_t outIx, int64_t n) { return op(true, true, kNone, kOutput, -1, outIx, n, false); }
  bool recvOutput(int64_t outIx, int64_t n) { return op(true, false, kNone, kOutput, -1, outIx, n, false); }
};

// calcCollChunking for one channel (src/enqueue.cc:1993-1999; tree LL128 :2043-2051; grain
// alignment :2062) → chunkCount in elements (ncclCollCbdPart, device.h:946-970).
int64_t chunkElems(const nexrRingComm* c, Geom g, size_t esz, bool tree, size_t nBytes) {
  int64_t chunk = (int64_t)c->stepBytes * (c->proto == nexrRingProtoSimple ? g.chunkSteps : 1);
  if (c->proto == nexrRingProtoLL) chunk /= 2;
  if (c->proto == nexrRingProtoLL128) chunk = chunk / 16 * 15;  // NCCL_LL128_LINEELEMS / DATAELEMS
  if (tree && c->proto == nexrRingProtoLL128) {
    const int L = c->cfg.treeRanksPerNode > 0 ? c->cfg.treeRanksPerNode : c->cfg.nRanks;
    const int nNodes = c->cfg.nRanks / L;
    int log2n = 0;
    while ((2 << log2n) <= nNodes) log2n++;
    const float ppn = (float)c->cfg.nRanks / (float)nNodes;
    const float nstepsLL128 = 1 + log2n + 0.1f * ppn;
    while ((float)(nBytes / (size_t)chunk) < nstepsLL128 * 64 / ppn && chunk > 131072) chunk /= 2;
    while ((float)(nBytes / (size_t)chunk) < nstepsLL128 * 16 / ppn && chunk > 32768) chunk /= 2;
  }
  const int64_t grain = c->proto == nexrRingProtoLL ? 16 : c->proto == nexrRingProtoLL128 ? 1920 : 512;
  chunk = chunk / grain * grain;
  return chunk / (int64_t)esz;
}

// ---- schedules (one rank's view; 1 channel, userRanks[i] = (rank + i) % nranks) ----------------

// runRing for ncclAllReduce (all_reduce.h:12-84).
void runRingAllReduce(Prims& p, int nranks, int64_t count) {
  const int ringIx = p.rank;
  int64_t chunkCount = chunkElems(p.c, kGeomRing, p.esz, false, 0);
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
    if (!p.sendInput(offset, nelem)) return;
    // k-2 steps: reduce and copy to next GPU
    for (int j = 2; j < nranks; ++j) {
      nelem = at(modRanks(ringIx + nranks - j), &offset);
      if (!p.recvReduceSend(offset, nelem)) return;
    }
    // step k-1: reduce this buffer and data -> final result, stored and pushed
    nelem = at(ringIx, &offset);
    if (!p.recvReduceCopySend(offset, offset, nelem, /*postOp=*/true)) return;
    // k-2 steps: copy to next GPU
    for (int j = 1; j < nranks - 1; ++j) {
      nelem = at(modRanks(ringIx + nranks - j), &offset);
      if (!p.recvCopySend(offset, nelem)) return;
    }
    // final copy from buffer to dest
    nelem = at(modRanks(ringIx + 1), &offset);
    if (!p.recvOutput(offset, nelem)) return;
  }
}

// runRing for ncclReduceScatter (reduce_scatter.h:12-52): `count` is the per-rank recvcount; the
// segment of rankDest starts at rankDest*count in every sendbuff.
void runRingReduceScatter(Prims& p, int nranks, int64_t count) {
  const int64_t chunkCount = chunkElems(p.c, kGeomRing, p.esz, false, 0);
  const int r = p.rank;
  for (int64_t elemOffset = 0; elemOffset < count; elemOffset += chunkCount) {
    const int64_t nelem = std::min(chunkCount, count - elemOffset);
    const int64_t dataOffset = elemOffset;
    int rankDest = (r + nranks - 1) % nranks;  // ringRanks[nranks-1]
    if (!p.sendInput(dataOffset + rankDest * count, nelem)) return;
    for (int j = 2; j < nranks; ++j) {
      rankDest = (r + nranks - j) % nranks;
      if (!p.recvReduceSend(dataOffset + rankDest * count, nelem)) return;
    }
    rankDest = r;  // ringRanks[0]
    if (!p.recvReduceCopy(dataOffset + rankDest * count, dataOffset, nelem, /*postOp=*/true)) return;
  }
}

// runRing for ncclAllGather (all_gather.h:12-66): `count` is the per-rank sendcount.
void runRingAllGather(Prims& p, int nranks, int64_t count) {
  const int64_t chunkCount = chunkElems(p.c, kGeomRing, p.esz, false, 0);
  const int r = p.rank;
  for (int64_t elemOffset = 0; elemOffset < count; elemOffset += chunkCount) {
    const int64_t nelem = std::min(chunkCount, count - elemOffset);
    const int64_t dataOffset = elemOffset;
    int64_t offset = dataOffset + (int64_t)r * count;
    // in place when the input chunk already sits at its place in the output (:52-56)
    const bool inPlace = p.userInput + dataOffset * p.esz == p.userOutput + offset * p.esz;
    if (!(inPlace ? p.sendInput(dataOffset, nelem) : p.copySend(dataOffset, offset, nelem))) return;
    for (int j = 1; j < nranks - 1; ++j) {
      const int rankDest = (r + nranks - j) % nranks;
      offset = dataOffset + (int64_t)rankDest * count;
      if (!p.recvCopySend(offset, nelem)) return;
    }
    offset = dataOffset + (int64_t)((r + 1) % nranks) * count;
    if (!p.recvOutput(offset, nelem)) return;
  }
}

// runRing for ncclReduce (reduce.h:12-50).
void runRingReduce(Prims& p, int nranks, int64_t count, int root) {
  const int64_t chunkCount = chunkElems(p.c, kGeomPipe, p.esz, false, 0);
  const int r = p.rank, prevRank = (r + nranks - 1) % nranks;
  for (int64_t offset = 0; offset < count; offset += chunkCount) {
    const int64_t nelem = std::min(chunkCount, count - offset);
    bool ok;
    if (prevRank == root) ok = p.sendInput(offset, nelem);
    else if (r == root) ok = p.recvReduceCopy(offset, offset, nelem, /*postOp=*/true);
    else ok = p.recvReduceSend(offset, nelem);
    if (!ok) return;
  }
}

// runRing for ncclBroadcast (broadcast.h:12-58).
void runRingBroadcast(Prims& p, int nranks, int64_t count, int root) {
  const int64_t chunkCount = chunkElems(p.c, kGeomPipe, p.esz, false, 0);
  const int r = p.rank, nextRank = (r + 1) % nranks;
  for (int64_t offset = 0; offset < count; offset += chunkCount) {
    const int64_t nelem = std::min(chunkCount, count - offset);
    bool ok;
    if (r == root) ok = p.userInput == p.userOutput ? p.sendInput(offset, nelem) : p.copySend(offset, offset, nelem);
    else if (nextRank == root) ok = p.recvOutput(offset, nelem);
    else ok = p.recvCopySend(offset, nelem);
    if (!ok) return;
  }
}

// runTreeSplit for ncclAllReduce (all_reduce.h:150-230), one role of one rank: the root reduces
// from and broadcasts to its children in one pass (FanSymmetric<NCCL_MAX_TREE_ARITY_TOP>); every
// other rank runs a reduce-up half (FanAsymmetric<3,1>) and a broadcast-down half
// (FanAsymmetric<1,3>) side by side.
enum TreeRole { kTreeRoot, kTreeReduceUp, kTreeBcastDown };
void runTree(Prims& p, int64_t count, TreeRole role, bool leaf) {
  const int64_t chunkCount = chunkElems(p.c, kGeomPipe, p.esz, true, (size_t)count * p.esz);
  for (int64_t offset = 0; offset < count; offset += chunkCount) {
    const int64_t nelem = std::min(chunkCount, count - offset);
    bool ok;
    if (role == kTreeRoot) ok = p.recvReduceCopySend(offset, offset, nelem, /*postOp=*/true);
    else if (role == kTreeReduceUp) ok = leaf ? p.sendInput(offset, nelem) : p.recvReduceSend(offset, nelem);
    else ok = leaf ? p.recvOutput(offset, nelem) : p.recvCopySend(offset, nelem);
    if (!ok) return;
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

Prims makePrims(nexrRingComm* c, Shared* sh, int rank, const void* sendbuff, void* recvbuff, size_t esz, int datatype,
                const nexrDevRedOpFull& red, Geom g, hipStream_t stream, uint32_t* status) {
  Prims p;
  p.c = c;
  p.sh = sh;
  p.rank = rank;
  p.userInput = (const char*)sendbuff;
  p.userOutput = (char*)recvbuff;
  p.esz = esz;
  p.stepSize = (int64_t)(c->stepBytes / esz);
  p.stepPerSlice = g.sliceSteps;
  p.slicePerChunk = g.chunkSteps / g.sliceSteps;
  p.datatype = datatype;
  p.devOp = red.op;
  p.redOpArgs[0] = red.scalarArg;
  p.fn = c->cfg.fn;
  p.llFn = c->cfg.llFn;
  p.ll128Fn = c->cfg.ll128Fn;
  p.status = status;
  p.stream = stream;
  p.device = c->cfg.memMode == nexrRingDeviceMemory;
  p.proto = c->proto;
  return p;
}

// ncclLaunchOneRank (onerank.cc:48-83) for rank `r`'s buffers: every collective with nRanks == 1
// (enqueue.cc:2354-2356).
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

// Common argument checks: datatype and op encoding (hostToDevRedOp, enqueue.cc:2185-2278).
nexrResult_t prepare(nexrRingComm* c, int datatype, int op, size_t* esz, nexrDevRedOpFull* red) {
  if (!c) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  *esz = nexrTypeSize(datatype);
  if (*esz == 0 || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2) return nexrInvalidArgument;
  return nexrHostToDevRedOp(red, op, datatype, c->cfg.nRanks);
}

// Runs `jobs` (one per emulated rank, or per tree half) on host threads and collects the first error.
nexrResult_t runThreads(nexrRingComm* c, Shared& sh, const std::vector<std::function<void()>>& jobs) {
  std::vector<std::thread> threads;
  threads.reserve(jobs.size());
  for (const auto& j : jobs) threads.emplace_back(j);
  for (auto& t : threads) t.join();
  if (sh.firstError.load() != 0) {
    c->broken = true;  // step counters are mid-protocol: the communicator cannot be reused
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

// NEXR_RING_HOST_PINNED=0 keeps host-memory FIFOs pageable (the staged path for every step).
bool pinnedHostFifos() {
  static const bool on = [] {
    const char* e = getenv("NEXR_RING_HOST_PINNED");
    return !(e && e[0] == '0');
  }();
  return on;
}

nexrResult_t allocFifo(nexrRingComm* c, Conn* k, int device, size_t bytes = 0) {
  k->device = device;
  if (bytes == 0) bytes = c->cfg.buffBytes;
  if (c->cfg.memMode == nexrRingDeviceMemory) {
    if (hipSetDevice(device) != hipSuccess || hipMalloc((void**)&k->fifo, bytes) != hipSuccess)
      return nexrUnhandledCudaError;
  } else if (c->needHip && pinnedHostFifos()) {
    // Host memory with the MI355X doing the steps: pinned, device-mapped FIFOs, so that a step whose
    // user buffers are pinned too runs as one zero-copy kernel over PCIe (nexrReduceCopyHost) instead
    // of staging every slice through device memory.
    if (hipHostMalloc((void**)&k->fifo, bytes, hipHostMallocMapped | hipHostMallocPortable) != hipSuccess)
      return nexrUnhandledCudaError;
    k->pinned = true;
  } else {
    k->fifo = (char*)aligned_alloc(4096, bytes);
    if (!k->fifo) return nexrSystemError;
  }
  return nexrSuccess;
}

nexrResult_t enablePeer(int a, int b) {
  if (a == b) return nexrSuccess;
  (void)hipSetDevice(a);
  hipError_t e = hipDeviceEnablePeerAccess(b, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) return nexrUnhandledCudaError;
  (void)hipGetLastError();
  return nexrSuccess;
}

nexrResult_t allocStatus(nexrRingComm* c, uint32_t** s) {
  if (c->needHip) {  // pinned, device-mapped status word for the LL kernel's timeout report
    if (hipHostMalloc((void**)s, sizeof(uint32_t), hipHostMallocMapped) != hipSuccess) return nexrUnhandledCudaError;
    **s = 0;
  } else {  // CPU-side LL implementation: an ordinary host word
    *s = (uint32_t*)calloc(1, sizeof(uint32_t));
    if (!*s) return nexrSystemError;
  }
  return nexrSuccess;
}

// A second stream and status word per rank, for ranks that run two halves at once (the tree's
// reduce-up / broadcast-down, a send beside a recv).
nexrResult_t ensureSecondStreams(nexrRingComm* c) {
  if (!c->streams2.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks;
  c->streams2.assign(n, nullptr);
  c->status2.assign(n, nullptr);
  for (int r = 0; r < n; r++) {
    if (c->streams[r]) {
      if (hipSetDevice(c->devices[r]) != hipSuccess || hipStreamCreate(&c->streams2[r]) != hipSuccess)
        return nexrUnhandledCudaError;
    }
    if (c->ll) {
      nexrResult_t res = allocStatus(c, &c->status2[r]);
      if (res != nexrSuccess) return res;
    }
  }
  return nexrSuccess;
}

// The tree's connections (and the second streams), made by the first tree call.
nexrResult_t ensureTree(nexrRingComm* c) {
  if (!c->treeUp.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks;
  c->treeUp.assign(n, nullptr);
  c->treeDown.assign(n, nullptr);
  nexrResult_t sres = ensureSecondStreams(c);
  if (sres != nexrSuccess) return sres;
  for (int r = 0; r < n; r++) {
    const int up = c->tree[r].up;
    if (up < 0) continue;
    c->treeUp[r] = new Conn();
    c->treeDown[r] = new Conn();
    nexrResult_t res = allocFifo(c, c->treeUp[r], c->devices[up]);
    if (res == nexrSuccess) res = allocFifo(c, c->treeDown[r], c->devices[r]);
    if (res == nexrSuccess && c->cfg.memMode == nexrRingDeviceMemory) {
      res = enablePeer(c->devices[r], c->devices[up]);
      if (res == nexrSuccess) res = enablePeer(c->devices[up], c->devices[r]);
    }
    if (res != nexrSuccess) return res;
  }
  return nexrSuccess;
}

void freeConn(nexrRingComm* c, Conn* k) {
  if (!k) return;
  if (k->fifo && k->ownsFifo) {
    if (c->cfg.memMode == nexrRingDeviceMemory) {
      (void)hipSetDevice(k->device);
      (void)hipFree(k->fifo);
    } else if (k->pinned) {
      (void)hipHostFree(k->fifo);
    } else {
      free(k->fifo);
    }
  }
  delete k;
}

bool validConfigBuff(const nexrRingComm* c) {
  return c->cfg.buffBytes % (kSteps * 16) == 0 && c->cfg.buffBytes >= kMinBuffBytes &&
         (c->proto != nexrRingProtoLL128 || c->cfg.buffBytes % (kSteps * 2048) == 0);  // whole LL128 slices
}

// Thread-rank collectives: the ring schedules on one thread per rank.
enum RingColl { kAllReduce, kReduceScatter, kAllGather, kReduce, kBroadcast };
nexrResult_t ringCollective(nexrRingComm* c, RingColl coll, const void* const* sendbuffs, void* const* recvbuffs,
                            size_t count, int datatype, int op, int root) {
  if (!c || c->peer) return nexrInvalidArgument;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = prepare(c, datatype, op, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks;
  if ((coll == kReduce || coll == kBroadcast) && (root < 0 || root >= n)) return nexrInvalidArgument;
  if (!sendbuffs || !recvbuffs) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  for (int i = 0; i < n; i++) {
    const bool needSend = coll != kBroadcast || i == root;
    const bool needRecv = coll != kReduce || i == root;
    if ((needSend && !sendbuffs[i]) || (needRecv && !recvbuffs[i])) return nexrInvalidArgument;
  }
  if (n == 1) return oneRank(c, 0, sendbuffs[0], recvbuffs[0], count, datatype, red, esz);
  const Geom g = (coll == kReduce || coll == kBroadcast) ? kGeomPipe : kGeomRing;
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (int rank = 0; rank < n; rank++) {
    jobs.emplace_back([&, rank] {
      if (c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
      Prims p = makePrims(c, &sh, rank, sendbuffs[rank], recvbuffs[rank], esz, datatype, red, g, c->streams[rank],
                          c->status[rank]);
      p.recv[p.nRecv++] = c->conns[rank];
      p.send[p.nSend++] = c->conns[(rank + 1) % n];
      p.attach();
      switch (coll) {
        case kAllReduce: runRingAllReduce(p, n, (int64_t)count); break;
        case kReduceScatter: runRingReduceScatter(p, n, (int64_t)count); break;
        case kAllGather: runRingAllGather(p, n, (int64_t)count); break;
        case kReduce: runRingReduce(p, n, (int64_t)count, root); break;
        case kBroadcast: runRingBroadcast(p, n, (int64_t)count, root); break;
      }
    });
  }
  return runThreads(c, sh, jobs);
}

// Process-rank collectives: this process's rank of the same ring schedules.
nexrResult_t peerCollective(nexrRingComm* c, RingColl coll, const void* sendbuff, void* recvbuff, size_t count,
                            int datatype, int op, int root) {
  if (!c || !c->peer) return nexrInvalidArgument;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = prepare(c, datatype, op, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks, me = c->self;
  if ((coll == kReduce || coll == kBroadcast) && (root < 0 || root >= n)) return nexrInvalidArgument;
  const bool needSend = coll != kBroadcast || me == root;
  const bool needRecv = coll != kReduce || me == root;
  if (count > 0 && ((needSend && !sendbuff) || (needRecv && !recvbuff))) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  (void)hipSetDevice(c->devices[me]);
  if (n == 1) return oneRank(c, me, sendbuff, recvbuff, count, datatype, red, esz);
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  const Geom g = (coll == kReduce || coll == kBroadcast) ? kGeomPipe : kGeomRing;
  Prims p = makePrims(c, &sh, me, sendbuff, recvbuff, esz, datatype, red, g, c->streams[me], c->status[me]);
  p.recv[p.nRecv++] = c->conns[me];
  p.send[p.nSend++] = c->conns[(me + 1) % n];
  p.attach();
  switch (coll) {
    case kAllReduce: runRingAllReduce(p, n, (int64_t)count); break;
    case kReduceScatter: runRingReduceScatter(p, n, (int64_t)count); break;
    case kAllGather: runRingAllGather(p, n, (int64_t)count); break;
    case kReduce: runRingReduce(p, n, (int64_t)count, root); break;
    case kBroadcast: runRingBroadcast(p, n, (int64_t)count, root); break;
  }
  if (sh.firstError.load() != 0) {
    c->broken = true;
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

// ---- PAT: ncclReduceScatter / ncclAllGather with NCCL_ALGO_PAT (SIMPLE) ----------------------------
// The reference runs PAT as one compute thread generating a stream of steps (PatRSAlgorithm /
// PatAGAlgorithm, src/device/collectives.h:433-906) that parallelFactor worker groups consume in
// lock-step batches: every group of step batch b waits for its peers, all groups meet at patBarrier
// (barrier over all NCCL_PAT_NWORKERS threads, prims_simple.h:76-78), each runs its reduceCopy, the
// step counters and accumulation marks are updated, all meet again, then tails/heads are published
// (patReduce :992-1088, patCopy :1090-1183). Here one host thread per rank runs the same batches
// in order: it reads every peer's step at the start of the batch, waits, issues the batch's
// reduce-copies, waits for them, then applies the updates and publishes. Rank r's dimension d
// connects it to r -/+ 2^d (prims_simple.h:694-717).

constexpr int kPatWorkers = 512;                        // NCCL_PAT_NWORKERS (collectives.h:402)
constexpr int kPatMaxParallel = kPatWorkers / 32;       // NCCL_PAT_NWORKERS/WARP_SIZE (reduce_scatter.h:100)
constexpr int kPatMaxDims = 32;                         // ncclPatShmem::sendDims[32] (collectives.h:429)

// One ncclPatStep (collectives.h:407-410); `skipped` is PatSkipped in ps->flags.
struct PatOp {
  int recvDim = -1, sendDim = -1, recvOffset = -1, sendOffset = -1, stepOffset = 0, postRecv = 0, postSend = 0;
  int nelem = 0, last = 0;
  bool skipped = false;
  int64_t inpIx = 0, outIx = 0;
};

int log2Up(int n) {
  int p = 0;
  while ((1 << p) < n) p++;
  return p;
}
int firstBitSet(int i, int max) { return i ? __builtin_ctz((unsigned)i) : max; }

// The aggregation geometry both generators compute in their constructors (collectives.h:515-536,
// :779-801): several small chunks share one FIFO step (postFreq), and up to stepDepth steps are in
// flight per peer (aggFactor), as long as aggFactor < nRanks/2.
struct PatGeometry {
  int nrPow2, aggFactor, aggDelta, postFreq, parallelFactor;
  PatGeometry(uint64_t stepBytes, int stepDepth, int maxParallel, uint64_t channelElems, size_t esz, int nranks) {
    parallelFactor = maxParallel;
    aggDelta = nrPow2 = 1 << log2Up(nranks);
    aggFactor = 1;
    while (stepBytes / (channelElems * esz * (uint64_t)aggFactor) >= 2 && aggFactor < nranks / 2) {
      aggFactor *= 2;
      aggDelta /= 2;
    }
    postFreq = aggFactor;
    if (postFreq < parallelFactor) parallelFactor = postFreq;
    for (int d = stepDepth; d > 1 && aggFactor < nranks / 2;) {
      d /= 2;
      aggFactor *= 2;
      aggDelta /= 2;
    }
  }
};

// PatRSAlgorithm::getNextOp (collectives.h:542-683): phase 0 sends this rank's input for far
// destinations, phase 1 receives partials on dimension recvDim, folds them into the step bound
// for sendDim, phases 2/3 repeat that for the aggregated low dimensions, phase 4 folds the
// partial arriving on dimension 0 with the own input into the output.
struct PatReduceScatterPlan : PatGeometry {
  int64_t offset, end, count;
  int chunkCount, nelem = 0, rank, nranks;
  int lastA = 0, as = 0, a = 0, sendSkipped = 0, stepOffset = 0, scale = 1, phase = 0;

  PatReduceScatterPlan(int chunkCount_, size_t esz, int64_t count_, int rank_, int nranks_)
      : PatGeometry((uint64_t)chunkCount_ * esz, kSteps, kPatMaxParallel, (uint64_t)count_, esz, nranks_),
        offset(0), end(count_), count(count_), chunkCount(chunkCount_), rank(rank_), nranks(nranks_) {
    reset();
  }
  static int mirrorInvert(int i, int max) {
    int r = 0;
    for (int mask = 1, imask = max / 2; mask < max; mask <<= 1, imask >>= 1)
      if ((i & mask) == 0) r += imask;
    return r;
  }
  // 1 when only the upper bits of i are set, e.g. 8, 12, 14, 15 for pow2 = 16 (collectives.h:507-512).
  static bool newPeer(int i, int pow2) { return __builtin_popcount((unsigned)((i ^ (pow2 - 1)) + 1)) == 1; }
  void resetA() {
    a = 0;
    sendSkipped = stepOffset = 0;
    lastA = aggFactor;
    if (phase >= 2) lastA /= 2 * scale;
    if (phase == 4) lastA = 1;
  }
  void reset() {
    nelem = (int)std::min<int64_t>(chunkCount, end - offset);
    phase = 0;
    scale = 1;
    as = aggDelta - 1;
    resetA();
  }
  bool posts(int x) const { return (x % postFreq) + 1 >= postFreq || x == lastA - 1; }
  void next(PatOp* ps) {
    ps->last = 0;
    ps->nelem = nelem;
    ps->outIx = offset;
    ps->stepOffset = stepOffset;
    bool skip = false;
    if (a >= lastA) {
      skip = true;
    } else if (phase == 0) {
      const int s = mirrorInvert(a, lastA) * aggDelta + as;
      if (s >= nranks) skip = true;
      ps->inpIx = (int64_t)((rank + s) % nranks) * count + offset;
      ps->recvDim = -1;
      ps->sendDim = 0;
      ps->outIx = 0;
      ps->recvOffset = -1;
      ps->sendOffset = (a % postFreq) * nelem;
      ps->postSend = posts(a) ? 1 : 0;
      ps->postRecv = 0;
    } else if (phase == 1) {
      int s = mirrorInvert(a, lastA) * aggDelta + as;
      if (s >= nranks) skip = true;
      ps->recvDim = firstBitSet(s, nrPow2);
      ps->sendOffset = (a % postFreq) * nelem;
      ps->recvOffset = (a % postFreq) * nelem;
      ps->postSend = (ps->recvDim == 0 && posts(a)) ? 1 : 0;
      ps->postRecv = posts(a) ? 1 : 0;
      s -= 1 << ps->recvDim;
      ps->inpIx = (int64_t)((rank + nranks + s) % nranks) * count + offset;
      ps->sendDim = s ? firstBitSet(s, nrPow2) : -1;
      if (ps->sendDim == -1) {
        ps->sendOffset = -1;
      } else if (as - (1 << ps->recvDim) == 0) {
        if (newPeer(a, aggFactor)) {
          sendSkipped = a;
          ps->stepOffset = stepOffset = 0;
        }
        ps->sendOffset = ((a - sendSkipped) % postFreq) * nelem;
      }
      const int recvDim = ps->recvDim;
      if (s < nranks && skip) {  // still fold the own input even though nothing arrives
        ps->recvDim = -1;
        ps->recvOffset = -1;
        ps->postRecv = 0;
        skip = false;
      }
      if (recvDim > 0 && ((a - sendSkipped) % postFreq) + 1 >= postFreq && !skip) stepOffset++;
    } else if (phase == 2) {
      int s = (2 * mirrorInvert(a, lastA) + 1) * scale * aggDelta + 1;
      ps->postRecv = 0;
      if (s >= nranks) skip = true;
      ps->recvDim = 0;
      ps->postSend = a == lastA - 1 ? 1 : 0;
      s -= 1;
      if (s < nranks && skip) {
        ps->recvDim = -1;
        ps->recvOffset = -1;
        skip = false;
      } else if (!skip) {
        const int foffset = a + aggFactor - aggFactor / scale;
        ps->postRecv |= ((foffset + 1) % postFreq) == 0 ? 1 : 0;
        ps->recvOffset = (foffset % postFreq) * nelem;
      }
      ps->inpIx = (int64_t)((rank + nranks + s) % nranks) * count + offset;
      ps->sendDim = s ? firstBitSet(s, nrPow2) : -1;
      ps->postSend |= ((a + 1) % postFreq) == 0 ? 1 : 0;
      ps->sendOffset = (a % postFreq) * nelem;
    } else if (phase == 3) {
      int s = (2 * mirrorInvert(a, lastA) + 1) * scale * aggDelta;
      ps->postRecv = a == lastA - 1 ? 1 : 0;
      if (s >= nranks) skip = true;
      ps->recvDim = firstBitSet(s, nrPow2);
      ps->postSend = 0;
      s -= 1 << ps->recvDim;
      ps->postRecv |= (a + 1) % postFreq == 0 ? 1 : 0;
      ps->recvOffset = (a % postFreq) * nelem;
      ps->inpIx = (int64_t)((rank + nranks + s) % nranks) * count + offset;
      ps->sendDim = s ? firstBitSet(s, nrPow2) : -1;
      if (s < nranks && skip) {
        ps->recvDim = -1;
        ps->recvOffset = -1;
        ps->postRecv = 0;
        skip = false;
      }
      if (newPeer(a, aggFactor / (2 * scale))) {
        sendSkipped = a;
        ps->stepOffset = stepOffset = 0;
      }
      const int foffset = a - sendSkipped;
      if ((foffset % postFreq) + 1 >= postFreq && !skip) stepOffset++;
      ps->sendOffset = ps->sendDim >= 0 ? (foffset % postFreq) * nelem : -1;
    } else if (phase == 4) {
      ps->recvDim = 0;
      ps->sendDim = -1;
      ps->inpIx = (int64_t)rank * count + offset;
      ps->recvOffset = ((aggFactor - 1) % postFreq) * nelem;
      ps->sendOffset = -1;
      ps->postRecv = 1;
      ps->postSend = 0;
      offset += chunkCount;
    }
    a++;
    if (a >= lastA && a >= parallelFactor) {
      const int p = phase;
      if (p == 1) as--;
      if (p == 3) scale *= 2;
      phase = p == 0   ? (as == 1 ? (aggFactor > 1 ? 2 : 4) : 1)
              : p == 1 ? (as % 2 == 1 ? 0 : 1)
              : p == 2 ? 3
              : p == 3 ? (scale < aggFactor ? 2 : 4)
                       : 5;
      if (p == 4) {
        if (offset >= end) ps->last = 2;
        else reset();
      } else {
        resetA();
      }
    } else if (phase == 4 && offset >= end) {
      ps->last = 1;
    }
    ps->skipped = skip;
  }
};

// PatAGAlgorithm::getNextOp (collectives.h:807-905): the mirror image. Phase 2 forwards the own
// chunk and received chunks up the aggregated dimensions, phase 1 forwards along one dimension
// while copying into the output, phase 0 only receives on dimension 0. `as` walks the aggregated
// sub-steps in the order nextAs() produces (:757-775).
struct PatAllGatherPlan : PatGeometry {
  int64_t offset, end, count;
  int chunkCount, nelem = 0, rank, nranks;
  int lastA = 0, as = 0, a = 0, scale = 0, phase = 0;
  int asDim, v = 0;
  int bitCount[32], bitZeroStep[32];

  PatAllGatherPlan(int chunkCount_, size_t esz, int64_t count_, int rank_, int nranks_)
      : PatGeometry((uint64_t)chunkCount_ * esz, kSteps, kPatMaxParallel, (uint64_t)count_, esz, nranks_),
        offset(0), end(count_), count(count_), chunkCount(chunkCount_), rank(rank_), nranks(nranks_) {
    asDim = log2Up(aggDelta);
    reset();
  }
  void resetA() {
    a = 0;
    lastA = aggFactor;
    if (phase >= 2) lastA /= 2 * scale;
  }
  void reset() {
    nelem = (int)std::min<int64_t>(chunkCount, end - offset);
    scale = aggFactor / 2;
    phase = scale ? 2 : 1;
    v = 0;
    for (int i = 0; i < asDim; i++) {
      bitCount[i] = asDim - i;
      bitZeroStep[i] = 1;
    }
    as = nextAs();
    resetA();
  }
  int nextAs() {
    for (int d = 0; d < asDim; d++) {
      const int p = 1 << d;
      if (--bitCount[d] == 0) {
        v ^= p;
        bitCount[d] = p;
        if ((v & p) == 0) {
          bitCount[d] += firstBitSet(bitZeroStep[d], asDim) - 1;
          if (bitCount[d] == 0) {
            v ^= p;
            bitCount[d] = p;
          }
          bitZeroStep[d]++;
        }
      }
    }
    return v;
  }
  void next(PatOp* ps) {
    ps->last = 0;
    ps->nelem = nelem;
    ps->inpIx = offset;
    bool skip = false;
    if (a >= lastA) {
      skip = true;
    } else if (phase == 0) {
      const int s = a * aggDelta + as;
      if (s >= nranks) skip = true;
      ps->outIx = (int64_t)((rank + s) % nranks) * count + offset;
      ps->sendDim = -1;
      ps->recvDim = 0;
      ps->inpIx = 0;
      ps->sendOffset = -1;
      ps->recvOffset = (a % postFreq) * nelem;
      ps->stepOffset = 0;
      ps->postRecv = (a % postFreq == postFreq - 1) || ((a + 1) * aggDelta + as >= nranks) ? 1 : 0;
      ps->postSend = 0;
    } else if (phase == 1) {
      int s = a * aggDelta + as;
      if (s >= nranks) skip = true;
      ps->sendDim = firstBitSet(s, nrPow2);
      s -= 1 << ps->sendDim;
      ps->outIx = (int64_t)((rank + nranks + s) % nranks) * count + offset;
      ps->recvDim = s ? firstBitSet(s, nrPow2) : -1;
      ps->sendOffset = ps->recvOffset = (a % postFreq) * nelem;
      ps->postSend = (a % postFreq == postFreq - 1) || ((a + 1) * aggDelta + as >= nranks) ? 1 : 0;
      ps->postRecv =
          (ps->sendDim == 0) && ((a % postFreq == postFreq - 1) || ((a + 1) * aggDelta + as - 1 >= nranks)) ? 1 : 0;
      ps->stepOffset = (ps->sendDim == 0) ? 0 : a / postFreq;
      if (ps->recvDim == -1) {
        ps->recvOffset = -1;
        ps->postRecv = 0;
      } else if (as - (1 << ps->sendDim) == 0) {
        const int foffset = (a * aggDelta) >> (ps->recvDim + 1);
        ps->recvOffset = (foffset % postFreq) * nelem;
        ps->postRecv = (ps->sendDim == 0) && ((foffset % postFreq == postFreq - 1) ||
                                              ((((foffset + 1) * 2) + 1) << ps->recvDim) >= nranks)
                           ? 1
                           : 0;
        ps->stepOffset = (ps->sendDim == 0) ? 0 : foffset / postFreq;
      }
      if (s < nranks && ps->sendDim == 0 && skip) {  // receive once even when nothing is sent on
        ps->sendDim = -1;
        ps->sendOffset = -1;
        ps->postSend = 0;
        skip = false;
      }
    } else if (phase == 2) {
      int s = (2 * a + 1) * scale * aggDelta;
      ps->postSend = (a % postFreq == postFreq - 1) || ((2 * (a + 1) + 1) * scale * aggDelta >= nranks) ? 1 : 0;
      ps->postRecv = 0;
      if (s >= nranks) skip = true;
      ps->sendDim = firstBitSet(s, nrPow2);
      s -= 1 << ps->sendDim;
      ps->sendOffset = (a % postFreq) * nelem;
      ps->stepOffset = a / postFreq;
      ps->outIx = (int64_t)((rank + nranks + s) % nranks) * count + offset;
      ps->recvDim = s ? firstBitSet(s, nrPow2) : -1;
      if (ps->recvDim == -1) {
        ps->recvOffset = -1;
      } else {
        const int foffset = (a * 2 * scale * aggDelta) >> (ps->recvDim + 1);
        ps->recvOffset = (foffset % postFreq) * nelem;
        ps->stepOffset = foffset / postFreq;
      }
    }
    a++;
    if (a >= lastA && a >= parallelFactor) {
      const int p = phase;
      if (p == 2) scale /= 2;
      phase = p == 2 ? (scale ? 2 : 1) : p == 1 ? (as % 2 == 1 ? 0 : 1) : 1;
      if (p == 0 || (p == 1 && as % 2 == 0)) as = nextAs();
      if (p == 0 && as == aggDelta / 2) {
        offset += chunkCount;
        if (offset >= end) ps->last = 2;
        else reset();
      } else {
        resetA();
      }
    } else if (phase == 0 && as == 1 && offset + chunkCount >= end &&
               a - 1 >= ((lastA - 1) / parallelFactor) * parallelFactor) {
      ps->last = 1;
    }
    ps->skipped = skip;
  }
};

// calcCollChunking for PAT on one channel (enqueue.cc:1993-1996, :2048-2051, :2062): one FIFO step
// per chunk, halved while the chunk is large next to the collective (nBytes = nRanks * count * esz,
// ncclFuncMaxSendRecvCount), never below 64 KiB by halving; aligned to the SIMPLE grain.
int64_t patChunkElems(const nexrRingComm* c, size_t esz, bool allGather, int64_t count) {
  int64_t chunk = (int64_t)c->stepBytes;
  const int64_t nBytes = (int64_t)c->cfg.nRanks * count * (int64_t)esz;
  while (chunk * (allGather ? 32 : 16) > nBytes && chunk > 65536) chunk /= 2;
  chunk = chunk / 512 * 512;
  return chunk / (int64_t)esz;
}

// The PAT op stream of one rank, for inspection (nexrPatSchedule) and for the executor.
template <typename Plan>
std::vector<PatOp> patOps(Plan plan, int* parallelFactor) {
  std::vector<PatOp> ops;
  *parallelFactor = plan.parallelFactor;
  for (;;) {
    PatOp op;
    plan.next(&op);
    ops.push_back(op);
    if (op.last == 2) break;
  }
  return ops;
}

struct PatPeer {
  Conn* conn = nullptr;
  uint64_t step = 0;     // ncclPatPeer::step, loaded from conn->step (prims_simple.h:699, :710)
  int64_t accSize = 0;   // elements of the FIFO's absolute index space already written / delivered
};

// One rank of a PAT collective: Prims supplies the rank's buffers, reduce-copy function, stream
// and bounded waits; the dims are its ncclPatShmem recvDims / sendDims.
struct PatRank {
  Prims p;
  bool reduceScatter;
  PatPeer recvDims[kPatMaxDims], sendDims[kPatMaxDims];
  int64_t localAccSize = 0;  // ncclPatShmem::localAccSize
  int64_t stepElems = 0;     // connStepSize

  const char* fifoAt(const PatPeer& q, uint64_t step, int off) const {
    return q.conn->fifo + ((int64_t)(step % kSteps) * stepElems + off) * (int64_t)p.esz;
  }
  bool waitData(PatPeer& q, uint64_t target) { return p.waitAtLeast(q.conn->st->tail, target); }
  bool waitCredit(PatPeer& q, uint64_t target) {
    return target <= (uint64_t)kSteps || p.waitAtLeast(q.conn->st->head, target - kSteps);
  }
  nexrResult_t issue(int k, const void* const* srcs, int m, void* const* dsts, int nelem) {
    if (nelem <= 0 || k == 0 || m == 0) return nexrSuccess;
    return p.fn(k, srcs, m, dsts, (size_t)nelem, p.datatype, p.devOp, p.redOpArgs[0], 0, nullptr, 0,
                (nexrStream_t)p.stream);
  }

  // One lock-step batch (parallelFactor consecutive ops).
  bool runBatch(const PatOp* ops, int nOps) {
    bool postRecv[kPatMaxDims] = {}, postSend[kPatMaxDims] = {};
    int64_t recvAcc[kPatMaxDims], sendAcc[kPatMaxDims];
    for (int d = 0; d < kPatMaxDims; d++) recvAcc[d] = sendAcc[d] = -1;
    int64_t localAcc = localAccSize;
    for (int j = 0; j < nOps; j++) {
      const PatOp& op = ops[j];
      if (op.skipped) continue;
      const int nelem = op.nelem < 0 ? 0 : op.nelem;
      nexrResult_t r;
      if (reduceScatter) {  // patReduce (prims_simple.h:992-1088)
        const void* srcs[2];
        void* dst;
        int k = 0;
        if (op.recvDim >= 0) {
          PatPeer& q = recvDims[op.recvDim];
          if (!waitData(q, q.step + 1)) return false;
          srcs[k++] = fifoAt(q, q.step, op.recvOffset);
        }
        const char* own = p.userInput + op.inpIx * (int64_t)p.esz;
        if (op.sendDim >= 0) {
          PatPeer& q = sendDims[op.sendDim];
          const uint64_t s = q.step + op.stepOffset;
          if (!waitCredit(q, s + 1)) return false;
          dst = const_cast<char*>(fifoAt(q, s, op.sendOffset));
          const int64_t mark = op.sendOffset + nelem + (int64_t)s * stepElems;
          if (q.accSize >= mark) own = (const char*)dst;  // data already there: accumulate into it
          sendAcc[op.sendDim] = std::max(sendAcc[op.sendDim], mark);
        } else {
          dst = p.userOutput + op.outIx * (int64_t)p.esz;
          if (localAccSize < op.outIx + nelem) localAcc = std::max(localAcc, op.outIx + nelem);
          else own = (const char*)dst;
        }
        srcs[k++] = own;  // srcs = [received partial, own input or accumulator]
        r = issue(k, srcs, 1, &dst, nelem);
      } else {  // patCopy (prims_simple.h:1090-1183)
        const void* src;
        void* dsts[2];
        int m = 0;
        char* out;
        if (op.recvDim >= 0) {
          PatPeer& q = recvDims[op.recvDim];
          const uint64_t s = q.step + op.stepOffset;
          if (!waitData(q, s + 1)) return false;
          src = fifoAt(q, s, op.recvOffset);
          const int64_t mark = op.recvOffset + nelem + (int64_t)s * stepElems;
          out = q.accSize < mark ? p.userOutput + op.outIx * (int64_t)p.esz : (char*)src;  // else: delivered
          recvAcc[op.recvDim] = std::max(recvAcc[op.recvDim], mark);
        } else {
          src = p.userInput + op.inpIx * (int64_t)p.esz;
          if (localAccSize < op.inpIx + nelem) {
            out = p.userOutput + op.outIx * (int64_t)p.esz;
            localAcc = std::max(localAcc, op.inpIx + nelem);
          } else {
            out = (char*)src;
          }
        }
        if (op.sendDim >= 0) {
          PatPeer& q = sendDims[op.sendDim];
          if (!waitCredit(q, q.step + 1)) return false;
          dsts[m++] = const_cast<char*>(fifoAt(q, q.step, op.sendOffset));
        }
        if (out != (const char*)src) dsts[m++] = out;  // in place, or already delivered
        r = issue(1, &src, m, dsts, nelem);
      }
      if (r != nexrSuccess) {
        p.sh->fail(r);
        return false;
      }
      if (op.postRecv && op.recvDim >= 0) postRecv[op.recvDim] = true;
      if (op.postSend && op.sendDim >= 0) postSend[op.sendDim] = true;
    }
    if (p.device && hipStreamSynchronize(p.stream) != hipSuccess) {
      p.sh->fail(nexrUnhandledCudaError);
      return false;
    }
    localAccSize = localAcc;
    for (int d = 0; d < kPatMaxDims; d++) {
      if (recvAcc[d] >= 0) recvDims[d].accSize = std::max(recvDims[d].accSize, recvAcc[d]);
      if (sendAcc[d] >= 0) sendDims[d].accSize = std::max(sendDims[d].accSize, sendAcc[d]);
    }
    for (int d = 0; d < kPatMaxDims; d++) {  // every post in a batch stores the batch-start step + 1
      if (postSend[d]) {
        PatPeer& q = sendDims[d];
        q.conn->sendStep = ++q.step;
        q.conn->st->tail.store(q.step, std::memory_order_release);
      }
      if (postRecv[d]) {
        PatPeer& q = recvDims[d];
        q.conn->recvStep = ++q.step;
        q.conn->st->head.store(q.step, std::memory_order_release);
      }
    }
    return true;
  }

  void run(int64_t count, int nranks) {
    const int64_t chunkCount = patChunkElems(p.c, p.esz, !reduceScatter, count);
    int pf = 1;
    const std::vector<PatOp> ops =
        reduceScatter ? patOps(PatReduceScatterPlan((int)chunkCount, p.esz, count, p.rank, nranks), &pf)
                      : patOps(PatAllGatherPlan((int)chunkCount, p.esz, count, p.rank, nranks), &pf);
    // Worker group g runs ops g, g+pf, ... and stops after its first op with `last` set
    // (reduce_scatter.h:127-138): the stream must end on a whole batch whose every op is marked.
    for (size_t b = 0; b < ops.size(); b += (size_t)pf) {
      const int nb = (int)std::min<size_t>((size_t)pf, ops.size() - b);
      if (!runBatch(&ops[b], nb)) return;
      int marked = 0;
      for (int j = 0; j < nb; j++) marked += ops[b + j].last != 0;
      if (marked == 0) continue;
      if (marked != pf || b + (size_t)pf != ops.size()) p.sh->fail(nexrInternalError);
      return;
    }
  }
};

// Connection r -> q for PAT (channel.peers[q]->send[0] of rank r): the ring connection when q = r+1,
// otherwise one made by the first PAT call, its FIFO on q's device.
Conn* patConn(nexrRingComm* c, int from, int to) {
  if (to == (from + 1) % c->cfg.nRanks) return c->conns[to];
  return c->patConns[(size_t)from * c->cfg.nRanks + to];
}

nexrResult_t ensurePat(nexrRingComm* c) {
  if (!c->patConns.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks;
  c->patConns.assign((size_t)n * n, nullptr);
  for (int r = 0; r < n; r++) {
    for (int d = 0; d < kPatMaxDims && (1 << d) < n; d++) {
      for (int q : {(r + (1 << d)) % n, (r - (1 << d) + n) % n}) {
        Conn*& k = c->patConns[(size_t)r * n + q];
        if (q == (r + 1) % n || k) continue;
        k = new Conn();
        nexrResult_t res = allocFifo(c, k, c->devices[q]);
        if (res == nexrSuccess && c->cfg.memMode == nexrRingDeviceMemory) res = enablePeer(c->devices[r], c->devices[q]);
        if (res != nexrSuccess) return res;
      }
    }
  }
  return nexrSuccess;
}


// One rank's PAT collective on the calling thread (thread ranks and process ranks alike).
void runPatRank(nexrRingComm* c, Shared* sh, int rank, bool reduceScatter, const void* sendbuff, void* recvbuff,
                size_t count, size_t esz, int datatype, const nexrDevRedOpFull& red) {
  const int n = c->cfg.nRanks;
  if (c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
  PatRank pr;
  pr.p = makePrims(c, sh, rank, sendbuff, recvbuff, esz, datatype, red, kGeomPipe, c->streams[rank], c->status[rank]);
  pr.reduceScatter = reduceScatter;
  pr.stepElems = (int64_t)(c->stepBytes / esz);
  for (int d = 0; d < kPatMaxDims && (1 << d) < n; d++) {
    const int delta = 1 << d;
    const int lo = (rank - delta + n) % n, hi = (rank + delta) % n;
    // ReduceScatter receives from rank-2^d and sends to rank+2^d; AllGather the other way round.
    const int recvPeer = reduceScatter ? lo : hi, sendPeer = reduceScatter ? hi : lo;
    pr.recvDims[d].conn = patConn(c, recvPeer, rank);
    pr.recvDims[d].step = pr.recvDims[d].conn->recvStep;
    pr.sendDims[d].conn = patConn(c, rank, sendPeer);
    pr.sendDims[d].step = pr.sendDims[d].conn->sendStep;
  }
  pr.run((int64_t)count, n);
}

// Argument checks shared by the thread-rank and process-rank PAT entry points.
nexrResult_t patPrepare(nexrRingComm* c, bool reduceScatter, int datatype, int op, size_t count, size_t* esz,
                        nexrDevRedOpFull* red) {
  nexrResult_t r = prepare(c, datatype, op, esz, red);
  if (r != nexrSuccess) return r;
  // PAT runs SIMPLE only (tuning.cc:264) and never for ReduceScatter with a pre/post-op scaling
  // (ncclAvg / user PreMulSum, enqueue.cc:1779-1780).
  if (c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  if (reduceScatter && (red->op == nexrDevPreMulSum || red->op == nexrDevSumPostDiv)) return nexrInvalidArgument;
  if (count > (size_t)INT32_MAX) return nexrInvalidArgument;  // ncclPatStep offsets are int
  return nexrSuccess;
}

nexrResult_t patCollective(nexrRingComm* c, bool reduceScatter, const void* const* sendbuffs, void* const* recvbuffs,
                           size_t count, int datatype, int op) {
  if (!c || c->peer) return nexrInvalidArgument;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = patPrepare(c, reduceScatter, datatype, op, count, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks;
  if (!sendbuffs || !recvbuffs) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  for (int i = 0; i < n; i++)
    if (!sendbuffs[i] || !recvbuffs[i]) return nexrInvalidArgument;
  if (n == 1) return oneRank(c, 0, sendbuffs[0], recvbuffs[0], count, datatype, red, esz);
  r = ensurePat(c);
  if (r != nexrSuccess) {
    c->broken = true;
    return r;
  }
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (int rank = 0; rank < n; rank++)
    jobs.emplace_back([&, rank] {
      runPatRank(c, &sh, rank, reduceScatter, sendbuffs[rank], recvbuffs[rank], count, esz, datatype, red);
    });
  return runThreads(c, sh, jobs);
}

// ---- ncclSend / ncclRecv (the P2P work batch, src/device/sendrecv.h) --------------------------------
// Every rank's send and recv run side by side, as the reference splits a work's warps between
// them (sendrecv.h:144-176): the send half on the rank's stream, the recv half on its second stream.
// runSend / runRecv (:15-62) move the message in chunks of the P2P chunk size through
// Primitives<FanAsymmetric<0,1> / <1,0>, ProtoSimple<1,1>> on connection index 1: directSend is
// genericOp(Input -> peer FIFO) and directRecv genericOp(peer FIFO -> Output). A send to self is one
// reduceCopy copy (:192-194). Messages are bytes (T = int8, :13).

// u32fp8Encode/Decode (src/include/bitops.h:384-410): the work descriptor carries the chunk size in
// 8 bits, so the chunk the kernels use is the encoded value decoded again (enqueue.cc:854-855).
uint32_t u32fp8RoundTrip(uint32_t x) {
  const int log2x = 31 - __builtin_clz(x | 1);
  const uint32_t mant = x >> (log2x >= 3 ? log2x - 3 : 0) & 7u;
  uint32_t expo = log2x >= 3 ? (uint32_t)(log2x - 2) : 0;
  const uint32_t m = mant | (expo != 0 ? 8u : 0u);
  if (expo != 0) expo -= 1;
  return m << expo;
}

Conn* p2pConn(nexrRingComm* c, int from, int to, bool ll) {
  return (ll ? c->p2pLLConns : c->p2pConns)[(size_t)from * c->cfg.nRanks + to];
}

// P2P messages of at most this many bytes take the LL protocol (NCCL_P2P_LL_THRESHOLD x 1 channel,
// enqueue.cc:786, :825-839), when an LL step implementation can reach the FIFO lines: device
// memory, or a caller-supplied llFn. Self-sends never do (:805).
constexpr size_t kP2pLLThreshold = 16384;
bool p2pUsesLL(const nexrRingComm* c, size_t bytes) {
  return bytes <= kP2pLLThreshold && (c->cfg.memMode == nexrRingDeviceMemory || c->cfg.llFn != defaultLLFn);
}

nexrResult_t ensureP2p(nexrRingComm* c, const int* sendPeers, bool ll) {
  const int n = c->cfg.nRanks;
  std::vector<Conn*>& conns = ll ? c->p2pLLConns : c->p2pConns;
  if (conns.empty()) conns.assign((size_t)n * n, nullptr);
  for (int r = 0; r < n; r++) {
    const int q = sendPeers[r];
    if (q < 0 || q == r || p2pConn(c, r, q, ll)) continue;
    Conn* k = new Conn();
    conns[(size_t)r * n + q] = k;
    // SIMPLE: 8 steps of the P2P chunk; LL: the LL buffer's 8 steps of 64 KiB lines (init.cc:618)
    k->slotBytes = ll ? kDefaultLLBuffBytes / kSteps : c->p2pChunkBytes;
    nexrResult_t res = allocFifo(c, k, c->devices[q], ll ? kDefaultLLBuffBytes : 0);
    if (res == nexrSuccess && c->cfg.memMode == nexrRingDeviceMemory) res = enablePeer(c->devices[r], c->devices[q]);
    if (res != nexrSuccess) return res;
  }
  return nexrSuccess;
}

// The halves of one rank's P2P work (sendrecv.h:174-194), each on the calling thread.
void runSelfCopy(nexrRingComm* c, Shared* sh, int rank, const void* src, void* dst, size_t bytes) {
  if (c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
  nexrResult_t r = c->cfg.fn(1, &src, 1, &dst, bytes, nexrInt8, nexrDevSum, 0, 0, nullptr, 0,
                             (nexrStream_t)c->streams[rank]);
  if (r == nexrSuccess && c->streams[rank] && c->cfg.memMode == nexrRingDeviceMemory &&
      hipStreamSynchronize(c->streams[rank]) != hipSuccess)
    r = nexrUnhandledCudaError;
  if (r != nexrSuccess) sh->fail(r);
}

void runP2pHalf(nexrRingComm* c, Shared* sh, int rank, bool send, int peer, const void* sendbuff, void* recvbuff,
                size_t bytes) {
  hipStream_t s = send ? c->streams[rank] : c->streams2[rank];
  if (s) (void)hipSetDevice(c->devices[rank]);
  const nexrDevRedOpFull copy = {nexrDevSum, 0, 0, 0};
  const bool ll = p2pUsesLL(c, bytes);
  Prims p = makePrims(c, sh, rank, sendbuff, recvbuff, 1, nexrInt8, copy, kGeomPipe, s,
                      send ? c->status[rank] : c->status2[rank]);
  p.proto = ll ? nexrRingProtoLL : nexrRingProtoSimple;
  p.stepSize = (int64_t)c->p2pChunkBytes;  // Primitives' P2P stepSize argument (sendrecv.h:27-29)
  if (send) p.send[p.nSend++] = p2pConn(c, rank, peer, ll);
  else p.recv[p.nRecv++] = p2pConn(c, peer, rank, ll);
  p.attach();
  // The chunk (enqueue.cc:840-856): SIMPLE moves p2pChunkSize per chunk, LL half an LL step of data;
  // either way after the 8-bit u32fp8 round trip of the work descriptor.
  const int64_t chunk = (int64_t)u32fp8RoundTrip((uint32_t)(ll ? kDefaultLLBuffBytes / kSteps / 2 : c->p2pChunkBytes));
  for (int64_t cursor = 0; cursor < (int64_t)bytes;) {  // runSend / runRecv (:15-62)
    const int64_t m = std::min<int64_t>(chunk, (int64_t)bytes - cursor);
    if (!(send ? p.sendInput(cursor, m) : p.recvOutput(cursor, m))) return;
    cursor += m;
  }
}

nexrResult_t sendRecv(nexrRingComm* c, const void* const* sendbuffs, const int* sendPeers, void* const* recvbuffs,
                      const int* recvPeers, size_t bytes) {
  if (!c || c->peer || !sendbuffs || !sendPeers || !recvbuffs || !recvPeers) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  if (c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  const int n = c->cfg.nRanks;
  for (int r = 0; r < n; r++) {  // every send matches the peer's recv, and the other way round
    const int s = sendPeers[r], v = recvPeers[r];
    if (s < -1 || s >= n || v < -1 || v >= n) return nexrInvalidArgument;
    if (s >= 0 && recvPeers[s] != r) return nexrInvalidArgument;
    if (v >= 0 && sendPeers[v] != r) return nexrInvalidArgument;
    if (bytes > 0 && ((s >= 0 && !sendbuffs[r]) || (v >= 0 && !recvbuffs[r]))) return nexrInvalidArgument;
  }
  if (bytes == 0) return nexrSuccess;
  nexrResult_t res = ensureSecondStreams(c);
  if (res == nexrSuccess) res = ensureP2p(c, sendPeers, p2pUsesLL(c, bytes));
  if (res != nexrSuccess) {
    c->broken = true;
    return res;
  }
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (int rank = 0; rank < n; rank++) {
    const int to = sendPeers[rank], from = recvPeers[rank];
    if (to == rank) {  // isCopy: one reduceCopy from the send buffer to the recv buffer
      jobs.emplace_back([&, rank] { runSelfCopy(c, &sh, rank, sendbuffs[rank], recvbuffs[rank], bytes); });
      continue;
    }
    if (to >= 0)
      jobs.emplace_back([&, rank, to] { runP2pHalf(c, &sh, rank, true, to, sendbuffs[rank], recvbuffs[rank], bytes); });
    if (from >= 0)
      jobs.emplace_back(
          [&, rank, from] { runP2pHalf(c, &sh, rank, false, from, sendbuffs[rank], recvbuffs[rank], bytes); });
  }
  return runThreads(c, sh, jobs);
}

// The op stream of one rank, as plain ints for inspection: 12 per op, in the order of PatOp's fields
// recvDim, sendDim, recvOffset, sendOffset, stepOffset, postRecv, postSend, nelem, last, skipped,
// inpIx, outIx.
nexrResult_t patSchedule(bool reduceScatter, int nRanks, int rank, size_t count, size_t esz, size_t stepBytes,
                         int64_t* out, size_t capOps, size_t* nOps, int* parallelFactor) {
  if (nRanks < 2 || rank < 0 || rank >= nRanks || count == 0 || count > (size_t)INT32_MAX || esz == 0 ||
      stepBytes < 512 || !nOps || !parallelFactor)
    return nexrInvalidArgument;
  nexrRingComm tmp;
  tmp.cfg.nRanks = nRanks;
  tmp.stepBytes = stepBytes;
  const int64_t chunkCount = patChunkElems(&tmp, esz, !reduceScatter, (int64_t)count);
  if (chunkCount <= 0) return nexrInvalidArgument;
  const std::vector<PatOp> ops =
      reduceScatter ? patOps(PatReduceScatterPlan((int)chunkCount, esz, (int64_t)count, rank, nRanks), parallelFactor)
                    : patOps(PatAllGatherPlan((int)chunkCount, esz, (int64_t)count, rank, nRanks), parallelFactor);
  *nOps = ops.size();
  if (out) {
    for (size_t i = 0; i < ops.size() && i < capOps; i++) {
      const PatOp& o = ops[i];
      const int64_t v[12] = {o.recvDim, o.sendDim, o.recvOffset, o.sendOffset, o.stepOffset, o.postRecv,
                             o.postSend, o.nelem,   o.last,       o.skipped ? 1 : 0, o.inpIx, o.outIx};
      memcpy(out + i * 12, v, sizeof(v));
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
  if (cfg->treeRanksPerNode < 0 || (cfg->treeRanksPerNode > 0 && cfg->nRanks % cfg->treeRanksPerNode != 0) ||
      (cfg->treeIndex != 0 && cfg->treeIndex != 1))
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
  if (!validConfigBuff(c)) {
    delete c;
    return nexrInvalidArgument;
  }
  if (!c->cfg.fn) c->cfg.fn = cfg->memMode == nexrRingDeviceMemory ? defaultDeviceFn : defaultHostFn;
  if (!c->cfg.llFn) c->cfg.llFn = defaultLLFn;
  if (!c->cfg.ll128Fn) c->cfg.ll128Fn = defaultLL128Fn;
  c->stepBytes = c->cfg.buffBytes / kSteps;
  // comm->p2pChunkSize (init.cc:637-642): NCCL_P2P_PCI_CHUNKSIZE (128 KiB, the single-node non-NVLink
  // default), at most one SIMPLE step.
  c->p2pChunkBytes = std::min<size_t>(128 << 10, c->stepBytes);
  const int n = cfg->nRanks;
  c->tree = treeTopology(n, cfg->treeRanksPerNode > 0 ? cfg->treeRanksPerNode : n, cfg->treeIndex);
  c->devices.assign(n, 0);
  c->streams.assign(n, nullptr);
  c->status.assign(n, nullptr);
  int nDev = 0;
  c->needHip = cfg->memMode == nexrRingDeviceMemory || (c->proto == nexrRingProtoSimple && !cfg->fn) ||
               (c->proto == nexrRingProtoLL && !cfg->llFn) || (c->proto == nexrRingProtoLL128 && !cfg->ll128Fn);
  c->pinnedStatus = c->needHip;
  if (c->needHip) {
    if (hipGetDeviceCount(&nDev) != hipSuccess || nDev < 1) {
      delete c;
      return nexrUnhandledCudaError;
    }
  }
  for (int r = 0; r < n; r++) c->devices[r] = nDev > 0 ? r % nDev : 0;
  for (int r = 0; r < n; r++) {
    c->conns.push_back(new Conn());
    if (nDev > 0) {
      if (hipSetDevice(c->devices[r]) != hipSuccess || hipStreamCreate(&c->streams[r]) != hipSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
    }
    nexrResult_t res = c->ll ? allocStatus(c, &c->status[r]) : nexrSuccess;
    if (res == nexrSuccess) res = allocFifo(c, c->conns[r], c->devices[r]);
    if (res != nexrSuccess) {
      nexrRingCommDestroy(c);
      return res;
    }
  }
  if (cfg->memMode == nexrRingDeviceMemory && nDev > 1) {  // sender writes into the receiver's FIFO
    for (int r = 0; r < n; r++) {
      if (enablePeer(c->devices[r], c->devices[(r + 1) % n]) != nexrSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
    }
  }
  *out = c;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingAllReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op) {
  return ringCollective(c, kAllReduce, sendbuffs, recvbuffs, count, datatype, op, 0);
}

NEXR_API nexrResult_t nexrRingReduceScatter(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                            size_t recvcount, int datatype, int op) {
  return ringCollective(c, kReduceScatter, sendbuffs, recvbuffs, recvcount, datatype, op, 0);
}

NEXR_API nexrResult_t nexrRingAllGather(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t sendcount, int datatype) {
  return ringCollective(c, kAllGather, sendbuffs, recvbuffs, sendcount, datatype, nexrSum, 0);  // ncclAllGather: ncclSum
}

NEXR_API nexrResult_t nexrRingReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                     size_t count, int datatype, int op, int root) {
  return ringCollective(c, kReduce, sendbuffs, recvbuffs, count, datatype, op, root);
}

NEXR_API nexrResult_t nexrRingBroadcast(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int root) {
  return ringCollective(c, kBroadcast, sendbuffs, recvbuffs, count, datatype, nexrSum, root);  // ncclBroadcast: ncclSum
}

NEXR_API nexrResult_t nexrTreeAllReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op) {
  if (!c || c->peer) return nexrInvalidArgument;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = prepare(c, datatype, op, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks;
  if (!sendbuffs || !recvbuffs) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  for (int i = 0; i < n; i++)
    if (!sendbuffs[i] || !recvbuffs[i]) return nexrInvalidArgument;
  if (n == 1) return oneRank(c, 0, sendbuffs[0], recvbuffs[0], count, datatype, red, esz);
  r = ensureTree(c);
  if (r != nexrSuccess) {
    c->broken = true;
    return r;
  }
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (int rank = 0; rank < n; rank++) {
    const TreeLinks& t = c->tree[rank];
    const bool leaf = t.down[0] == -1;
    auto make = [&, rank](hipStream_t s, uint32_t* st) {
      return makePrims(c, &sh, rank, sendbuffs[rank], recvbuffs[rank], esz, datatype, red, kGeomPipe, s, st);
    };
    if (t.up == -1) {  // root: recv from and send to every child
      jobs.emplace_back([&, rank, make] {
        if (c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
        Prims p = make(c->streams[rank], c->status[rank]);
        const TreeLinks& tl = c->tree[rank];
        for (int i = 0; i < tl.nDown(); i++) {
          p.recv[p.nRecv++] = c->treeUp[tl.down[i]];
          p.send[p.nSend++] = c->treeDown[tl.down[i]];
        }
        p.attach();
        runTree(p, (int64_t)count, kTreeRoot, false);
      });
      continue;
    }
    jobs.emplace_back([&, rank, leaf, make] {  // reduce up: recv from children, send to the parent
      if (c->streams[rank]) (void)hipSetDevice(c->devices[rank]);
      Prims p = make(c->streams[rank], c->status[rank]);
      const TreeLinks& tl = c->tree[rank];
      for (int i = 0; i < tl.nDown(); i++) p.recv[p.nRecv++] = c->treeUp[tl.down[i]];
      p.send[p.nSend++] = c->treeUp[rank];
      p.attach();
      runTree(p, (int64_t)count, kTreeReduceUp, leaf);
    });
    jobs.emplace_back([&, rank, leaf, make] {  // broadcast down: recv from the parent, send to children
      if (c->streams2[rank]) (void)hipSetDevice(c->devices[rank]);
      Prims p = make(c->streams2[rank], c->status2[rank]);
      const TreeLinks& tl = c->tree[rank];
      p.recv[p.nRecv++] = c->treeDown[rank];
      for (int i = 0; i < tl.nDown(); i++) p.send[p.nSend++] = c->treeDown[tl.down[i]];
      p.attach();
      runTree(p, (int64_t)count, kTreeBcastDown, leaf);
    });
  }
  return runThreads(c, sh, jobs);
}

NEXR_API nexrResult_t nexrPatReduceScatter(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                           size_t recvcount, int datatype, int op) {
  return patCollective(c, true, sendbuffs, recvbuffs, recvcount, datatype, op);
}

NEXR_API nexrResult_t nexrPatAllGather(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                       size_t sendcount, int datatype) {
  return patCollective(c, false, sendbuffs, recvbuffs, sendcount, datatype, nexrSum);  // ncclAllGather: ncclSum
}

NEXR_API nexrResult_t nexrSendRecv(nexrRingComm_t c, const void* const* sendbuffs, const int* sendPeers,
                                   void* const* recvbuffs, const int* recvPeers, size_t bytes) {
  return sendRecv(c, sendbuffs, sendPeers, recvbuffs, recvPeers, bytes);
}

NEXR_API nexrResult_t nexrPatSchedule(int reduceScatter, int nRanks, int rank, size_t count, int datatype,
                                      size_t buffBytes, int64_t* ops, size_t capOps, size_t* nOps,
                                      int* parallelFactor) {
  const size_t esz = nexrTypeSize(datatype);
  if (esz == 0 || buffBytes % (kSteps * 16) != 0) return nexrInvalidArgument;
  return patSchedule(reduceScatter != 0, nRanks, rank, count, esz, (buffBytes ? buffBytes : kDefaultBuffBytes) / kSteps,
                     ops, capOps, nOps, parallelFactor);
}

NEXR_API nexrResult_t nexrTreeTopology(nexrRingComm_t c, int rank, int* up, int* down) {
  if (!c || !up || !down || rank < 0 || rank >= c->cfg.nRanks || c->tree.empty()) return nexrInvalidArgument;
  *up = c->tree[rank].up;
  for (int i = 0; i < kMaxArity; i++) down[i] = c->tree[rank].down[i];
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingCommDestroy(nexrRingComm_t c) {
  if (!c) return nexrInvalidArgument;
  if (c->peer) {
    if (!c->streams.empty() && c->streams[c->self]) (void)hipStreamSynchronize(c->streams[c->self]);
    const int next = (c->self + 1) % c->cfg.nRanks;
    if (next != c->self && c->conns.size() > (size_t)next && c->conns[next]->fifo && !c->conns[next]->ownsFifo)
      (void)hipIpcCloseMemHandle(c->conns[next]->fifo);
    if (c->shm) {
      PeerHeader* h = peerHeader(c->shm);
      // The last rank to leave removes the segment's name (each rank still unmaps its own view).
      if (h->joined.load() > 0 && h->left.fetch_add(1) + 1 == h->nRanks) shm_unlink(c->shmName);
      munmap(c->shm, c->shmBytes);
    }
    for (size_t r = 0; r < c->conns.size(); r++) {
      c->conns[r]->st = &c->conns[r]->own;  // counters lived in the unmapped segment
      if ((int)r != c->self) c->conns[r]->fifo = nullptr;  // only this rank's FIFO is owned here
    }
    for (auto* v : {&c->patConns, &c->p2pConns, &c->p2pLLConns})
      for (Conn* k : *v) {
        if (!k) continue;
        k->st = &k->own;
        if (!k->ownsFifo && k->fifo) {
          (void)hipIpcCloseMemHandle(k->fifo);
          k->fifo = nullptr;
        }
      }
  }
  for (Conn* k : c->conns) freeConn(c, k);
  for (Conn* k : c->treeUp) freeConn(c, k);
  for (Conn* k : c->treeDown) freeConn(c, k);
  for (Conn* k : c->patConns) freeConn(c, k);
  for (Conn* k : c->p2pConns) freeConn(c, k);
  for (Conn* k : c->p2pLLConns) freeConn(c, k);
  for (auto* v : {&c->status, &c->status2})
    for (uint32_t* s : *v)
      if (s) {
        if (c->pinnedStatus) (void)hipHostFree(s);
        else free(s);
      }
  for (auto* v : {&c->streams, &c->streams2})
    for (size_t r = 0; r < v->size(); r++)
      if ((*v)[r]) {
        (void)hipSetDevice(c->devices[r]);
        (void)hipStreamDestroy((*v)[r]);
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
  if (!validConfigBuff(c)) {
    delete c;
    return nexrInvalidArgument;
  }
  c->cfg.fn = defaultDeviceFn;
  c->cfg.llFn = defaultLLFn;
  c->cfg.ll128Fn = defaultLL128Fn;
  c->stepBytes = c->cfg.buffBytes / kSteps;
  c->p2pChunkBytes = std::min<size_t>(128 << 10, c->stepBytes);  // as nexrRingCommCreate
  c->peer = true;
  c->needHip = true;
  const int n = cfg->nRanks, me = cfg->rank, next = (me + 1) % n;
  c->self = me;
  c->devices.assign(n, cfg->device);
  c->streams.assign(n, nullptr);
  c->status.assign(n, nullptr);
  c->pinnedStatus = true;
  for (int r = 0; r < n; r++) {
    c->conns.push_back(new Conn());
    c->conns[r]->device = cfg->device;
  }
  strncpy(c->shmName, cfg->shmName, sizeof(c->shmName) - 1);
  auto fail = [&](nexrResult_t r) {
    if (c->shm) peerHeader(c->shm)->abort.store(1);
    nexrRingCommDestroy(c);
    return r;
  };
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreate(&c->streams[me]) != hipSuccess)
    return fail(nexrUnhandledCudaError);
  if (c->ll && allocStatus(c, &c->status[me]) != nexrSuccess) return fail(nexrUnhandledCudaError);
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
    char* mapped = nullptr;
    if (hipIpcOpenMemHandle((void**)&mapped, hd, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
      return fail(nexrUnhandledCudaError);
    c->conns[next]->fifo = mapped;
    c->conns[next]->ownsFifo = false;
    c->conns[next]->st = &peerSlot(c->shm, next)->conn;
  }
  *out = c;
  return nexrSuccess;
}

}  // extern "C"

namespace {

bool isPatPair(int n, int from, int to) {
  for (int d = 0; (1 << d) < n; d++)
    if (to == (from + (1 << d)) % n || to == (from - (1 << d) + n) % n) return true;
  return false;
}

// Process ranks: the first PAT (p2p = false) or Send/Recv (p2p = true) call on a communicator
// connects this rank's extra links. Every rank allocates the FIFOs it receives into, publishes
// their IPC handles in the shared segment, and, once all ranks have, maps the FIFOs it sends into.
// Collective: every rank makes its first call of each kind together.
nexrResult_t ensurePeerLinks(nexrRingComm* c, bool p2p) {
  std::vector<Conn*>& first = p2p ? c->p2pConns : c->patConns;
  if (!first.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks, me = c->self;
  if (n > kPeerLinkMaxRanks) return nexrInvalidUsage;
  auto isLink = [&](int from, int to) {
    return from != to && (p2p || (to != (from + 1) % n && isPatPair(n, from, to)));  // r -> r+1 is the ring's
  };
  // The link sets this kind connects: PAT's; or P2P's SIMPLE buffers and their LL buffers.
  struct Set {
    std::vector<Conn*>* conns;
    size_t bytes, slot;
    ConnState PeerLink::*state;
    hipIpcMemHandle_t PeerLink::*handle;
  };
  std::vector<Set> sets;
  if (p2p) {
    sets.push_back({&c->p2pConns, c->p2pChunkBytes * kSteps, c->p2pChunkBytes, &PeerLink::p2p, &PeerLink::p2pFifo});
    sets.push_back({&c->p2pLLConns, kDefaultLLBuffBytes, kDefaultLLBuffBytes / kSteps, &PeerLink::p2pLL,
                    &PeerLink::p2pLLFifo});
  } else {
    sets.push_back({&c->patConns, c->cfg.buffBytes, 0, &PeerLink::pat, &PeerLink::patFifo});
  }
  const char* unc = getenv("NEXR_PEER_FIFO_UNCACHED");
  const bool uncached = !(unc && unc[0] == '0');
  if (hipSetDevice(c->devices[me]) != hipSuccess) return nexrUnhandledCudaError;
  for (Set& st : sets) {
    st.conns->assign((size_t)n * n, nullptr);
    for (int q = 0; q < n; q++) {
      if (!isLink(q, me)) continue;
      PeerLink* l = peerLink(c->shm, n, q, me);
      Conn* k = (*st.conns)[(size_t)q * n + me] = new Conn();
      k->device = c->devices[me];
      k->slotBytes = st.slot;
      k->st = &(l->*st.state);
      if ((uncached ? hipExtMallocWithFlags((void**)&k->fifo, st.bytes, hipDeviceMallocUncached)
                    : hipMalloc((void**)&k->fifo, st.bytes)) != hipSuccess ||
          hipIpcGetMemHandle(&(l->*st.handle), k->fifo) != hipSuccess)
        return nexrUnhandledCudaError;
    }
  }
  PeerHeader* h = peerHeader(c->shm);
  std::atomic<uint32_t>& joined = p2p ? h->p2pJoined : h->patJoined;
  joined.fetch_add(1, std::memory_order_acq_rel);  // publishes the handles
  const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
  const auto t0 = std::chrono::steady_clock::now();
  while (joined.load(std::memory_order_acquire) < (uint32_t)n) {
    if (h->abort.load(std::memory_order_acquire)) return nexrRemoteError;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return nexrRemoteError;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  for (Set& st : sets) {
    for (int q = 0; q < n; q++) {
      if (!isLink(me, q)) continue;
      PeerLink* l = peerLink(c->shm, n, me, q);
      Conn* k = (*st.conns)[(size_t)me * n + q] = new Conn();
      k->device = c->devices[me];
      k->slotBytes = st.slot;
      k->st = &(l->*st.state);
      k->ownsFifo = false;
      char* mapped = nullptr;
      if (hipIpcOpenMemHandle((void**)&mapped, l->*st.handle, hipIpcMemLazyEnablePeerAccess) != hipSuccess)
        return nexrUnhandledCudaError;
      k->fifo = mapped;
    }
  }
  return nexrSuccess;
}

nexrResult_t peerFinish(nexrRingComm* c, Shared& sh) {
  if (sh.firstError.load() != 0) {
    c->broken = true;
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

nexrResult_t peerPat(nexrRingComm* c, bool reduceScatter, const void* sendbuff, void* recvbuff, size_t count,
                     int datatype, int op) {
  if (!c || !c->peer) return nexrInvalidArgument;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = patPrepare(c, reduceScatter, datatype, op, count, &esz, &red);
  if (r != nexrSuccess) return r;
  if (count == 0) return nexrSuccess;
  if (!sendbuff || !recvbuff) return nexrInvalidArgument;
  const int me = c->self;
  (void)hipSetDevice(c->devices[me]);
  if (c->cfg.nRanks == 1) return oneRank(c, me, sendbuff, recvbuff, count, datatype, red, esz);
  r = ensurePeerLinks(c, false);
  if (r != nexrSuccess) {
    c->broken = true;
    if (c->shm) peerHeader(c->shm)->abort.store(1);
    return r;
  }
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  runPatRank(c, &sh, me, reduceScatter, sendbuff, recvbuff, count, esz, datatype, red);
  return peerFinish(c, sh);
}

}  // namespace

extern "C" {

NEXR_API nexrResult_t nexrPeerPatReduceScatter(nexrRingComm_t c, const void* sendbuff, void* recvbuff,
                                               size_t recvcount, int datatype, int op) {
  return peerPat(c, true, sendbuff, recvbuff, recvcount, datatype, op);
}

NEXR_API nexrResult_t nexrPeerPatAllGather(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t sendcount,
                                           int datatype) {
  return peerPat(c, false, sendbuff, recvbuff, sendcount, datatype, nexrSum);
}

NEXR_API nexrResult_t nexrPeerSendRecv(nexrRingComm_t c, const void* sendbuff, int sendPeer, void* recvbuff,
                                       int recvPeer, size_t bytes) {
  if (!c || !c->peer) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  if (c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  const int n = c->cfg.nRanks, me = c->self;
  if (sendPeer < -1 || sendPeer >= n || recvPeer < -1 || recvPeer >= n) return nexrInvalidArgument;
  if ((sendPeer == me) != (recvPeer == me)) return nexrInvalidArgument;  // a self-send is its own recv
  if (bytes > 0 && ((sendPeer >= 0 && !sendbuff) || (recvPeer >= 0 && !recvbuff))) return nexrInvalidArgument;
  (void)hipSetDevice(c->devices[me]);
  nexrResult_t r = n > 1 ? ensureSecondStreams(c) : nexrSuccess;
  if (r == nexrSuccess && n > 1) r = ensurePeerLinks(c, true);
  if (r != nexrSuccess) {
    c->broken = true;
    if (c->shm) peerHeader(c->shm)->abort.store(1);
    return r;
  }
  if (bytes == 0) return nexrSuccess;
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  if (sendPeer == me) {
    runSelfCopy(c, &sh, me, sendbuff, recvbuff, bytes);
    return peerFinish(c, sh);
  }
  std::thread sender;
  if (sendPeer >= 0) sender = std::thread([&] { runP2pHalf(c, &sh, me, true, sendPeer, sendbuff, recvbuff, bytes); });
  if (recvPeer >= 0) runP2pHalf(c, &sh, me, false, recvPeer, sendbuff, recvbuff, bytes);
  if (sender.joinable()) sender.join();
  return peerFinish(c, sh);
}

NEXR_API nexrResult_t nexrPeerRingAllReduce(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int op) {
  return peerCollective(c, kAllReduce, sendbuff, recvbuff, count, datatype, op, 0);
}

NEXR_API nexrResult_t nexrPeerRingReduceScatter(nexrRingComm_t c, const void* sendbuff, void* recvbuff,
                                                size_t recvcount, int datatype, int op) {
  return peerCollective(c, kReduceScatter, sendbuff, recvbuff, recvcount, datatype, op, 0);
}

NEXR_API nexrResult_t nexrPeerRingAllGather(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t sendcount,
                                            int datatype) {
  return peerCollective(c, kAllGather, sendbuff, recvbuff, sendcount, datatype, nexrSum, 0);
}

NEXR_API nexrResult_t nexrPeerRingReduce(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                         int datatype, int op, int root) {
  return peerCollective(c, kReduce, sendbuff, recvbuff, count, datatype, op, root);
}

NEXR_API nexrResult_t nexrPeerRingBroadcast(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int root) {
  return peerCollective(c, kBroadcast, sendbuff, recvbuff, count, datatype, nexrSum, root);
}

}  // extern "C"
