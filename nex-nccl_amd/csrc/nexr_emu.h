// nexr_emu.h — internal to the CPU-emulated collectives (nexr_ring.cpp; the extras library's
// nexr_p2p.cpp and nexr_resident_host.cpp): the connection and FIFO state, the communicator, and the
// host-side Primitives every schedule drives. Not installed; the public surface is
// include/nexr_ring.h (and include/nexr_extras.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <functional>
#include <thread>
#include <vector>

#include "../../include/nexr_ring.h"

namespace nexr_emu {

constexpr int kSteps = 8;                                // NCCL_STEPS (src/include/device.h:649)
constexpr int kMaxChannels = 64;                         // MAXCHANNELS (src/include/device.h:711)
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

// Keeps the calling thread's current HIP device across an entry point, as NCCL's entry points keep
// the caller's CUDA device (init.cc:1873 ncclCommInitAll, enqueue.cc:2422 ncclEnqueueCheck). The
// entry points select each rank's device while they build streams and FIFOs or run a process rank's
// steps; without the guard the caller (and PyTorch, whose current device is HIP's) would be left on
// the last rank's device. Inactive for communicators that never touch HIP (CPU checkers).
struct DeviceGuard {
  int dev = -1;
  explicit DeviceGuard(bool active) {
    if (active && hipGetDevice(&dev) != hipSuccess) {
      (void)hipGetLastError();
      dev = -1;
    }
  }
  ~DeviceGuard() {
    if (dev >= 0) (void)hipSetDevice(dev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

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
  // Thread ranks, FIFO in device memory: the receiver's head words for runs of LL steps on the device
  // (nexrReduceCopyLLSteps), NEXR_LL_HEAD_BYTES right behind the FIFO in the same zeroed allocation.
  uint64_t* devHead = nullptr;
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
constexpr size_t kPeerResidentRecordBytes = 128 * 256;  // kResMaxTeam x kResCtrBytes (nexr_resident.h)
struct alignas(64) PeerHeader {
  std::atomic<uint32_t> initState;  // 0 fresh, 1 being configured, 2 configured
  std::atomic<uint32_t> joined;
  std::atomic<uint32_t> left;
  std::atomic<uint32_t> abort;
  std::atomic<uint32_t> p2pJoined;  // ranks that published their P2P receive FIFOs
  uint32_t magic, nRanks, protocol, pad;
  uint64_t buffBytes;
};
struct PeerSlot {
  hipIpcMemHandle_t fifoHandle;
  std::atomic<uint32_t> claimed;  // set once by rank r when it joins; already set = stale segment
  alignas(64) ConnState conn;
  // Resident all-reduces rank r has completed (nexrPeerRingAllReduceResident): its kernel no longer
  // reads its receive FIFO. The ring link's two users hand over through this and conn (ringLinkHandover).
  alignas(64) std::atomic<uint64_t> residentDone;
  // Rank r's first resident call publishes its GPU (PCI domain/bus/device) and the team its GPU can
  // keep resident; every rank then runs the minimum (member g only meets member g of its neighbours).
  std::atomic<uint64_t> residentGpu;
  std::atomic<int64_t> residentCap;   // workgroups per part rank r's GPU keeps resident
  std::atomic<int32_t> residentTeam;  // rank r's proposed team; 0 = not published yet
  std::atomic<uint64_t> gpu;          // rank r's GPU (PCI domain/bus/device + 1), published when it joins
};
// Links beyond the ring for P2P (any r -> q, the extras library's send/recv), one per ordered pair:
// the receiver's FIFO handles and the link's counters. Only for communicators of up to
// kPeerLinkMaxRanks.
constexpr int kPeerLinkMaxRanks = 64;
struct PeerLink {
  hipIpcMemHandle_t p2pFifo, p2pLLFifo;
  alignas(64) ConnState p2p;
  alignas(64) ConnState p2pLL;
};
inline size_t peerShmBytes(int n) {
  return sizeof(PeerHeader) + (size_t)n * sizeof(PeerSlot) +
         (n <= kPeerLinkMaxRanks ? (size_t)n * n * sizeof(PeerLink) : 0);
}
inline PeerHeader* peerHeader(void* base) { return (PeerHeader*)base; }
inline PeerSlot* peerSlot(void* base, int r) { return (PeerSlot*)((char*)base + sizeof(PeerHeader)) + r; }
inline PeerLink* peerLink(void* base, int n, int from, int to) {
  return (PeerLink*)((char*)base + sizeof(PeerHeader) + (size_t)n * sizeof(PeerSlot)) + (size_t)from * n + to;
}

inline int64_t divUp(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t alignUp(int64_t a, int64_t b) { return divUp(a, b) * b; }

struct TreeLinks {
  int up = -1;
  int down[kMaxArity] = {-1, -1, -1};
  int nDown() const {
    int k = 0;
    while (k < kMaxArity && down[k] >= 0) k++;
    return k;
  }
};

}  // namespace nexr_emu

using namespace nexr_emu;

struct nexrRingComm {
  nexrRingConfig cfg;
  size_t stepBytes = 0;
  std::vector<Conn*> conns;     // ring: conns[r] is the connection into rank r from rank r-1
  std::vector<TreeLinks> tree;  // tree topology (computed at creation)
  std::vector<Conn*> treeUp;    // treeUp[r]: r -> parent(r) (reduce); created by the first tree call
  std::vector<Conn*> treeDown;  // treeDown[r]: parent(r) -> r (broadcast)
  std::vector<Conn*> p2pConns;  // ncclSend/ncclRecv: p2pConns[from*nRanks+to] (connIndex 1), made on first use
  std::vector<Conn*> p2pLLConns;  // the same links' LL buffers, for messages <= 16 KiB
  // Channels 1..nChannels-1, each a communicator of its own (links, FIFOs, streams, tree) over the
  // same ranks; channel 0 is this one. Only the top-level communicator is called by the API.
  std::vector<nexrRingComm*> channels;
  size_t p2pChunkBytes = 0;     // comm->p2pChunkSize
  std::vector<int> devices;
  std::vector<hipStream_t> streams, streams2;  // streams2: the tree's broadcast-half threads
  std::vector<uint32_t*> status, status2;      // LL: pinned status words the kernel reports timeouts in
  std::vector<uint32_t*> done, done2;          // per stream: pinned step-completion words (Prims::streamDone)
  bool ll = false;     // LL or LL128: one FIFO step per primitive call, data readiness in line flags
  int proto = nexrRingProtoSimple;
  bool needHip = false;
  bool pinnedStatus = false;  // status words from hipHostMalloc (else calloc)
  bool broken = false;
  // How a rank thread waits for its step (Prims::streamDone): the completion word when every rank of
  // the communicator runs on one GPU, hipStreamSynchronize when the ranks span GPUs (the step's stores
  // then land in a peer GPU's memory, and only the synchronisation is documented to cover them).
  // NEXR_STEP_WAIT=word / sync forces either (stepWaitMode).
  bool stepWaitWord = true;
  // How the last thread-rank ring collective ran its LL steps (diagnostics, nexrRingCommGetQueued):
  // 0 host-sequenced, 1 queued launches (Prims::enableLLAsync), 2 runs with device credits (enableLLRun).
  int lastLLMode = 0;
  bool ownQueues = true;  // every rank stream has a hardware queue of its own (createRankStream)
  // Frees what the extras library attached to this communicator (set by its first resident call).
  void (*freeExtras)(nexrRingComm*) = nullptr;
  // Resident ring (nexrRingAllReduceResident), made by its first call: for every device hosting ranks
  // (resDevs, in order of first appearance), the (channel, rank) connection table and the step-counter
  // block in that device's memory, and a pinned, device-mapped status word.
  std::vector<int> resDevs;
  std::vector<void*> resTable, resCtr;
  std::vector<void*> resFifo;  // ranks on several GPUs: uncached receive FIFOs [channel * nRanks + rank]
  // The tree's (nexrTreeAllReduceResident), made by its first call: per device the (channel, rank)
  // table and the records of connections up[r] (id r) and down[r] (id nRanks + r); on several GPUs
  // also uncached FIFOs [channel * 2 nRanks + id].
  std::vector<void*> resTreeTable, resTreeCtr, resTreeFifo;
  std::vector<uint32_t*> resStatus;
  // Process ranks: this process is rank `self` only.
  bool peer = false;
  int ringLinkUser = 0;          // last user of the ring link r -> r+1: 0 none, 1 host-sequenced, 2 resident
  uint64_t residentCalls = 0;    // resident all-reduces this rank has completed
  int residentTeamAgreed = 0;    // process ranks: the team size all ranks agreed on (first resident call)
  int residentSharing = 1;       // process ranks: ranks on this rank's GPU (published at that agreement)
  int self = 0;
  void* shm = nullptr;
  size_t shmBytes = 0;
  char shmName[256] = {0};
};

namespace nexr_emu {

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
  uint32_t* done = nullptr;  // the stream's completion word: [0] written by the GPU, [1] last ticket
  bool device;
  int proto = nexrRingProtoSimple;  // the communicator's, or LL for a small P2P message (sendrecv.h)
  // Queued LL steps (enableLLAsync): a step's kernel is followed on the stream by a completion ticket,
  // and the receive slots it consumed are released (head published) only once the ticket has landed.
  bool llAsync = false;
  struct PendingStep {
    uint32_t ticket;
    int n;
    Conn* conn[kMaxArity];
    uint64_t head[kMaxArity];
  };
  std::deque<PendingStep> pending;
  // Releases of queued steps not yet behind a ticket: one ticket (a hipStreamWriteValue32, ~3 us of host
  // time) per ticketEvery steps, and always before this thread blocks (flushTicket in waitAtLeast), so
  // a thread never waits while holding a release a peer may need.
  PendingStep acc{0, 0, {}, {}};
  int accSteps = 0;
  int ticketEvery = 4;
  // Runs of LL steps with the credits on the device (enableLLRun): steps collected here, launched
  // kLLRunFlush at a time; runRecv0 / runSend0 are the connections' steps at the run's first step.
  bool llRun = false;
  std::vector<nexrLLStep> run;
  uint64_t runRecv0[kMaxArity] = {}, runSend0[kMaxArity] = {};
  static constexpr size_t kLLRunFlush = 96;  // one launch's worth (kLLStepsMax, nexr_internal.h)

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

  // The step queued on `stream` is complete (its bytes are in place before postPeer publishes them,
  // prims_simple.h:177-188). Two ways to wait, chosen per communicator (stepWaitWord, below):
  //   word: a hipStreamWriteValue32 of a fresh ticket into the stream's pinned, device-mapped word
  //     follows the step, and the thread spins on the word. The command processor writes it only
  //     after the step's kernel has finished, its end-of-kernel release included, so the next rank's
  //     launch on the SAME GPU sees the bytes exactly as after hipStreamSynchronize — 2.6-2.8 us
  //     cheaper per step on MI355X (tools/step_sync_probe.cpp, profiles/r03z_step_wait_ab.txt).
  //   sync: hipStreamSynchronize, whose completion also covers stores to a peer GPU's memory.
  // Without a word, if the write cannot be queued, or after the communicator's timeout, the word
  // mode falls back to hipStreamSynchronize (so it never returns with the step still in flight).
  bool streamDone() {
    if (done && c->stepWaitWord) {
      const uint32_t t = ++done[1];
      if (hipStreamWriteValue32(stream, done, t, 0) == hipSuccess) {
        const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
        auto t0 = std::chrono::steady_clock::now();
        for (unsigned spins = 0;; spins++) {
          if (__atomic_load_n(done, __ATOMIC_ACQUIRE) == t) return true;
          if (spins >= 4096) {
            if ((spins & 255) == 0 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs))
              break;
            std::this_thread::yield();
          }
        }
      }
    }
    return hipStreamSynchronize(stream) == hipSuccess;
  }

  // LL steps without a host round trip per step (round 6). Host sequencing waits for every step's
  // kernel before publishing it (streamDone), so each step costs a launch plus a wait, and the two
  // ranks of C1 take turns. LL does not need that: its lines carry their own flags (prims_ll.h:38-93)
  // and the kernel polls them (bounded: a flag that never comes is a timeout error, nexr_ll.hip). So a
  // queued step publishes its send steps (incSend) as soon as its kernel is on the stream, the
  // receiver queues the consuming kernel at once, and only the credits wait for the GPU: the slots a
  // step read are released (postRecv, head) when a completion ticket behind it lands (progress(),
  // polled from every wait of this thread and by finishLL()). A ticket is a hipStreamWriteValue32,
  // ~3 us of host time like the launch itself (tools/api_cost_probe.cpp), so one ticket covers
  // ticketEvery steps, and the accumulated releases are always ticketed before this thread blocks.
  // No kernel waits behind its producer: a consumer is queued only after its producer (the tail is
  // published after the launch returns), so on a hardware queue the two share the producer is ahead,
  // and on separate queues both run; by induction over queueing order every polled flag arrives. The
  // conditions (llAsyncAllowed in nexr_ring.cpp): every rank on one GPU (the completion word is the
  // step wait), steps on the device, and the rank streams within the device's hardware queues.
  void enableLLAsync(int every = 4) {
    if (proto != nexrRingProtoLL || !device || !done || !status || !c->stepWaitWord) return;
    llAsync = true;
    ticketEvery = every < 1 ? 1 : every;
    __atomic_store_n(status, 0u, __ATOMIC_RELEASE);
  }
  // Puts the accumulated releases behind a fresh ticket on the stream; false if the write could not be
  // queued (the caller then drains the stream: drainLL).
  bool flushTicket() {
    if (acc.n == 0) return true;
    const uint32_t t = ++done[1];
    if (hipStreamWriteValue32(stream, done, t, 0) != hipSuccess) return false;
    acc.ticket = t;
    pending.push_back(acc);
    acc.n = 0;
    accSteps = 0;
    return true;
  }
  // Every queued step complete (stream synchronised): publish every release, leave queued mode.
  bool drainLL() {
    llAsync = false;
    const bool ok = hipStreamSynchronize(stream) == hipSuccess;
    for (const PendingStep& ps : pending)
      for (int i = 0; i < ps.n; i++) ps.conn[i]->st->head.store(ps.head[i], std::memory_order_release);
    for (int i = 0; i < acc.n; i++) acc.conn[i]->st->head.store(acc.head[i], std::memory_order_release);
    pending.clear();
    acc.n = 0;
    if (!ok) {
      sh->fail(nexrUnhandledCudaError);
      return false;
    }
    if (__atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) {
      sh->fail(nexrInternalError);
      return false;
    }
    return true;
  }
  // Publishes the heads of every queued step whose ticket has landed; false (and the communicator
  // failed) when a step's kernel reported a flag timeout.
  bool progress() {
    if (!llAsync) return true;
    const uint32_t d = __atomic_load_n(done, __ATOMIC_ACQUIRE);
    while (!pending.empty() && (int32_t)(d - pending.front().ticket) >= 0) {
      const PendingStep& ps = pending.front();
      for (int i = 0; i < ps.n; i++) ps.conn[i]->st->head.store(ps.head[i], std::memory_order_release);
      pending.pop_front();
    }
    if (__atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) {
      sh->fail(nexrInternalError);
      return false;
    }
    return true;
  }
  // The end of a collective with queued steps: wait (polling, so that the heads this rank owes keep
  // flowing to senders that still need credits) until the last step has completed.
  bool finishLL() {
    if (llRun) return finishRun();
    if (!llAsync) return true;
    if (!flushTicket()) return drainLL();
    const uint32_t t = ++done[1];
    bool landed = false;
    if (hipStreamWriteValue32(stream, done, t, 0) == hipSuccess) {
      const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
      auto t0 = std::chrono::steady_clock::now();
      for (unsigned spins = 0;; spins++) {
        if (!progress()) {
          llAsync = false;
          (void)hipStreamSynchronize(stream);
          return false;
        }
        if ((int32_t)(__atomic_load_n(done, __ATOMIC_ACQUIRE) - t) >= 0) {
          landed = true;
          break;
        }
        if ((spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs))
          break;
        if (spins >= 4096) std::this_thread::yield();
      }
    }
    llAsync = false;
    if (!landed && hipStreamSynchronize(stream) != hipSuccess) {
      sh->fail(nexrUnhandledCudaError);
      return false;
    }
    for (const PendingStep& ps : pending)  // every queued step is complete: release what it read
      for (int i = 0; i < ps.n; i++) ps.conn[i]->st->head.store(ps.head[i], std::memory_order_release);
    pending.clear();
    if (__atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) {
      sh->fail(nexrInternalError);
      return false;
    }
    return true;
  }

  // Runs of LL steps on the device (round 6): the steps of a collective are queued as launches of up
  // to 96 steps each (nexrReduceCopyLLSteps), whose workgroups poll the peers' line flags for the data
  // (readLL, prims_ll.h:91-109) AND the receivers' head words for the credits (waitSend :55-75), and
  // publish their own heads once they have read a step (postRecv :80-83) — the reference's LL loop, so
  // the rank thread waits for nothing until the end of the collective (finishLL). The launch per step
  // and the host hand-offs of the queued mode are gone. Conditions (llRunAllowed, nexr_ring.cpp): those
  // of the queued mode (every rank's kernels can run at once on the one GPU), the library's own LL
  // kernels, and device head words on every connection.
  void enableLLRun() {
    if (proto != nexrRingProtoLL || !device || !done || !status || !c->stepWaitWord) return;
    if (nRecv > NEXR_LL_STEPS_MAX_PEERS || nSend > NEXR_LL_STEPS_MAX_PEERS) return;
    for (int i = 0; i < nRecv; i++)
      if (!recv[i]->devHead || slot(recv[i]) != c->stepBytes) return;
    for (int i = 0; i < nSend; i++)
      if (!send[i]->devHead || slot(send[i]) != c->stepBytes) return;
    llRun = true;
    run.clear();
    __atomic_store_n(status, 0u, __ATOMIC_RELEASE);
  }
  bool flushRun() {
    if (run.empty()) return true;
    nexrLLConnSet cs;
    memset(&cs, 0, sizeof(cs));
    cs.input = userInput;
    cs.output = userOutput;
    cs.nRecv = nRecv;
    cs.nSend = nSend;
    for (int i = 0; i < nRecv; i++) {
      cs.recvFifo[i] = recv[i]->fifo;
      cs.recvHead[i] = recv[i]->devHead;
      cs.recvStep[i] = runRecv0[i];
    }
    for (int i = 0; i < nSend; i++) {
      cs.sendFifo[i] = send[i]->fifo;
      cs.sendHead[i] = send[i]->devHead;
      cs.sendStep[i] = runSend0[i];
    }
    cs.slotBytes = c->stepBytes;
    cs.nSlots = kSteps;
    const uint32_t tmo = (uint32_t)((c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 1000u);
    const nexrResult_t r = nexrReduceCopyLLSteps(&cs, run.data(), (int)run.size(), datatype, devOp, redOpArgs[0],
                                                 status, tmo, (nexrStream_t)stream);
    run.clear();
    if (r != nexrSuccess) {
      sh->fail(r);
      return false;
    }
    return true;
  }
  // The end of a collective run on the device: the last launch queued, the stream complete, then the
  // host counters (which host-sequenced collectives read) published as if every step had posted. When
  // another rank has failed, the steps not yet launched are dropped and the abort is relayed into this
  // rank's status word, which the run's polls read now and then (nexr_ll.hip): its kernels end at once
  // instead of at their timeout (checkAbort, primitives.h:142-156).
  bool finishRun() {
    llRun = false;
    bool ok;
    if (sh->aborted()) {
      run.clear();
      __atomic_store_n(status, 2u, __ATOMIC_RELEASE);
      ok = false;
    } else {
      ok = flushRun();
    }
    const uint32_t t = ++done[1];
    bool landed = false;
    if (hipStreamWriteValue32(stream, done, t, 0) == hipSuccess) {
      const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
      auto t0 = std::chrono::steady_clock::now();
      for (unsigned spins = 0;; spins++) {
        if ((int32_t)(__atomic_load_n(done, __ATOMIC_ACQUIRE) - t) >= 0) {
          landed = true;
          break;
        }
        if (sh->aborted() && __atomic_load_n(status, __ATOMIC_ACQUIRE) == 0)
          __atomic_store_n(status, 2u, __ATOMIC_RELEASE);
        if ((spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs))
          break;
        if (spins >= 4096) std::this_thread::yield();
      }
    }
    if (!landed && hipStreamSynchronize(stream) != hipSuccess) {
      sh->fail(nexrUnhandledCudaError);
      ok = false;
    }
    for (int i = 0; i < nRecv; i++) recv[i]->st->head.store(recv[i]->recvStep, std::memory_order_release);
    for (int i = 0; i < nSend; i++) send[i]->st->tail.store(send[i]->sendStep, std::memory_order_release);
    const uint32_t st = __atomic_load_n(status, __ATOMIC_ACQUIRE);
    if (ok && st != 0) {
      sh->fail(nexrInternalError);
      ok = false;
    }
    return ok;
  }

  // Spin until `a` >= target (waitPeer's connStepCache loop, prims_simple.h:116-123), bounded and
  // abortable like checkAbort (primitives.h:142-156).
  bool waitAtLeast(std::atomic<uint64_t>& a, uint64_t target) {
    if (a.load(std::memory_order_acquire) >= target) return true;
    if (llAsync && acc.n) {
      // Never block holding a release: but a peer's post usually comes within a launch's time (~3 us),
      // and a ticket costs as much as a launch, so look for 20 us before putting the releases behind one.
      const auto tw = std::chrono::steady_clock::now();
      for (unsigned spins = 1;; spins++) {
        if (a.load(std::memory_order_acquire) >= target) return true;
        if ((spins & 63) == 0 && std::chrono::steady_clock::now() - tw > std::chrono::microseconds(20)) break;
      }
      if (!flushTicket() && !drainLL()) return false;
    }
    const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
    auto t0 = std::chrono::steady_clock::now();
    for (unsigned spins = 0;; spins++) {
      if (llAsync && !progress()) return false;
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
          if (!streamDone()) r = nexrUnhandledCudaError;  // data complete before the step is posted
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
  // Host-sequenced, the host additionally waits for the sender's step so that the kernel's flag poll
  // succeeds at once; queued (enableLLAsync), the sender's tail means its kernel is on its stream, and
  // the consuming kernel polls the flags as they arrive.
  bool genericOpLL(bool Recv, bool Send, int srcBuf, int dstBuf, int64_t srcIx, int64_t dstIx, int64_t nelem,
                   bool postOp) {
    const int nr = Recv ? nRecv : 0, ns = Send ? nSend : 0;
    nelem = nelem < 0 ? 0 : nelem;
    if (llRun) {  // no host wait: the run's kernel polls the flags and the credits itself
      if (sh->aborted()) {
        sh->fail(nexrRemoteError);
        return false;
      }
      if (run.empty()) {
        for (int i = 0; i < nRecv; i++) runRecv0[i] = recv[i]->recvStep;
        for (int i = 0; i < nSend; i++) runSend0[i] = send[i]->sendStep;
      }
      nexrLLStep s;
      memset(&s, 0, sizeof(s));
      s.srcBuf = (int8_t)(srcBuf == kNone ? -1 : srcBuf);
      s.dstBuf = (int8_t)(dstBuf == kNone ? -1 : dstBuf);
      s.srcIx = srcBuf == kNone ? 0 : srcIx;
      s.dstIx = dstBuf == kNone ? 0 : dstIx;
      s.nElts = (uint32_t)nelem;
      s.recv = nr > 0;
      s.send = ns > 0;
      s.postOp = postOp ? 1 : 0;
      run.push_back(s);
      for (int i = 0; i < nr; i++) recv[i]->recvStep += 1;
      for (int i = 0; i < ns; i++) send[i]->sendStep += 1;
      return run.size() < kLLRunFlush || flushRun();
    }
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
      if (status && !llAsync) *status = 0;
      const uint32_t tmo = (uint32_t)((c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 1000u);
      nexrResult_t r;
      if (proto == nexrRingProtoLL128)
        r = ll128Fn(src, srcIsInput, nr, recvLines, rf64, dst, ns, sendLines, sf64, (size_t)nelem, datatype, devOp,
                    redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      else
        r = llFn(src, srcIsInput, nr, recvLines, rf32, dst, ns, sendLines, sf32, (size_t)nelem, datatype, devOp,
                 redOpArgs[0], postOp ? 1 : 0, status, tmo, (nexrStream_t)stream);
      if (!llAsync) {
        if (r == nexrSuccess && device && !streamDone()) r = nexrUnhandledCudaError;
        if (r == nexrSuccess && status && __atomic_load_n(status, __ATOMIC_ACQUIRE) != 0) r = nexrInternalError;
      }
      if (r != nexrSuccess) {
        sh->fail(r);
        return false;
      }
    }
    if (llAsync) {  // queued (also an empty step, whose release must not overtake the queued ones)
      for (int i = 0; i < nr; i++) {  // postRecv waits for a ticket (progress)
        int j = 0;
        while (j < acc.n && acc.conn[j] != recv[i]) j++;
        if (j == acc.n) acc.conn[acc.n++] = recv[i];
        acc.head[j] = ++recv[i]->recvStep;
      }
      for (int i = 0; i < ns; i++) {  // incSend now: the receiver's kernel finds the data by its flags
        send[i]->sendStep += 1;
        send[i]->st->tail.store(send[i]->sendStep, std::memory_order_release);
      }
      if (++accSteps >= ticketEvery && !flushTicket()) return drainLL();
      return progress();
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

// One channel's share of a collective (ncclCollCbdPart, src/include/device.h:946-970): elements
// [offset, offset + count) of every rank's buffers, moved in chunks of chunkCount elements.
struct ChannelPart {
  int channel;
  int64_t offset, count, chunkCount;
};
inline nexrRingComm* channelComm(nexrRingComm* c, int k) { return k == 0 ? c : c->channels[(size_t)k - 1]; }

// ---- shared helpers (nexr_ring.cpp) ----------------------------------------------------------------
// The channels a collective of `count` elements uses and each one's part (scheduleCollTasksToPlan for
// one task, src/enqueue.cc:539-690): trafficPerByte = ncclFuncTrafficPerByte (:74-81). chunkCount is
// left 0 for the caller (calcCollChunking of each part).
std::vector<ChannelPart> channelParts(const nexrRingComm* c, int64_t count, size_t esz, int trafficPerByte);
nexrResult_t defaultLLFn(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                         const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                         const uint32_t* sendFlags, size_t n, int dt, int op, uint64_t arg, int post, uint32_t* status,
                         uint32_t timeoutUs, nexrStream_t s);
Prims makePrims(nexrRingComm* c, Shared* sh, int rank, const void* sendbuff, void* recvbuff, size_t esz, int datatype,
                const nexrDevRedOpFull& red, Geom g, hipStream_t stream, uint32_t* status);
nexrResult_t oneRank(nexrRingComm* c, int r, const void* sendbuff, void* recvbuff, size_t count, int datatype,
                     const nexrDevRedOpFull& red, size_t esz);
nexrResult_t prepare(nexrRingComm* c, int datatype, int op, size_t* esz, nexrDevRedOpFull* red);
nexrResult_t runThreads(nexrRingComm* c, Shared& sh, const std::vector<std::function<void()>>& jobs);
nexrResult_t allocFifo(nexrRingComm* c, Conn* k, int device, size_t bytes = 0);
nexrResult_t enablePeer(int a, int b);
nexrResult_t ensureSecondStreams(nexrRingComm* c);
nexrResult_t peerFinish(nexrRingComm* c, Shared& sh);
nexrResult_t ringLinkHandover(nexrRingComm* c, bool resident);
// NEXR_STEP_WAIT: 1 = word, 0 = sync, -1 = unset (auto: word only when all ranks share one GPU).
int stepWaitMode();
// calcCollChunking for one channel in elements (enqueue.cc:1993-1999).
int64_t chunkElems(const nexrRingComm* c, Geom g, size_t esz, bool tree, size_t nBytes);
nexrResult_t ensureTree(nexrRingComm* c);
bool envFlagOn(const char* name, bool dflt);
enum RingColl { kAllReduce, kReduceScatter, kAllGather, kReduce, kBroadcast };

}  // namespace nexr_emu
