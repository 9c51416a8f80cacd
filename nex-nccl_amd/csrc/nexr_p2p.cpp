// nexr_p2p.cpp — ncclSend / ncclRecv on the emulated communicator (the P2P work batch of
// src/device/sendrecv.h), thread ranks and process ranks (include/nexr_extras.h nexrSendRecv,
// nexrPeerSendRecv). Part of the opt-in extras library (make EXTRAS=1 -> libnexr_extras.so): the
// P2P schedule goes beyond SURVEY §8's rows.
#include "nexr_emu.h"

namespace nexr_emu {

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
  const nexrDevRedOpFull copy = {nexrDevSum, 0, false, 0};
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

// Process ranks: the first Send/Recv call on a communicator connects this rank's P2P links (any
// r -> q at connection index 1, SIMPLE buffers and their LL buffers). Every rank allocates the FIFOs
// it receives into, publishes their IPC handles in the shared segment, and, once all ranks have,
// maps the FIFOs it sends into. Collective: every rank makes its first call together.
nexrResult_t ensurePeerLinks(nexrRingComm* c) {
  if (!c->p2pConns.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks, me = c->self;
  if (n > kPeerLinkMaxRanks) return nexrInvalidUsage;
  struct Set {
    std::vector<Conn*>* conns;
    size_t bytes, slot;
    ConnState PeerLink::*state;
    hipIpcMemHandle_t PeerLink::*handle;
  };
  Set sets[2] = {{&c->p2pConns, c->p2pChunkBytes * kSteps, c->p2pChunkBytes, &PeerLink::p2p, &PeerLink::p2pFifo},
                 {&c->p2pLLConns, kDefaultLLBuffBytes, kDefaultLLBuffBytes / kSteps, &PeerLink::p2pLL,
                  &PeerLink::p2pLLFifo}};
  const char* unc = getenv("NEXR_PEER_FIFO_UNCACHED");
  const bool uncached = !(unc && unc[0] == '0');
  if (hipSetDevice(c->devices[me]) != hipSuccess) return nexrUnhandledCudaError;
  for (Set& st : sets) {
    st.conns->assign((size_t)n * n, nullptr);
    for (int q = 0; q < n; q++) {
      if (q == me) continue;
      PeerLink* l = peerLink(c->shm, n, q, me);
      Conn* k = (*st.conns)[(size_t)q * n + me] = new Conn();
      k->device = c->devices[me];
      k->slotBytes = st.slot;
      k->st = &(l->*st.state);
      if ((uncached ? hipExtMallocWithFlags((void**)&k->fifo, st.bytes, hipDeviceMallocUncached)
                    : hipMalloc((void**)&k->fifo, st.bytes)) != hipSuccess ||
          hipMemset(k->fifo, 0, st.bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||  // no stale LL lines
          hipIpcGetMemHandle(&(l->*st.handle), k->fifo) != hipSuccess)
        return nexrUnhandledCudaError;
    }
  }
  PeerHeader* h = peerHeader(c->shm);
  h->p2pJoined.fetch_add(1, std::memory_order_acq_rel);  // publishes the handles
  const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
  const auto t0 = std::chrono::steady_clock::now();
  while (h->p2pJoined.load(std::memory_order_acquire) < (uint32_t)n) {
    if (h->abort.load(std::memory_order_acquire)) return nexrRemoteError;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) return nexrRemoteError;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
  for (Set& st : sets) {
    for (int q = 0; q < n; q++) {
      if (q == me) continue;
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

}  // namespace nexr_emu

extern "C" {

NEXR_API nexrResult_t nexrSendRecv(nexrRingComm_t c, const void* const* sendbuffs, const int* sendPeers,
                                   void* const* recvbuffs, const int* recvPeers, size_t bytes) {
  DeviceGuard dg(c && c->needHip);
  return sendRecv(c, sendbuffs, sendPeers, recvbuffs, recvPeers, bytes);
}
NEXR_API nexrResult_t nexrPeerSendRecv(nexrRingComm_t c, const void* sendbuff, int sendPeer, void* recvbuff,
                                       int recvPeer, size_t bytes) {
  DeviceGuard dg(c && c->needHip);
  if (!c || !c->peer) return nexrInvalidArgument;
  if (c->broken) return nexrInvalidUsage;
  if (c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  const int n = c->cfg.nRanks, me = c->self;
  if (sendPeer < -1 || sendPeer >= n || recvPeer < -1 || recvPeer >= n) return nexrInvalidArgument;
  if ((sendPeer == me) != (recvPeer == me)) return nexrInvalidArgument;  // a self-send is its own recv
  if (bytes > 0 && ((sendPeer >= 0 && !sendbuff) || (recvPeer >= 0 && !recvbuff))) return nexrInvalidArgument;
  (void)hipSetDevice(c->devices[me]);
  nexrResult_t r = n > 1 ? ensureSecondStreams(c) : nexrSuccess;
  if (r == nexrSuccess && n > 1) r = ensurePeerLinks(c);
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
  try {
    if (sendPeer >= 0) sender = std::thread([&] { runP2pHalf(c, &sh, me, true, sendPeer, sendbuff, recvbuff, bytes); });
  } catch (...) {
    sh.fail(nexrSystemError);  // no send half: the peers see the abort word, this rank's recv is skipped
  }
  if (recvPeer >= 0 && !sh.aborted()) runP2pHalf(c, &sh, me, false, recvPeer, sendbuff, recvbuff, bytes);
  if (sender.joinable()) sender.join();
  return peerFinish(c, sh);
}

}  // extern "C"
