// nexr_resident_host.cpp — host side of the device-resident ring / tree collectives
// (nexrRing*Resident, nexrTreeAllReduceResident, nexrPeerRingAllReduceResident; include/nexr_extras.h).
// Part of the opt-in extras library (make EXTRAS=1 -> libnexr_extras.so), not of the default
// product: these schedules are the reference's L3 device code (all_reduce.h & co.), which SURVEY §2
// marks out of scope, run inside one launch per GPU (nexr_resident.hip).
#include <map>
#include <mutex>
#include <tuple>

#include "nexr_emu.h"
#include "nexr_resident.h"

namespace nexr_emu {
// ---- resident ring (nexr_resident.hip) ----------------------------------------------------------
void freeResident(nexrRingComm* c) {
  for (size_t i = 0; i < c->resDevs.size(); i++) {
    (void)hipSetDevice(c->resDevs[i]);
    if (c->resTable[i]) (void)hipFree(c->resTable[i]);
    if (c->resCtr[i]) (void)hipFree(c->resCtr[i]);
    if (c->resStatus[i]) (void)hipHostFree(c->resStatus[i]);
  }
  for (size_t k = 0; k < c->resFifo.size(); k++) {
    if (!c->resFifo[k]) continue;
    (void)hipSetDevice(c->devices[k % c->cfg.nRanks]);
    (void)hipFree(c->resFifo[k]);
  }
  c->resFifo.clear();
  for (auto* v : {&c->resTreeTable, &c->resTreeCtr, &c->resTreeFifo})
    for (void* q : *v)
      if (q) (void)hipFree(q);  // hipFree finds the owning device itself
  c->resTreeTable.clear();
  c->resTreeCtr.clear();
  c->resTreeFifo.clear();
  c->resDevs.clear();
  c->resTable.clear();
  c->resCtr.clear();
  c->resStatus.clear();
}

int resDevIndex(const nexrRingComm* c, int rank) {
  for (size_t i = 0; i < c->resDevs.size(); i++)
    if (c->resDevs[i] == c->devices[rank]) return (int)i;
  return -1;
}

// First call: per device, a zeroed step-counter block with one record per (channel, rank, team
// member) for the ranks it hosts, a status word, and the (channel, rank) connection table. When the
// ranks span several GPUs, the step records and the FIFOs are uncached device memory
// (hipDeviceMallocUncached, as RCCL allocates its P2P FIFOs and flags): their writers then sit on
// another GPU, whose stores the owner's L2 does not see. On one GPU the communicator's own FIFOs
// serve, and the records are ordinary device memory.
bool residentMulti(const nexrRingComm* c) {
  static const bool forceUncached = [] {  // NEXR_RESIDENT_UNCACHED=1: the multi-GPU layout on one GPU (tests)
    const char* v = getenv("NEXR_RESIDENT_UNCACHED");
    return v && v[0] == '1';
  }();
  return c->resDevs.size() > 1 || forceUncached;
}

nexrResult_t ensureResident(nexrRingComm* c) {
  if (!c->resDevs.empty()) return nexrSuccess;
  c->freeExtras = freeResident;
  const int n = c->cfg.nRanks, nCh = c->cfg.nChannels;
  for (int r = 0; r < n; r++)
    if (std::find(c->resDevs.begin(), c->resDevs.end(), c->devices[r]) == c->resDevs.end())
      c->resDevs.push_back(c->devices[r]);
  const size_t nd = c->resDevs.size();
  c->resTable.assign(nd, nullptr);
  c->resCtr.assign(nd, nullptr);
  c->resStatus.assign(nd, nullptr);
  const size_t ctrBytes = (size_t)nCh * n * nexr::kResMaxTeam * nexr::kResCtrBytes;
  const bool multi = residentMulti(c);
  auto devAlloc = [&](void** p, size_t bytes) {
    return multi ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) : hipMalloc(p, bytes);
  };
  for (size_t i = 0; i < nd; i++) {
    if (hipSetDevice(c->resDevs[i]) != hipSuccess || devAlloc(&c->resCtr[i], ctrBytes) != hipSuccess ||
        hipMemset(c->resCtr[i], 0, ctrBytes) != hipSuccess ||
        hipHostMalloc((void**)&c->resStatus[i], sizeof(uint32_t), hipHostMallocMapped | hipHostMallocPortable) !=
            hipSuccess ||
        hipMalloc(&c->resTable[i], sizeof(nexr::ResConn) * nCh * n) != hipSuccess) {
      freeResident(c);
      return nexrUnhandledCudaError;
    }
  }
  if (multi) {  // resFifo[ch * n + r]: rank r's receive FIFO of channel ch, on rank r's GPU
    c->resFifo.assign((size_t)nCh * n, nullptr);
    for (size_t k = 0; k < c->resFifo.size(); k++) {
      if (hipSetDevice(c->devices[k % n]) != hipSuccess || devAlloc(&c->resFifo[k], c->cfg.buffBytes) != hipSuccess) {
        freeResident(c);
        return nexrUnhandledCudaError;
      }
    }
  }
  auto fifo = [&](int ch, int r) {
    return multi ? (char*)c->resFifo[(size_t)ch * n + r] : channelComm(c, ch)->conns[r]->fifo;
  };
  std::vector<nexr::ResConn> table((size_t)nCh * n);
  for (int ch = 0; ch < nCh; ch++) {
    for (int r = 0; r < n; r++) {
      const int nx = (r + 1) % n;
      auto rec = [&](int rank) {
        return (char*)c->resCtr[resDevIndex(c, rank)] +
               ((size_t)(ch * n + rank) * nexr::kResMaxTeam) * nexr::kResCtrBytes;
      };
      table[(size_t)ch * n + r] = {fifo(ch, r), fifo(ch, nx), rec(r), rec(nx)};
    }
  }
  for (size_t i = 0; i < nd; i++) {
    *c->resStatus[i] = 0;
    if (hipSetDevice(c->resDevs[i]) != hipSuccess ||
        hipMemcpy(c->resTable[i], table.data(), sizeof(nexr::ResConn) * table.size(), hipMemcpyHostToDevice) !=
            hipSuccess) {
      freeResident(c);
      return nexrUnhandledCudaError;
    }
  }
  return nexrSuccess;
}

// First tree call (after ensureResident): every channel's tree links (ensureTree), per device a
// zeroed record block for the tree's connections and the (channel, rank) ResTreeConn table. The
// record and FIFO of up[r] sit on the parent's GPU, those of down[r] on r's.
nexrResult_t ensureResidentTree(nexrRingComm* c, bool multi) {
  if (!c->resTreeTable.empty()) return nexrSuccess;
  const int n = c->cfg.nRanks, nCh = c->cfg.nChannels;
  for (int ch = 0; ch < nCh; ch++) {
    nexrResult_t r = ensureTree(channelComm(c, ch));
    if (r != nexrSuccess) return r;
  }
  const size_t nd = c->resDevs.size();
  c->resTreeTable.assign(nd, nullptr);
  c->resTreeCtr.assign(nd, nullptr);
  const size_t ctrBytes = (size_t)nCh * 2 * n * nexr::kResMaxTeam * nexr::kResCtrBytes;
  auto devAlloc = [&](void** p, size_t bytes) {
    return multi ? hipExtMallocWithFlags(p, bytes, hipDeviceMallocUncached) : hipMalloc(p, bytes);
  };
  auto fail = [&] {
    freeResident(c);
    return nexrUnhandledCudaError;
  };
  for (size_t i = 0; i < nd; i++) {
    if (hipSetDevice(c->resDevs[i]) != hipSuccess || devAlloc(&c->resTreeCtr[i], ctrBytes) != hipSuccess ||
        hipMemset(c->resTreeCtr[i], 0, ctrBytes) != hipSuccess ||
        hipMalloc(&c->resTreeTable[i], sizeof(nexr::ResTreeConn) * nCh * n) != hipSuccess)
      return fail();
  }
  // receiver of connection id (r: up[r], n + r: down[r]) on channel ch
  auto receiver = [&](int ch, int id) { return id < n ? channelComm(c, ch)->tree[id].up : id - n; };
  if (multi) {
    c->resTreeFifo.assign((size_t)nCh * 2 * n, nullptr);
    for (int ch = 0; ch < nCh; ch++)
      for (int id = 0; id < 2 * n; id++) {
        const int rcv = receiver(ch, id);
        if (rcv < 0) continue;  // up[root]
        if (hipSetDevice(c->devices[rcv]) != hipSuccess ||
            devAlloc(&c->resTreeFifo[(size_t)ch * 2 * n + id], c->cfg.buffBytes) != hipSuccess)
          return fail();
      }
  }
  auto fifo = [&](int ch, int id) -> char* {
    if (multi) return (char*)c->resTreeFifo[(size_t)ch * 2 * n + id];
    nexrRingComm* ck = channelComm(c, ch);
    return id < n ? ck->treeUp[id]->fifo : ck->treeDown[id - n]->fifo;
  };
  auto rec = [&](int ch, int id) {
    return (char*)c->resTreeCtr[resDevIndex(c, receiver(ch, id))] +
           ((size_t)(ch * 2 * n + id) * nexr::kResMaxTeam) * nexr::kResCtrBytes;
  };
  std::vector<nexr::ResTreeConn> table((size_t)nCh * n);
  for (int ch = 0; ch < nCh; ch++) {
    const std::vector<TreeLinks>& tl = channelComm(c, ch)->tree;
    for (int r = 0; r < n; r++) {
      nexr::ResTreeConn t{};
      t.nDown = tl[r].nDown();
      t.root = tl[r].up < 0 ? 1 : 0;
      for (int i = 0; i < t.nDown; i++) {
        const int child = tl[r].down[i];
        t.upRecvFifo[i] = fifo(ch, child);
        t.upRecvCtr[i] = rec(ch, child);
        t.downSendFifo[i] = fifo(ch, n + child);
        t.downSendCtr[i] = rec(ch, n + child);
      }
      if (!t.root) {
        t.upSendFifo = fifo(ch, r);
        t.upSendCtr = rec(ch, r);
        t.downRecvFifo = fifo(ch, n + r);
        t.downRecvCtr = rec(ch, n + r);
      }
      table[(size_t)ch * n + r] = t;
    }
  }
  for (size_t i = 0; i < nd; i++) {
    if (hipSetDevice(c->resDevs[i]) != hipSuccess ||
        hipMemcpy(c->resTreeTable[i], table.data(), sizeof(nexr::ResTreeConn) * table.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
      return fail();
  }
  return nexrSuccess;
}

// Workgroups of the (datatype, op, collective) resident kernel that `device` keeps resident at once:
// blocks per CU x CUs, queried once per process and kernel (a resident call is ~30 us; the queries
// are host work the C1 path would otherwise repeat).
nexrResult_t residentCapacity(int device, int kdt, int devOp, uint64_t redArg, int coll, long* capacity) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, bool, int>, long> cache;
  const auto key = std::make_tuple(device, kdt, devOp, (redArg & 1) == 0, coll);
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(key);
  if (it != cache.end()) {
    *capacity = it->second;
    return nexrSuccess;
  }
  int perCU = 0, cus = 0;
  if (nexr::resident_blocks_per_cu(kdt, devOp, redArg, coll, &perCU) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
    return nexrUnhandledCudaError;
  *capacity = cache[key] = (long)perCU * cus;
  return nexrSuccess;
}

// Workgroups per (rank, channel): NEXR_RESIDENT_TEAM, else as many as give every member at least
// 16 KiB of a full slice (StepPerSlice steps), at most about 512 workgroups on the busiest device (two
// per CU) and at most kResMaxTeam. Measured on MI355X (tools/resident_time.py, 2 ranks, 256 MiB):
// 16 KiB pieces beat 8 KiB ones (0.89 vs 1.03 ms on one channel) and 32/64 KiB ones at 4 channels.
int residentTeam(int ranksOnDevice, int nParts, size_t sliceBytes) {
  static const long env = [] {
    const char* v = getenv("NEXR_RESIDENT_TEAM");
    return v && *v ? strtol(v, nullptr, 0) : 0l;
  }();
  long t = env > 0 ? env
                   : std::min<long>((long)(sliceBytes / (16 << 10)), 512 / std::max(1, ranksOnDevice * nParts));
  return (int)std::max(1l, std::min<long>(t, nexr::kResMaxTeam));
}

nexrResult_t residentCollective(nexrRingComm* c, RingColl coll, const void* const* sendbuffs, void* const* recvbuffs,
                                size_t count, int datatype, int op, int root, bool tree = false) {
  if (!c || c->peer) return nexrInvalidArgument;
  if (c->cfg.memMode != nexrRingDeviceMemory || c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  int sem = nexrSemanticsNccl;
  if (nexrGetSemantics(&sem) != nexrSuccess || sem == nexrSemanticsShipped) return nexrInvalidUsage;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = prepare(c, datatype, op, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks;
  if ((coll == kReduce || coll == kBroadcast) && (root < 0 || root >= n)) return nexrInvalidArgument;
  if (!sendbuffs || !recvbuffs) return nexrInvalidArgument;
  for (int i = 0; i < n; i++) {  // as ringCollective: Broadcast needs only the root's send buffer,
    const bool needSend = coll != kBroadcast || i == root;  // Reduce only the root's recv buffer
    const bool needRecv = coll != kReduce || i == root;
    if ((needSend && !sendbuffs[i]) || (needRecv && !recvbuffs[i])) return nexrInvalidArgument;
  }
  if (count == 0) return nexrSuccess;
  if (n == 1) return oneRank(c, 0, sendbuffs[0], recvbuffs[0], count, datatype, red, esz);
  if (n > nexr::kResMaxRanks) return nexrInvalidUsage;
  // The fork's dispatch runs signed Min/Max on the unsigned kernel (generate.py:128-136).
  int kdt = datatype;
  if (sem == nexrSemanticsFork && red.op == nexrDevMinMax)
    kdt = datatype == nexrInt8 ? nexrUint8 : datatype == nexrInt32 ? nexrUint32 : datatype == nexrInt64 ? nexrUint64 : datatype;
  r = ensureResident(c);
  if (r == nexrSuccess && tree) r = ensureResidentTree(c, residentMulti(c));
  if (r != nexrSuccess) return r;
  const Geom g = (coll == kReduce || coll == kBroadcast || tree) ? kGeomPipe : kGeomRing;
  const int trafficPerByte = coll == kAllReduce ? 2 : (coll == kReduceScatter || coll == kAllGather) ? n : 1;
  std::vector<ChannelPart> parts = channelParts(c, (int64_t)count, esz, trafficPerByte);
  nexr::ResParams a{};
  a.coll = tree                     ? nexr::kResTreeAllReduce
           : coll == kAllReduce     ? nexr::kResAllReduce
           : coll == kReduceScatter ? nexr::kResReduceScatter
           : coll == kAllGather     ? nexr::kResAllGather
           : coll == kReduce        ? nexr::kResReduce
                                    : nexr::kResBroadcast;
  a.root = root;
  a.count = (int64_t)count;
  a.nRanks = n;
  a.nParts = (int)parts.size();
  for (size_t i = 0; i < parts.size(); i++) {
    a.partOffset[i] = parts[i].offset;
    a.partCount[i] = parts[i].count;
    a.partChannel[i] = parts[i].channel;
  }
  // calcCollChunking per part (enqueue.cc:1993-1999); for SIMPLE every part gets the same chunk
  a.chunkCount = chunkElems(c, g, esz, tree, parts.empty() ? 0 : (size_t)parts[0].count * esz);
  a.stepElems = (int64_t)(c->stepBytes / esz);
  a.stepBytes = c->stepBytes;
  a.stepPerSlice = g.sliceSteps;
  a.slicePerChunk = g.chunkSteps / g.sliceSteps;
  a.redArg = red.scalarArg;
  a.timeoutTicks = (uint64_t)(c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 100000ull;  // 100 MHz
  for (int i = 0; i < n; i++) {
    a.input[i] = (const char*)sendbuffs[i];
    a.output[i] = (char*)recvbuffs[i];
  }
  int busiest = 0;
  std::vector<std::vector<int>> onDev(c->resDevs.size());
  for (int i = 0; i < n; i++) onDev[resDevIndex(c, i)].push_back(i);
  for (const auto& v : onDev) busiest = std::max(busiest, (int)v.size());
  const int roles = tree ? 2 : 1;  // the tree's reduce-up and broadcast-down teams
  a.team = residentTeam(busiest * roles, a.nParts, c->stepBytes * (size_t)a.stepPerSlice);
  // Every workgroup of a device's grid must be resident at once (a rank's workgroups wait on others'):
  // the team shrinks to what the kernel's occupancy allows on every device used.
  long capacity = -1;
  for (size_t d = 0; d < c->resDevs.size(); d++) {
    long cap = 0;
    if (hipSetDevice(c->resDevs[d]) != hipSuccess ||
        residentCapacity(c->resDevs[d], kdt, red.op, red.scalarArg, a.coll, &cap) != nexrSuccess)
      return nexrUnhandledCudaError;
    capacity = capacity < 0 ? cap : std::min(capacity, cap);
  }
  if ((long)busiest * roles * a.nParts * a.team > capacity) a.team = (int)(capacity / ((long)busiest * roles * a.nParts));
  if (a.team < 1) return nexrInvalidUsage;
  std::vector<hipStream_t> used;
  for (size_t d = 0; d < onDev.size() && r == nexrSuccess; d++) {
    a.conns = (const nexr::ResConn*)c->resTable[d];
    a.tree = tree ? (const nexr::ResTreeConn*)c->resTreeTable[d] : nullptr;
    a.status = c->resStatus[d];
    for (size_t k = 0; k < onDev[d].size(); k++) a.rankOf[k] = onDev[d][k];
    hipStream_t s = c->streams[onDev[d][0]];
    if (hipSetDevice(c->resDevs[d]) != hipSuccess ||
        nexr::launch_resident(kdt, red.op, a, (int)onDev[d].size() * roles * a.nParts * a.team, s) != hipSuccess)
      r = nexrUnhandledCudaError;
    else
      used.push_back(s);
  }
  if (r != nexrSuccess)  // a GPU's launch failed: the ones already running would wait for its ranks
    for (size_t d = 0; d < used.size(); d++) __atomic_store_n(c->resStatus[d], 2u, __ATOMIC_RELEASE);
  for (size_t d = 0; d < used.size(); d++) {
    (void)hipSetDevice(c->resDevs[d]);
    if (hipStreamSynchronize(used[d]) != hipSuccess)
      r = nexrUnhandledCudaError;
    else if (__atomic_load_n(c->resStatus[d], __ATOMIC_ACQUIRE) != 0 && r == nexrSuccess)
      r = nexrInternalError;  // a step wait timed out: the counters are mid-protocol
  }
  if (r != nexrSuccess) c->broken = true;
  return r;
}

// Process ranks, first resident call: publish this rank's GPU and its proposed team (`want`, capped
// by what its GPU keeps resident, `perPartCap` workgroups per part), wait for every rank, then run
// min over ranks of min(want, perPartCap / ranks sharing that GPU): every rank launches the same
// team, and the grids of ranks that share a GPU fit on it together. Collective, bounded by the
// communicator's timeout and abort word.
nexrResult_t residentPeerTeam(nexrRingComm* c, int want, long perPartCap) {
  const int n = c->cfg.nRanks, me = c->self;
  int dom = 0, bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, c->devices[me]) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, c->devices[me]) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, c->devices[me]) != hipSuccess)
    return nexrUnhandledCudaError;
  PeerSlot* mine = peerSlot(c->shm, me);
  mine->residentGpu.store(((uint64_t)(uint32_t)dom << 32) | ((uint64_t)(bus & 0xffff) << 16) | (uint64_t)(dev & 0xffff),
                          std::memory_order_relaxed);
  mine->residentCap.store(perPartCap, std::memory_order_relaxed);
  mine->residentTeam.store(std::max(1, want), std::memory_order_release);
  PeerHeader* h = peerHeader(c->shm);
  const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
  const auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < n; r++) {
    while (peerSlot(c->shm, r)->residentTeam.load(std::memory_order_acquire) == 0) {
      if (h->abort.load(std::memory_order_acquire) ||
          std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) {
        c->broken = true;
        h->abort.store(1);
        return nexrRemoteError;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  // Every rank evaluates the same expression over the same published values.
  long team = nexr::kResMaxTeam;
  for (int r = 0; r < n; r++) {
    const PeerSlot* sr = peerSlot(c->shm, r);
    const uint64_t gpu = sr->residentGpu.load(std::memory_order_relaxed);
    int sharing = 0;
    for (int q = 0; q < n; q++) sharing += peerSlot(c->shm, q)->residentGpu.load(std::memory_order_relaxed) == gpu;
    team = std::min<long>(team, sr->residentTeam.load(std::memory_order_relaxed));
    team = std::min<long>(team, sr->residentCap.load(std::memory_order_relaxed) / std::max(1, sharing));
  }
  const uint64_t myGpu = mine->residentGpu.load(std::memory_order_relaxed);
  int sharing = 0;
  for (int q = 0; q < n; q++) sharing += peerSlot(c->shm, q)->residentGpu.load(std::memory_order_relaxed) == myGpu;
  if (team < 1) return nexrInvalidUsage;
  c->residentTeamAgreed = (int)std::min<long>(team, nexr::kResMaxTeam);
  c->residentSharing = std::max(1, sharing);
  return nexrSuccess;
}

// Process ranks: this process's rank of the resident ring all-reduce. The schedule runs in one
// launch on this rank's GPU; the other ranks' launches in their own processes meet it only through
// the FIFOs and the step records behind them (the receiver's allocation, mapped by the sender over
// IPC). Every rank must make the same sequence of calls.
nexrResult_t residentPeerAllReduce(nexrRingComm* c, const void* sendbuff, void* recvbuff, size_t count, int datatype,
                                   int op) {
  if (!c || !c->peer) return nexrInvalidArgument;
  if (c->proto != nexrRingProtoSimple) return nexrInvalidUsage;
  int sem = nexrSemanticsNccl;
  if (nexrGetSemantics(&sem) != nexrSuccess || sem == nexrSemanticsShipped) return nexrInvalidUsage;
  size_t esz;
  nexrDevRedOpFull red;
  nexrResult_t r = prepare(c, datatype, op, &esz, &red);
  if (r != nexrSuccess) return r;
  const int n = c->cfg.nRanks, me = c->self, next = (me + 1) % n;
  if (count > 0 && (!sendbuff || !recvbuff)) return nexrInvalidArgument;
  if (count == 0) return nexrSuccess;
  (void)hipSetDevice(c->devices[me]);
  if (n == 1) return oneRank(c, me, sendbuff, recvbuff, count, datatype, red, esz);
  if (n > nexr::kResMaxRanks) return nexrInvalidUsage;
  int kdt = datatype;
  if (sem == nexrSemanticsFork && red.op == nexrDevMinMax)
    kdt = datatype == nexrInt8 ? nexrUint8 : datatype == nexrInt32 ? nexrUint32 : datatype == nexrInt64 ? nexrUint64 : datatype;
  if (c->resDevs.empty()) {  // the (rank) table with this rank's entry, and a status word
    c->resDevs.assign(1, c->devices[me]);
    c->resTable.assign(1, nullptr);
    c->resCtr.assign(1, nullptr);
    c->resStatus.assign(1, nullptr);
    c->freeExtras = freeResident;
    char* fifoIn = c->conns[me]->fifo;
    char* fifoOut = c->conns[next]->fifo;
    std::vector<nexr::ResConn> table((size_t)n);
    table[(size_t)me] = {fifoIn, fifoOut, fifoIn + c->cfg.buffBytes, fifoOut + c->cfg.buffBytes};
    if (hipMalloc(&c->resTable[0], sizeof(nexr::ResConn) * table.size()) != hipSuccess ||
        hipMemcpy(c->resTable[0], table.data(), sizeof(nexr::ResConn) * table.size(), hipMemcpyHostToDevice) !=
            hipSuccess ||
        hipHostMalloc((void**)&c->resStatus[0], sizeof(uint32_t), hipHostMallocMapped | hipHostMallocPortable) !=
            hipSuccess) {
      freeResident(c);
      c->broken = true;
      peerHeader(c->shm)->abort.store(1);  // the other ranks would wait for this one's kernel
      return nexrUnhandledCudaError;
    }
    *c->resStatus[0] = 0;
  }
  const Geom g = kGeomRing;
  std::vector<ChannelPart> parts = channelParts(c, (int64_t)count, esz, 2);  // process ranks: 1 channel
  nexr::ResParams a{};
  a.coll = nexr::kResAllReduce;
  a.count = (int64_t)count;
  a.nRanks = n;
  a.nParts = (int)parts.size();
  for (size_t i = 0; i < parts.size(); i++) {
    a.partOffset[i] = parts[i].offset;
    a.partCount[i] = parts[i].count;
    a.partChannel[i] = 0;
  }
  a.chunkCount = chunkElems(c, g, esz, false, 0);
  a.stepElems = (int64_t)(c->stepBytes / esz);
  a.stepBytes = c->stepBytes;
  a.stepPerSlice = g.sliceSteps;
  a.slicePerChunk = g.chunkSteps / g.sliceSteps;
  a.redArg = red.scalarArg;
  a.timeoutTicks = (uint64_t)(c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000) * 100000ull;
  a.input[me] = (const char*)sendbuff;
  a.output[me] = (char*)recvbuff;
  a.rankOf[0] = me;
  a.conns = (const nexr::ResConn*)c->resTable[0];
  a.status = c->resStatus[0];
  // The team size must be the same on every rank (member g meets member g), and every rank's grid
  // must stay resident beside the other ranks' grids on the same GPU: agreed once, through the
  // shared segment (residentPeerTeam).
  // A failure from here on leaves the other ranks waiting for this one: mark the communicator broken
  // and raise the shared abort word, so they leave at once instead of after the timeout.
  auto failAll = [&](nexrResult_t res) {
    c->broken = true;
    peerHeader(c->shm)->abort.store(1);
    return res;
  };
  long capacity = 0;
  if (residentCapacity(c->devices[me], kdt, red.op, red.scalarArg, a.coll, &capacity) != nexrSuccess)
    return failAll(nexrUnhandledCudaError);
  if (c->residentTeamAgreed == 0) {
    int team = residentTeam(1, a.nParts, c->stepBytes * (size_t)a.stepPerSlice);
    r = residentPeerTeam(c, team, capacity / a.nParts);
    if (r != nexrSuccess) return failAll(r);
  }
  a.team = c->residentTeamAgreed;
  // The team was agreed on the first call's kernel; this call's (datatype, op) kernel may keep fewer
  // workgroups per CU resident. Its grid, beside the grids of the ranks sharing this GPU, must still
  // fit at once, or member g would wait for peers that are never scheduled: fail fast instead.
  if ((long)a.nParts * a.team * c->residentSharing > capacity) return failAll(nexrInvalidUsage);
  r = ringLinkHandover(c, true);
  if (r != nexrSuccess) return r;
  hipStream_t s = c->streams[me];
  if (nexr::launch_resident(kdt, red.op, a, a.nParts * a.team, s) != hipSuccess) r = nexrUnhandledCudaError;
  // Wait for the kernel while relaying the communicator's abort word (set by a failing rank in another
  // process) into this GPU's status word, which the kernel's waits poll: a rank's failure then ends
  // every rank's kernel at once instead of after the full timeout.
  // Poll without sleeping for the first 2 ms (a C1-size call takes tens of microseconds, and a sleep
  // costs the timer slack, ~50 us), then every 20 us.
  PeerHeader* ph = peerHeader(c->shm);
  const auto pollStart = std::chrono::steady_clock::now();
  static const bool relay = envFlagOn("NEXR_RESIDENT_RELAY", true);  // A/B knob (tools/xgmi_probe.py)
  for (bool relayed = !relay; r == nexrSuccess && relay;) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) {
      r = nexrUnhandledCudaError;
      break;
    }
    if (!relayed && ph->abort.load(std::memory_order_acquire)) {
      // Only over a clean word: a timeout the kernel already reported (1) must stay visible.
      uint32_t clean = 0;
      __atomic_compare_exchange_n(c->resStatus[0], &clean, 2u, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE);
      relayed = true;
    }
    if (std::chrono::steady_clock::now() - pollStart > std::chrono::milliseconds(2))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    else
      std::this_thread::yield();
  }
  if (hipStreamSynchronize(s) != hipSuccess && r == nexrSuccess) r = nexrUnhandledCudaError;
  // 1: a step wait timed out; 3: a workgroup gave up on the relayed abort (mid-protocol either way).
  // 2 left as relayed: no wait saw it, the kernel ran this rank's whole schedule before the relay
  // arrived (another rank failed a LATER call, e.g. at the capacity guard above): this call succeeded.
  const uint32_t st = __atomic_load_n(c->resStatus[0], __ATOMIC_ACQUIRE);
  if (st == 2) __atomic_store_n(c->resStatus[0], 0u, __ATOMIC_RELEASE);
  else if (r == nexrSuccess && st != 0) r = nexrInternalError;
  if (r != nexrSuccess) {
    c->broken = true;
    peerHeader(c->shm)->abort.store(1);
    return r;
  }
  peerSlot(c->shm, me)->residentDone.store(++c->residentCalls, std::memory_order_release);
  return r;
}

}  // namespace nexr_emu

extern "C" {

NEXR_API nexrResult_t nexrPeerRingAllReduceResident(nexrRingComm_t c, const void* sendbuff, void* recvbuff,
                                                    size_t count, int datatype, int op) {
  DeviceGuard dg(true);
  return residentPeerAllReduce(c, sendbuff, recvbuff, count, datatype, op);
}

NEXR_API nexrResult_t nexrRingAllReduceResident(nexrRingComm_t c, const void* const* sendbuffs,
                                                void* const* recvbuffs, size_t count, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kAllReduce, sendbuffs, recvbuffs, count, datatype, op, 0);
}

NEXR_API nexrResult_t nexrTreeAllReduceResident(nexrRingComm_t c, const void* const* sendbuffs,
                                                void* const* recvbuffs, size_t count, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kAllReduce, sendbuffs, recvbuffs, count, datatype, op, 0, /*tree=*/true);
}

NEXR_API nexrResult_t nexrRingReduceScatterResident(nexrRingComm_t c, const void* const* sendbuffs,
                                                    void* const* recvbuffs, size_t recvcount, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kReduceScatter, sendbuffs, recvbuffs, recvcount, datatype, op, 0);
}

NEXR_API nexrResult_t nexrRingAllGatherResident(nexrRingComm_t c, const void* const* sendbuffs,
                                                void* const* recvbuffs, size_t sendcount, int datatype) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kAllGather, sendbuffs, recvbuffs, sendcount, datatype, nexrSum, 0);
}

NEXR_API nexrResult_t nexrRingReduceResident(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                             size_t count, int datatype, int op, int root) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kReduce, sendbuffs, recvbuffs, count, datatype, op, root);
}

NEXR_API nexrResult_t nexrRingBroadcastResident(nexrRingComm_t c, const void* const* sendbuffs,
                                                void* const* recvbuffs, size_t count, int datatype, int root) {
  DeviceGuard dg(c && c->needHip);
  return residentCollective(c, kBroadcast, sendbuffs, recvbuffs, count, datatype, nexrSum, root);
}

}  // extern "C"
