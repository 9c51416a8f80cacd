// nexr_ring.cpp — CPU-emulated collectives (include/nexr_ring.h): the reference's own collective
// schedules, restated on host threads, calling the reduce-copy ABI at exactly the reduceCopy sites
// of Primitives::genericOp. This is the drop-in demonstration for BASELINE configs[0] ("fp32 sum
// all-reduce, 4 MiB, 2 CPU-emulated ranks") and for every other caller of the primitive: the
// schedules are unchanged, only the primitive underneath is the MI355X kernel.
#include <fcntl.h>
#include <map>
#include <mutex>
#include <system_error>
#include <tuple>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "nexr_emu.h"
#include "nexr_resident.h"

namespace nexr_emu {

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
std::vector<ChannelPart> channelParts(const nexrRingComm* c, int64_t count, size_t esz, int trafficPerByteFn) {
  const int64_t kMinTrafficPerChannel = 16 << 10;  // enqueue.cc:539
  const int64_t nMaxChannels = c->cfg.nChannels > 0 ? c->cfg.nChannels : 1;
  // Plan-level traffic split (:548-573) for this one task; the task may use every channel.
  const int64_t taskTraffic = std::max<int64_t>(kMinTrafficPerChannel, count * (int64_t)esz * trafficPerByteFn);
  const int64_t trafficPerChannel = std::max<int64_t>(kMinTrafficPerChannel, taskTraffic / nMaxChannels);
  // Cell partition (:608-646).
  int64_t channelId = 0;
  const int64_t currentTraffic = 0;
  const int64_t trafficPerByte = trafficPerByteFn * (c->proto == nexrRingProtoLL ? 4 : 1);
  const int64_t cellSize = divUp(divUp(kMinTrafficPerChannel, trafficPerByte), 16) * 16;
  const int64_t elementsPerCell = cellSize / (int64_t)esz;
  const int64_t cells = divUp(count * (int64_t)esz, cellSize);
  const int64_t trafficPerCell = cellSize * trafficPerByte;
  int64_t cellsPerChannel = std::min(cells, divUp(trafficPerChannel, trafficPerCell));
  int64_t cellsLo = channelId + 1 == nMaxChannels
                        ? cells
                        : std::min(cells, divUp(trafficPerChannel - currentTraffic, trafficPerCell));
  int64_t nMidChannels = (cells - cellsLo) / cellsPerChannel;
  int64_t cellsHi = (cells - cellsLo) % cellsPerChannel;
  int64_t nChannels = (cellsLo != 0 ? 1 : 0) + nMidChannels + (cellsHi != 0 ? 1 : 0);
  if (nMaxChannels < channelId + nChannels) {  // overflowed the available channels
    nMidChannels = nMaxChannels - channelId - 2;
    cellsPerChannel = (cells - cellsLo) / (nMidChannels + 1);
    cellsHi = cellsPerChannel + (cells - cellsLo) % (nMidChannels + 1);
  }
  if (cellsHi == 0 && nMidChannels != 0) {
    cellsHi = cellsPerChannel;
    nMidChannels -= 1;
  }
  if (cellsLo == 0) {  // least channel skipped
    channelId += 1;
    if (nMidChannels == 0) {
      cellsLo = cellsHi;
      cellsHi = 0;
    } else {
      cellsLo = cellsPerChannel;
      nMidChannels -= 1;
    }
  }
  const int64_t countMid = nMidChannels != 0 ? cellsPerChannel * elementsPerCell : 0;
  int64_t countLo = cellsLo * elementsPerCell;
  int64_t countHi = cellsHi * elementsPerCell;
  (countHi != 0 ? countHi : countLo) -= cells * elementsPerCell - count;
  nChannels = (countLo != 0 ? 1 : 0) + nMidChannels + (cellsHi != 0 ? 1 : 0);
  // ncclCollCbdPart (device.h:946-970) for channels channelLo .. channelLo + nChannels - 1.
  std::vector<ChannelPart> parts;
  const int64_t lo = channelId, hi = channelId + nChannels - 1;
  for (int64_t ch = lo; ch <= hi; ch++) {
    ChannelPart part{(int)ch, 0, 0, 0};
    if (ch == lo) {
      part.count = countLo;
    } else if (ch == hi) {
      part.offset = countLo + nMidChannels * countMid;
      part.count = countHi;
    } else {
      part.offset = countLo + (ch - lo - 1) * countMid;
      part.count = countMid;
    }
    parts.push_back(part);
  }
  return parts;
}

// ---- schedules (one rank's view of one channel, userRanks[i] = (rank + i) % nranks) -------------
// Every schedule works on its channel's part of the data (ncclCollCbdPart, device.h:946-970):
// elements [part.offset, part.offset + part.count) in chunks of part.chunkCount.

// runRing for ncclAllReduce (all_reduce.h:12-84).
void runRingAllReduce(Prims& p, int nranks, const ChannelPart& part) {
  const int ringIx = p.rank;
  int64_t chunkCount = part.chunkCount;
  const int64_t loopCount = nranks * chunkCount;
  auto modRanks = [&](int r) { return r - (r >= nranks ? nranks : 0); };
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += loopCount) {
    const int64_t remCount = part.count - elemOffset;
    if (remCount < loopCount) chunkCount = alignUp(divUp(remCount, nranks), 16 / (int64_t)p.esz);
    auto at = [&](int chunk, int64_t* offset) {
      const int64_t chunkOffset = chunk * chunkCount;
      *offset = part.offset + elemOffset + chunkOffset;
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
void runRingReduceScatter(Prims& p, int nranks, int64_t count, const ChannelPart& part) {
  const int r = p.rank;
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += part.chunkCount) {
    const int64_t nelem = std::min(part.chunkCount, part.count - elemOffset);
    const int64_t dataOffset = part.offset + elemOffset;
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
void runRingAllGather(Prims& p, int nranks, int64_t count, const ChannelPart& part) {
  const int r = p.rank;
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += part.chunkCount) {
    const int64_t nelem = std::min(part.chunkCount, part.count - elemOffset);
    const int64_t dataOffset = part.offset + elemOffset;
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
void runRingReduce(Prims& p, int nranks, int root, const ChannelPart& part) {
  const int r = p.rank, prevRank = (r + nranks - 1) % nranks;
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += part.chunkCount) {
    const int64_t offset = part.offset + elemOffset;
    const int64_t nelem = std::min(part.chunkCount, part.count - elemOffset);
    bool ok;
    if (prevRank == root) ok = p.sendInput(offset, nelem);
    else if (r == root) ok = p.recvReduceCopy(offset, offset, nelem, /*postOp=*/true);
    else ok = p.recvReduceSend(offset, nelem);
    if (!ok) return;
  }
}

// runRing for ncclBroadcast (broadcast.h:12-58).
void runRingBroadcast(Prims& p, int nranks, int root, const ChannelPart& part) {
  const int r = p.rank, nextRank = (r + 1) % nranks;
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += part.chunkCount) {
    const int64_t offset = part.offset + elemOffset;
    const int64_t nelem = std::min(part.chunkCount, part.count - elemOffset);
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
void runTree(Prims& p, TreeRole role, bool leaf, const ChannelPart& part) {
  for (int64_t elemOffset = 0; elemOffset < part.count; elemOffset += part.chunkCount) {
    const int64_t offset = part.offset + elemOffset;
    const int64_t nelem = std::min(part.chunkCount, part.count - elemOffset);
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

// The pinned, device-mapped completion word of one stream (Prims::streamDone): [0] is written by
// the stream's hipStreamWriteValue32, [1] holds the last ticket handed out.
nexrResult_t allocDone(uint32_t** w) {
  if (hipHostMalloc((void**)w, 2 * sizeof(uint32_t), hipHostMallocMapped | hipHostMallocPortable) != hipSuccess) {
    *w = nullptr;
    return nexrUnhandledCudaError;
  }
  (*w)[0] = (*w)[1] = 0;
  return nexrSuccess;
}

// The completion word of `stream` (one of the communicator's streams), or nullptr.
uint32_t* doneFor(const nexrRingComm* c, hipStream_t stream) {
  if (!stream) return nullptr;
  for (size_t r = 0; r < c->streams.size() && r < c->done.size(); r++)
    if (c->streams[r] == stream) return c->done[r];
  for (size_t r = 0; r < c->streams2.size() && r < c->done2.size(); r++)
    if (c->streams2[r] == stream) return c->done2[r];
  return nullptr;
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
  p.done = doneFor(c, stream);
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

// Test hook: NEXR_TEST_SPAWN_FAIL_AT=k makes the k-th thread creation (1-based) of the next
// runThreads calls throw, as std::thread does when the system is out of threads.
static void spawnHook(size_t k) {
  const char* e = getenv("NEXR_TEST_SPAWN_FAIL_AT");
  if (e && *e && (size_t)strtoull(e, nullptr, 10) == k)
    throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again), "spawn hook");
}

// Runs `jobs` (one per emulated rank, or per tree half) on host threads and collects the first error.
// If a thread cannot be created, the ones already running are told to give up (their spins see the
// abort), joined, and the call reports nexrSystemError with the communicator broken: nothing throws
// through the C entry points and no joinable thread is ever destroyed.
nexrResult_t runThreads(nexrRingComm* c, Shared& sh, const std::vector<std::function<void()>>& jobs) {
  std::vector<std::thread> threads;
  try {
    threads.reserve(jobs.size());
    for (const auto& j : jobs) {
      spawnHook(threads.size() + 1);
      threads.emplace_back(j);
    }
  } catch (...) {
    sh.fail(nexrSystemError);
  }
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

nexrResult_t allocFifo(nexrRingComm* c, Conn* k, int device, size_t bytes) {
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
  c->done2.assign(n, nullptr);
  for (int r = 0; r < n; r++) {
    if (c->streams[r]) {
      if (hipSetDevice(c->devices[r]) != hipSuccess || hipStreamCreate(&c->streams2[r]) != hipSuccess)
        return nexrUnhandledCudaError;
      if (allocDone(&c->done2[r]) != nexrSuccess) return nexrUnhandledCudaError;
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
  const int trafficPerByte = coll == kAllReduce ? 2 : (coll == kReduceScatter || coll == kAllGather) ? n : 1;
  std::vector<ChannelPart> parts = channelParts(c, (int64_t)count, esz, trafficPerByte);
  for (ChannelPart& part : parts) part.chunkCount = chunkElems(channelComm(c, part.channel), g, esz, false, 0);
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (const ChannelPart& part : parts) {
    for (int rank = 0; rank < n; rank++) {
      jobs.emplace_back([&, rank, part] {
        nexrRingComm* ck = channelComm(c, part.channel);
        if (ck->streams[rank]) (void)hipSetDevice(ck->devices[rank]);
        Prims p = makePrims(ck, &sh, rank, sendbuffs[rank], recvbuffs[rank], esz, datatype, red, g,
                            ck->streams[rank], ck->status[rank]);
        p.recv[p.nRecv++] = ck->conns[rank];
        p.send[p.nSend++] = ck->conns[(rank + 1) % n];
        p.attach();
        switch (coll) {
          case kAllReduce: runRingAllReduce(p, n, part); break;
          case kReduceScatter: runRingReduceScatter(p, n, (int64_t)count, part); break;
          case kAllGather: runRingAllGather(p, n, (int64_t)count, part); break;
          case kReduce: runRingReduce(p, n, root, part); break;
          case kBroadcast: runRingBroadcast(p, n, root, part); break;
        }
      });
    }
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
  r = ringLinkHandover(c, false);
  if (r != nexrSuccess) return r;
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  const Geom g = (coll == kReduce || coll == kBroadcast) ? kGeomPipe : kGeomRing;
  Prims p = makePrims(c, &sh, me, sendbuff, recvbuff, esz, datatype, red, g, c->streams[me], c->status[me]);
  p.recv[p.nRecv++] = c->conns[me];
  p.send[p.nSend++] = c->conns[(me + 1) % n];
  p.attach();
  const ChannelPart part{0, 0, (int64_t)count, chunkElems(c, g, esz, false, 0)};  // process ranks: 1 channel
  switch (coll) {
    case kAllReduce: runRingAllReduce(p, n, part); break;
    case kReduceScatter: runRingReduceScatter(p, n, (int64_t)count, part); break;
    case kAllGather: runRingAllGather(p, n, (int64_t)count, part); break;
    case kReduce: runRingReduce(p, n, root, part); break;
    case kBroadcast: runRingBroadcast(p, n, root, part); break;
  }
  if (sh.firstError.load() != 0) {
    c->broken = true;
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

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

bool envFlagOn(const char* name, bool dflt) {
  const char* v = getenv(name);
  return v && *v ? v[0] != '0' : dflt;
}

// Process ranks: the ring link r -> r+1 (rank r+1's receive FIFO) serves two users with separate
// step counters: the host-sequenced collectives (head/tail in the shared segment, also PAT's ring
// link) and the resident all-reduce (records behind the FIFO). Either returns once this rank's own
// schedule is done, while rank r+1 may still be reading the last slots it was sent. Before this
// rank writes the link as the other user, it waits until rank r+1 has consumed everything the
// previous user sent: head == tail after host-sequenced calls, or rank r+1's kernel done after
// resident ones. Bounded by the communicator's timeout and its abort word, as every other wait.
nexrResult_t ringLinkHandover(nexrRingComm* c, bool resident) {
  const int want = resident ? 2 : 1;
  const int prev = c->ringLinkUser;
  c->ringLinkUser = want;
  if (prev == 0 || prev == want) return nexrSuccess;
  const int n = c->cfg.nRanks, next = (c->self + 1) % n;
  PeerSlot* s = peerSlot(c->shm, next);
  PeerHeader* h = peerHeader(c->shm);
  const int timeoutMs = c->cfg.timeoutMs > 0 ? c->cfg.timeoutMs : 60000;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const bool drained = resident
                             ? s->conn.head.load(std::memory_order_acquire) >= s->conn.tail.load(std::memory_order_acquire)
                             : s->residentDone.load(std::memory_order_acquire) >= c->residentCalls;
    if (drained) return nexrSuccess;
    if (h->abort.load(std::memory_order_acquire)) break;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeoutMs)) break;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
  c->broken = true;
  h->abort.store(1);
  return nexrRemoteError;
}

nexrResult_t peerFinish(nexrRingComm* c, Shared& sh) {
  if (sh.firstError.load() != 0) {
    c->broken = true;
    return (nexrResult_t)sh.firstError.load();
  }
  return nexrSuccess;
}

// A communicator touches HIP when its FIFOs live in device memory or when any of its steps runs the
// built-in (HIP) reduce-copy; one whose steps are all caller-supplied (a CPU checker) never does.
bool needsHip(const nexrRingConfig& cfg) {
  return cfg.memMode == nexrRingDeviceMemory || (cfg.protocol == nexrRingProtoSimple && !cfg.fn) ||
         (cfg.protocol == nexrRingProtoLL && !cfg.llFn) || (cfg.protocol == nexrRingProtoLL128 && !cfg.ll128Fn);
}

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
  if (team < 1) return nexrInvalidUsage;
  c->residentTeamAgreed = (int)std::min<long>(team, nexr::kResMaxTeam);
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
  if (c->residentTeamAgreed == 0) {
    int team = residentTeam(1, a.nParts, c->stepBytes * (size_t)a.stepPerSlice);
    long capacity = 0;
    if (residentCapacity(c->devices[me], kdt, red.op, red.scalarArg, a.coll, &capacity) != nexrSuccess)
      return nexrUnhandledCudaError;
    r = residentPeerTeam(c, team, capacity / a.nParts);
    if (r != nexrSuccess) return r;
  }
  a.team = c->residentTeamAgreed;
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
      __atomic_store_n(c->resStatus[0], 2u, __ATOMIC_RELEASE);
      relayed = true;
    }
    if (std::chrono::steady_clock::now() - pollStart > std::chrono::milliseconds(2))
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    else
      std::this_thread::yield();
  }
  if (hipStreamSynchronize(s) != hipSuccess && r == nexrSuccess) r = nexrUnhandledCudaError;
  if (r == nexrSuccess && __atomic_load_n(c->resStatus[0], __ATOMIC_ACQUIRE) != 0) r = nexrInternalError;
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

NEXR_API nexrResult_t nexrRingCommCreate(nexrRingComm_t* out, const nexrRingConfig* cfg) {
  DeviceGuard dg(cfg && needsHip(*cfg));
  if (!out || !cfg || cfg->nRanks < 1 || cfg->nRanks > 1024) return nexrInvalidArgument;
  if (cfg->memMode != nexrRingHostMemory && cfg->memMode != nexrRingDeviceMemory) return nexrInvalidArgument;
  if (cfg->protocol != nexrRingProtoSimple && cfg->protocol != nexrRingProtoLL && cfg->protocol != nexrRingProtoLL128)
    return nexrInvalidArgument;
  if (cfg->treeRanksPerNode < 0 || (cfg->treeRanksPerNode > 0 && cfg->nRanks % cfg->treeRanksPerNode != 0) ||
      (cfg->treeIndex != 0 && cfg->treeIndex != 1))
    return nexrInvalidArgument;
  if (cfg->nChannels < 0 || cfg->nChannels > kMaxChannels) return nexrInvalidArgument;
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
  c->done.assign(n, nullptr);
  int nDev = 0;
  c->needHip = needsHip(*cfg);
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
      if (hipSetDevice(c->devices[r]) != hipSuccess || hipStreamCreate(&c->streams[r]) != hipSuccess ||
          allocDone(&c->done[r]) != nexrSuccess) {
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
  // Channels 1..nChannels-1: the same communicator again. The reference duplicates its channels and
  // gives the copies the other tree of the double binary tree (graph/connect.cc:146-160).
  const int nCh = cfg->nChannels > 0 ? cfg->nChannels : 1;
  c->cfg.nChannels = nCh;
  for (int k = 1; k < nCh; k++) {
    nexrRingConfig sub = *cfg;
    sub.nChannels = 1;
    sub.treeIndex = (cfg->treeIndex + (nCh >= 2 && k >= nCh / 2 ? 1 : 0)) % 2;
    nexrRingComm_t sc = nullptr;
    nexrResult_t res = nexrRingCommCreate(&sc, &sub);
    if (res != nexrSuccess) {
      nexrRingCommDestroy(c);
      return res;
    }
    c->channels.push_back(sc);
  }
  *out = c;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingAllReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return ringCollective(c, kAllReduce, sendbuffs, recvbuffs, count, datatype, op, 0);
}

NEXR_API nexrResult_t nexrRingReduceScatter(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                            size_t recvcount, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return ringCollective(c, kReduceScatter, sendbuffs, recvbuffs, recvcount, datatype, op, 0);
}

NEXR_API nexrResult_t nexrRingAllGather(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t sendcount, int datatype) {
  DeviceGuard dg(c && c->needHip);
  return ringCollective(c, kAllGather, sendbuffs, recvbuffs, sendcount, datatype, nexrSum, 0);  // ncclAllGather: ncclSum
}

NEXR_API nexrResult_t nexrRingReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                     size_t count, int datatype, int op, int root) {
  DeviceGuard dg(c && c->needHip);
  return ringCollective(c, kReduce, sendbuffs, recvbuffs, count, datatype, op, root);
}

NEXR_API nexrResult_t nexrRingBroadcast(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int root) {
  DeviceGuard dg(c && c->needHip);
  return ringCollective(c, kBroadcast, sendbuffs, recvbuffs, count, datatype, nexrSum, root);  // ncclBroadcast: ncclSum
}

NEXR_API nexrResult_t nexrTreeAllReduce(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
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
  std::vector<ChannelPart> parts = channelParts(c, (int64_t)count, esz, /*ncclFuncAllReduce*/ 2);
  for (ChannelPart& part : parts) {
    nexrRingComm* ck = channelComm(c, part.channel);
    r = ensureTree(ck);
    if (r != nexrSuccess) {
      c->broken = true;
      return r;
    }
    // calcCollChunking for the part: nBytes = its count x esz (enqueue.cc:664-679)
    part.chunkCount = chunkElems(ck, kGeomPipe, esz, true, (size_t)part.count * esz);
  }
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (const ChannelPart& part : parts) {
    nexrRingComm* ck = channelComm(c, part.channel);
    for (int rank = 0; rank < n; rank++) {
      const TreeLinks& t = ck->tree[rank];
      const bool leaf = t.down[0] == -1;
      auto make = [&, rank, ck](hipStream_t s, uint32_t* st) {
        return makePrims(ck, &sh, rank, sendbuffs[rank], recvbuffs[rank], esz, datatype, red, kGeomPipe, s, st);
      };
      if (t.up == -1) {  // root: recv from and send to every child
        jobs.emplace_back([&, rank, make, ck, part] {
          if (ck->streams[rank]) (void)hipSetDevice(ck->devices[rank]);
          Prims p = make(ck->streams[rank], ck->status[rank]);
          const TreeLinks& tl = ck->tree[rank];
          for (int i = 0; i < tl.nDown(); i++) {
            p.recv[p.nRecv++] = ck->treeUp[tl.down[i]];
            p.send[p.nSend++] = ck->treeDown[tl.down[i]];
          }
          p.attach();
          runTree(p, kTreeRoot, false, part);
        });
        continue;
      }
      jobs.emplace_back([&, rank, leaf, make, ck, part] {  // reduce up: recv from children, send to the parent
        if (ck->streams[rank]) (void)hipSetDevice(ck->devices[rank]);
        Prims p = make(ck->streams[rank], ck->status[rank]);
        const TreeLinks& tl = ck->tree[rank];
        for (int i = 0; i < tl.nDown(); i++) p.recv[p.nRecv++] = ck->treeUp[tl.down[i]];
        p.send[p.nSend++] = ck->treeUp[rank];
        p.attach();
        runTree(p, kTreeReduceUp, leaf, part);
      });
      jobs.emplace_back([&, rank, leaf, make, ck, part] {  // broadcast down: recv from the parent, send to children
        if (ck->streams2[rank]) (void)hipSetDevice(ck->devices[rank]);
        Prims p = make(ck->streams2[rank], ck->status2[rank]);
        const TreeLinks& tl = ck->tree[rank];
        p.recv[p.nRecv++] = ck->treeDown[rank];
        for (int i = 0; i < tl.nDown(); i++) p.send[p.nSend++] = ck->treeDown[tl.down[i]];
        p.attach();
        runTree(p, kTreeBcastDown, leaf, part);
      });
    }
  }
  return runThreads(c, sh, jobs);
}

NEXR_API nexrResult_t nexrTreeTopology(nexrRingComm_t c, int rank, int* up, int* down) {
  if (!c || !up || !down || rank < 0 || rank >= c->cfg.nRanks || c->tree.empty()) return nexrInvalidArgument;
  *up = c->tree[rank].up;
  for (int i = 0; i < kMaxArity; i++) down[i] = c->tree[rank].down[i];
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingCommDestroy(nexrRingComm_t c) {
  DeviceGuard dg(c && c->needHip);
  if (!c) return nexrInvalidArgument;
  freeResident(c);
  for (nexrRingComm* ch : c->channels) nexrRingCommDestroy(ch);
  c->channels.clear();
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
  for (auto* v : {&c->done, &c->done2})
    for (uint32_t* w : *v)
      if (w) (void)hipHostFree(w);
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
  DeviceGuard dg(true);
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
  c->done.assign(n, nullptr);
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
  if (hipSetDevice(cfg->device) != hipSuccess || hipStreamCreate(&c->streams[me]) != hipSuccess ||
      allocDone(&c->done[me]) != nexrSuccess)
    return fail(nexrUnhandledCudaError);
  if (c->ll && allocStatus(c, &c->status[me]) != nexrSuccess) return fail(nexrUnhandledCudaError);
  // The FIFO into this rank. Uncached device memory: it is written by another process's kernels
  // (over xGMI when that process drives another GPU) between this rank's launches.
  // NEXR_PEER_FIFO_UNCACHED=0 selects ordinary (coarse-grained) device memory instead.
  const char* unc = getenv("NEXR_PEER_FIFO_UNCACHED");
  const bool uncached = !(unc && unc[0] == '0');
  // Behind the FIFO, in the same allocation (so the sender maps both with the one IPC handle): the
  // step records of the resident all-reduce's connection into this rank, zeroed before the handle is
  // published (nexrPeerRingAllReduceResident).
  const size_t allocBytes = c->cfg.buffBytes + kPeerResidentRecordBytes;
  if ((uncached ? hipExtMallocWithFlags((void**)&c->conns[me]->fifo, allocBytes, hipDeviceMallocUncached)
                : hipMalloc((void**)&c->conns[me]->fifo, allocBytes)) != hipSuccess ||
      hipMemset(c->conns[me]->fifo + c->cfg.buffBytes, 0, kPeerResidentRecordBytes) != hipSuccess ||
      hipDeviceSynchronize() != hipSuccess)
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
    // The first rank configures the segment; every slot, link and counter starts from zero even if
    // the name was reused (the others touch nothing before initState == 2).
    memset((char*)c->shm + sizeof(PeerHeader), 0, c->shmBytes - sizeof(PeerHeader));
    h->joined.store(0);
    h->left.store(0);
    h->abort.store(0);
    h->patJoined.store(0);
    h->p2pJoined.store(0);
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
  // A segment left behind by an earlier communicator under the same name (a crashed run) still holds
  // its ranks' claims and counters: joining it would inherit stale head/tail steps and handles, so it
  // is refused. So is a second process claiming the same rank.
  PeerSlot* mine = peerSlot(c->shm, me);
  uint32_t unclaimed = 0;
  if (h->left.load(std::memory_order_acquire) != 0 || !mine->claimed.compare_exchange_strong(unclaimed, 1)) {
    munmap(c->shm, c->shmBytes);  // not ours: leave its abort word and counters alone
    c->shm = nullptr;
    nexrRingCommDestroy(c);
    return nexrInvalidUsage;
  }
  if (hipIpcGetMemHandle(&mine->fifoHandle, c->conns[me]->fifo) != hipSuccess) return fail(nexrUnhandledCudaError);
  c->conns[me]->st = &mine->conn;
  if (h->joined.fetch_add(1, std::memory_order_acq_rel) >= (uint32_t)n)  // publishes the handle
    return fail(nexrInvalidUsage);
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

NEXR_API nexrResult_t nexrPeerRingAllReduce(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return peerCollective(c, kAllReduce, sendbuff, recvbuff, count, datatype, op, 0);
}

NEXR_API nexrResult_t nexrPeerRingReduceScatter(nexrRingComm_t c, const void* sendbuff, void* recvbuff,
                                                size_t recvcount, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return peerCollective(c, kReduceScatter, sendbuff, recvbuff, recvcount, datatype, op, 0);
}

NEXR_API nexrResult_t nexrPeerRingAllGather(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t sendcount,
                                            int datatype) {
  DeviceGuard dg(c && c->needHip);
  return peerCollective(c, kAllGather, sendbuff, recvbuff, sendcount, datatype, nexrSum, 0);
}

NEXR_API nexrResult_t nexrPeerRingReduce(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                         int datatype, int op, int root) {
  DeviceGuard dg(c && c->needHip);
  return peerCollective(c, kReduce, sendbuff, recvbuff, count, datatype, op, root);
}

NEXR_API nexrResult_t nexrPeerRingBroadcast(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int root) {
  DeviceGuard dg(c && c->needHip);
  return peerCollective(c, kBroadcast, sendbuff, recvbuff, count, datatype, nexrSum, root);
}

}  // extern "C"
