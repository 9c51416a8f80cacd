// nexr_ring.cpp — CPU-emulated collectives (include/nexr_ring.h): the reference's own collective
// schedules, restated on host threads, calling the reduce-copy ABI at exactly the reduceCopy sites
// of Primitives::genericOp. This is the drop-in demonstration for BASELINE configs[0] ("fp32 sum
// all-reduce, 4 MiB, 2 CPU-emulated ranks") and for every other caller of the primitive: the
// schedules are unchanged, only the primitive underneath is the MI355X kernel.
// ncclSend/ncclRecv (nexr_p2p.cpp) and the device-resident forms (nexr_resident_host.cpp) go beyond
// SURVEY §8 and are built only into the opt-in extras library (include/nexr_extras.h).
#include <fcntl.h>
#include <system_error>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include "nexr_emu.h"

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

// A rank stream. Runs of LL steps on the device (Prims::enableLLRun) need the ranks' kernels to run at
// the same time: HIP shares its GPU_MAX_HW_QUEUES hardware queues among streams (once they are all made,
// a new stream takes the least used one), and two streams on one queue run their kernels one after the
// other, so a run waiting for its peer's would end only at its timeout. A stream made with a CU mask gets a
// hardware queue of its own (the runtime does not share those); with every CU in the mask it runs like any
// other stream (tools/ll_run_queue_probe.py). Device-memory LL communicators, the ones whose steps may
// run so, make their rank streams that way (NEXR_RING_OWN_QUEUES=0: plain streams, and no device runs);
// *own reports whether it worked.
hipError_t createRankStream(const nexrRingComm* c, hipStream_t* s, bool* own) {
  static const bool off = [] {
    const char* e = getenv("NEXR_RING_OWN_QUEUES");
    return e && e[0] == '0';
  }();
  *own = false;
  int dev = 0, cus = 0;
  if (c->cfg.memMode == nexrRingDeviceMemory && c->proto == nexrRingProtoLL && !off && hipGetDevice(&dev) == hipSuccess &&
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0) {
    std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
    if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
    if (hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data()) == hipSuccess) {
      *own = true;
      return hipSuccess;
    }
    (void)hipGetLastError();
  }
  return hipStreamCreate(s);
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
// runThreads calls throw, as std::thread does when the system is out of threads. Read once per call
// (tests set it between calls), never per thread.
static size_t spawnFailAt() {
  const char* e = getenv("NEXR_TEST_SPAWN_FAIL_AT");
  return e && *e ? (size_t)strtoull(e, nullptr, 10) : 0;
}

nexrResult_t runThreads(nexrRingComm* c, Shared& sh, const std::vector<std::function<void()>>& jobs) {
  std::vector<std::thread> threads;
  const size_t failAt = spawnFailAt();
  try {
    threads.reserve(jobs.size());
    for (const auto& j : jobs) {
      if (threads.size() + 1 == failAt)
        throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again), "spawn hook");
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
    // Zeroed, as NCCL clears its buffers: hipMalloc may hand back a freed FIFO of an earlier
    // communicator, whose LL lines carry flags (step + 1) the new one will wait for; a queued LL
    // consumer polls its slot before the producer writes it and must not accept such a stale line.
    // The receiver's head words for runs of LL steps (Conn::devHead) follow the FIFO, zeroed with it.
    if (hipSetDevice(device) != hipSuccess || hipMalloc((void**)&k->fifo, bytes + NEXR_LL_HEAD_BYTES) != hipSuccess ||
        hipMemset(k->fifo, 0, bytes + NEXR_LL_HEAD_BYTES) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
      return nexrUnhandledCudaError;
    k->devHead = (uint64_t*)(k->fifo + bytes);
  } else if (c->needHip && pinnedHostFifos()) {
    // Host memory with the MI355X doing the steps: pinned, device-mapped FIFOs, so that a step whose
    // user buffers are pinned too runs as one zero-copy kernel over PCIe (nexrReduceCopyHost) instead
    // of staging every slice through device memory. nexrHostMemAlloc records the FIFO in libnexr's
    // registration cache, so no step queries the runtime to classify it.
    nexrResult_t r = nexrHostMemAlloc((void**)&k->fifo, bytes);
    if (r != nexrSuccess) return r;
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
      bool own = false;
      if (hipSetDevice(c->devices[r]) != hipSuccess || createRankStream(c, &c->streams2[r], &own) != hipSuccess)
        return nexrUnhandledCudaError;
      c->ownQueues = c->ownQueues && own;
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
      (void)nexrHostMemFree(k->fifo);
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

// Queued LL steps (Prims::enableLLAsync) for thread ranks. LL only: an LL128 line carries one flag per
// 128 bytes (prims_ll128.h), and a consumer polling while its producer writes could see the flag's
// 16-B unit new and another unit of the line still old (only 16-B granules are untorn on this GPU;
// a queued LL128 ring failed the oracle this way), while LL's flag per 8-byte granule has no such
// window; ordering queued LL128 consumers behind producer events instead ran slower than host
// sequencing (0.26-0.28 against 0.22 ms for C1, profiles/r06g_ll_queue_probe.json), so LL128 stays
// host-sequenced. The kernels' progress does not depend on the hardware queues (Prims comment), but
// as a margin the rank streams of the device (all channels, the tree's second streams included) must
// fit in its hardware queues beside the default stream's: at most GPU_MAX_HW_QUEUES - 1 of them (HIP's
// default is 4 per device). Every rank on one GPU and FIFOs in device memory, as enableLLAsync
// requires. NEXR_LL_ASYNC=0 keeps host sequencing, =1 skips the queue count.
bool llAsyncAllowed(const nexrRingComm* c) {
  static const int forced = [] {
    const char* e = getenv("NEXR_LL_ASYNC");
    return e && *e ? (e[0] == '0' ? 0 : 1) : -1;
  }();
  static const long hwQueues = [] {
    const char* e = getenv("GPU_MAX_HW_QUEUES");
    const long v = e && *e ? strtol(e, nullptr, 10) : 4;
    return v > 0 ? v : 4;
  }();
  if (forced == 0 || c->proto != nexrRingProtoLL || !c->stepWaitWord || c->cfg.memMode != nexrRingDeviceMemory)
    return false;
  if (forced == 1) return true;
  std::vector<std::pair<int, int>> perDev;  // (device, rank streams on it)
  const int nCh = 1 + (int)c->channels.size();
  for (int k = 0; k < nCh; k++) {
    const nexrRingComm* ck = k == 0 ? c : c->channels[(size_t)k - 1];
    for (size_t r = 0; r < ck->streams.size(); r++) {
      const int streams = (ck->streams[r] ? 1 : 0) + (r < ck->streams2.size() && ck->streams2[r] ? 1 : 0);
      auto it = std::find_if(perDev.begin(), perDev.end(), [&](const std::pair<int, int>& x) { return x.first == ck->devices[r]; });
      if (it == perDev.end()) perDev.emplace_back(ck->devices[r], streams);
      else it->second += streams;
    }
  }
  for (const auto& d : perDev)
    if (d.second > hwQueues - 1) return false;
  return true;
}

// Runs of LL steps on the device (Prims::enableLLRun): where the queued mode may run (every rank's
// kernels can run at once on the one GPU), with the library's own LL kernels (not a caller's llFn).
// NEXR_LL_RUN=0 falls back to queued launches.
bool llRunAllowed(const nexrRingComm* c, bool llAsync) {
  static const bool off = [] {
    const char* e = getenv("NEXR_LL_RUN");
    return e && e[0] == '0';
  }();
  if (!llAsync || off || c->cfg.llFn != defaultLLFn || !c->ownQueues) return false;
  for (const nexrRingComm* ck : c->channels)
    if (!ck->ownQueues) return false;
  return true;
}

// Queued LL steps per completion ticket (Prims::flushTicket): NEXR_LL_TICKET_EVERY, default 4 (half the
// FIFO's 8 slots, so a sender always has credits for 4 more steps while the next ticket is pending).
int llTicketEvery() {
  static const int every = [] {
    const char* e = getenv("NEXR_LL_TICKET_EVERY");
    const long v = e && *e ? strtol(e, nullptr, 10) : 4;
    return (int)(v < 1 ? 1 : v > 64 ? 64 : v);
  }();
  return every;
}

// Thread-rank collectives: the ring schedules on one thread per rank.
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
  const bool llAsync = llAsyncAllowed(c);
  const bool llRun = llRunAllowed(c, llAsync);
  c->lastLLMode = llRun ? 2 : llAsync ? 1 : 0;
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
        if (llRun) p.enableLLRun();
        if (llAsync && !p.llRun) p.enableLLAsync(llTicketEvery());
        switch (coll) {
          case kAllReduce: runRingAllReduce(p, n, part); break;
          case kReduceScatter: runRingReduceScatter(p, n, (int64_t)count, part); break;
          case kAllGather: runRingAllGather(p, n, (int64_t)count, part); break;
          case kReduce: runRingReduce(p, n, root, part); break;
          case kBroadcast: runRingBroadcast(p, n, root, part); break;
        }
        p.finishLL();  // queued LL steps complete before the collective returns (even after a failure)
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

int stepWaitMode() {
  static const int mode = [] {
    const char* e = getenv("NEXR_STEP_WAIT");
    if (e && !strcmp(e, "word")) return 1;
    if (e && !strcmp(e, "sync")) return 0;
    return -1;
  }();
  return mode;
}

// A GPU's identity across processes: PCI domain / bus / device (+1, so that 0 means "not published").
uint64_t gpuIdentity(int device) {
  int dom = 0, bus = 0, dev = 0;
  if (hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess ||
      hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return (((uint64_t)(uint32_t)dom << 32) | ((uint64_t)(bus & 0xffff) << 16) | (uint64_t)(dev & 0xffff)) + 1;
}

bool envFlagOn(const char* name, bool dflt) {
  const char* v = getenv(name);
  return v && *v ? v[0] != '0' : dflt;
}

// Process ranks: the ring link r -> r+1 (rank r+1's receive FIFO) serves two users with separate
// step counters: the host-sequenced collectives (head/tail in the shared segment) and the resident
// all-reduce of the extras library (records behind the FIFO). Either returns once this rank's own
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

}  // namespace nexr_emu

extern "C" {


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
  // Ranks on one GPU hand steps over through the completion word; ranks spanning GPUs synchronise.
  c->stepWaitWord = stepWaitMode() >= 0 ? stepWaitMode() == 1
                                        : std::all_of(c->devices.begin(), c->devices.end(),
                                                      [&](int d) { return d == c->devices[0]; });
  for (int r = 0; r < n; r++) {
    c->conns.push_back(new Conn());
    if (nDev > 0) {
      bool own = false;
      if (hipSetDevice(c->devices[r]) != hipSuccess || createRankStream(c, &c->streams[r], &own) != hipSuccess ||
          allocDone(&c->done[r]) != nexrSuccess) {
        nexrRingCommDestroy(c);
        return nexrUnhandledCudaError;
      }
      c->ownQueues = c->ownQueues && own;
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

NEXR_API nexrResult_t nexrRingCommGetStepWait(nexrRingComm_t c, int* word) {
  if (!c || !word) return nexrInvalidArgument;
  *word = c->stepWaitWord ? 1 : 0;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrRingCommGetQueued(nexrRingComm_t c, int* queued) {
  if (!c || !queued) return nexrInvalidArgument;
  *queued = c->lastLLMode;
  return nexrSuccess;
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
  if (c->freeExtras) c->freeExtras(c);
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
    for (auto* v : {&c->p2pConns, &c->p2pLLConns})
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
      hipMemset(c->conns[me]->fifo, 0, allocBytes) != hipSuccess ||  // no stale LL lines (allocFifo)
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
  mine->gpu.store(gpuIdentity(cfg->device), std::memory_order_relaxed);
  c->conns[me]->st = &mine->conn;
  if (h->joined.fetch_add(1, std::memory_order_acq_rel) >= (uint32_t)n)  // publishes the handle
    return fail(nexrInvalidUsage);
  if (!waitFor([&] { return h->joined.load(std::memory_order_acquire) >= (uint32_t)n; })) return fail(nexrRemoteError);
  // The step wait (Prims::streamDone): the completion word only when every rank's GPU is this one (a
  // GPU whose identity could not be read counts as another GPU).
  const uint64_t myGpu = mine->gpu.load(std::memory_order_relaxed);
  bool oneGpu = myGpu != 0;
  for (int r = 0; r < n; r++) oneGpu = oneGpu && peerSlot(c->shm, r)->gpu.load(std::memory_order_relaxed) == myGpu;
  c->stepWaitWord = stepWaitMode() >= 0 ? stepWaitMode() == 1 : oneGpu;
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
