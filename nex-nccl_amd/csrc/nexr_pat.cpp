// nexr_pat.cpp — the PAT ReduceScatter / AllGather schedules (NCCL_ALGO_PAT) on the emulated
// communicator, thread ranks and process ranks (include/nexr_ring.h nexrPat*, nexrPeerPat*).
#include "nexr_emu.h"

namespace nexr_emu {

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

  // The channel's part is [offset_, end_) of the `count_` elements per rank (reduce_scatter.h:100,
  // all_gather.h:133: channelOffset, channelOffset + channelCount).
  PatReduceScatterPlan(int chunkCount_, size_t esz, int64_t offset_, int64_t end_, int64_t count_, int rank_, int nranks_)
      : PatGeometry((uint64_t)chunkCount_ * esz, kSteps, kPatMaxParallel, (uint64_t)(end_ - offset_), esz, nranks_),
        offset(offset_), end(end_), count(count_), chunkCount(chunkCount_), rank(rank_), nranks(nranks_) {
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

  // The channel's part is [offset_, end_) of the `count_` elements per rank (reduce_scatter.h:100,
  // all_gather.h:133: channelOffset, channelOffset + channelCount).
  PatAllGatherPlan(int chunkCount_, size_t esz, int64_t offset_, int64_t end_, int64_t count_, int rank_, int nranks_)
      : PatGeometry((uint64_t)chunkCount_ * esz, kSteps, kPatMaxParallel, (uint64_t)(end_ - offset_), esz, nranks_),
        offset(offset_), end(end_), count(count_), chunkCount(chunkCount_), rank(rank_), nranks(nranks_) {
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
    if (p.device && !p.streamDone()) {
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

  void run(const ChannelPart& part, int64_t count, int nranks) {
    const int chunkCount = (int)part.chunkCount;
    const int64_t lo = part.offset, hi = part.offset + part.count;
    int pf = 1;
    const std::vector<PatOp> ops =
        reduceScatter ? patOps(PatReduceScatterPlan(chunkCount, p.esz, lo, hi, count, p.rank, nranks), &pf)
                      : patOps(PatAllGatherPlan(chunkCount, p.esz, lo, hi, count, p.rank, nranks), &pf);
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
                size_t count, size_t esz, int datatype, const nexrDevRedOpFull& red, const ChannelPart& part) {
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
  pr.run(part, (int64_t)count, n);
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
  // split over the channels as any collective (ncclFuncTrafficPerByte = nRanks for both)
  std::vector<ChannelPart> parts = channelParts(c, (int64_t)count, esz, n);
  for (ChannelPart& part : parts) {
    nexrRingComm* ck = channelComm(c, part.channel);
    r = ensurePat(ck);
    if (r != nexrSuccess) {
      c->broken = true;
      return r;
    }
    part.chunkCount = patChunkElems(ck, esz, !reduceScatter, part.count);
  }
  Shared sh;
  std::vector<std::function<void()>> jobs;
  for (const ChannelPart& part : parts)
    for (int rank = 0; rank < n; rank++)
      jobs.emplace_back([&, rank, part] {
        runPatRank(channelComm(c, part.channel), &sh, rank, reduceScatter, sendbuffs[rank], recvbuffs[rank], count,
                   esz, datatype, red, part);
      });
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
      reduceScatter
          ? patOps(PatReduceScatterPlan((int)chunkCount, esz, 0, (int64_t)count, (int64_t)count, rank, nRanks),
                   parallelFactor)
          : patOps(PatAllGatherPlan((int)chunkCount, esz, 0, (int64_t)count, (int64_t)count, rank, nRanks),
                   parallelFactor);
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
  r = ringLinkHandover(c, false);  // PAT's r -> r+1 link is the ring's
  if (r != nexrSuccess) return r;
  Shared sh;
  sh.remoteAbort = &peerHeader(c->shm)->abort;
  const ChannelPart part{0, 0, (int64_t)count, patChunkElems(c, esz, !reduceScatter, (int64_t)count)};
  runPatRank(c, &sh, me, reduceScatter, sendbuff, recvbuff, count, esz, datatype, red, part);
  return peerFinish(c, sh);
}

}  // namespace nexr_emu

extern "C" {

NEXR_API nexrResult_t nexrPatReduceScatter(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                           size_t recvcount, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return patCollective(c, true, sendbuffs, recvbuffs, recvcount, datatype, op);
}

NEXR_API nexrResult_t nexrPatAllGather(nexrRingComm_t c, const void* const* sendbuffs, void* const* recvbuffs,
                                       size_t sendcount, int datatype) {
  DeviceGuard dg(c && c->needHip);
  return patCollective(c, false, sendbuffs, recvbuffs, sendcount, datatype, nexrSum);  // ncclAllGather: ncclSum
}
NEXR_API nexrResult_t nexrPatSchedule(int reduceScatter, int nRanks, int rank, size_t count, int datatype,
                                      size_t buffBytes, int64_t* ops, size_t capOps, size_t* nOps,
                                      int* parallelFactor) {
  const size_t esz = nexrTypeSize(datatype);
  if (esz == 0 || buffBytes % (kSteps * 16) != 0) return nexrInvalidArgument;
  return patSchedule(reduceScatter != 0, nRanks, rank, count, esz, (buffBytes ? buffBytes : kDefaultBuffBytes) / kSteps,
                     ops, capOps, nOps, parallelFactor);
}
NEXR_API nexrResult_t nexrPeerPatReduceScatter(nexrRingComm_t c, const void* sendbuff, void* recvbuff,
                                               size_t recvcount, int datatype, int op) {
  DeviceGuard dg(c && c->needHip);
  return peerPat(c, true, sendbuff, recvbuff, recvcount, datatype, op);
}

NEXR_API nexrResult_t nexrPeerPatAllGather(nexrRingComm_t c, const void* sendbuff, void* recvbuff, size_t sendcount,
                                           int datatype) {
  DeviceGuard dg(c && c->needHip);
  return peerPat(c, false, sendbuff, recvbuff, sendcount, datatype, nexrSum);
}

}  // extern "C"
