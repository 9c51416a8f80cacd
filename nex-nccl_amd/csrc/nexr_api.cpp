// nexr_api.cpp — the C ABI (include/nexr.h): argument validation, datatype/op dispatch, launch
// geometry, the host-staged variant and the op encoder. Host code only; the kernels live in
// nexr_kernels.hip (one object per datatype).
#include <hip/hip_runtime.h>
#include <string.h>
#include <stdlib.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <shared_mutex>
#include <thread>
#include <vector>

#include "nexr_internal.h"

namespace nexr {
namespace {

thread_local int tLastHipError = 0;

inline nexrResult_t hipFail(hipError_t e) {
  tLastHipError = (int)e;
  return nexrUnhandledCudaError;
}
#define NEXR_HIP(call)                          \
  do {                                          \
    hipError_t e_ = (call);                     \
    if (e_ != hipSuccess) return hipFail(e_);   \
  } while (0)

// ---- host-path counters (nexrGetHostPathStats): where a nexrReduceCopyHost call spends its time
std::atomic<uint64_t> gHpCalls{0}, gHpZeroCopy{0}, gHpRegHits{0}, gHpQueries{0};
std::atomic<uint64_t> gHpClassifyNs{0}, gHpCopyNs{0}, gHpLaunchNs{0}, gHpWaitNs{0};
inline uint64_t nowNs() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}


size_t typeSize(int dt) {
  switch (dt) {
    case nexrInt8: case nexrUint8: case nexrFloat8e4m3: case nexrFloat8e5m2: return 1;
    case nexrFloat16: case nexrBfloat16: return 2;
    case nexrInt32: case nexrUint32: case nexrFloat32: return 4;
    case nexrInt64: case nexrUint64: case nexrFloat64: return 8;
  }
  return 0;
}
bool isInteger(int dt) { return dt >= nexrInt8 && dt <= nexrUint64; }
bool isSignedInt(int dt) { return dt == nexrInt8 || dt == nexrInt32 || dt == nexrInt64; }

long envLong(const char* name, long dflt) {
  const char* v = getenv(name);
  if (!v || !*v) return dflt;
  return strtol(v, nullptr, 0);
}

// Reduction semantics (include/nexr.h, nexrSetSemantics): process-wide, like an NCCL parameter; the
// initial value comes from NEXR_SEMANTICS the first time a call needs it.
std::atomic<int> gSemantics{-1};

int semantics() {
  int s = gSemantics.load(std::memory_order_relaxed);
  if (s >= 0) return s;
  const char* v = getenv("NEXR_SEMANTICS");
  int init = nexrSemanticsNccl;
  if (v && (!strcmp(v, "fork") || !strcmp(v, "1"))) init = nexrSemanticsFork;
  if (v && (!strcmp(v, "shipped") || !strcmp(v, "2"))) init = nexrSemanticsShipped;
  gSemantics.compare_exchange_strong(s, init);
  return gSemantics.load(std::memory_order_relaxed);
}

// The fork's kernel dispatch (equivalent_primary, generate.py:128-136): signed Min/Max run on the
// unsigned kernel, whose FuncMinMax never applies the sign xormask hostToDevRedOp encodes.
int forkDispatchType(int dt, int op) {
  if (op != nexrDevMinMax) return dt;
  switch (dt) {
    case nexrInt8: return nexrUint8;
    case nexrInt32: return nexrUint32;
    case nexrInt64: return nexrUint64;
  }
  return dt;
}

// The parts of a validated SIMPLE call the semantics can change. Shipped (SKIP_COMP): every reduce
// returns acc = src0, the pre-op and post-op return their input — a K = 1 copy with no arithmetic.
struct CallShape {
  int dt, op, nSrcs, nPreOp, postOp;
  const void* prePtr;
};
void applySemantics(CallShape& c) {
  const int s = semantics();
  if (s == nexrSemanticsFork) {
    c.dt = forkDispatchType(c.dt, c.op);
  } else if (s == nexrSemanticsShipped) {
    c.op = nexrDevSum;
    c.nSrcs = 1;
    c.nPreOp = 0;
    c.postOp = 0;
    c.prePtr = nullptr;
  }
}

// The kernel a (semantics-shaped) call runs: kernel_compiled (nexr_internal.h) names the compiled
// ones; every other call maps onto one of them with the same output bytes. A K = 1 copy becomes a
// byte copy (*nElts counted in bytes from then on); signed Sum / Prod / PreMulSum / SumPostDiv run the
// unsigned kernel; PreMulSum without pre-op sources and SumPostDiv without the divide run Sum.
int unsignedOf(int dt) {
  return dt == nexrInt8 ? nexrUint8 : dt == nexrInt32 ? nexrUint32 : dt == nexrInt64 ? nexrUint64 : dt;
}
void routeKernel(CallShape& c, size_t* nElts) {
  if (c.op == nexrDevPreMulSum && c.nPreOp == 0) c.op = nexrDevSum;
  if (c.op == nexrDevSumPostDiv && !c.postOp) c.op = nexrDevSum;
  if (c.nSrcs == 1 && c.op != nexrDevPreMulSum && c.op != nexrDevSumPostDiv) {
    *nElts *= typeSize(c.dt);
    c.dt = nexrUint8;
    c.op = nexrDevSum;
    return;
  }
  if (c.op != nexrDevMinMax) c.dt = unsignedOf(c.dt);
}

// The same for an LL / LL128 step (after validation): shipped → every reduce returns its first operand,
// the peer (prims_ll.h:288-294, prims_ll128.h:225-255), with no pre-op and no post-op.
void llSemantics(int* dt, int* op, int* srcIsInput, int* postOp, int* firstWins) {
  const int s = semantics();
  *firstWins = 0;
  if (s == nexrSemanticsFork) {
    *dt = forkDispatchType(*dt, *op);
  } else if (s == nexrSemanticsShipped) {
    *op = nexrDevSum;
    *srcIsInput = 0;
    *postOp = 0;
    *firstWins = 1;
  }
}

// Cache policy by the bytes a call streams (every src read once, every dst written once): plain below
// NEXR_NT_LOAD_MIN_BYTES (64 MiB: the data likely sits in L2/MALL and the consumer wants the output
// there too), non-temporal loads above it, non-temporal loads and stores above
// NEXR_NT_STORE_MIN_BYTES (512 MiB = 2x the Infinity Cache). NEXR_POLICY (0/1/3) overrides it for
// sweeps. The workgroup geometry follows the policy (unroll_for/block_for, nexr_internal.h).
// One exception (round 5): calls with few sources take nt stores as well from
// NEXR_NT_STORE_K2_MIN_BYTES (96 MiB streamed), for the (K, M) measured to gain at 96-510 MiB
// (tools/occupancy_ab.hip ntstore / ntstore2 / ntstore3 / c4pol / ntstore4): K = 1 with M = 1-4
// (1.1-4.8 %), K = 2 with M = 1-7 (2.2-6.3 %; M = 7, round 6: 0.7-2.4 %), K = 3 with M = 2-7 (3.1-5.6 %;
// M = 6-7, round 6: 0-5.0 %, never slower) (profiles/r05q_occupancy_ntstore.txt,
// r05zd_occupancy_ntstore2.txt, r05zg_occupancy_ntstore3.txt, r05zj_occupancy_ntstore3_m5.txt,
// r06w_occupancy_ntstore4.txt). Outside it nt stores were mixed (K = 3 M = 1, K = 1 M = 5, K = 2 M = 8
// and K = 3 M = 8: 1.3-4.8 % slower at 110-120 MiB, 2.3-4.7 % faster at 290-300) or lost (K = 1 M = 8:
// 2.9-5.9 %, K = 4 M = 2, K = 8). nDsts = 0: unknown (a batch), the general rule.
constexpr int kNtStoreMinM[4] = {0, 1, 1, 2}, kNtStoreMaxM[4] = {0, 4, 7, 7};
int pickPolicy(uint64_t streamBytes, int nSrcs = 0, int nDsts = 0) {
  static const long polOverride = envLong("NEXR_POLICY", -1);
  static const long ntLoadMin = envLong("NEXR_NT_LOAD_MIN_BYTES", 64l << 20);
  static const long ntStoreMin = envLong("NEXR_NT_STORE_MIN_BYTES", 512l << 20);
  static const long ntStoreK2Min = envLong("NEXR_NT_STORE_K2_MIN_BYTES", 96l << 20);
  if (polOverride >= 0) return polOverride == 0 ? 0 : (polOverride == 1 ? 1 : 3);
  const bool fewSrcs = nSrcs >= 1 && nSrcs <= 3 && nDsts >= kNtStoreMinM[nSrcs] && nDsts <= kNtStoreMaxM[nSrcs];
  if (fewSrcs && streamBytes >= (uint64_t)ntStoreK2Min) return 3;
  return streamBytes >= (uint64_t)ntStoreMin ? 3 : (streamBytes >= (uint64_t)ntLoadMin ? 1 : 0);
}

// Grid: one workgroup per kTripPacks-pack trip ("one-shot"), capped so that grid x block stays
// within HIP's 2^32 - 1 work-item limit (2^24 workgroups of 256 lanes, 2^22 of 1024); beyond the
// cap the kernel grid-strides. NEXR_GRID overrides the grid for sweeps.
uint64_t gridCap(int block) { return 0xffffffffull / (uint64_t)block; }

nexrResult_t pickGeometry(uint64_t workgroups, int pol, int block, Geometry* g) {
  static const long gridOverride = envLong("NEXR_GRID", 0);
  const uint64_t cap = gridCap(block);
  uint64_t need = workgroups < 1 ? 1 : workgroups;
  g->grid = (int)(need < cap ? need : cap);
  if (gridOverride > 0) g->grid = (int)gridOverride;
  g->pol = pol;
  return nexrSuccess;
}

hipError_t launchDt(int dt, const RCParams& p, int op, int nSrcs, const Geometry& g, hipStream_t s) {
  switch (dt) {
    case 0: return launch_dt0(p, op, nSrcs, g, s);
    case 1: return launch_dt1(p, op, nSrcs, g, s);
    case 2: return launch_dt2(p, op, nSrcs, g, s);
    case 3: return launch_dt3(p, op, nSrcs, g, s);
    case 4: return launch_dt4(p, op, nSrcs, g, s);
    case 5: return launch_dt5(p, op, nSrcs, g, s);
    case 6: return launch_dt6(p, op, nSrcs, g, s);
    case 7: return launch_dt7(p, op, nSrcs, g, s);
    case 8: return launch_dt8(p, op, nSrcs, g, s);
    case 9: return launch_dt9(p, op, nSrcs, g, s);
  }
  return hipErrorInvalidValue;
}

// Shared validation for every reduce-copy entry point (error convention: SURVEY §8(b)).
nexrResult_t validate(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                      int datatype, int op, uint64_t redOpArg, int nPreOpSrcs, const uint64_t* preOpArgs) {
  if (nSrcs < 1 || nSrcs > NEXR_MAX_SRCS) return nexrInvalidArgument;
  if (nDsts < 0 || nDsts > NEXR_MAX_DSTS) return nexrInvalidArgument;
  if (datatype < 0 || datatype >= nexrNumTypes) return nexrInvalidArgument;
  if (datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2) return nexrInvalidArgument;
  if (op < 0 || op >= nexrNumDevRedOps) return nexrInvalidArgument;
  // SumPostDiv kernels exist for integer types only (generate.py:108 required_cuda).
  if (op == nexrDevSumPostDiv && !isInteger(datatype)) return nexrInvalidArgument;
  if (op == nexrDevSumPostDiv && isSignedInt(datatype)) {
    // The signed quotient divides by the divisor truncated to T (reduce_kernel.h:94): a
    // divisor that truncates to 0 would divide by zero.
    uint32_t divisor = (uint32_t)(redOpArg >> 1);
    if (divisor == 0) divisor = 1;
    size_t sz = typeSize(datatype);
    if (sz == 1 && (int8_t)divisor == 0) return nexrInvalidArgument;
  }
  if (nPreOpSrcs < 0 || nPreOpSrcs > nSrcs) return nexrInvalidArgument;
  if (nPreOpSrcs > 0 && preOpArgs == nullptr) return nexrInvalidArgument;
  if (nElts == 0 || nDsts == 0) return nexrSuccess;
  if (srcs == nullptr || (nDsts > 0 && dsts == nullptr)) return nexrInvalidArgument;
  for (int s = 0; s < nSrcs; s++)
    if (srcs[s] == nullptr) return nexrInvalidArgument;
  for (int d = 0; d < nDsts; d++)
    if (dsts[d] == nullptr) return nexrInvalidArgument;
  return nexrSuccess;
}

// Split [0, nElts) into head edge / packed body / tail edge (RCParams comment). Pack i of the body
// is the 16 contiguous bytes at offset 16 i of every buffer, at that buffer's own alignment: when all
// pointers share a 16-B phase every access is aligned; otherwise the misaligned ones are unaligned
// 16-B loads / stores (one instruction per lane on gfx950, no element-by-element path). The head
// brings the first destination to a 128-B boundary when its offset is a whole number of elements, so
// that each wave's 1 KiB store instruction writes whole 128-B lines: misaligned stores cost more than
// misaligned loads (tools/misalign_rate.py).
constexpr uintptr_t kLineBytes = 128;
void planLayout(RCParams& p, int nSrcs, size_t esz) {
  const uintptr_t phase16 = (uintptr_t)p.src[0] & 15;
  bool common = (phase16 % esz) == 0;
  for (int s = 1; s < nSrcs && common; s++) common = (((uintptr_t)p.src[s]) & 15) == phase16;
  for (int d = 0; d < p.nDsts && common; d++) common = (((uintptr_t)p.dst[d]) & 15) == phase16;
  p.unaligned = common ? 0 : 1;
  uintptr_t phase = (uintptr_t)p.dst[0] & (kLineBytes - 1);
  if (phase % esz) phase = 0;
  uint64_t head = phase ? (kLineBytes - phase) / esz : 0;
  if (head > p.nElts) head = p.nElts;
  p.head = head;
  p.nPacks = (p.nElts - head) * esz / 16;
}

void fillParams(RCParams& p, int nSrcs, const void* const* srcs, int nDsts, void* const* dsts, size_t nElts,
                size_t esz, uint64_t redOpArg, int nPreOpSrcs, const uint64_t* preOpArgs, const void* prePtr,
                int postOp) {
  memset(&p, 0, sizeof(p));
  for (int s = 0; s < nSrcs; s++) p.src[s] = (const char*)srcs[s];
  for (int d = 0; d < nDsts; d++) p.dst[d] = (char*)dsts[d];
  for (int s = 0; s < nPreOpSrcs; s++) p.pre[s] = preOpArgs[s];
  p.prePtr = prePtr;
  p.redArg = redOpArg;
  p.nElts = nElts;
  p.nDsts = nDsts;
  p.nPreOp = nPreOpSrcs;
  p.postOp = postOp ? 1 : 0;
  planLayout(p, nSrcs, esz);
}

// One-shot workgroups of one reduce-copy: one per B lane work items, a work item being a U-pack
// group, with (U, B) = the kernel's geometry for (dt, K, policy).
uint64_t workgroupsFor(const RCParams& p, int nSrcs, int dt, int pol) {
  const uint64_t u = (uint64_t)unroll_for(dt, nSrcs, pol), b = (uint64_t)block_for(dt, nSrcs, pol);
  const uint64_t items = (p.nPacks + u - 1) / u;  // >= 1 workgroup (pickGeometry) covers the edges
  return (items + b - 1) / b;
}

hipError_t launchBatchDt(int dt, const BatchParams& b, int op, int nSrcs, int pol, int grid, hipStream_t s) {
  switch (dt) {
    case 0: return launch_batch_dt0(b, op, nSrcs, pol, grid, s);
    case 1: return launch_batch_dt1(b, op, nSrcs, pol, grid, s);
    case 2: return launch_batch_dt2(b, op, nSrcs, pol, grid, s);
    case 3: return launch_batch_dt3(b, op, nSrcs, pol, grid, s);
    case 4: return launch_batch_dt4(b, op, nSrcs, pol, grid, s);
    case 5: return launch_batch_dt5(b, op, nSrcs, pol, grid, s);
    case 6: return launch_batch_dt6(b, op, nSrcs, pol, grid, s);
    case 7: return launch_batch_dt7(b, op, nSrcs, pol, grid, s);
    case 8: return launch_batch_dt8(b, op, nSrcs, pol, grid, s);
    case 9: return launch_batch_dt9(b, op, nSrcs, pol, grid, s);
  }
  return hipErrorInvalidValue;
}

nexrResult_t launchSingle(const RCParams& p, int dt, int op, int nSrcs, hipStream_t stream, uint64_t maxGrid);

// One batch launch per run of <= kMaxBatch works that run the same kernel: the works as the semantics
// and the kernel routing (routeKernel) run them, grouped by (datatype, op, K, and for MinMax isMin),
// each group in order of first appearance. Work i gets max(1, workgroupsFor(work i)) workgroups (its
// one-shot grid), total capped at gridCap(block) by shrinking the largest shares (the kernel
// grid-strides inside each work's range). A run that would stream enough for non-temporal stores runs
// its works as single launches instead (kBatchPolicies, nexr_internal.h).
nexrResult_t reduceCopyBatch(const nexrReduceCopyWork* works, int nWorks, int datatype, int op, hipStream_t stream) {
  if (nWorks < 0 || (nWorks > 0 && works == nullptr)) return nexrInvalidArgument;
  for (int i = 0; i < nWorks; i++) {
    const nexrReduceCopyWork& w = works[i];
    nexrResult_t r = validate(w.nSrcs, w.srcs, w.nDsts, w.dsts, w.nElts, datatype, op, w.redOpArg, w.nPreOpSrcs,
                              w.preOpArgs);
    if (r != nexrSuccess) return r;
  }
  struct Routed {
    CallShape c;
    int minClass;  // MinMax: 1 = min ((redOpArg & 1) == 0), 0 = max
    size_t nElts;
    const nexrReduceCopyWork* w;
  };
  std::vector<Routed> rw;
  rw.reserve((size_t)nWorks);
  for (int i = 0; i < nWorks; i++) {
    const nexrReduceCopyWork& w = works[i];
    if (w.nElts == 0 || w.nDsts == 0) continue;
    Routed x{{datatype, op, w.nSrcs, w.nPreOpSrcs, w.postOp, nullptr}, 0, w.nElts, &w};
    applySemantics(x.c);
    routeKernel(x.c, &x.nElts);
    x.minClass = x.c.op == nexrDevMinMax && (w.redOpArg & 1) == 0 ? 1 : 0;
    rw.push_back(x);
  }
  std::vector<char> taken(rw.size(), 0);
  for (size_t i0 = 0; i0 < rw.size(); i0++) {
    if (taken[i0]) continue;
    const CallShape key = rw[i0].c;
    const int keyMin = rw[i0].minClass, k = key.nSrcs;
    const size_t esz = typeSize(key.dt);
    BatchParams b;
    b.nWorks = 0;
    uint64_t blocks[kMaxBatch];
    uint64_t streamBytes = 0;
    auto flush = [&]() -> nexrResult_t {
      if (b.nWorks == 0) return nexrSuccess;
      const int pol = pickPolicy(streamBytes);
      if (pol >= kBatchPolicies) {  // non-temporal stores: one launch per work, each at its own policy
        for (int i = 0; i < b.nWorks; i++) {
          nexrResult_t r = launchSingle(b.w[i], key.dt, key.op, k, stream, 0);
          if (r != nexrSuccess) return r;
        }
        b.nWorks = 0;
        streamBytes = 0;
        return nexrSuccess;
      }
      const int block = block_for(key.dt, k, pol);
      const uint64_t cap = gridCap(block);
      uint64_t total = 0;
      for (int i = 0; i < b.nWorks; i++) {
        const uint64_t need = workgroupsFor(b.w[i], k, key.dt, pol);
        blocks[i] = need < 1 ? 1 : (need < cap ? need : cap);
        total += blocks[i];
      }
      while (total > cap) {
        int big = 0;
        for (int i = 1; i < b.nWorks; i++)
          if (blocks[i] > blocks[big]) big = i;
        uint64_t cut = blocks[big] / 2;
        blocks[big] -= cut;
        total -= cut;
      }
      b.start[0] = 0;
      for (int i = 0; i < b.nWorks; i++) b.start[i + 1] = b.start[i] + (uint32_t)blocks[i];
      Geometry g;
      nexrResult_t r = pickGeometry(total, pol, block, &g);
      if (r != nexrSuccess) return r;
      NEXR_HIP(launchBatchDt(key.dt, b, key.op, k, g.pol, (int)total, stream));
      b.nWorks = 0;
      streamBytes = 0;
      return nexrSuccess;
    };
    for (size_t i = i0; i < rw.size(); i++) {
      const Routed& x = rw[i];
      if (taken[i] || x.c.dt != key.dt || x.c.op != key.op || x.c.nSrcs != k || x.minClass != keyMin) continue;
      taken[i] = 1;
      const nexrReduceCopyWork& w = *x.w;
      fillParams(b.w[b.nWorks], k, w.srcs, w.nDsts, w.dsts, x.nElts, esz, w.redOpArg, x.c.nPreOp, w.preOpArgs, nullptr,
                 x.c.postOp);
      streamBytes += (uint64_t)(k + w.nDsts) * x.nElts * esz;
      if (++b.nWorks == kMaxBatch) {
        nexrResult_t r = flush();
        if (r != nexrSuccess) return r;
      }
    }
    nexrResult_t r = flush();
    if (r != nexrSuccess) return r;
  }
  return nexrSuccess;
}

// One launch of a routed call whose parameters are filled: policy by the bytes it streams, one-shot grid
// (capped at maxGrid when > 0).
nexrResult_t launchSingle(const RCParams& p, int dt, int op, int nSrcs, hipStream_t stream, uint64_t maxGrid) {
  const uint64_t esz = (uint64_t)typeSize(dt);
  const int pol = pickPolicy((uint64_t)(nSrcs + p.nDsts) * p.nElts * esz, nSrcs, p.nDsts);
  uint64_t wgs = workgroupsFor(p, nSrcs, dt, pol);
  if (maxGrid > 0 && wgs > maxGrid) wgs = maxGrid;
  Geometry g;
  nexrResult_t r = pickGeometry(wgs, pol, block_for(dt, nSrcs, pol), &g);
  if (r != nexrSuccess) return r;
  NEXR_HIP(launchDt(dt, p, op, nSrcs, g, stream));
  return nexrSuccess;
}

// maxGrid > 0 caps the grid (the kernel grid-strides): launches that read or write host memory over
// PCIe use hostGrid() workgroups. With a one-shot grid every workgroup's loads are interleaved over the
// whole transfer, so every workgroup's last load lands near its end and the writes start only then;
// 32 workgroups keep ~1 MiB of reads in flight (more than the link's bandwidth x latency) and let the
// early workgroups write while the others still read: +4-9 % at 1 MiB, +10-20 % at 4 MiB and +6-12 % at
// 64 MiB per buffer over the one-shot grid (tools/zero_copy_sizes.py, profiles/r05f_zero_copy_grid.txt).
uint64_t hostGrid() {
  static const long g = envLong("NEXR_HOST_GRID", 32);
  return g > 0 ? (uint64_t)g : 0;
}

nexrResult_t reduceCopyDevice(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                              size_t nElts, int datatype, int op, uint64_t redOpArg, int nPreOpSrcs,
                              const uint64_t* preOpArgs, const void* prePtr, int postOp, hipStream_t stream,
                              uint64_t maxGrid = 0) {
  nexrResult_t r = validate(nSrcs, srcs, nDsts, dsts, nElts, datatype, op, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != nexrSuccess) return r;
  if (nElts == 0 || nDsts == 0) return nexrSuccess;  // common_kernel.h:288-289: nothing to store
  CallShape c{datatype, op, nSrcs, nPreOpSrcs, postOp, prePtr};
  applySemantics(c);
  size_t n = nElts;
  routeKernel(c, &n);
  const size_t esz = typeSize(c.dt);
  RCParams p;
  fillParams(p, c.nSrcs, srcs, nDsts, dsts, n, esz, redOpArg, c.nPreOp, preOpArgs, c.prePtr, c.postOp);
  return launchSingle(p, c.dt, c.op, c.nSrcs, stream, maxGrid);
}

// ---- independent chunks on several GPUs from one host call -------------------
// One host thread per work: hipSetDevice, a stream of its own, the shared start barrier, `reps`
// launches, hipStreamSynchronize. A thread whose setup fails still arrives at the barrier (so the
// others are released) and reports its error.
// Streams come from a process-wide per-device pool: a stream is checked out for one work of one
// call and handed back drained. (A fresh stream per call cost ~1.5 ms on its first launches, which
// dominated calls of tens of MiB; profiles/r01s5_c_examples_gpu.txt.)
std::mutex gMdStreamMu;
std::vector<std::pair<int, hipStream_t>> gMdStreamIdle;
uint64_t gMdStreamsCreated = 0;  // under gMdStreamMu (nexrGetPoolStats)

hipError_t mdStreamTake(int dev, hipStream_t* st) {
  {
    std::lock_guard<std::mutex> g(gMdStreamMu);
    for (size_t i = 0; i < gMdStreamIdle.size(); i++)
      if (gMdStreamIdle[i].first == dev) {
        *st = gMdStreamIdle[i].second;
        gMdStreamIdle.erase(gMdStreamIdle.begin() + (long)i);
        return hipSuccess;
      }
  }
  hipError_t e = hipStreamCreateWithFlags(st, hipStreamNonBlocking);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> g(gMdStreamMu);
    gMdStreamsCreated++;
  }
  return e;
}

void mdStreamGive(int dev, hipStream_t st) {  // st was synchronised without error
  std::lock_guard<std::mutex> g(gMdStreamMu);
  gMdStreamIdle.emplace_back(dev, st);
}
// nSets works per thread (works[i * nSets + s], all on devices[i]): launch k of thread i runs set
// k mod nSets, the rotation the N = 1 bench uses so no launch re-reads cache-resident bytes.
nexrResult_t reduceCopyMultiDevice(const nexrReduceCopyWork* works, const int* devices, int nWorks, int nSets,
                                   int datatype, int op, int reps, double* seconds) {
  if (nWorks < 0 || nWorks > NEXR_MAX_MULTI_DEVICE_WORKS || reps < 1) return nexrInvalidArgument;
  if (nSets < 1 || nSets > NEXR_MAX_MULTI_DEVICE_SETS) return nexrInvalidArgument;
  if (nWorks > 0 && (works == nullptr || devices == nullptr)) return nexrInvalidArgument;
  for (int i = 0; i < nWorks * nSets; i++) {
    const nexrReduceCopyWork& w = works[i];
    nexrResult_t r = validate(w.nSrcs, w.srcs, w.nDsts, w.dsts, w.nElts, datatype, op, w.redOpArg, w.nPreOpSrcs,
                              w.preOpArgs);
    if (r != nexrSuccess) return r;
  }
  if (seconds) *seconds = 0.0;
  if (nWorks == 0) return nexrSuccess;
  int nDev = 0;
  NEXR_HIP(hipGetDeviceCount(&nDev));
  for (int i = 0; i < nWorks; i++)
    if (devices[i] < 0 || devices[i] >= nDev) return nexrInvalidArgument;

  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  std::chrono::steady_clock::time_point t0;
  std::vector<std::chrono::steady_clock::time_point> t1(nWorks);
  std::vector<nexrResult_t> res(nWorks, nexrSuccess);
  std::vector<int> hipErr(nWorks, 0);
  bool cancel = false;  // set (under mu) when not every work got a thread: nothing runs
  auto run = [&](int i) {
    hipStream_t st = nullptr;
    hipError_t e = hipSetDevice(devices[i]);
    if (e == hipSuccess) e = mdStreamTake(devices[i], &st);
    if (e != hipSuccess) {
      res[i] = nexrUnhandledCudaError;
      hipErr[i] = (int)e;
    }
    {
      std::unique_lock<std::mutex> lk(mu);
      if (++arrived == nWorks) {
        t0 = std::chrono::steady_clock::now();
        cv.notify_all();
      } else {
        cv.wait(lk, [&] { return arrived == nWorks; });
      }
      if (cancel && res[i] == nexrSuccess) res[i] = nexrSystemError;
    }
    for (int k = 0; k < reps && res[i] == nexrSuccess; k++) {
      const nexrReduceCopyWork& w = works[(size_t)i * nSets + k % nSets];
      res[i] = reduceCopyDevice(w.nSrcs, w.srcs, w.nDsts, w.dsts, w.nElts, datatype, op, w.redOpArg, w.nPreOpSrcs,
                                w.preOpArgs, nullptr, w.postOp, st);
    }
    if (res[i] == nexrUnhandledCudaError && hipErr[i] == 0) hipErr[i] = tLastHipError;
    if (st) {
      e = hipStreamSynchronize(st);
      t1[i] = std::chrono::steady_clock::now();
      if (e != hipSuccess && res[i] == nexrSuccess) {
        res[i] = nexrUnhandledCudaError;
        hipErr[i] = (int)e;
      }
      if (e == hipSuccess) mdStreamGive(devices[i], st);
      else (void)hipStreamDestroy(st);
    } else {
      t1[i] = std::chrono::steady_clock::now();
    }
  };
  std::vector<std::thread> threads;
  bool spawnFailed = false;
  try {
    threads.reserve(nWorks);
    for (int i = 0; i < nWorks; i++) threads.emplace_back(run, i);
  } catch (...) {
    // A thread could not be created: the works that never got one count as arrived (so the started
    // threads leave the barrier), but none of them may run, and the call reports a system error.
    std::lock_guard<std::mutex> lk(mu);
    spawnFailed = true;
    cancel = true;
    for (int i = (int)threads.size(); i < nWorks; i++) res[i] = nexrSystemError;
    arrived += nWorks - (int)threads.size();
    if (arrived == nWorks) t0 = std::chrono::steady_clock::now();
    cv.notify_all();
  }
  for (auto& t : threads) t.join();
  if (spawnFailed) return nexrSystemError;
  for (int i = 0; i < nWorks; i++)
    if (res[i] != nexrSuccess) {
      tLastHipError = hipErr[i];
      return res[i];
    }
  if (seconds) {
    auto last = t1[0];
    for (int i = 1; i < nWorks; i++) last = t1[i] > last ? t1[i] : last;
    *seconds = std::chrono::duration<double>(last - t0).count();
  }
  return nexrSuccess;
}

// ---- host-staged variant: a process-wide pool of staging rings ----------------------------------
// A ring is two device slots of (K+1) x chunk bytes: chunk c is copied in (H2D) and reduced on the
// caller's stream while chunk c-1 is copied out (D2H) on the ring's own stream, so the two PCIe
// directions run concurrently. A call checks a ring out for its duration and hands it back, so the
// pool holds, per device, as many rings as host calls have ever run there at once. (The emulated
// collectives run each call's ranks on fresh threads: a ring cached per thread would be a new device
// allocation and stream per thread, never freed.)
struct HostStage {
  int device = -1;
  char* buf = nullptr;
  size_t slotBytes = 0;  // bytes per slot
  hipStream_t out = nullptr;
  hipEvent_t kernelDone[2] = {nullptr, nullptr};
  hipEvent_t outDone[2] = {nullptr, nullptr};
};
std::mutex gStageMu;
std::vector<HostStage*> gStageIdle;
uint64_t gStagesCreated = 0;  // under gStageMu (nexrGetPoolStats)

// Checks a ring out for the current device (the largest idle one, or a new one) and hands it back
// when the call ends. Release drains the ring's stream and the caller's stream first, so that no
// copy of this call still targets the slots when another call takes the ring; a ring whose streams
// report an error is dropped rather than reused.
struct StageLease {
  HostStage* st = nullptr;
  hipStream_t caller = nullptr;
  ~StageLease() {
    if (!st) return;
    bool ok = hipStreamSynchronize(st->out) == hipSuccess;
    ok = hipStreamSynchronize(caller) == hipSuccess && ok;
    if (!ok) {
      (void)hipGetLastError();
      return;
    }
    std::lock_guard<std::mutex> g(gStageMu);
    gStageIdle.push_back(st);
  }
};

nexrResult_t stageFor(size_t slotBytes, hipStream_t caller, StageLease* lease) {
  int dev = 0;
  NEXR_HIP(hipGetDevice(&dev));
  HostStage* st = nullptr;
  {
    std::lock_guard<std::mutex> g(gStageMu);
    size_t best = gStageIdle.size();
    for (size_t i = 0; i < gStageIdle.size(); i++)
      if (gStageIdle[i]->device == dev && (best == gStageIdle.size() || gStageIdle[i]->slotBytes > gStageIdle[best]->slotBytes))
        best = i;
    if (best < gStageIdle.size()) {
      st = gStageIdle[best];
      gStageIdle.erase(gStageIdle.begin() + (long)best);
    }
  }
  if (!st) {
    st = new HostStage();
    hipError_t e = hipStreamCreateWithFlags(&st->out, hipStreamNonBlocking);
    for (int i = 0; i < 2 && e == hipSuccess; i++) {
      e = hipEventCreateWithFlags(&st->kernelDone[i], hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&st->outDone[i], hipEventDisableTiming);
    }
    if (e != hipSuccess) {  // free the half-built ring; it is never pooled
      for (int i = 0; i < 2; i++) {
        if (st->kernelDone[i]) (void)hipEventDestroy(st->kernelDone[i]);
        if (st->outDone[i]) (void)hipEventDestroy(st->outDone[i]);
      }
      if (st->out) (void)hipStreamDestroy(st->out);
      delete st;
      return hipFail(e);
    }
    st->device = dev;
    std::lock_guard<std::mutex> g(gStageMu);
    gStagesCreated++;
  }
  lease->st = st;
  lease->caller = caller;
  if (st->slotBytes < slotBytes) {  // idle ring: its stream was drained when it was handed back
    if (st->buf) NEXR_HIP(hipFree(st->buf));
    st->buf = nullptr;
    st->slotBytes = 0;
    NEXR_HIP(hipMalloc((void**)&st->buf, 2 * slotBytes));
    st->slotBytes = slotBytes;
  }
  return nexrSuccess;
}

// ---- host-staged variant, large pageable calls: a CPU copy team and pinned zero-copy slots -------
// The runtime's pageable hipMemcpyAsync copies through its own staging buffer with one CPU memcpy
// before each DMA, which held the C2 mix to 49 GB/s against an ~86 GB/s PCIe floor
// (profiles/r01_h2d_probe.log). For a call with at least NEXR_HOST_MT_MIN_BYTES of pageable
// buffers: a team of host threads copies each chunk of the pageable sources into a pinned,
// device-mapped slot; the kernel reads the slot and writes its output slot in place over PCIe
// (zero-copy, both link directions at once; pinned user buffers are read/written in place as
// well); the team copies the output slot to the pageable destinations. Three slots: chunk c is
// filled while chunk c-1 is reduced and chunk c-2 is drained.
constexpr int kPinnedSlots = 3;
struct PinnedStage {
  int device = -1;
  char* host = nullptr;  // hipHostMalloc (pinned, mapped, coherent): kPinnedSlots x slotBytes
  char* dev = nullptr;   // the same bytes as the device addresses them
  size_t slotBytes = 0;
  hipEvent_t done[kPinnedSlots] = {};
};
std::mutex gPinMu;
std::vector<PinnedStage*> gPinIdle;
uint64_t gPinCreated = 0;  // under gPinMu (nexrGetPoolStats)

// Checks a pinned ring out for the current device; the lease drains the caller's stream (every
// kernel this call queued, even one whose completion event could not be recorded) and every slot's
// event before handing the ring back; a ring that reports an error is dropped, not reused.
struct PinLease {
  PinnedStage* st = nullptr;
  hipStream_t caller = nullptr;
  ~PinLease() {
    if (!st) return;
    bool ok = hipStreamSynchronize(caller) == hipSuccess;
    for (int i = 0; i < kPinnedSlots; i++) ok = hipEventSynchronize(st->done[i]) == hipSuccess && ok;
    if (!ok) {
      (void)hipGetLastError();
      return;
    }
    std::lock_guard<std::mutex> g(gPinMu);
    gPinIdle.push_back(st);
  }
};

nexrResult_t pinnedFor(size_t slotBytes, hipStream_t caller, PinLease* lease) {
  int dev = 0;
  NEXR_HIP(hipGetDevice(&dev));
  PinnedStage* st = nullptr;
  {
    std::lock_guard<std::mutex> g(gPinMu);
    for (size_t i = 0; i < gPinIdle.size(); i++)
      if (gPinIdle[i]->device == dev && (!st || gPinIdle[i]->slotBytes > st->slotBytes)) st = gPinIdle[i];
    if (st) gPinIdle.erase(std::find(gPinIdle.begin(), gPinIdle.end(), st));
  }
  if (!st) {
    st = new PinnedStage();
    hipError_t e = hipSuccess;
    for (int i = 0; i < kPinnedSlots && e == hipSuccess; i++)
      e = hipEventCreateWithFlags(&st->done[i], hipEventDisableTiming);
    if (e == hipSuccess) {  // the events start "complete": record each once on the null stream
      for (int i = 0; i < kPinnedSlots && e == hipSuccess; i++) e = hipEventRecord(st->done[i], nullptr);
    }
    if (e != hipSuccess) {
      for (int i = 0; i < kPinnedSlots; i++)
        if (st->done[i]) (void)hipEventDestroy(st->done[i]);
      delete st;
      return hipFail(e);
    }
    st->device = dev;
    std::lock_guard<std::mutex> g(gPinMu);
    gPinCreated++;
  }
  lease->st = st;
  lease->caller = caller;
  if (st->slotBytes < slotBytes) {  // idle ring: its events were synchronised when it was handed back
    if (st->host) NEXR_HIP(hipHostFree(st->host));
    st->host = st->dev = nullptr;
    st->slotBytes = 0;
    NEXR_HIP(hipHostMalloc((void**)&st->host, kPinnedSlots * slotBytes, hipHostMallocDefault));
    NEXR_HIP(hipHostGetDevicePointer((void**)&st->dev, st->host, 0));
    st->slotBytes = slotBytes;
  }
  return nexrSuccess;
}

// Parallel memcpy: `run` splits every task into one contiguous, 4 KiB-aligned piece per thread and
// returns when all pieces are copied. The calling thread copies a piece too; the others are
// created for one host call and joined when it ends.
class CopyTeam {
 public:
  struct Task {
    char* dst;
    const char* src;
    size_t bytes;
  };
  explicit CopyTeam(int n) {
    for (int i = 1; i < n; i++) {
      try {
        workers_.emplace_back([this, i] { loop(i); });
      } catch (...) {  // fewer threads than asked for: the pieces are re-split over those that exist
        break;
      }
    }
    n_ = 1 + (int)workers_.size();
  }
  ~CopyTeam() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  void run(const Task* tasks, int nTasks) {
    {
      std::lock_guard<std::mutex> g(mu_);
      tasks_ = tasks;
      nTasks_ = nTasks;
      pending_ = n_ - 1;
      gen_++;
    }
    cv_.notify_all();
    piece(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void piece(int idx) const {
    for (int t = 0; t < nTasks_; t++) {
      const Task& k = tasks_[t];
      const size_t per = ((k.bytes + n_ - 1) / n_ + 4095) & ~(size_t)4095;
      const size_t b0 = per * (size_t)idx;
      if (b0 >= k.bytes) continue;
      memcpy(k.dst + b0, k.src + b0, per < k.bytes - b0 ? per : k.bytes - b0);
    }
  }
  void loop(int idx) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      piece(idx);
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> workers_;
  int n_ = 1;
  std::mutex mu_;
  std::condition_variable cv_, done_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  const Task* tasks_ = nullptr;
  int nTasks_ = 0;
};

// srcs/dsts: the caller's host pointers; psrc/pdst: which are pinned (zsrc/zdst: their device
// addresses, used in place).
nexrResult_t reduceCopyHostTeam(int nSrcs, const void* const* srcs, const bool* psrc, const void* const* zsrc,
                                int nDsts, void* const* dsts, const bool* pdst, void* const* zdst, size_t nElts,
                                int datatype, int op, uint64_t redOpArg, int nPreOpSrcs, const uint64_t* preOpArgs,
                                int postOp, hipStream_t s, int nThreads) {
  const size_t esz = typeSize(datatype);
  // A team's chunk is an eighth of a buffer, between 4 MiB and NEXR_HOST_MT_CHUNK_BYTES (32 MiB), so
  // that a call runs at least 8 chunks through the 3 slots; alone, NEXR_HOST_SMALL_CHUNK_BYTES (4 MiB).
  static const long chunkTeam = envLong("NEXR_HOST_MT_CHUNK_BYTES", 32l << 20);
  static const long chunkSolo = envLong("NEXR_HOST_SMALL_CHUNK_BYTES", 4l << 20);
  long chunkOverride = chunkSolo;
  if (nThreads > 1) {
    const long eighth = (long)(nElts * esz / 8);
    chunkOverride = eighth < (4l << 20) ? (4l << 20) : eighth;
    if (chunkOverride > chunkTeam) chunkOverride = chunkTeam;
  }
  size_t chunkElts = ((size_t)(chunkOverride > 4096 ? chunkOverride : 4096) / esz) & ~(size_t)15;
  if (chunkElts > nElts) chunkElts = nElts;
  const size_t chunkBytes = ((chunkElts * esz) + 4095) & ~(size_t)4095;
  int nPageSrc = 0;
  bool outStaged = false;
  for (int k = 0; k < nSrcs; k++) nPageSrc += psrc[k] ? 0 : 1;
  for (int d = 0; d < nDsts; d++) outStaged |= !pdst[d];
  PinLease lease;
  nexrResult_t r = pinnedFor(chunkBytes * (size_t)(nPageSrc + (outStaged ? 1 : 0)), s, &lease);
  if (r != nexrSuccess) return r;
  PinnedStage* st = lease.st;
  CopyTeam team(nThreads);
  const size_t nChunks = (nElts + chunkElts - 1) / chunkElts;
  auto span = [&](size_t c, size_t* e0, size_t* n) {
    *e0 = c * chunkElts;
    *n = nElts - *e0 < chunkElts ? nElts - *e0 : chunkElts;
  };
  auto outOffset = [&] { return chunkBytes * (size_t)nPageSrc; };
  // Copy-in tasks of chunk c (its pageable sources into slot c % 3) and copy-out tasks of chunk c
  // (slot c % 3's output to the pageable destinations), appended to `tasks`.
  CopyTeam::Task tasks[NEXR_MAX_SRCS + NEXR_MAX_DSTS];
  int nTasks = 0;
  auto copyIn = [&](size_t c) {
    size_t e0, n;
    span(c, &e0, &n);
    const size_t slot = (c % kPinnedSlots) * st->slotBytes;
    for (int k = 0, j = 0; k < nSrcs; k++)
      if (!psrc[k]) tasks[nTasks++] = {st->host + slot + chunkBytes * j++, (const char*)srcs[k] + e0 * esz, n * esz};
  };
  auto copyOut = [&](size_t c) {
    size_t e0, n;
    span(c, &e0, &n);
    const char* out = st->host + (c % kPinnedSlots) * st->slotBytes + outOffset();
    for (int d = 0; d < nDsts; d++)
      if (!pdst[d]) tasks[nTasks++] = {(char*)dsts[d] + e0 * esz, out, n * esz};
  };
  auto launch = [&](size_t c) -> nexrResult_t {
    size_t e0, n;
    span(c, &e0, &n);
    const size_t slot = (c % kPinnedSlots) * st->slotBytes;
    const void* dsrc[NEXR_MAX_SRCS];
    for (int k = 0, j = 0; k < nSrcs; k++)
      dsrc[k] = psrc[k] ? (const void*)((const char*)zsrc[k] + e0 * esz) : (const void*)(st->dev + slot + chunkBytes * j++);
    void* ddst[NEXR_MAX_DSTS + 1];
    int m = 0;
    for (int d = 0; d < nDsts; d++)
      if (pdst[d]) ddst[m++] = (char*)zdst[d] + e0 * esz;
    if (outStaged) ddst[m++] = st->dev + slot + outOffset();
    nexrResult_t rr = reduceCopyDevice(nSrcs, dsrc, m, ddst, n, datatype, op, redOpArg, nPreOpSrcs, preOpArgs,
                                       nullptr, postOp, s, hostGrid());
    if (rr != nexrSuccess) return rr;
    NEXR_HIP(hipEventRecord(st->done[c % kPinnedSlots], s));
    return nexrSuccess;
  };
  // Iteration c: wait for chunk c-2's kernel, then ONE team pass copies chunk c-2's output out of
  // slot (c-2) % 3 and chunk c's sources into slot c % 3 (drained one iteration ago) while the GPU
  // reduces chunk c-1; then chunk c's kernel is queued.
  for (size_t c = 0; c < nChunks + 2; c++) {
    nTasks = 0;
    uint64_t t0 = nowNs();
    if (c >= 2) {
      NEXR_HIP(hipEventSynchronize(st->done[(c - 2) % kPinnedSlots]));
      const uint64_t t1 = nowNs();
      gHpWaitNs.fetch_add(t1 - t0, std::memory_order_relaxed);
      t0 = t1;
      if (outStaged) copyOut(c - 2);
    }
    if (c < nChunks) copyIn(c);
    if (nTasks > 0) team.run(tasks, nTasks);
    const uint64_t t1 = nowNs();
    gHpCopyNs.fetch_add(t1 - t0, std::memory_order_relaxed);
    if (c < nChunks) {
      r = launch(c);
      if (r != nexrSuccess) return r;
      gHpLaunchNs.fetch_add(nowNs() - t1, std::memory_order_relaxed);
    }
  }
  return nexrSuccess;
}

// ---- host-side half/bfloat16 rounding used by the op encoder (RNE, NaN -> 0x7fff) ------------
uint16_t floatToHalfRne(float f) {
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  const uint32_t a = x & 0x7fffffffu;
  if (a > 0x7f800000u) return 0x7fffu;
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to +-inf
  if (a < 0x33000001u) return (uint16_t)sign;               // <= 2^-25 rounds to 0
  uint32_t mant, shift;
  if (a >= 0x38800000u) {  // normal half
    mant = a - 0x38000000u;
    shift = 13;
  } else {  // subnormal half
    const uint32_t e = a >> 23;
    mant = (a & 0x7fffffu) | 0x800000u;
    shift = 126 - e;
  }
  uint32_t q = mant >> shift;
  const uint32_t rem = mant & ((1u << shift) - 1);
  const uint32_t halfway = 1u << (shift - 1);
  if (rem > halfway || (rem == halfway && (q & 1))) q++;
  return (uint16_t)(sign | q);
}
uint16_t floatToBf16Rne(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fffu;
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// ---- host registration cache (reference: ncclCommRegister's per-comm regCache, sorted by begin
// address, src/register/register.cc:40-60; ncclMemAlloc, src/allocator.cc:11-) -----------------
// Pinned, device-mapped host ranges the library registered (nexrHostRegister) or allocated
// (nexrHostMemAlloc), sorted by begin address. nexrReduceCopyHost looks a buffer up here first, so a
// call on registered memory costs no HIP query per buffer; because the library made every entry, it
// also knows when one ends (nexrHostDeregister / nexrHostMemFree), so nothing here goes stale.
// Entries hold exact byte ranges. hipHostRegister pins every page a range touches, and on this ROCm it
// accepts a second range that shares a page with a registered one (adjacent heap buffers do, e.g. the
// C1 bench's numpy arrays), giving it a mapping of its own, so such neighbours are separate entries
// whose deregistrations are independent (tests/test_host_register_gpu.py); should the runtime refuse
// one, the call returns nexrInvalidUsage, not a raw HIP error. Handles are monotonic ids, never
// addresses: a handle whose entry is gone stays invalid even when a later entry lands at the same
// address.
struct HostReg {
  uintptr_t beg = 0, end = 0;
  char* dev = nullptr;         // device address of beg
  void* hipPtr = nullptr;      // the pointer hipHostRegister / hipHostMalloc returned or took
  bool owned = false;          // allocated by nexrHostMemAlloc (freed by nexrHostMemFree), else registered
  int regs = 0;                // live nexrHostRegister references to this entry (its handles)
  uint64_t id = 0;
};
std::shared_mutex gRegMu;
std::vector<HostReg*> gRegs;  // sorted by beg, non-overlapping
uint64_t gRegNextId = 1;      // under gRegMu

uintptr_t pageSize() {
  static const uintptr_t ps = [] {
    const long v = sysconf(_SC_PAGESIZE);
    return (uintptr_t)(v > 0 ? v : 4096);
  }();
  return ps;
}
uintptr_t pageFloor(uintptr_t a) { return a & ~(pageSize() - 1); }
uintptr_t pageCeil(uintptr_t a) { return (a + pageSize() - 1) & ~(pageSize() - 1); }

// The device address of [p, p + bytes) when the whole range lies inside one entry.
bool regLookup(const void* p, size_t bytes, void** dev) {
  const uintptr_t a = (uintptr_t)p;
  std::shared_lock<std::shared_mutex> lk(gRegMu);
  auto it = std::upper_bound(gRegs.begin(), gRegs.end(), a, [](uintptr_t v, const HostReg* r) { return v < r->beg; });
  if (it == gRegs.begin()) return false;
  const HostReg* r = *(it - 1);
  if (a + bytes > r->end || a + bytes < a) return false;
  *dev = r->dev + (a - r->beg);
  return true;
}

// Index of the entry containing [a, a + n), -1 if none; overlap: some entry intersects it; sharesPage:
// some entry shares a page with it.
int regFind(uintptr_t a, size_t n, bool* overlap, bool* sharesPage) {
  *overlap = *sharesPage = false;
  const uintptr_t pb = pageFloor(a), pe = pageCeil(a + n);
  for (size_t i = 0; i < gRegs.size(); i++) {
    const HostReg* r = gRegs[i];
    if (a >= r->beg && a + n <= r->end) return (int)i;
    if (a < r->end && a + n > r->beg) *overlap = true;
    if (pb < pageCeil(r->end) && pe > pageFloor(r->beg)) *sharesPage = true;
  }
  return -1;
}

void regInsert(HostReg* r) {
  r->id = gRegNextId++;
  auto it = std::upper_bound(gRegs.begin(), gRegs.end(), r->beg, [](uintptr_t v, const HostReg* x) { return v < x->beg; });
  gRegs.insert(it, r);
}

std::vector<HostReg*>::iterator regById(const void* handle) {
  const uint64_t id = (uint64_t)(uintptr_t)handle;
  return std::find_if(gRegs.begin(), gRegs.end(), [&](const HostReg* r) { return r->id == id; });
}

}  // namespace
}  // namespace nexr

using namespace nexr;

extern "C" {

NEXR_API nexrResult_t nexrReduceCopy(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                     size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                                     int nPreOpSrcs, const uint64_t* preOpArgs, int postOp,
                                     nexrStream_t stream) {
  return reduceCopyDevice(nSrcs, srcs, nDsts, dsts, nElts, datatype, devRedOp, redOpArg, nPreOpSrcs,
                          preOpArgs, nullptr, postOp, (hipStream_t)stream);
}

NEXR_API nexrResult_t nexrGetPoolStats(uint64_t* multiDeviceStreams, uint64_t* hostStagingRings) {
  if (multiDeviceStreams) {
    std::lock_guard<std::mutex> g(gMdStreamMu);
    *multiDeviceStreams = gMdStreamsCreated;
  }
  if (hostStagingRings) {
    uint64_t n = 0;
    {
      std::lock_guard<std::mutex> g(gStageMu);
      n = gStagesCreated;
    }
    std::lock_guard<std::mutex> g(gPinMu);
    *hostStagingRings = n + gPinCreated;
  }
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrQueryLaunch(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                      size_t nElts, int datatype, nexrLaunchInfo* info) {
  if (info == nullptr) return nexrInvalidArgument;
  memset(info, 0, sizeof(*info));
  nexrResult_t r = validate(nSrcs, srcs, nDsts, dsts, nElts, datatype, nexrDevSum, 0, 0, nullptr);
  if (r != nexrSuccess) return r;
  if (nElts == 0 || nDsts == 0) return nexrSuccess;  // nothing would be launched
  CallShape c{datatype, nexrDevSum, nSrcs, 0, 0, nullptr};
  applySemantics(c);
  routeKernel(c, &nElts);  // a K = 1 call is a byte copy: headElts / bodyPacks of the uint8 kernel
  nSrcs = c.nSrcs;
  datatype = c.dt;
  const size_t esz = typeSize(datatype);
  RCParams p;
  fillParams(p, nSrcs, srcs, nDsts, dsts, nElts, esz, 0, 0, nullptr, nullptr, 0);
  Geometry g;
  const int pol = pickPolicy((uint64_t)(nSrcs + nDsts) * nElts * esz, nSrcs, nDsts);
  const int block = block_for(datatype, nSrcs, pol);
  r = pickGeometry(workgroupsFor(p, nSrcs, datatype, pol), pol, block, &g);
  if (r != nexrSuccess) return r;
  info->grid = (uint32_t)g.grid;
  info->block = block;
  info->packsPerLane = unroll_for(datatype, nSrcs, pol);
  info->policy = g.pol;
  info->unaligned = p.unaligned;
  info->headElts = p.head;
  info->bodyPacks = p.nPacks;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrReduceCopyBatch(const nexrReduceCopyWork* works, int nWorks, int datatype, int devRedOp,
                                          nexrStream_t stream) {
  return reduceCopyBatch(works, nWorks, datatype, devRedOp, (hipStream_t)stream);
}

NEXR_API nexrResult_t nexrReduceCopyMultiDevice(const nexrReduceCopyWork* works, const int* devices, int nWorks,
                                                int datatype, int devRedOp, int reps, double* seconds) {
  return reduceCopyMultiDevice(works, devices, nWorks, 1, datatype, devRedOp, reps, seconds);
}
NEXR_API nexrResult_t nexrReduceCopyMultiDeviceSets(const nexrReduceCopyWork* works, const int* devices, int nWorks,
                                                    int nSets, int datatype, int devRedOp, int reps, double* seconds) {
  return reduceCopyMultiDevice(works, devices, nWorks, nSets, datatype, devRedOp, reps, seconds);
}

NEXR_API nexrResult_t nexrReduceCopyHost(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                         size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                                         int nPreOpSrcs, const uint64_t* preOpArgs, int postOp,
                                         nexrStream_t stream) {
  nexrResult_t r = validate(nSrcs, srcs, nDsts, dsts, nElts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs);
  if (r != nexrSuccess) return r;
  if (nElts == 0 || nDsts == 0) return nexrSuccess;
  hipStream_t s = (hipStream_t)stream;
  // Zero-copy: when every buffer is pinned (page-locked, device-mapped) host memory the kernel reads
  // and writes it directly over PCIe, both directions at once, with no staging copies (measured
  // 80.7 GB/s vs 71.5 GB/s staged for the C2 mix: profiles/r01_h2d_probe.log).
  const void* zsrc[NEXR_MAX_SRCS];
  void* zdst[NEXR_MAX_DSTS];
  bool psrc[NEXR_MAX_SRCS], pdst[NEXR_MAX_DSTS];  // pinned (device-mapped) buffers
  // Classification: the registration cache first (no HIP call); otherwise the runtime's pointer
  // query, trusted only when the whole buffer lies inside the pinned range it reports.
  static const long zeroCopy = envLong("NEXR_HOST_ZERO_COPY", 1);
  const size_t esz = typeSize(datatype);
  const size_t bufBytes = nElts * esz;
  const uint64_t tc0 = nowNs();
  gHpCalls.fetch_add(1, std::memory_order_relaxed);
  int nPinned = 0;
  for (int k = 0; k < nSrcs + nDsts; k++) {
    const void* hp = k < nSrcs ? srcs[k] : dsts[k - nSrcs];
    void* dev = nullptr;
    bool pin = false;
    if (zeroCopy != 0) {
      if (regLookup(hp, bufBytes, &dev)) {
        pin = true;
        gHpRegHits.fetch_add(1, std::memory_order_relaxed);
      } else {
        gHpQueries.fetch_add(1, std::memory_order_relaxed);
        hipPointerAttribute_t a;
        pin = hipPointerGetAttributes(&a, hp) == hipSuccess && a.type == hipMemoryTypeHost && a.devicePointer != nullptr;
        if (pin) {
          dev = a.devicePointer;
          // A pointer inside a registered range whose buffer runs past its end must not be read in
          // place: the device mapping covers only the range. Without the range, nothing is.
          uintptr_t beg = 0;
          size_t size = 0;
          if (hipPointerGetAttribute(&beg, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)hp) != hipSuccess ||
              hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)hp) != hipSuccess ||
              (uintptr_t)hp < beg || (uintptr_t)hp + bufBytes > beg + size)
            pin = false;
        }
        (void)hipGetLastError();  // pageable memory reports an error: not a failure of this call
      }
    }
    if (k < nSrcs) {
      psrc[k] = pin;
      zsrc[k] = pin ? dev : nullptr;
    } else {
      pdst[k - nSrcs] = pin;
      zdst[k - nSrcs] = pin ? dev : nullptr;
    }
    nPinned += pin ? 1 : 0;
  }
  const uint64_t tc1 = nowNs();
  gHpClassifyNs.fetch_add(tc1 - tc0, std::memory_order_relaxed);
  if (nPinned == nSrcs + nDsts) {
    gHpZeroCopy.fetch_add(1, std::memory_order_relaxed);
    r = reduceCopyDevice(nSrcs, zsrc, nDsts, zdst, nElts, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs,
                         nullptr, postOp, s, hostGrid());
    const uint64_t tc2 = nowNs();
    gHpLaunchNs.fetch_add(tc2 - tc1, std::memory_order_relaxed);
    if (r != nexrSuccess) return r;
    NEXR_HIP(hipStreamSynchronize(s));
    gHpWaitNs.fetch_add(nowNs() - tc2, std::memory_order_relaxed);
    return nexrSuccess;
  }
  // Pageable buffers, by the pageable bytes the call moves (profiles/r02_host_sizes_sweep.log):
  //   <= NEXR_HOST_SOLO_MAX_BYTES (4 MiB; the emulated ring's slices): the calling thread copies them
  //      into pinned zero-copy slots (reduceCopyHostTeam, one thread): 1.2-1.9x the runtime copies;
  //   >= NEXR_HOST_MT_MIN_BYTES (256 MiB): a team of NEXR_HOST_COPY_THREADS (8) threads does: 1.1-1.2x;
  //   in between, and always with NEXR_HOST_COPY_THREADS=0: the runtime-copy chunk pipeline below,
  //      which is as fast or faster there.
  static const long mtMin = envLong("NEXR_HOST_MT_MIN_BYTES", 256l << 20);
  static const long soloMax = envLong("NEXR_HOST_SOLO_MAX_BYTES", 4l << 20);
  static const long mtThreads = envLong("NEXR_HOST_COPY_THREADS", 8);
  const uint64_t pageable = (uint64_t)(nSrcs + nDsts - nPinned) * nElts * esz;
  if (mtThreads >= 1 && (pageable >= (uint64_t)mtMin || pageable <= (uint64_t)soloMax)) {
    const bool large = pageable >= (uint64_t)mtMin;
    return reduceCopyHostTeam(nSrcs, srcs, psrc, zsrc, nDsts, dsts, pdst, zdst, nElts, datatype, devRedOp, redOpArg,
                              nPreOpSrcs, preOpArgs, postOp, s, large ? (int)(mtThreads > 64 ? 64 : mtThreads) : 1);
  }
  // Some buffers pageable: a two-stream chunk pipeline through device memory for those only; the
  // pinned ones (e.g. the emulated transport's FIFOs) are read and written in place by the kernel.
  static const long chunkOverride = envLong("NEXR_HOST_CHUNK_BYTES", 8l << 20);
  size_t chunkElts = ((size_t)(chunkOverride > 4096 ? chunkOverride : 4096) / esz) & ~(size_t)15;
  if (chunkElts > nElts) chunkElts = nElts;
  const size_t chunkBytes = ((chunkElts * esz) + 255) & ~(size_t)255;
  StageLease lease;
  r = stageFor(chunkBytes * (size_t)(nSrcs + 1), s, &lease);
  if (r != nexrSuccess) return r;
  HostStage* st = lease.st;
  bool anyPageableDst = false;
  for (int d = 0; d < nDsts; d++) anyPageableDst |= !pdst[d];
  const size_t nChunks = (nElts + chunkElts - 1) / chunkElts;
  const uint64_t tp = nowNs();
  for (size_t c = 0; c < nChunks; c++) {
    const int slot = (int)(c & 1);
    const size_t e0 = c * chunkElts;
    const size_t n = (nElts - e0 < chunkElts) ? nElts - e0 : chunkElts;
    char* base = st->buf + (size_t)slot * st->slotBytes;
    if (c >= 2) NEXR_HIP(hipStreamWaitEvent(s, st->outDone[slot], 0));  // slot drained by chunk c-2's D2H
    const void* dsrc[NEXR_MAX_SRCS];
    for (int k = 0; k < nSrcs; k++) {
      if (psrc[k]) {
        dsrc[k] = (const char*)zsrc[k] + e0 * esz;
        continue;
      }
      dsrc[k] = base + chunkBytes * k;
      NEXR_HIP(hipMemcpyAsync((void*)dsrc[k], (const char*)srcs[k] + e0 * esz, n * esz, hipMemcpyHostToDevice, s));
    }
    void* ddst[NEXR_MAX_DSTS + 1];
    int m = 0;
    for (int d = 0; d < nDsts; d++)
      if (pdst[d]) ddst[m++] = (char*)zdst[d] + e0 * esz;
    char* staged = base + chunkBytes * nSrcs;
    if (anyPageableDst) ddst[m++] = staged;
    r = reduceCopyDevice(nSrcs, dsrc, m, ddst, n, datatype, devRedOp, redOpArg, nPreOpSrcs, preOpArgs, nullptr,
                         postOp, s, nPinned > 0 ? hostGrid() : 0);
    if (r != nexrSuccess) return r;
    NEXR_HIP(hipEventRecord(st->kernelDone[slot], s));
    NEXR_HIP(hipStreamWaitEvent(st->out, st->kernelDone[slot], 0));
    for (int d = 0; d < nDsts; d++)
      if (!pdst[d])
        NEXR_HIP(hipMemcpyAsync((char*)dsts[d] + e0 * esz, staged, n * esz, hipMemcpyDeviceToHost, st->out));
    NEXR_HIP(hipEventRecord(st->outDone[slot], st->out));
  }
  const uint64_t tw = nowNs();
  gHpLaunchNs.fetch_add(tw - tp, std::memory_order_relaxed);
  NEXR_HIP(hipStreamSynchronize(st->out));
  NEXR_HIP(hipStreamSynchronize(s));
  gHpWaitNs.fetch_add(nowNs() - tw, std::memory_order_relaxed);
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrHostRegister(void* buff, size_t size, void** handle) {
  if (buff == nullptr || size == 0 || handle == nullptr) return nexrInvalidArgument;
  const uintptr_t a = (uintptr_t)buff;
  if (a + size < a) return nexrInvalidArgument;
  std::unique_lock<std::shared_mutex> lk(gRegMu);
  bool overlap = false, sharesPage = false;
  const int i = regFind(a, size, &overlap, &sharesPage);
  if (i >= 0) {  // inside a range this library already maps (registered or allocated): share it (register.cc:49-76)
    gRegs[i]->regs++;
    *handle = (void*)(uintptr_t)gRegs[i]->id;
    return nexrSuccess;
  }
  if (overlap) return nexrInvalidUsage;  // partly inside another entry: hipHostRegister would refuse it
  hipError_t e = hipHostRegister(buff, size, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) {
    if (sharesPage) {  // a page-sharing neighbour the runtime refused: the documented usage error
      (void)hipGetLastError();
      return nexrInvalidUsage;
    }
    return hipFail(e);
  }
  void* dev = nullptr;
  e = hipHostGetDevicePointer(&dev, buff, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister(buff);
    return hipFail(e);
  }
  HostReg* r = new HostReg();
  r->beg = a;
  r->end = a + size;
  r->dev = (char*)dev;
  r->hipPtr = buff;
  r->regs = 1;
  regInsert(r);
  *handle = (void*)(uintptr_t)r->id;
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrHostDeregister(void* handle) {
  if (handle == nullptr) return nexrSuccess;  // ncclCommDeregister accepts a NULL handle
  std::unique_lock<std::shared_mutex> lk(gRegMu);
  auto it = regById(handle);
  if (it == gRegs.end() || (*it)->regs == 0) return nexrInvalidUsage;  // register.cc:150-153
  HostReg* r = *it;
  if (--r->regs > 0 || r->owned) return nexrSuccess;  // an allocation's pages stay until nexrHostMemFree
  gRegs.erase(it);
  hipError_t e = hipHostUnregister(r->hipPtr);
  delete r;
  NEXR_HIP(e);
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrHostMemAlloc(void** ptr, size_t size) {
  if (ptr == nullptr || size == 0) return nexrInvalidArgument;
  *ptr = nullptr;
  void* host = nullptr;
  NEXR_HIP(hipHostMalloc(&host, size, hipHostMallocMapped | hipHostMallocPortable));
  void* dev = nullptr;
  hipError_t e = hipHostGetDevicePointer(&dev, host, 0);
  if (e != hipSuccess) {
    (void)hipHostFree(host);
    return hipFail(e);
  }
  HostReg* r = new HostReg();
  r->beg = (uintptr_t)host;
  r->end = (uintptr_t)host + size;
  r->dev = (char*)dev;
  r->hipPtr = host;
  r->owned = true;
  std::unique_lock<std::shared_mutex> lk(gRegMu);
  regInsert(r);
  *ptr = host;
  return nexrSuccess;
}

// Refused (nexrInvalidUsage) while registrations inside the allocation remain: their handles would
// otherwise name freed memory (the caller deregisters first, as ncclCommDeregister before ncclMemFree).
NEXR_API nexrResult_t nexrHostMemFree(void* ptr) {
  if (ptr == nullptr) return nexrSuccess;
  std::unique_lock<std::shared_mutex> lk(gRegMu);
  auto it = std::find_if(gRegs.begin(), gRegs.end(), [&](const HostReg* r) { return r->owned && r->hipPtr == ptr; });
  if (it == gRegs.end()) return nexrInvalidArgument;
  HostReg* r = *it;
  if (r->regs > 0) return nexrInvalidUsage;
  gRegs.erase(it);
  delete r;
  NEXR_HIP(hipHostFree(ptr));
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrGetHostPathStats(nexrHostPathStats* stats, int reset) {
  if (stats == nullptr) return nexrInvalidArgument;
  auto take = [&](std::atomic<uint64_t>& a) { return reset ? a.exchange(0) : a.load(); };
  stats->calls = take(gHpCalls);
  stats->zeroCopyCalls = take(gHpZeroCopy);
  stats->registeredHits = take(gHpRegHits);
  stats->pointerQueries = take(gHpQueries);
  stats->classifyNs = take(gHpClassifyNs);
  stats->copyNs = take(gHpCopyNs);
  stats->launchNs = take(gHpLaunchNs);
  stats->waitNs = take(gHpWaitNs);
  return nexrSuccess;
}

// Restates hostToDevRedOp (reference src/enqueue.cc:2185-2278) for the built-in ops.
NEXR_API nexrResult_t nexrHostToDevRedOp(nexrDevRedOpFull* opFull, int op, int datatype, int nRanks) {
  if (opFull == nullptr) return nexrInvalidArgument;
  const int nbits = 8 * (int)typeSize(datatype);
  if (nbits <= 0) return nexrInvalidArgument;
  const uint64_t allBits = ~(uint64_t)0 >> (64 - nbits);
  const uint64_t signBit = allBits ^ (allBits >> 1);
  opFull->scalarArgIsPtr = false;
  opFull->proxyOp = op;
  opFull->scalarArg = 0;
  switch (op) {
    case nexrSum: opFull->op = nexrDevSum; break;
    case nexrProd: opFull->op = nexrDevProd; break;
    case nexrMin:
    case nexrMax:
      opFull->op = nexrDevMinMax;
      if (isSignedInt(datatype)) opFull->scalarArg ^= signBit;
      opFull->scalarArg ^= (op == nexrMax) ? allBits : 0;
      break;
    case nexrAvg: {
      if (nRanks < 1) return nexrInvalidArgument;
      uint64_t u64 = 0;
      switch (datatype) {
        case nexrInt8: case nexrInt32: case nexrInt64:
        case nexrUint8: case nexrUint32: case nexrUint64:
          opFull->op = nexrDevSumPostDiv;
          u64 = ((uint64_t)nRanks << 1) | (isSignedInt(datatype) ? 1u : 0u);
          break;
        case nexrFloat16:
          opFull->op = nexrDevPreMulSum;
          u64 = floatToHalfRne((float)(1.0 / nRanks));
          break;
        case nexrBfloat16:
          opFull->op = nexrDevPreMulSum;
          u64 = floatToBf16Rne((float)(1.0 / nRanks));
          break;
        case nexrFloat32: {
          opFull->op = nexrDevPreMulSum;
          float f = (float)(1.0 / nRanks);
          uint32_t b;
          memcpy(&b, &f, 4);
          u64 = b;
          break;
        }
        case nexrFloat64: {
          opFull->op = nexrDevPreMulSum;
          double f = 1.0 / nRanks;
          memcpy(&u64, &f, 8);
          break;
        }
        default:  // fp8: the fork compiles this case out (enqueue.cc:2229-2238 guard)
          return nexrInvalidArgument;
      }
      opFull->scalarArg = u64;
      break;
    }
    default:  // user-created ops need a communicator's op table: not part of this boundary
      return nexrInvalidArgument;
  }
  return nexrSuccess;
}

// Restates ncclLaunchOneRank (reference src/device/onerank.cc:48-83).
NEXR_API nexrResult_t nexrLaunchOneRank(void* dst, const void* src, size_t nElts, nexrDevRedOpFull redOp,
                                        int datatype, nexrStream_t stream) {
  const size_t esz = typeSize(datatype);
  if (esz == 0) return nexrInvalidArgument;
  hipStream_t s = (hipStream_t)stream;
  if (redOp.op != nexrDevPreMulSum) {
    if (dst != src && nElts > 0) NEXR_HIP(hipMemcpyAsync(dst, src, nElts * esz, hipMemcpyDeviceToDevice, s));
    return nexrSuccess;
  }
  if (datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2) return nexrInvalidArgument;
  const void* srcs[1] = {src};
  void* dsts[1] = {dst};
  uint64_t arg = redOp.scalarArg;
  const void* prePtr = redOp.scalarArgIsPtr ? (const void*)(uintptr_t)redOp.scalarArg : nullptr;
  return reduceCopyDevice(1, srcs, 1, dsts, nElts, datatype, nexrDevPreMulSum, arg, 1, &arg, prePtr,
                          /*postOp=*/1, s);
}

NEXR_API nexrResult_t nexrReduceCopyLL(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                                       const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                                       const uint32_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                       uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                       nexrStream_t stream) {
  if (nRecv < 0 || nRecv > NEXR_MAX_SRCS || nSend < 0 || nSend > NEXR_MAX_DSTS) return nexrInvalidArgument;
  if (!src && nRecv == 0) return nexrInvalidArgument;   // LLGenericOp needs SRC or RECV
  if (!dst && nSend == 0) return nexrInvalidArgument;   // ... and DST or SEND
  if (datatype < 0 || datatype >= nexrNumTypes || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2)
    return nexrInvalidArgument;
  if (devRedOp < 0 || devRedOp >= nexrNumDevRedOps) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && !isInteger(datatype)) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && isSignedInt(datatype) && typeSize(datatype) == 1) {
    uint32_t divisor = (uint32_t)(redOpArg >> 1);
    if (divisor == 0) divisor = 1;
    if ((int8_t)divisor == 0) return nexrInvalidArgument;
  }
  if ((nRecv && (!recvLines || !recvFlags)) || (nSend && (!sendLines || !sendFlags))) return nexrInvalidArgument;
  if (nElts == 0) return nexrSuccess;
  LLParams a;
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < nRecv; i++) {
    if (!recvLines[i] || ((uintptr_t)recvLines[i] & 15)) return nexrInvalidArgument;
    a.recv[i] = (const char*)recvLines[i];
    a.recvFlag[i] = recvFlags[i];
  }
  for (int i = 0; i < nSend; i++) {
    if (!sendLines[i] || ((uintptr_t)sendLines[i] & 15)) return nexrInvalidArgument;
    a.send[i] = (char*)sendLines[i];
    a.sendFlag[i] = sendFlags[i];
  }
  a.src = (const char*)src;
  a.dst = (char*)dst;
  a.nElts = nElts;
  a.redArg = redOpArg;
  a.status = status;
  a.timeoutTicks = (uint64_t)(timeoutUs ? timeoutUs : 1000000u) * 100u;  // s_memrealtime: 100 MHz
  a.nRecv = nRecv;
  a.nSend = nSend;
  a.srcIsInput = srcIsInput ? 1 : 0;
  a.postOp = postOp ? 1 : 0;
  llSemantics(&datatype, &devRedOp, &a.srcIsInput, &a.postOp, &a.firstWins);
  const uint64_t nLines = (nElts * typeSize(datatype) + 7) / 8;
  uint64_t grid = (nLines + kLLTileLines - 1) / kLLTileLines;
  if (grid > (1u << 20)) grid = 1u << 20;
  NEXR_HIP(launch_ll(datatype, a, devRedOp, (int)grid, (hipStream_t)stream));
  return nexrSuccess;
}

// The steps run as if one at a time: a launch's workgroups walk its steps independently, which is
// only the same when no step touches user bytes that an earlier step of the launch wrote (or, for a
// write, read) at another element position. The same range at the same position is handled by the
// same lanes in both steps, in order.
namespace {
struct UserRange {
  uintptr_t beg, end;
  bool write;
};
bool rangesConflict(const std::vector<UserRange>& seen, const UserRange& r) {
  for (const UserRange& q : seen) {
    if (!r.write && !q.write) continue;
    if (r.beg < q.end && q.beg < r.end && !(r.beg == q.beg && r.end == q.end)) return true;
  }
  return false;
}
}  // namespace

NEXR_API nexrResult_t nexrReduceCopyLLSteps(const nexrLLConnSet* cs, const nexrLLStep* steps, int nSteps,
                                            int datatype, int devRedOp, uint64_t redOpArg, uint32_t* status,
                                            uint32_t timeoutUs, nexrStream_t stream) {
  if (!cs || nSteps < 0 || (nSteps > 0 && !steps)) return nexrInvalidArgument;
  if (cs->nRecv < 0 || cs->nRecv > NEXR_LL_STEPS_MAX_PEERS || cs->nSend < 0 || cs->nSend > NEXR_LL_STEPS_MAX_PEERS)
    return nexrInvalidArgument;
  if (cs->slotBytes == 0 || cs->slotBytes % 16 || cs->nSlots == 0) return nexrInvalidArgument;
  if (datatype < 0 || datatype >= nexrNumTypes || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2)
    return nexrInvalidArgument;
  if (devRedOp < 0 || devRedOp >= nexrNumDevRedOps) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && !isInteger(datatype)) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && isSignedInt(datatype) && typeSize(datatype) == 1) {
    uint32_t divisor = (uint32_t)(redOpArg >> 1);
    if (divisor == 0) divisor = 1;
    if ((int8_t)divisor == 0) return nexrInvalidArgument;
  }
  for (int i = 0; i < cs->nRecv; i++)
    if (!cs->recvFifo[i] || ((uintptr_t)cs->recvFifo[i] & 15) || !cs->recvHead[i] || ((uintptr_t)cs->recvHead[i] & 7))
      return nexrInvalidArgument;
  for (int i = 0; i < cs->nSend; i++)
    if (!cs->sendFifo[i] || ((uintptr_t)cs->sendFifo[i] & 15) || !cs->sendHead[i] || ((uintptr_t)cs->sendHead[i] & 7))
      return nexrInvalidArgument;
  const size_t esz = typeSize(datatype);
  const uint64_t slotData = cs->slotBytes / 2;  // 8 data bytes per 16-byte line
  for (int k = 0; k < nSteps; k++) {
    const nexrLLStep& s = steps[k];
    if (s.srcBuf < -1 || s.srcBuf > 1 || s.dstBuf < -1 || s.dstBuf > 1) return nexrInvalidArgument;
    if ((s.recv && cs->nRecv == 0) || (s.send && cs->nSend == 0)) return nexrInvalidArgument;
    if ((s.srcBuf == 0 && !cs->input) || (s.srcBuf == 1 && !cs->output) || (s.dstBuf == 0 && !cs->input) ||
        (s.dstBuf == 1 && !cs->output))
      return nexrInvalidArgument;
    if (s.srcIx < 0 || s.dstIx < 0) return nexrInvalidArgument;
    if (s.nElts == 0) continue;
    if ((s.srcBuf < 0 && !s.recv) || (s.dstBuf < 0 && !s.send)) return nexrInvalidArgument;
    if ((s.recv || s.send) && (uint64_t)s.nElts * esz > slotData) return nexrInvalidArgument;
  }
  if (nSteps == 0) return nexrSuccess;
  int srcIsInput = 1, postOp = 1;
  LLStepsParams P;
  memset(&P, 0, sizeof(P));
  llSemantics(&datatype, &devRedOp, &srcIsInput, &postOp, &P.firstWins);
  P.input = (const char*)cs->input;
  P.output = (char*)cs->output;
  for (int i = 0; i < NEXR_LL_STEPS_MAX_PEERS; i++) {
    P.recvFifo[i] = (const char*)cs->recvFifo[i];
    P.recvHead[i] = cs->recvHead[i];
    P.sendFifo[i] = (char*)cs->sendFifo[i];
    P.sendHead[i] = cs->sendHead[i];
  }
  P.slotBytes = cs->slotBytes;
  P.redArg = redOpArg;
  P.status = status;
  P.timeoutTicks = (uint64_t)(timeoutUs ? timeoutUs : 1000000u) * 100u;
  P.nRecv = cs->nRecv;
  P.nSend = cs->nSend;
  P.nSlots = (int)cs->nSlots;
  // One workgroup per line tile of a full slot (the same grid on both ends of every connection).
  const uint64_t slotTiles = (cs->slotBytes / 16 + kLLTileLines - 1) / kLLTileLines;
  const int grid = (int)(slotTiles < 1 ? 1 : slotTiles > (uint64_t)kLLStepsMaxGrid ? kLLStepsMaxGrid : slotTiles);
  uint64_t rs[NEXR_LL_STEPS_MAX_PEERS], ss[NEXR_LL_STEPS_MAX_PEERS];
  for (int i = 0; i < NEXR_LL_STEPS_MAX_PEERS; i++) rs[i] = cs->recvStep[i], ss[i] = cs->sendStep[i];
  std::vector<UserRange> seen;
  auto launch = [&]() -> nexrResult_t {
    if (P.nSteps == 0) return nexrSuccess;
    NEXR_HIP(launch_ll_steps(datatype, P, devRedOp, grid, (hipStream_t)stream));
    P.nSteps = 0;
    seen.clear();
    return nexrSuccess;
  };
  for (int k = 0; k < nSteps; k++) {
    const nexrLLStep& s = steps[k];
    UserRange rd{0, 0, false}, wr{0, 0, true};
    if (s.nElts && s.srcBuf >= 0) {
      rd.beg = (uintptr_t)(s.srcBuf == 0 ? cs->input : cs->output) + (uintptr_t)s.srcIx * esz;
      rd.end = rd.beg + (uintptr_t)s.nElts * esz;
    }
    if (s.nElts && s.dstBuf >= 0) {
      wr.beg = (uintptr_t)(s.dstBuf == 0 ? cs->input : cs->output) + (uintptr_t)s.dstIx * esz;
      wr.end = wr.beg + (uintptr_t)s.nElts * esz;
    }
    if (P.nSteps == kLLStepsMax || (rd.end && rangesConflict(seen, rd)) || (wr.end && rangesConflict(seen, wr))) {
      nexrResult_t r = launch();
      if (r != nexrSuccess) return r;
    }
    if (P.nSteps == 0)
      for (int i = 0; i < NEXR_LL_STEPS_MAX_PEERS; i++) P.recvStep[i] = rs[i], P.sendStep[i] = ss[i];
    P.step[P.nSteps++] = s;
    if (rd.end) seen.push_back(rd);
    if (wr.end) seen.push_back(wr);
    if (s.recv)
      for (uint64_t& v : rs) v++;
    if (s.send)
      for (uint64_t& v : ss) v++;
  }
  return launch();
}

NEXR_API nexrResult_t nexrReduceCopyLL128(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                                          const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                                          const uint64_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                          uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                          nexrStream_t stream) {
  if (nRecv < 0 || nRecv > NEXR_MAX_SRCS || nSend < 0 || nSend > NEXR_MAX_DSTS) return nexrInvalidArgument;
  if ((!src && nRecv == 0) || (!dst && nSend == 0)) return nexrInvalidArgument;
  if (datatype < 0 || datatype >= nexrNumTypes || datatype == nexrFloat8e4m3 || datatype == nexrFloat8e5m2)
    return nexrInvalidArgument;
  if (devRedOp < 0 || devRedOp >= nexrNumDevRedOps) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && !isInteger(datatype)) return nexrInvalidArgument;
  if (devRedOp == nexrDevSumPostDiv && isSignedInt(datatype) && typeSize(datatype) == 1) {
    uint32_t divisor = (uint32_t)(redOpArg >> 1);
    if (divisor == 0) divisor = 1;
    if ((int8_t)divisor == 0) return nexrInvalidArgument;
  }
  if ((nRecv && (!recvWire || !recvFlags)) || (nSend && (!sendWire || !sendFlags))) return nexrInvalidArgument;
  if (nElts == 0) return nexrSuccess;
  LL128Params a;
  memset(&a, 0, sizeof(a));
  for (int i = 0; i < nRecv; i++) {
    if (!recvWire[i] || ((uintptr_t)recvWire[i] & 15)) return nexrInvalidArgument;
    a.recv[i] = (const char*)recvWire[i];
    a.recvFlag[i] = recvFlags[i];
  }
  for (int i = 0; i < nSend; i++) {
    if (!sendWire[i] || ((uintptr_t)sendWire[i] & 15)) return nexrInvalidArgument;
    a.send[i] = (char*)sendWire[i];
    a.sendFlag[i] = sendFlags[i];
  }
  a.src = (const char*)src;
  a.dst = (char*)dst;
  a.nElts = nElts;
  a.redArg = redOpArg;
  a.status = status;
  a.timeoutTicks = (uint64_t)(timeoutUs ? timeoutUs : 1000000u) * 100u;
  a.nRecv = nRecv;
  a.nSend = nSend;
  a.srcIsInput = srcIsInput ? 1 : 0;
  a.postOp = postOp ? 1 : 0;
  llSemantics(&datatype, &devRedOp, &a.srcIsInput, &a.postOp, &a.firstWins);
  const uint64_t nUnits = (nElts * typeSize(datatype) + kLL128SliceData - 1) / kLL128SliceData * 128;
  uint64_t grid = (nUnits + kLL128TileUnits - 1) / kLL128TileUnits;
  if (grid > (1u << 20)) grid = 1u << 20;
  NEXR_HIP(launch_ll128(datatype, a, devRedOp, (int)grid, (hipStream_t)stream));
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrSetSemantics(int mode) {
  if (mode < 0 || mode >= nexrNumSemantics) return nexrInvalidArgument;
  gSemantics.store(mode, std::memory_order_relaxed);
  return nexrSuccess;
}

NEXR_API nexrResult_t nexrGetSemantics(int* mode) {
  if (mode == nullptr) return nexrInvalidArgument;
  *mode = semantics();
  return nexrSuccess;
}

NEXR_API size_t nexrTypeSize(int datatype) { return typeSize(datatype); }

NEXR_API const char* nexrGetErrorString(nexrResult_t result) {
  switch (result) {
    case nexrSuccess: return "no error";
    case nexrUnhandledCudaError: return "unhandled HIP error (run with nexrGetLastHipError for details)";
    case nexrSystemError: return "unhandled system error";
    case nexrInternalError: return "internal error";
    case nexrInvalidArgument: return "invalid argument";
    case nexrInvalidUsage: return "invalid usage";
    case nexrRemoteError: return "remote process exited or there was a network error";
    case nexrInProgress: return "operation in progress";
    default: return "unknown result code";
  }
}

NEXR_API int nexrGetVersion(void) {
  return NEXR_VERSION_MAJOR * 10000 + NEXR_VERSION_MINOR * 100 + NEXR_VERSION_PATCH;
}

NEXR_API int nexrGetLastHipError(void) { return tLastHipError; }

}  // extern "C"
