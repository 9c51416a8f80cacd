// Where the time of a device LL run goes (tuning harness): C1's LL schedule (fp32 sum
// all-reduce of 4 MiB per rank over 2 ranks: 64 loops of send / recvReduceCopySend / recv, 32 KiB of
// data per step, 64 KiB slots, 8 slots, 96 steps per launch) run straight through the run kernel of
// nex-nccl_amd/csrc/nexr_ll.hip, compiled here with its per-step timestamps on (NEXR_LL_STEPS_TRACE:
// lane 0 of every workgroup stamps step start, after the credit, after the tile, after the end-of-step
// barrier, after postRecv, with s_memrealtime, 100 MHz). Two ranks on two own-queue streams; 10 calls;
// the last call's stamps summarised per step kind, and the kernel time of each launch from events.
// Without NEXR_LL_STEPS_TRACE only the kernel times (A/B of the NEXR_LL_* tuning macros of nexr_ll.hip).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNEXR_LL_STEPS_TRACE [-DNEXR_LL_CLOCK_EVERY=16] \
//     tools/ll_steps_trace.hip -o tools/ll_steps_trace
#include "../nex-nccl_amd/csrc/nexr_ll.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

using namespace nexr;

int main() {
  const int nRanks = 2, loops = 64, slots = 8;
  const uint64_t slot = 64 << 10, chunk = slot / 2 / 4;  // fp32 elements per step
  const uint64_t count = (uint64_t)loops * nRanks * chunk;  // 1 Mi elements = 4 MiB per rank
  const int grid = (int)(slot / 16 / kLLTileLines);
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
  // LL_TRACE_MASK (A/B of placement): "full" (default), "same" (both ranks on logical CUs 0-31),
  // "split" (rank 0 on 0-31, rank 1 on 32-63)
  const char* mm = getenv("LL_TRACE_MASK");
  const std::string maskMode = mm ? mm : "full";
  hipStream_t st[2];
  char *in[2], *out[2], *fifo[2];
  uint64_t* tr[2];
  uint32_t* status;
  CK(hipHostMalloc((void**)&status, 64, hipHostMallocMapped));
  memset(status, 0, 64);
  for (int r = 0; r < nRanks; r++) {
    std::vector<uint32_t> m = mask;
    if (maskMode != "full") {
      for (auto& x : m) x = 0;
      m[maskMode == "split" ? r : 0] = 0xffffffffu;
    }
    CK(hipExtStreamCreateWithCUMask(&st[r], (uint32_t)m.size(), m.data()));
    CK(hipMalloc((void**)&in[r], count * 4));
    CK(hipMalloc((void**)&out[r], count * 4));
    CK(hipMalloc((void**)&fifo[r], slot * slots + NEXR_LL_HEAD_BYTES));  // FIFO INTO rank r
    CK(hipMemset(fifo[r], 0, slot * slots + NEXR_LL_HEAD_BYTES));
    CK(hipMemset(in[r], 0, count * 4));
    CK(hipMalloc((void**)&tr[r], (size_t)grid * kLLStepsMax * 5 * 8));
  }
  // Rank r's steps of one call (runRing of all_reduce.h for 2 ranks): per loop, send chunk (r + 1) % 2
  // of the input, recvReduceCopySend chunk r into the output, recv chunk (r + 1) % 2 into the output.
  auto schedule = [&](int r) {
    std::vector<nexrLLStep> s;
    for (int l = 0; l < loops; l++) {
      const int64_t base = (int64_t)l * nRanks * chunk;
      const int64_t cSend = base + ((r + 1) % 2) * chunk, cOwn = base + r * chunk;
      nexrLLStep a{}, b{}, c{};
      a.srcBuf = 0, a.dstBuf = -1, a.srcIx = cSend, a.nElts = (uint32_t)chunk, a.send = 1;
      b.srcBuf = 0, b.dstBuf = 1, b.srcIx = cOwn, b.dstIx = cOwn, b.nElts = (uint32_t)chunk, b.recv = 1, b.send = 1;
      c.srcBuf = -1, c.dstBuf = 1, c.dstIx = cSend, c.nElts = (uint32_t)chunk, c.recv = 1;
      s.push_back(a), s.push_back(b), s.push_back(c);
    }
    return s;
  };
  const std::vector<nexrLLStep> sched[2] = {schedule(0), schedule(1)};
  uint64_t rs[2] = {0, 0}, ss[2] = {0, 0};
  hipEvent_t ev[2][3][2];
  for (auto& a : ev)
    for (auto& b : a)
      for (auto& e : b) CK(hipEventCreate(&e));
  double callMs = 0;
  for (int call = 0; call < 10; call++) {
    CK(hipDeviceSynchronize());
    for (int launch = 0; launch * kLLStepsMax < (int)sched[0].size(); launch++) {
      for (int r = 0; r < nRanks; r++) {
        LLStepsParams P;
        memset(&P, 0, sizeof(P));
        P.input = in[r];
        P.output = out[r];
        P.recvFifo[0] = fifo[r];
        P.recvHead[0] = (uint64_t*)(fifo[r] + slot * slots);
        P.sendFifo[0] = fifo[(r + 1) % 2];
        P.sendHead[0] = (const uint64_t*)(fifo[(r + 1) % 2] + slot * slots);
        P.recvStep[0] = rs[r];
        P.sendStep[0] = ss[r];
        P.slotBytes = slot;
        P.status = status + r;
        P.timeoutTicks = 100000000ull;  // 1 s
        P.nRecv = P.nSend = 1;
        P.nSlots = slots;
#ifdef NEXR_LL_STEPS_TRACE
        P.trace = tr[r];
#endif
        const int first = launch * kLLStepsMax;
        P.nSteps = std::min<int>(kLLStepsMax, (int)sched[r].size() - first);
        for (int k = 0; k < P.nSteps; k++) {
          P.step[k] = sched[r][first + k];
          rs[r] += P.step[k].recv;
          ss[r] += P.step[k].send;
        }
        CK(hipEventRecord(ev[r][launch][0], st[r]));
        CK(launch_ll_steps(nexrFloat32, P, nexrDevSum, grid, st[r]));
        CK(hipEventRecord(ev[r][launch][1], st[r]));
      }
    }
    CK(hipDeviceSynchronize());
    if (status[0] || status[1]) {
      printf("status %u %u\n", status[0], status[1]);
      return 1;
    }
    float ms = 0, tot = 0;
    for (int launch = 0; launch < 2; launch++) {
      CK(hipEventElapsedTime(&ms, ev[0][launch][0], ev[0][launch][1]));
      tot += ms;
    }
    callMs = tot;
    printf("call %d: rank 0 kernels %.1f us\n", call, tot * 1e3);
  }
#ifndef NEXR_LL_STEPS_TRACE
  printf("last call: rank 0 kernels %.1f us for %zu steps\n", callMs * 1e3, sched[0].size());
  return 0;
#endif
  // The last call's stamps (second launch of rank 0, every workgroup): per step kind (k % 3), the mean
  // of each phase in microseconds, and the whole step.
  std::vector<uint64_t> h((size_t)grid * kLLStepsMax * 5);
  for (int r = 0; r < 1; r++) {
    CK(hipMemcpy(h.data(), tr[r], h.size() * 8, hipMemcpyDeviceToHost));
    double ph[3][5] = {}, n[3] = {};
    for (int w = 0; w < grid; w++)
      for (int k = 1; k < kLLStepsMax; k++) {
        const uint64_t* t = &h[((size_t)w * kLLStepsMax + k) * 5];
        const uint64_t* tp = &h[((size_t)w * kLLStepsMax + k - 1) * 5];
        const int kind = (kLLStepsMax + k) % 3;  // the second launch starts at step 96 = 0 mod 3
        ph[kind][0] += (t[1] - t[0]) / 100.0;   // credit
        ph[kind][1] += (t[2] - t[1]) / 100.0;   // tile: loads, polls, fold, stores issued
        ph[kind][2] += (t[3] - t[2]) / 100.0;   // end-of-step barrier
        ph[kind][3] += (t[4] - t[3]) / 100.0;   // postRecv
        ph[kind][4] += (t[0] - tp[4]) / 100.0;  // between steps (kernel-argument reads)
        n[kind]++;
      }
    const char* names[3] = {"send", "recvReduceCopySend", "recv"};
    printf("rank %d, us per step (mean over %d workgroups): credit / tile / barrier / postRecv / gap\n", r, grid);
    for (int kind = 0; kind < 3; kind++)
      printf("  %-20s %6.2f %6.2f %6.2f %6.2f %6.2f\n", names[kind], ph[kind][0] / n[kind], ph[kind][1] / n[kind],
             ph[kind][2] / n[kind], ph[kind][3] / n[kind], ph[kind][4] / n[kind]);
    const uint64_t* a = &h[0];
    const uint64_t* b = &h[(size_t)(kLLStepsMax - 1) * 5];
    printf("  workgroup 0: %d steps in %.1f us (%.2f us per step)\n", kLLStepsMax, (b[4] - a[0]) / 100.0,
           (b[4] - a[0]) / 100.0 / kLLStepsMax);
  }
  printf("last call: rank 0 kernels %.1f us for %zu steps\n", callMs * 1e3, sched[0].size());
  return 0;
}
