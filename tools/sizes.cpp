// Throughput and per-call time of nexrReduceCopy (the product ABI) across message sizes, fp32 sum,
// K=2 M=1, back-to-back launches on one stream, 3 rotating buffer sets (tuning harness).
//   hipcc -O2 -std=c++17 tools/sizes.cpp -Lnex-nccl_amd -lnexr -Wl,-rpath,$PWD/nex-nccl_amd -o tools/sizes
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../include/nexr.h"
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  const size_t sizes[] = {4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20};
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("%12s %10s %12s %12s\n", "bytes/buf", "us/call", "GB/s(alg)", "launches");
  for (size_t bytes : sizes) {
    const int R = 3;
    void *a[R], *b[R], *o[R];
    for (int r = 0; r < R; r++) {
      CK(hipMalloc(&a[r], bytes)); CK(hipMalloc(&b[r], bytes)); CK(hipMalloc(&o[r], bytes));
      CK(hipMemset(a[r], 0x3c, bytes)); CK(hipMemset(b[r], 0x3d, bytes));
    }
    const size_t n = bytes / 4;
    const int iters = bytes >= (64 << 20) ? 50 : 2000;
    auto call = [&](int r) {
      const void* srcs[2] = {a[r], b[r]};
      void* dsts[1] = {o[r]};
      return nexrReduceCopy(2, srcs, 1, dsts, n, nexrFloat32, nexrDevSum, 0, 0, nullptr, 0, s);
    };
    for (int w = 0; w < 20; w++) call(w % R);
    CK(hipStreamSynchronize(s));
    std::vector<float> best;
    for (int rep = 0; rep < 5; rep++) {
      CK(hipEventRecord(e0, s));
      for (int i = 0; i < iters; i++) call(i % R);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best.push_back(ms / iters);
    }
    std::sort(best.begin(), best.end());
    float ms = best[best.size() / 2];
    printf("%12zu %10.2f %12.1f %12d\n", bytes, ms * 1e3, 3.0 * bytes / ms / 1e6, iters);
    for (int r = 0; r < R; r++) { (void)hipFree(a[r]); (void)hipFree(b[r]); (void)hipFree(o[r]); }
  }

  // Batched: W independent works of `bytes` each, one nexrReduceCopyBatch call vs W nexrReduceCopy calls.
  const int W = NEXR_MAX_BATCH_WORKS;
  printf("\nbatch of %d works (fp32 sum K=2 M=1)\n%12s %14s %14s %14s %14s %14s %14s\n", W, "bytes/work",
         "sep us/work", "batch us/work", "graph us/work", "host us/call", "sep GB/s", "batch GB/s");
  const size_t bsizes[] = {4 << 10, 64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20};
  for (size_t bytes : bsizes) {
    std::vector<void*> a(W), b(W), o(W);
    for (int w = 0; w < W; w++) {
      CK(hipMalloc(&a[w], bytes)); CK(hipMalloc(&b[w], bytes)); CK(hipMalloc(&o[w], bytes));
      CK(hipMemset(a[w], 0x3c, bytes)); CK(hipMemset(b[w], 0x3d, bytes));
    }
    std::vector<nexrReduceCopyWork> works(W);
    for (int w = 0; w < W; w++) {
      nexrReduceCopyWork& x = works[w];
      memset(&x, 0, sizeof(x));
      x.nSrcs = 2; x.nDsts = 1; x.srcs[0] = a[w]; x.srcs[1] = b[w]; x.dsts[0] = o[w]; x.nElts = bytes / 4;
    }
    const int iters = bytes >= (16 << 20) ? 50 : 500;
    auto sep = [&]() {
      for (int w = 0; w < W; w++)
        nexrReduceCopy(2, works[w].srcs, 1, works[w].dsts, works[w].nElts, nexrFloat32, nexrDevSum, 0, 0, nullptr, 0, s);
    };
    auto bat = [&]() { nexrReduceCopyBatch(works.data(), W, nexrFloat32, nexrDevSum, s); };
    // mode 2: the W separate calls captured once into a HIP graph and replayed.
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    sep();
    CK(hipStreamEndCapture(s, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    auto run = [&](int mode) {
      if (mode == 0) sep();
      else if (mode == 1) bat();
      else (void)hipGraphLaunch(exec, s);
    };
    // host-side cost of one nexrReduceCopy call (enqueue only)
    CK(hipStreamSynchronize(s));
    auto h0 = std::chrono::steady_clock::now();
    for (int i = 0; i < 200; i++) sep();
    auto h1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    const double hostUs = std::chrono::duration<double, std::micro>(h1 - h0).count() / (200.0 * W);
    float res[3];
    for (int mode = 0; mode < 3; mode++) {
      for (int i = 0; i < 10; i++) run(mode);
      CK(hipStreamSynchronize(s));
      std::vector<float> best;
      for (int rep = 0; rep < 5; rep++) {
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < iters; i++) run(mode);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best.push_back(ms / iters / W);
      }
      std::sort(best.begin(), best.end());
      res[mode] = best[best.size() / 2];
    }
    printf("%12zu %14.3f %14.3f %14.3f %14.3f %14.1f %14.1f\n", bytes, res[0] * 1e3, res[1] * 1e3, res[2] * 1e3, hostUs,
           3.0 * bytes / res[0] / 1e6, 3.0 * bytes / res[1] / 1e6);
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    for (int w = 0; w < W; w++) { (void)hipFree(a[w]); (void)hipFree(b[w]); (void)hipFree(o[w]); }
  }
  return 0;
}
