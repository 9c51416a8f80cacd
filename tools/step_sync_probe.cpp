// What one emulated ring step costs the host, by the way it waits for the step's reduce-copy
// (diagnostic for DESIGN §8.1: "one launch plus hipStreamSynchronize of a 128 KiB-2 MiB reduce-copy costs
// 12.0-12.5 us"). Each iteration launches one nexrReduceCopy (fp32 sum, K = 2, M = 2: the ring's
// recvReduceCopySend shape) on a non-blocking stream and waits for it with:
//   sync       hipStreamSynchronize
//   event      hipEventRecord + hipEventSynchronize
//   query      hipEventRecord + spin on hipEventQuery
//   value      hipStreamWriteValue32 of the iteration number into pinned host memory + spin on it
// Wall time per iteration (steady_clock), median of 2,000 iterations, per size. Tuning harness.
//   hipcc -O2 -std=c++17 -Iinclude tools/step_sync_probe.cpp -Lnex-nccl_amd -lnexr \
//         -Wl,-rpath,$PWD/nex-nccl_amd -o tools/step_sync_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "nexr.h"

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  uint32_t* flag;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocMapped));
  *flag = 0;
  const size_t sizes[] = {32 << 10, 512 << 10, 1 << 20, 2 << 20};
  const size_t maxBytes = 2 << 20;
  void* buf[4];
  for (auto& b : buf) {
    CK(hipMalloc(&b, maxBytes));
    CK(hipMemset(b, 0, maxBytes));
  }
  CK(hipDeviceSynchronize());
  const char* names[] = {"sync", "event", "query", "value"};
  printf("%-8s %10s %10s %10s %10s   (us per launch + wait, median of %d)\n", "bytes", names[0], names[1], names[2],
         names[3], iters);
  uint32_t tick = 0;
  for (size_t bytes : sizes) {
    const size_t n = bytes / 4;
    const void* srcs[2] = {buf[0], buf[1]};
    void* dsts[2] = {buf[2], buf[3]};
    double med[4];
    for (int mode = 0; mode < 4; mode++) {
      std::vector<double> us;
      for (int it = 0; it < iters + 50; it++) {
        auto t0 = std::chrono::steady_clock::now();
        if (nexrReduceCopy(2, srcs, 2, dsts, n, nexrFloat32, nexrDevSum, 0, 0, nullptr, 0, st) != nexrSuccess) {
          fprintf(stderr, "nexrReduceCopy failed\n");
          return 1;
        }
        if (mode == 0) {
          CK(hipStreamSynchronize(st));
        } else if (mode == 1) {
          CK(hipEventRecord(ev, st));
          CK(hipEventSynchronize(ev));
        } else if (mode == 2) {
          CK(hipEventRecord(ev, st));
          hipError_t q;
          while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
          }
          CK(q);
        } else {
          ++tick;
          CK(hipStreamWriteValue32(st, flag, tick, 0));
          auto spin0 = std::chrono::steady_clock::now();
          while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != tick) {
            if (std::chrono::steady_clock::now() - spin0 > std::chrono::seconds(5)) {
              fprintf(stderr, "write-value never arrived\n");
              return 1;
            }
          }
        }
        auto t1 = std::chrono::steady_clock::now();
        if (it >= 50) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      CK(hipStreamSynchronize(st));
      std::sort(us.begin(), us.end());
      med[mode] = us[us.size() / 2];
    }
    printf("%-8zu %10.2f %10.2f %10.2f %10.2f\n", bytes, med[0], med[1], med[2], med[3]);
  }
  return 0;
}
