// Host cost of the stream operations a queued ring step issues (tuning harness): the
// LL step launch (nexrReduceCopyLL, 32 KiB of data = one C1 LL step), hipStreamWriteValue32 (the
// completion ticket), hipEventRecord, hipStreamWaitEvent and hipStreamWaitValue32, each issued 2,000
// times back to back on its own stream; one thread, then two threads on two streams at once (the two
// rank threads of C1). Prints the mean host microseconds per call.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/api_cost_probe.cpp -Lnex-nccl_amd -lnexr -lpthread \
//     -Wl,-rpath,'$ORIGIN/../nex-nccl_amd' -o tools/api_cost_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <thread>
#include <vector>
#include "../include/nexr.h"
#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

struct Lane {
  hipStream_t s;
  char *src, *dst, *lines;
  uint32_t* word;
  hipEvent_t ev;
  uint32_t ticket = 0;
  uint32_t flag = 1;
};

static double timeCalls(int n, const std::function<void(int)>& f) {
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; i++) f(i);
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
  const size_t nElts = 8192;  // 32 KiB of fp32: one C1 LL step
  std::vector<Lane> lanes(2);
  for (Lane& l : lanes) {
    CK(hipStreamCreate(&l.s));
    CK(hipMalloc((void**)&l.src, nElts * 4));
    CK(hipMalloc((void**)&l.dst, nElts * 4));
    CK(hipMalloc((void**)&l.lines, nElts * 4 * 2));
    CK(hipHostMalloc((void**)&l.word, 64, hipHostMallocMapped));
    CK(hipEventCreateWithFlags(&l.ev, hipEventDisableTiming));
    *l.word = 0;
  }
  const int N = 2000;
  auto launchLL = [&](Lane& l) {
    void* send[1] = {l.lines};
    const uint32_t f = l.flag++;
    nexrResult_t r = nexrReduceCopyLL(l.src, 1, 0, nullptr, nullptr, l.dst, 1, send, &f, nElts, nexrFloat32, nexrDevSum,
                                      0, 0, nullptr, 0, l.s);
    if (r != nexrSuccess) {
      printf("nexrReduceCopyLL %d\n", (int)r);
      exit(1);
    }
  };
  struct Op {
    const char* name;
    std::function<void(Lane&)> f;
  } ops[] = {
      {"nexrReduceCopyLL (32 KiB step)", launchLL},
      {"hipStreamWriteValue32", [](Lane& l) { CK(hipStreamWriteValue32(l.s, l.word, ++l.ticket, 0)); }},
      {"hipEventRecord", [](Lane& l) { CK(hipEventRecord(l.ev, l.s)); }},
      {"hipStreamWaitEvent (other lane's event)", nullptr},
      {"hipStreamWaitValue32 (value already there)", [](Lane& l) {
         CK(hipStreamWaitValue32(l.s, l.word, 0, hipStreamWaitValueGte, 0xffffffffu));
       }},
      {"launch + write value (a queued step)", [&](Lane& l) {
         launchLL(l);
         CK(hipStreamWriteValue32(l.s, l.word, ++l.ticket, 0));
       }},
  };
  ops[3].f = [&](Lane& l) { CK(hipStreamWaitEvent(l.s, lanes[&l == &lanes[0] ? 1 : 0].ev, 0)); };
  for (Lane& l : lanes) CK(hipEventRecord(l.ev, l.s));
  for (int w = 0; w < 50; w++)
    for (auto& op : ops) op.f(lanes[0]), op.f(lanes[1]);
  CK(hipDeviceSynchronize());
  printf("%-44s %14s %22s\n", "host us per call", "one thread", "two threads (each)");
  for (auto& op : ops) {
    const double one = timeCalls(N, [&](int) { op.f(lanes[0]); });
    CK(hipDeviceSynchronize());
    double two[2];
    std::thread t0([&] { two[0] = timeCalls(N, [&](int) { op.f(lanes[0]); }); });
    std::thread t1([&] { two[1] = timeCalls(N, [&](int) { op.f(lanes[1]); }); });
    t0.join();
    t1.join();
    CK(hipDeviceSynchronize());
    printf("%-44s %14.2f %10.2f / %-10.2f\n", op.name, one, two[0], two[1]);
  }
  return 0;
}
