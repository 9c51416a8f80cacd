// Host-side copy rates behind nexrReduceCopyHost's copy-team path (tuning harness, not product code):
// T threads memcpy 256 MiB between pageable memory and hipHostMalloc'd pinned memory (default =
// coherent, and non-coherent), each direction, and pageable -> pageable for reference.
//   hipcc -O2 -std=c++17 tools/host_copy_probe.cpp -o tools/host_copy_probe && ./tools/host_copy_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double copyRate(char* dst, const char* src, size_t bytes, int threads, int reps) {
  auto run = [&] {
    std::vector<std::thread> ts;
    const size_t per = (bytes / threads + 4095) & ~(size_t)4095;
    for (int t = 0; t < threads; t++)
      ts.emplace_back([=] {
        const size_t b0 = per * t;
        if (b0 < bytes) memcpy(dst + b0, src + b0, per < bytes - b0 ? per : bytes - b0);
      });
    for (auto& t : ts) t.join();
  };
  run();
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < reps; r++) run();
  double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
  return bytes / s / 1e9;
}

int main() {
  const size_t bytes = 256u << 20;
  char* pa = (char*)aligned_alloc(4096, bytes);
  char* pb = (char*)aligned_alloc(4096, bytes);
  memset(pa, 1, bytes);
  memset(pb, 2, bytes);
  char *coh = nullptr, *nc = nullptr;
  if (hipHostMalloc((void**)&coh, bytes, hipHostMallocDefault) != hipSuccess) return 1;
  if (hipHostMalloc((void**)&nc, bytes, hipHostMallocNonCoherent) != hipSuccess) return 1;
  memset(coh, 3, bytes);
  memset(nc, 4, bytes);
  printf("%-8s %14s %14s %14s %14s %14s\n", "threads", "page->page", "page->pinned", "pinned->page", "page->pinnedNC",
         "pinnedNC->page");
  for (int t : {1, 2, 4, 8, 12, 16}) {
    printf("%-8d %14.1f %14.1f %14.1f %14.1f %14.1f\n", t, copyRate(pb, pa, bytes, t, 5), copyRate(coh, pa, bytes, t, 5),
           copyRate(pb, coh, bytes, t, 5), copyRate(nc, pa, bytes, t, 5), copyRate(pb, nc, bytes, t, 5));
    fflush(stdout);
  }
  return 0;
}
