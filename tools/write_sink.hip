// Where does the write stream's cost arise? (diagnostic for DESIGN §6.3 (docs/HISTORY.md §6): 8 read streams alone stream at
// ~6.6-6.8 TB/s, with one write stream beside them at ~5.9-6.05.) S read streams (fold = xor), then the
// write stream in one of these forms:
//   none        no store (the fold is kept live by a never-taken store)
//   hbm         the reduce-copy's store: pack i to out + 16 i (256 MiB, written to HBM), nt
//   win 512K    the same store instructions, addresses folded into a 512 KiB window (out + 16 (i mod
//               2^15), plain stores): the lines stay dirty in each XCD's 4 MiB L2 and almost nothing
//               leaves the XCD — the cost of the stores up to the L2
//   win 64M     a 64 MiB window: more than an L2, less than the 256 MiB Infinity Cache — the lines are
//               written back across the fabric into the memory-side cache but (mostly) not to DRAM
//   half_hbm    every second wave-instruction's store to HBM (nt), the others into the 512 KiB window
// Reads are the production kernel's (nt, 16 B per lane, one-shot grid of 256 x 4 packs); median of
// blocks of 10 launches over 3 rotating buffer sets. Tuning harness, not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNEXR_DT=7 tools/write_sink.hip -o tools/write_sink
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                  \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)
using namespace nexr;

struct Srcs {
  const char* p[8];
};
// MODE: 0 none, 1 hbm, 2 half_hbm, >= 8: window of 2^MODE packs
enum { kNone = 0, kHbm = 1, kHalf = 2, kWinL2 = 15, kWinMall = 22 };

template <int S, int MODE>
__global__ __launch_bounds__(256) void k_sink(Srcs s, char* o, size_t nPacks) {
  constexpr int U = 4;
  const size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  if (i + (U - 1) * 256 >= nPacks) return;
  u32x4 v[U][S];
#pragma unroll
  for (int k = 0; k < S; k++)
#pragma unroll
    for (int u = 0; u < U; u++) v[u][k] = ld16<kPolNt>(s.p[k] + (i + u * 256) * 16);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 a = v[u][0];
#pragma unroll
    for (int k = 1; k < S; k++) a ^= v[u][k];
    const size_t j = i + u * 256;
    if constexpr (MODE == kNone) {
      if (a.x == 0x9e3779b9u && a.y == 1u) *(u32x4*)o = a;
    } else if constexpr (MODE == kHbm) {
      st16<kPolNt>(o + j * 16, a);
    } else if constexpr (MODE == kHalf) {
      if (u & 1) st16<kPolPlain>(o + (j & ((1ull << kWinL2) - 1)) * 16, a);
      else st16<kPolNt>(o + j * 16, a);
    } else {
      st16<kPolPlain>(o + (j & ((1ull << MODE) - 1)) * 16, a);
    }
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)256 << 20, P = bytes / 16;
  const int R = 3, iters = argc > 1 ? atoi(argv[1]) : 8;
  std::vector<Srcs> ss(R);
  std::vector<char*> outs(R);
  for (int r = 0; r < R; r++) {
    for (int k = 0; k < 8; k++) {
      char* q;
      CK(hipMalloc((void**)&q, bytes));
      CK(hipMemset(q, 0x11 * (k + 1) + r, bytes));
      ss[r].p[k] = q;
    }
    CK(hipMalloc((void**)&outs[r], bytes));
  }
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = (int)(P / 1024);
  struct Case {
    const char* name;
    int s, mode;
    void (*fn)(Srcs, char*, size_t);
    std::vector<float> ms;
  };
  std::vector<Case> cs;
#define CASES(S)                                                           \
  cs.push_back({#S "R none", S, kNone, k_sink<S, kNone>, {}});             \
  cs.push_back({#S "R + W hbm", S, kHbm, k_sink<S, kHbm>, {}});            \
  cs.push_back({#S "R + W win 512K", S, kWinL2, k_sink<S, kWinL2>, {}});   \
  cs.push_back({#S "R + W win 64M", S, kWinMall, k_sink<S, kWinMall>, {}}); \
  cs.push_back({#S "R + W half_hbm", S, kHalf, k_sink<S, kHalf>, {}});
  CASES(2) CASES(4) CASES(8)
  for (auto& c : cs)
    for (int w = 0; w < 2; w++) c.fn<<<grid, 256>>>(ss[w % R], outs[w % R], P);
  CK(hipDeviceSynchronize());
  const int BLK = 10;
  for (int it = 0; it < iters; it++)
    for (auto& c : cs) {
      CK(hipEventRecord(e0));
      for (int b = 0; b < BLK; b++) c.fn<<<grid, 256>>>(ss[(it + b) % R], outs[(it + b) % R], P);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      c.ms.push_back(ms / BLK);
    }
  printf("median of %d blocks of %d launches, 256 MiB per stream; GB/s of HBM bytes (reads + written-to-HBM)\n",
         iters, BLK);
  for (auto& c : cs) {
    std::sort(c.ms.begin(), c.ms.end());
    const float med = c.ms[c.ms.size() / 2];
    const double rd = (double)c.s * bytes;
    const double wr = c.mode == kHbm ? (double)bytes : c.mode == kHalf ? bytes / 2.0 : 0.0;
    printf("%-18s %8.2f us  reads %6.0f GB/s  HBM total %6.0f GB/s  (all stored bytes %6.0f GB/s)\n", c.name,
           med * 1e3, rd / med / 1e6, (rd + wr) / med / 1e6,
           (rd + (c.mode == kNone ? 0.0 : (double)bytes)) / med / 1e6);
  }
  return 0;
}
