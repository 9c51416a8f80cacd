// How the HBM read rate depends on the number of concurrent input streams read at the same
// offsets (the access shape of a K-input reduce-copy), with and without the output stream.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DNEXR_DT=7 tools/streams.hip -o tools/streams
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
using namespace nexr;

struct Srcs { const char* p[8]; };

// S streams, U packs per lane, xor-fold, optional store of the fold (W=1)
template <int S, int U, int W>
__global__ __launch_bounds__(256) void k_streams(Srcs s, char* o, size_t nPacks) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  if (i + (U - 1) * 256 >= nPacks) return;
  u32x4 v[U][S];
#pragma unroll
  for (int k = 0; k < S; k++)
#pragma unroll
    for (int u = 0; u < U; u++) v[u][k] = ld16<1>(s.p[k] + (i + u * 256) * 16);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 a = v[u][0];
#pragma unroll
    for (int k = 1; k < S; k++) a ^= v[u][k];
    if (W) st16<2>(o + (i + u * 256) * 16, a);
    else if (a.x == 0x9e3779b9u && a.y == 1u) *(u32x4*)o = a;
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)256 << 20, P = bytes / 16;
  const int R = 3, iters = argc > 1 ? atoi(argv[1]) : 4;
  std::vector<Srcs> ss(R);
  std::vector<char*> outs(R);
  for (int r = 0; r < R; r++) {
    for (int k = 0; k < 8; k++) { char* q; CK(hipMalloc((void**)&q, bytes)); CK(hipMemset(q, 0x11 * (k + 1), bytes)); ss[r].p[k] = q; }
    CK(hipMalloc((void**)&outs[r], bytes));
  }
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  auto bench = [&](const char* name, double alg, auto launch) {
    std::vector<float> ms;
    for (int it = 0; it < iters; it++) {
      launch(it % R);
      CK(hipEventRecord(e0));
      for (int b = 0; b < 10; b++) launch((it + b) % R);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float t; CK(hipEventElapsedTime(&t, e0, e1)); ms.push_back(t / 10);
    }
    std::sort(ms.begin(), ms.end());
    printf("%-28s %8.1f us %7.0f GB/s\n", name, ms[ms.size() / 2] * 1e3, alg / ms[ms.size() / 2] / 1e6);
  };
  const int g = (int)(P / 1024);
#define RUN(S, U, W) bench("S=" #S " U=" #U " W=" #W, (double)(S + W) * bytes, [&](int r) { k_streams<S, U, W><<<(int)(P / (256 * U)), 256>>>(ss[r], outs[r], P); });
  RUN(1, 4, 0) RUN(2, 4, 0) RUN(4, 4, 0) RUN(8, 4, 0) RUN(8, 2, 0) RUN(8, 1, 0)
  RUN(1, 4, 1) RUN(2, 4, 1) RUN(4, 4, 1) RUN(8, 4, 1) RUN(8, 2, 1) RUN(8, 1, 1)
  (void)g;
  return 0;
}
