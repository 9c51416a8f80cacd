// Cache-policy sweep (buffer_load / buffer_store aux bits: 1 = sc0, 2 = nt, 16 = sc1) for the
// K-read + 1-write stream of a reduce-copy (tuning harness).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/cachepol.hip -o tools/cachepol
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct Srcs { const char* p[8]; };

template <int S, int LAUX, int SAUX>
__global__ __launch_bounds__(256) void k(Srcs s, char* o, uint32_t bytes) {
  constexpr int U = 4;
  const uint32_t i = (blockIdx.x * 256 * U + threadIdx.x) * 16;
  u32x4 v[U][S];
#pragma unroll
  for (int q = 0; q < S; q++) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)s.p[q], 0, bytes, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) v[u][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, i + u * 4096, 0, LAUX));
  }
  __amdgpu_buffer_rsrc_t w = __builtin_amdgcn_make_buffer_rsrc((void*)o, 0, bytes, 0x00020000);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 a = v[u][0];
#pragma unroll
    for (int q = 1; q < S; q++) a += v[u][q];
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, a), w, i + u * 4096, 0, SAUX);
  }
}

int main(int argc, char** argv) {
  const size_t bytes = (size_t)256 << 20, P = bytes / 16;
  const int R = 3, iters = argc > 1 ? atoi(argv[1]) : 4;
  std::vector<Srcs> ss(R);
  std::vector<char*> outs(R);
  for (int r = 0; r < R; r++) {
    for (int q = 0; q < 8; q++) { char* p; CK(hipMalloc((void**)&p, bytes)); CK(hipMemset(p, 0x11 * (q + 1), bytes)); ss[r].p[q] = p; }
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
    printf("%-32s %8.1f us %7.0f GB/s\n", name, ms[ms.size() / 2] * 1e3, alg / ms[ms.size() / 2] / 1e6);
  };
  const int g = (int)(P / 1024);
#define RUN(S, L, W) bench("S=" #S " load=" #L " store=" #W, (double)(S + 1) * bytes, [&](int r) { k<S, L, W><<<g, 256>>>(ss[r], outs[r], (uint32_t)bytes); });
  RUN(2, 2, 2) RUN(2, 2, 0) RUN(2, 2, 16) RUN(2, 2, 17) RUN(2, 2, 18) RUN(2, 2, 1) RUN(2, 2, 3) RUN(2, 18, 2) RUN(2, 16, 2) RUN(2, 0, 2) RUN(2, 3, 2) RUN(2, 19, 19)
  RUN(8, 2, 2) RUN(8, 2, 0) RUN(8, 2, 16) RUN(8, 2, 17) RUN(8, 2, 18) RUN(8, 2, 1) RUN(8, 2, 3) RUN(8, 18, 2) RUN(8, 16, 16) RUN(8, 3, 3) RUN(8, 19, 19)
  return 0;
}
