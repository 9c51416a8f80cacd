// Geometry sweep of the PRODUCTION reduce-copy kernel (nexr_kernels.hip included directly) on
// random data, interleaved rounds in one process (tuning harness, not product code).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 -DTK_K=2 \
//         tools/tune_kernel.hip -o tools/tune_kernel_dt7_k2
//   ./tools/tune_kernel_dt7_k2 <MiB per buffer> <iters>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#ifndef TK_K
#define TK_K 2
#endif
#ifndef TK_OP
#define TK_OP 0
#endif

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

__global__ void fill_random(uint32_t* p, size_t n, uint64_t seed, int dt) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint32_t v;
    if (dt == nexrFloat32) {
      float f = (float)(z >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
      v = __builtin_bit_cast(uint32_t, f);
    } else if (dt == nexrFloat16) {
      _Float16 a = (_Float16)((float)(z >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f);
      _Float16 b = (_Float16)((float)((z >> 16) & 0xffffff) * (1.0f / 16777216.0f) * 2.0f - 1.0f);
      v = __builtin_bit_cast(uint16_t, a) | ((uint32_t)__builtin_bit_cast(uint16_t, b) << 16);
    } else if (dt == nexrBfloat16) {
      float a = (float)(z >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
      float b = (float)((z >> 16) & 0xffffff) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
      v = (__builtin_bit_cast(uint32_t, a) >> 16) | (__builtin_bit_cast(uint32_t, b) & 0xffff0000u);
    } else {
      v = (uint32_t)z;
    }
    p[i] = v;
  }
}

using namespace nexr;
struct Var {
  std::string name;
  std::function<void(int)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const size_t skew = argc > 3 ? (size_t)atol(argv[3]) : 0;
  constexpr int D = NEXR_DT, K = TK_K, OP = TK_OP;
  constexpr int esz = 16 / Ty<D>::EPP;
  const int R = 3;
  std::vector<RCParams> ps(R);
  for (int r = 0; r < R; r++) {
    RCParams& p = ps[r];
    std::memset((void*)&p, 0, sizeof(p));
    char* base;
    CK(hipMalloc((void**)&base, (K + 1) * (bytes + (K + 1) * skew) + 4096));
    for (int s = 0; s < K; s++) {
      char* q = base + s * (bytes + skew * (s + 1));
      fill_random<<<2048, 256>>>((uint32_t*)q, bytes / 4, 1000 + r * 16 + s, D);
      p.src[s] = (const char*)q;
    }
    p.dst[0] = base + K * (bytes + skew * (K + 1));
    p.nDsts = 1;
    p.nElts = bytes / esz;
    p.nPacks = bytes / 16;
    p.redArg = (OP == nexrDevMinMax) ? 0 : 0;
  }
  CK(hipDeviceSynchronize());
  std::vector<Var> vs;
  const double alg = (double)(K + 1) * bytes;
#define V(POL, U, B, G)                                                                               \
  vs.push_back({"pol=" #POL " U=" #U " B=" #B " grid=" + std::to_string(G), [&, g = (G)](int r) {    \
                  reduce_copy_kernel<D, OP, K, POL, U, B><<<g, B>>>(ps[r]);                           \
                }, {}});
  const int P = (int)(bytes / 16);
  V(3, 4, 256, P / 1024) V(3, 2, 256, P / 512) V(3, 1, 256, P / 256) V(3, 1, 1024, P / 1024)
  V(1, 4, 256, P / 1024) V(3, 8, 256, P / 2048) V(3, 2, 512, P / 1024)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  // Steady state: each variant runs BLK launches back to back (rotating buffers) between two
  // events, so dirty lines a plain-store variant leaves in L2/MALL are paid by itself, not by
  // the next variant.
  const int BLK = 10;
  for (int it = 0; it < iters; it++)
    for (auto& v : vs) {
      v.run((it + BLK - 1) % R);
      CK(hipEventRecord(e0));
      for (int b = 0; b < BLK; b++) v.run((it + b) % R);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / BLK);
    }
  printf("dt=%d K=%d op=%d buffer=%zu MiB skew=%zu alg bytes=%.0f\n", D, K, OP, bytes >> 20, skew, alg);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-28s med %8.1f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, alg / med / 1e6, alg / mn / 1e6);
  }
  return 0;
}
