// HBM ceilings on this MI355X for the access mixes the reduce-copy uses (tuning harness):
// pure read, pure write, copy (1:1), 2-read:1-write (the K=2 reduce-copy itself), on random vs
// constant data, nt vs default policy. Interleaved rounds in one process.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 -DTK_K=2 tools/hbm_ceiling.hip -o tools/hbm_ceiling
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

using namespace nexr;

__global__ void fill_random(uint32_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    float f = (float)(z >> 40) * (1.0f / 16777216.0f) * 2.0f - 1.0f;
    p[i] = __builtin_bit_cast(uint32_t, f);
  }
}

// pure read: U packs per lane per trip, xor-reduced, one store per thread at the end
template <int NT, int U>
__global__ __launch_bounds__(256) void k_read(const char* a, size_t nPacks, u32x4* sink) {
  u32x4 acc = (u32x4)0u;
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < nPacks; i += (size_t)gridDim.x * 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld16<NT>(a + (i + u * 256) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) acc ^= v[u];
  }
  if (acc.x == 0x12345678u) sink[threadIdx.x] = acc;
}
template <int NT, int U>
__global__ __launch_bounds__(256) void k_write(char* o, size_t nPacks, uint32_t seed) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < nPacks; i += (size_t)gridDim.x * 256 * U) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t x = (uint32_t)(i + u * 256) * 2654435761u ^ seed;
      st16<NT>(o + (i + u * 256) * 16, (u32x4){x, x * 3u, x * 5u, x * 7u});
    }
  }
}
template <int NT, int U>
__global__ __launch_bounds__(256) void k_copy(const char* a, char* o, size_t nPacks) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < nPacks; i += (size_t)gridDim.x * 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld16<NT>(a + (i + u * 256) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) st16<NT>(o + (i + u * 256) * 16, v[u]);
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_copy2(const char* a, char* o, size_t nPacks) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  for (; i + (U - 1) * 256 < nPacks; i += (size_t)gridDim.x * 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) v[u] = ld16<1>(a + (i + u * 256) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) st16<0>(o + (i + u * 256) * 16, v[u]);
  }
}

struct Var {
  std::string name;
  double bytes;
  std::function<void(int)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 15;
  const size_t P = bytes / 16;
  const int R = 3;
  char *A[R], *Bf[R], *O[R], *CA[R], *CB[R];
  for (int r = 0; r < R; r++) {
    CK(hipMalloc((void**)&A[r], bytes));
    CK(hipMalloc((void**)&Bf[r], bytes));
    CK(hipMalloc((void**)&O[r], bytes));
    CK(hipMalloc((void**)&CA[r], bytes));
    CK(hipMalloc((void**)&CB[r], bytes));
    fill_random<<<2048, 256>>>((uint32_t*)A[r], bytes / 4, 11 + r);
    fill_random<<<2048, 256>>>((uint32_t*)Bf[r], bytes / 4, 97 + r);
    CK(hipMemset(CA[r], 0x3c, bytes));
    CK(hipMemset(CB[r], 0x3d, bytes));
  }
  u32x4* sink;
  CK(hipMalloc((void**)&sink, 4096));
  std::vector<RCParams> pr(R), pc(R);
  for (int r = 0; r < R; r++) {
    for (auto* pp : {&pr[r], &pc[r]}) {
      std::memset((void*)pp, 0, sizeof(RCParams));
      pp->nDsts = 1;
      pp->nElts = bytes / 4;
      pp->nPacks = P;
      pp->dst[0] = O[r];
    }
    pr[r].src[0] = A[r];
    pr[r].src[1] = Bf[r];
    pc[r].src[0] = CA[r];
    pc[r].src[1] = CB[r];
  }
  CK(hipDeviceSynchronize());
  std::vector<Var> vs;
  const int g1 = (int)(P / 1024);
  vs.push_back({"reduce K=2 pol0 U4 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 0, 4><<<g1, 256>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol1 U4 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 1, 4><<<g1, 256>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol2 U4 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 2, 4><<<g1, 256>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol3 U4 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 3, 4><<<g1, 256>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol1 U2 B512 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 1, 2, 512><<<g1, 512>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol3 U2 B512 oneshot", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 3, 2, 512><<<g1, 512>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol1 U4 g2048", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 1, 4><<<2048, 256>>>(pr[r]); }, {}});
  vs.push_back({"reduce K=2 pol3 U4 g2048", 3.0 * bytes, [&](int r) { reduce_copy_kernel<7, 0, 2, 3, 4><<<2048, 256>>>(pr[r]); }, {}});
  vs.push_back({"read random nt U4 oneshot", 1.0 * bytes, [&](int r) { k_read<3, 4><<<g1, 256>>>(A[r], P, sink); }, {}});
  vs.push_back({"read random plain U4 oneshot", 1.0 * bytes, [&](int r) { k_read<0, 4><<<g1, 256>>>(A[r], P, sink); }, {}});
  vs.push_back({"read random nt U8 g2048", 1.0 * bytes, [&](int r) { k_read<3, 8><<<2048, 256>>>(A[r], P, sink); }, {}});
  vs.push_back({"read const nt U4 oneshot", 1.0 * bytes, [&](int r) { k_read<3, 4><<<g1, 256>>>(CA[r], P, sink); }, {}});
  vs.push_back({"write nt U4 oneshot", 1.0 * bytes, [&](int r) { k_write<3, 4><<<g1, 256>>>(O[r], P, r); }, {}});
  vs.push_back({"write plain U4 oneshot", 1.0 * bytes, [&](int r) { k_write<0, 4><<<g1, 256>>>(O[r], P, r); }, {}});
  vs.push_back({"copy random nt U4 oneshot", 2.0 * bytes, [&](int r) { k_copy<3, 4><<<g1, 256>>>(A[r], O[r], P); }, {}});
  vs.push_back({"copy const nt U4 oneshot", 2.0 * bytes, [&](int r) { k_copy<3, 4><<<g1, 256>>>(CA[r], O[r], P); }, {}});
  vs.push_back({"copy ntload-plainstore U4 oneshot", 2.0 * bytes, [&](int r) { k_copy2<4><<<g1, 256>>>(A[r], O[r], P); }, {}});
  vs.push_back({"copy random plain U4 oneshot", 2.0 * bytes, [&](int r) { k_copy<0, 4><<<g1, 256>>>(A[r], O[r], P); }, {}});
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
  printf("buffer=%zu MiB iters=%d\n", bytes >> 20, iters);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s med %8.1f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, v.bytes / med / 1e6, v.bytes / mn / 1e6);
  }
  return 0;
}
