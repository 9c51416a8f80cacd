// Cache-control bits of the reduce-copy's loads and stores (tuning harness, not product code).
//
// Question: the production kernel streams with `nt` loads and `nt` stores (the only two policies
// hipcc's builtins reach: __builtin_nontemporal_load/_store). gfx950's vector memory instructions
// carry three bits — sc0, sc1, nt — and MI355X_MICROARCH.md (stores of each flavour) says plain /
// sc0 / nt stores KEEP the line in the XCD's L2 while sc1 / sc0 sc1 DROP it (write-through). Does
// any other combination move the HBM rate of the write stream (the K = 8 configurations lose ~10 %
// to the read/write mix, DESIGN §6.3 (docs/HISTORY.md §6)) or of the read streams?
//
// Each variant is the production trip (same geometry: unroll_for / block_for, one-shot grid, same
// fold: Fold<> from nexr_kernels.hip) with either the stores or the loads issued as
// raw_buffer_{load,store}_b128 with explicit aux bits (bit 0 sc0, bit 1 nt, bit 4 sc1) through a
// per-trip buffer descriptor built from kernel arguments and blockIdx (wave-uniform). Every
// variant's output is compared byte for byte with the production kernel's before timing.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 -DTK_K=2 \
//         tools/cache_bits.hip -o tools/cache_bits_dt7_k2
//   ./tools/cache_bits_dt7_k2 <MiB per buffer> <iters>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#ifndef TK_K
#define TK_K 2
#endif

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

using namespace nexr;

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0x83ff83ffu;  // small finite values for every float type
  }
}

// LAUX / SAUX: aux bits of the buffer loads / stores, or -1 for the production global nt access.
template <int D, int K, int U, int B, int LAUX, int SAUX>
__global__ __launch_bounds__(B) void k_bits(RCParams p) {
  Fold<D, nexrDevSum, K, false> f(p);
  constexpr uint32_t tile = (uint32_t)B * U * 16;
  const uint64_t base = (uint64_t)blockIdx.x * tile;
  u32x4 in[U][K];
#pragma unroll
  for (int s = 0; s < K; s++) {
    if constexpr (LAUX < 0) {
#pragma unroll
      for (int u = 0; u < U; u++) in[u][s] = ld16<kPolNt>(p.src[s] + base + (threadIdx.x + u * B) * 16);
    } else {
      auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(p.src[s] + base), 0, tile, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++)
        in[u][s] = bc<u32x4>(__builtin_amdgcn_raw_buffer_load_b128(r, (threadIdx.x + u * B) * 16, 0, LAUX));
    }
  }
  u32x4 out[U];
#pragma unroll
  for (int u = 0; u < U; u++) out[u] = f.run(in[u]);
  if constexpr (SAUX < 0) {
#pragma unroll
    for (int u = 0; u < U; u++) st16<kPolNt>(p.dst[0] + base + (threadIdx.x + u * B) * 16, out[u]);
  } else {
    auto r = __builtin_amdgcn_make_buffer_rsrc((void*)(p.dst[0] + base), 0, tile, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) __builtin_amdgcn_raw_buffer_store_b128(out[u], r, (threadIdx.x + u * B) * 16, 0, SAUX);
  }
}

struct Var {
  std::string name;
  std::function<void(int)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 8;
  constexpr int D = NEXR_DT, K = TK_K;
  constexpr int esz = 16 / Ty<D>::EPP;
  constexpr int U = unroll_for(D, K, kPolNt), B = block_for(D, K, kPolNt);
  const int R = 3;  // rotating buffer sets, as the bench
  std::vector<RCParams> ps(R);
  for (int r = 0; r < R; r++) {
    RCParams& p = ps[r];
    std::memset((void*)&p, 0, sizeof(p));
    for (int s = 0; s < K; s++) {
      char* q;
      CK(hipMalloc((void**)&q, bytes));
      fill_bits<<<2048, 256>>>((uint32_t*)q, bytes / 4, 1000 + r * 16 + s);
      p.src[s] = q;
    }
    CK(hipMalloc((void**)&p.dst[0], bytes));
    p.nDsts = 1;
    p.nElts = bytes / esz;
    p.nPacks = bytes / 16;
  }
  CK(hipDeviceSynchronize());
  const double alg = (double)(K + 1) * bytes;
  const int grid = (int)(bytes / 16 / (U * B));
  std::vector<Var> vs;
  vs.push_back({"production (global nt ld, nt st)",
                [&](int r) { reduce_copy_kernel<D, nexrDevSum, K, kPolNt, U, B><<<grid, B>>>(ps[r]); }, {}});
#define VS(SAUX, NAME) \
  vs.push_back({"st " NAME, [&](int r) { k_bits<D, K, U, B, -1, SAUX><<<grid, B>>>(ps[r]); }, {}});
#define VL(LAUX, NAME) \
  vs.push_back({"ld " NAME, [&](int r) { k_bits<D, K, U, B, LAUX, -1><<<grid, B>>>(ps[r]); }, {}});
  VS(-1, "global nt (= production)")
  VS(0, "buffer plain") VS(2, "buffer nt") VS(1, "buffer sc0") VS(3, "buffer sc0 nt") VS(16, "buffer sc1")
  VS(18, "buffer sc1 nt") VS(17, "buffer sc0 sc1") VS(19, "buffer sc0 sc1 nt")
  VL(2, "buffer nt") VL(0, "buffer plain") VL(16, "buffer sc1") VL(18, "buffer sc1 nt") VL(17, "buffer sc0 sc1")
  VL(19, "buffer sc0 sc1 nt")
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {  // every variant must produce the production kernel's bytes
    std::vector<char> ref(bytes), got(bytes);
    vs[0].run(0);
    CK(hipMemcpy(ref.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
    for (size_t i = 1; i < vs.size(); i++) {
      CK(hipMemset(ps[0].dst[0], 0, bytes));
      vs[i].run(0);
      CK(hipMemcpy(got.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      if (memcmp(ref.data(), got.data(), bytes) != 0) printf("MISMATCH: %s\n", vs[i].name.c_str());
    }
  }
  const int BLK = 6;
  for (int it = 0; it < iters; it++)
    for (auto& v : vs) {
      v.run((it + BLK - 1) % R);
      CK(hipEventRecord(e0));
      for (int bb = 0; bb < BLK; bb++) v.run((it + bb) % R);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms / BLK);
    }
  printf("dt=%d K=%d U=%d B=%d buffer=%zu MiB alg bytes=%.0f (median / best of %d blocks of %d launches)\n", D, K, U,
         B, bytes >> 20, alg, iters, BLK);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s med %8.1f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6);
  }
  return 0;
}
