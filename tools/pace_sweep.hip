// Pacing the stores (tuning harness, not product code). On the same buffers the bf16 K = 8 kernel,
// whose software rounding costs far more VALU work than fp16's packed adds, runs 1-3 % faster than the
// fp16 kernel and than a plain uint32 sum (tools/k8_types_ab.py), and round 1 found the hardware bf16
// conversion (fewer VALU instructions) 2 % slower than the software rounding. If work between a wave's
// loads returning and its stores issuing helps because it spreads the write stream out in time, a
// bare s_sleep there should do the same for every type. Variants: the production trip body with
// s_sleep(P) after the fold and before the stores, P in {0, 1, 2, 4, 8, 16} (one unit = 64 clocks),
// one-shot grid, production geometry and cache policy; outputs byte-checked against P = 0.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=<dt> tools/pace_sweep.hip \
//         -o tools/pace_sweep_dt<dt>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

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
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0x3bff3bffu;  // finite values for every float type
  }
}

constexpr int D = NEXR_DT;

// The production full-trip loop of body() (nexr_kernels.hip) for a one-shot grid of whole trips, with
// s_sleep(P) between the fold and the stores.
template <int OP, int K, int POL, int P, int U = unroll_for(D, K, POL), int B = block_for(D, K, POL)>
__global__ __launch_bounds__(B) void paced_kernel(RCParams p) {
  Fold<D, OP, K, false> f(p);
  const uint64_t off = ((uint64_t)blockIdx.x * (B * U) + threadIdx.x) * 16;
  u32x4 in[U][K];
#pragma unroll
  for (int s = 0; s < K; s++)
#pragma unroll
    for (int u = 0; u < U; u++) in[u][s] = ld16<POL>(p.src[s] + off + u * B * 16);
  u32x4 out[U];
#pragma unroll
  for (int u = 0; u < U; u++) out[u] = f.run(in[u]);
  if constexpr (P > 0) __builtin_amdgcn_s_sleep(P);
#pragma unroll
  for (int u = 0; u < U; u++) st16<POL>(p.dst[0] + off + u * B * 16, out[u]);
}

struct Var {
  std::string name;
  int k;
  size_t bytes;
  std::function<void(int)> run;
  int ref;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8;
  constexpr int esz = 16 / Ty<D>::EPP;
  const size_t maxBytes = 256u << 20;
  const int R = 3;
  std::vector<RCParams> base(R);
  for (int r = 0; r < R; r++) {
    std::memset((void*)&base[r], 0, sizeof(RCParams));
    for (int s = 0; s < 8; s++) {
      char* q;
      CK(hipMalloc((void**)&q, maxBytes));
      fill_bits<<<2048, 256>>>((uint32_t*)q, maxBytes / 4, 1000 + r * 16 + s);
      base[r].src[s] = q;
    }
    CK(hipMalloc((void**)&base[r].dst[0], maxBytes));
    base[r].nDsts = 1;
  }
  CK(hipDeviceSynchronize());
  auto params = [&](int r, size_t bytes) {
    RCParams q = base[r];
    q.nElts = bytes / esz;
    q.nPacks = bytes / 16;
    return q;
  };
  std::vector<Var> vs;
#define VAR(KK, POL, P, BYTES, REF)                                                                     \
  {                                                                                                   \
    char nm[96];                                                                                      \
    snprintf(nm, sizeof nm, "sum K%d %3zu MiB s_sleep(%2d)", KK, (size_t)(BYTES) >> 20, P);            \
    const int grid = (int)((BYTES) / 16 / (unroll_for(D, KK, POL) * block_for(D, KK, POL)));          \
    vs.push_back({nm, KK, BYTES,                                                                      \
                  [=, &params](int r) {                                                               \
                    paced_kernel<nexrDevSum, KK, POL, P><<<grid, block_for(D, KK, POL)>>>(params(r, BYTES)); \
                  },                                                                                  \
                  REF, {}});                                                                          \
  }
#define SWEEP(KK, POL, BYTES)                    \
  {                                              \
    const int ref = (int)vs.size();              \
    VAR(KK, POL, 0, BYTES, -1)                   \
    VAR(KK, POL, 1, BYTES, ref)                  \
    VAR(KK, POL, 2, BYTES, ref)                  \
    VAR(KK, POL, 4, BYTES, ref)                  \
    VAR(KK, POL, 8, BYTES, ref)                  \
    VAR(KK, POL, 16, BYTES, ref)                 \
  }
  if constexpr (D == nexrFloat32) {
    SWEEP(2, kPolNt, (size_t)256 << 20)
  } else if constexpr (D == nexrInt32 || D == nexrUint32) {
    SWEEP(4, kPolNtLoad, (size_t)64 << 20)
    SWEEP(8, kPolNt, (size_t)256 << 20)
  } else {
    SWEEP(8, kPolNt, (size_t)256 << 20)
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {
    std::vector<char> want(maxBytes), got(maxBytes);
    for (size_t i = 0; i < vs.size(); i++) {
      CK(hipMemset(base[0].dst[0], 0, vs[i].bytes));
      vs[i].run(0);
      CK(hipMemcpy(vs[i].ref < 0 ? want.data() : got.data(), base[0].dst[0], vs[i].bytes, hipMemcpyDeviceToHost));
      if (vs[i].ref >= 0 && memcmp(want.data(), got.data(), vs[i].bytes) != 0)
        printf("MISMATCH: %s\n", vs[i].name.c_str());
    }
  }
  const int BLK = 8;
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
  printf("dt=%d: median (best) of %d blocks of %d launches; vs = median vs s_sleep(0)\n", D, iters, BLK);
  double refMed = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double alg = (double)(v.k + 1) * v.bytes;
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    if (v.ref < 0) refMed = med;
    printf("%-36s %8.2f us  %6.0f GB/s (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6, (refMed / med - 1) * 100);
  }
  return 0;
}
