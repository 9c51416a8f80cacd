// Trip size per workgroup for the production reduce-copy kernel (tuning harness, not product code).
// Rounds 1-2 swept (U, B) with the trip fixed at 16 KiB per buffer (1,024 packs) at C2/C3's size; at
// C4's 64 MiB a launch is only ~2 generations of workgroups long, so a smaller trip (shorter workgroup
// lifetime, finer drain) or a larger one (fewer workgroups) might pay there. Variants: U x B in
// {1x256 (4 KiB), 2x256 / 1x512 (8 KiB), production (16 KiB), 2x1024 / 8x256 (32 KiB), 4x1024
// (64 KiB)}, one-shot grids of nPacks / (U x B) workgroups, the cache policy production picks. Every
// variant's output is compared byte for byte with the production geometry's; timing is the median of
// blocks of 8 launches over 3 rotating buffer sets, all variants interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=<dt> tools/trip_sweep.hip \
//         -o tools/trip_sweep_dt<dt>
//   ./tools/trip_sweep_dt<dt> <iters>
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
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0xbfffbfffu;  // finite values for every float type
  }
}

struct Var {
  std::string name;
  int k;
  size_t bytes;
  std::function<void(int)> run;
  int ref;  // index of the production variant this one must match (-1: itself the reference)
  std::vector<float> ms;
};

constexpr int D = NEXR_DT;

template <int OP, int K, int POL, int U, int B>
void launch(const RCParams& p) {
  reduce_copy_kernel<D, OP, K, POL, U, B><<<(int)(p.nPacks / (U * B)), B>>>(p);
}

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
  auto params = [&](int r, size_t bytes, uint64_t arg) {
    RCParams q = base[r];
    q.nElts = bytes / esz;
    q.nPacks = bytes / 16;
    q.redArg = arg;
    return q;
  };
  const bool isSigned = D == nexrInt8 || D == nexrInt32 || D == nexrInt64;
  const uint64_t maxArg = isSigned ? ((1ull << (esz * 8 - 1)) ^ ((esz == 8) ? ~0ull : ((1ull << (esz * 8)) - 1))) : ~0ull;
  std::vector<Var> vs;
#define VAR(OP, KK, POL, U, B, BYTES, ARG, LABEL)                                                              \
  {                                                                                                          \
    char nm[96];                                                                                             \
    snprintf(nm, sizeof nm, "%s K%d %3zu MiB U%d B%d (%2d KiB)%s", LABEL, KK, (size_t)(BYTES) >> 20, U, B,   \
             U * B * 16 / 1024, (U == unroll_for(D, KK, POL) && B == block_for(D, KK, POL)) ? " *prod" : ""); \
    vs.push_back({nm, KK, BYTES, [&](int r) { launch<OP, KK, POL, U, B>(params(r, BYTES, ARG)); }, ref, {}}); \
  }
#define SWEEP(OP, KK, POL, BYTES, ARG, LABEL)                                                       \
  {                                                                                                 \
    const int ref = -1;                                                                             \
    VAR(OP, KK, POL, (unroll_for(D, KK, POL)), (block_for(D, KK, POL)), BYTES, ARG, LABEL)          \
  }                                                                                                 \
  {                                                                                                 \
    const int ref = (int)vs.size() - 1;                                                             \
    VAR(OP, KK, POL, 1, 256, BYTES, ARG, LABEL) VAR(OP, KK, POL, 2, 256, BYTES, ARG, LABEL)         \
    VAR(OP, KK, POL, 1, 512, BYTES, ARG, LABEL) VAR(OP, KK, POL, 2, 1024, BYTES, ARG, LABEL)        \
    VAR(OP, KK, POL, 8, 256, BYTES, ARG, LABEL) VAR(OP, KK, POL, 4, 1024, BYTES, ARG, LABEL)        \
  }
  if constexpr (D == nexrInt32 || D == nexrInt8) {
    SWEEP(nexrDevMinMax, 4, kPolNtLoad, (size_t)64 << 20, maxArg, "max")
    SWEEP(nexrDevProd, 4, kPolNtLoad, (size_t)64 << 20, 0, "prod")
  } else if constexpr (D == nexrFloat32) {
    SWEEP(nexrDevSum, 2, kPolNt, (size_t)256 << 20, 0, "sum")
    SWEEP(nexrDevSum, 2, kPolNtLoad, (size_t)64 << 20, 0, "sum")
  } else {
    SWEEP(nexrDevSum, 8, kPolNt, (size_t)256 << 20, 0, "sum")
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
  printf("dt=%d: median (best) of %d blocks of %d launches; vs = median vs production\n", D, iters, BLK);
  double refMed = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double alg = (double)(v.k + 1) * v.bytes;
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    if (v.ref < 0) refMed = med;
    printf("%-40s %8.2f us  %6.0f GB/s (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6, (refMed / med - 1) * 100);
  }
  return 0;
}
