// XCD-aware tile order for the production reduce-copy kernel (tuning harness, not product code).
// The hardware hands workgroup b to XCD b mod 8, so with the production one-shot grid (tile = b) each
// XCD's L2 sees 16 KiB tiles at a 128 KiB stride. Round 1 measured the other extreme — each XCD
// sweeping its own eighth of the buffers — at 3-13 % slower (tools/tune_sched.hip). This sweep tries the
// middle: within every group of 8 x G consecutive workgroups, XCD x takes G consecutive tiles
// (tile = group base + x * G + j), so each XCD streams G x 16 KiB contiguous runs while the chip-wide
// in-flight window stays as narrow as production's. G in {1 (production), 2, 4, 16}, plus the
// reversed order (last tile first). Every variant's output is compared byte for byte with production's;
// timing is the median of blocks of 8 launches over 3 rotating buffer sets, variants interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=<dt> tools/xcd_order.hip \
//         -o tools/xcd_order_dt<dt>
//   ./tools/xcd_order_dt<dt> <iters>
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

constexpr int D = NEXR_DT;

// G > 0: XCD-grouped order; G == 0: production (tile = b); G < 0: reversed.
template <int G>
__device__ __forceinline__ uint64_t tile_of(uint64_t b, uint64_t nblk) {
  if constexpr (G == 0) {
    return b;
  } else if constexpr (G < 0) {
    return nblk - 1 - b;
  } else {
    const uint64_t grp = 8ull * G, full = nblk / grp * grp;
    if (b >= full) return b;  // a ragged last group keeps the production order (still a bijection)
    const uint64_t base = b / grp * grp, r = b - base;
    return base + (r % 8) * G + r / 8;
  }
}

template <int OP, int K, int POL, int G, int U = unroll_for(D, K, POL), int B = block_for(D, K, POL)>
__global__ __launch_bounds__(B) void ordered_kernel(RCParams p) {
  dispatch_minmax<D, OP, K, POL, U, B>(p, tile_of<G>(blockIdx.x, gridDim.x), gridDim.x);
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
#define VAR(OP, KK, POL, G, BYTES, ARG, LABEL, REF)                                                          \
  {                                                                                                        \
    char nm[96];                                                                                           \
    snprintf(nm, sizeof nm, "%s K%d %3zu MiB %s", LABEL, KK, (size_t)(BYTES) >> 20,                        \
             G == 0 ? "production (tile = b)" : G < 0 ? "reversed" : "XCD runs of G=" #G " tiles");        \
    const int grid = (int)((BYTES) / 16 / (unroll_for(D, KK, POL) * block_for(D, KK, POL)));               \
    vs.push_back({nm, KK, BYTES,                                                                           \
                  [=, &params](int r) {                                                                    \
                    ordered_kernel<OP, KK, POL, G><<<grid, block_for(D, KK, POL)>>>(params(r, BYTES, ARG)); \
                  },                                                                                       \
                  REF, {}});                                                                               \
  }
#define SWEEP(OP, KK, POL, BYTES, ARG, LABEL)                              \
  {                                                                        \
    const int ref = (int)vs.size();                                        \
    VAR(OP, KK, POL, 0, BYTES, ARG, LABEL, -1)                             \
    VAR(OP, KK, POL, 2, BYTES, ARG, LABEL, ref)                            \
    VAR(OP, KK, POL, 4, BYTES, ARG, LABEL, ref)                            \
    VAR(OP, KK, POL, 16, BYTES, ARG, LABEL, ref)                           \
    VAR(OP, KK, POL, -1, BYTES, ARG, LABEL, ref)                           \
  }
  if constexpr (D == nexrInt32 || D == nexrInt8) {
    SWEEP(nexrDevMinMax, 4, kPolNtLoad, (size_t)64 << 20, maxArg, "max")
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
    printf("%-44s %8.2f us  %6.0f GB/s (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6, (refMed / med - 1) * 100);
  }
  return 0;
}
