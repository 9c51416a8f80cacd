// Workgroup geometry per (datatype, fan-in) for the production reduce-copy kernel (tuning harness, not
// product code). Every geometry keeps the 16 KiB trip (U packs per lane x B lanes = 1024 packs), so the
// grid, the bytes and the access order are the same; what changes is how many packs each lane folds
// in series (U) and how many waves share a workgroup (B / 64).
//
// For one datatype (-DNEXR_DT), K in 2..8, ops Sum and Min (Min only where it is not Sum's
// arithmetic twin), buffers of 64 MiB (C4's size) and 256 MiB (C2/C3's), each (U, B) in
// {4x256 (shipped default), 2x512, 1x1024}, the cache policy production picks for that size. Every
// variant's output is compared byte for byte with the 4x256 twin before timing; timing is the median
// of blocks of 8 launches over 3 rotating buffer sets, all variants interleaved.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=<dt> tools/geom_sweep.hip \
//         -o tools/geom_sweep_dt<dt>
//   ./tools/geom_sweep_dt<dt> <iters>
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
  int twin;  // index of the 4x256 variant this one must match (-1: itself the reference)
  std::vector<float> ms;
};

constexpr int D = NEXR_DT;

template <int OP, int K, int POL, int U, int B>
void launch(const RCParams& p) {
  reduce_copy_kernel<D, OP, K, POL, U, B><<<(int)(p.nPacks / 1024), B>>>(p);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8;
  constexpr int esz = 16 / Ty<D>::EPP;
  const size_t sizes[2] = {64u << 20, 256u << 20};
  const int R = 3;
  // one allocation of 9 x 256 MiB per set; the 64 MiB runs use the first quarter of each buffer
  std::vector<RCParams> base(R);
  for (int r = 0; r < R; r++) {
    std::memset((void*)&base[r], 0, sizeof(RCParams));
    for (int s = 0; s < 8; s++) {
      char* q;
      CK(hipMalloc((void**)&q, sizes[1]));
      fill_bits<<<2048, 256>>>((uint32_t*)q, sizes[1] / 4, 1000 + r * 16 + s);
      base[r].src[s] = q;
    }
    CK(hipMalloc((void**)&base[r].dst[0], sizes[1]));
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
  const bool isInt = Ty<D>::kIsInt;
  const bool isSigned = D == nexrInt8 || D == nexrInt32 || D == nexrInt64;
  const uint64_t minArg = isSigned ? (1ull << (esz * 8 - 1)) : 0;  // hostToDevRedOp: min (bit 0 clear)
  std::vector<Var> vs;
#define GEO3(OP, OPNAME, KK, ARG)                                                                                 \
  for (int si = 0; si < 2; si++) {                                                                                \
    const size_t bytes = sizes[si];                                                                               \
    const bool ntStore = (size_t)(KK + 1) * bytes >= (512u << 20);                                                \
    const int ref = (int)vs.size();                                                                               \
    char nm[96];                                                                                                  \
    for (int g = 0; g < 3; g++) {                                                                                 \
      snprintf(nm, sizeof nm, "%s K%d %3zu MiB %s", OPNAME, KK, bytes >> 20, g == 0 ? "U4 B256" : g == 1 ? "U2 B512" : "U1 B1024"); \
      std::function<void(int)> f;                                                                                 \
      if (g == 0) f = [&, bytes, ntStore](int r) { ntStore ? launch<OP, KK, kPolNt, 4, 256>(params(r, bytes, ARG)) : launch<OP, KK, kPolNtLoad, 4, 256>(params(r, bytes, ARG)); }; \
      if (g == 1) f = [&, bytes, ntStore](int r) { ntStore ? launch<OP, KK, kPolNt, 2, 512>(params(r, bytes, ARG)) : launch<OP, KK, kPolNtLoad, 2, 512>(params(r, bytes, ARG)); }; \
      if (g == 2) f = [&, bytes, ntStore](int r) { ntStore ? launch<OP, KK, kPolNt, 1, 1024>(params(r, bytes, ARG)) : launch<OP, KK, kPolNtLoad, 1, 1024>(params(r, bytes, ARG)); }; \
      vs.push_back({nm, KK, bytes, f, g == 0 ? -1 : ref, {}});                                                   \
    }                                                                                                             \
  }
#define GEOK(OP, OPNAME, ARG)                                                                                \
  GEO3(OP, OPNAME, 2, ARG) GEO3(OP, OPNAME, 3, ARG) GEO3(OP, OPNAME, 4, ARG) GEO3(OP, OPNAME, 5, ARG)           \
  GEO3(OP, OPNAME, 6, ARG) GEO3(OP, OPNAME, 7, ARG) GEO3(OP, OPNAME, 8, ARG)
  GEOK(nexrDevSum, "sum", 0)
  if (isInt || D == nexrFloat16 || D == nexrBfloat16 || D == nexrFloat32) { GEOK(nexrDevMinMax, "min", minArg) }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {
    std::vector<char> ref(sizes[1]), got(sizes[1]);
    for (size_t i = 0; i < vs.size(); i++) {
      if (vs[i].twin < 0) {
        CK(hipMemset(base[0].dst[0], 0, vs[i].bytes));
        vs[i].run(0);
        CK(hipMemcpy(ref.data(), base[0].dst[0], vs[i].bytes, hipMemcpyDeviceToHost));
        continue;
      }
      CK(hipMemset(base[0].dst[0], 0, vs[i].bytes));
      vs[i].run(0);
      CK(hipMemcpy(got.data(), base[0].dst[0], vs[i].bytes, hipMemcpyDeviceToHost));
      if (memcmp(ref.data(), got.data(), vs[i].bytes) != 0) printf("MISMATCH: %s\n", vs[i].name.c_str());
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
  printf("dt=%d: GB/s of (K+1) x buffer, median (best) of %d blocks of %d launches; vs = median vs U4 B256\n", D, iters,
         BLK);
  double refMed = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double alg = (double)(v.k + 1) * v.bytes;
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    if (v.twin < 0) refMed = med;
    printf("%-30s %8.1f us  %6.0f (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6, alg / mn / 1e6,
           (refMed / med - 1) * 100);
  }
  return 0;
}
