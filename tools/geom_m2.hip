// Workgroup geometry for two-destination reduce-copies (tuning harness, not product code): the ring's
// recvReduceCopySend (K = 2, M = 2) and copySend (K = 1, M = 2) shapes, fp32 sum, 64 and 256 MiB per
// buffer, (U, B) in {4x256 (shipped), 2x512, 1x1024}, the cache policy production picks for the bytes
// streamed. Each variant's outputs are compared byte for byte with the 4x256 twin before timing; the
// timing is the median of blocks of 8 launches over 3 rotating buffer sets, variants interleaved.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 tools/geom_m2.hip -o tools/geom_m2
//   ./tools/geom_m2 <iters>
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
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0xbfffbfffu;
  }
}

struct Var {
  std::string name;
  int k, m;
  size_t bytes;
  std::function<void(int)> run;
  int twin;
  std::vector<float> ms;
};

template <int K, int POL, int U, int B>
void launch(const RCParams& p) {
  reduce_copy_kernel<nexrFloat32, nexrDevSum, K, POL, U, B><<<(int)(p.nPacks / 1024), B>>>(p);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8;
  const size_t sizes[2] = {64u << 20, 256u << 20};
  const int R = 3;
  std::vector<RCParams> base(R);
  for (int r = 0; r < R; r++) {
    std::memset((void*)&base[r], 0, sizeof(RCParams));
    for (int s = 0; s < 2; s++) {
      char* q;
      CK(hipMalloc((void**)&q, sizes[1]));
      fill_bits<<<2048, 256>>>((uint32_t*)q, sizes[1] / 4, 1000 + r * 16 + s);
      base[r].src[s] = q;
    }
    for (int d = 0; d < 2; d++) CK(hipMalloc((void**)&base[r].dst[d], sizes[1]));
  }
  CK(hipDeviceSynchronize());
  auto params = [&](int r, size_t bytes, int m) {
    RCParams q = base[r];
    q.nElts = bytes / 4;
    q.nPacks = bytes / 16;
    q.nDsts = m;
    return q;
  };
  std::vector<Var> vs;
#define GEO(KK, MM)                                                                                              \
  for (int si = 0; si < 2; si++) {                                                                               \
    const size_t bytes = sizes[si];                                                                              \
    const bool ntStore = (size_t)(KK + MM) * bytes >= (512u << 20);                                              \
    const int ref = (int)vs.size();                                                                              \
    char nm[96];                                                                                                 \
    for (int g = 0; g < 3; g++) {                                                                                \
      snprintf(nm, sizeof nm, "K%d M%d %3zu MiB %s", KK, MM, bytes >> 20, g == 0 ? "U4 B256" : g == 1 ? "U2 B512" : "U1 B1024"); \
      std::function<void(int)> f;                                                                                \
      if (g == 0) f = [&, bytes, ntStore](int r) { ntStore ? launch<KK, kPolNt, 4, 256>(params(r, bytes, MM)) : launch<KK, kPolNtLoad, 4, 256>(params(r, bytes, MM)); }; \
      if (g == 1) f = [&, bytes, ntStore](int r) { ntStore ? launch<KK, kPolNt, 2, 512>(params(r, bytes, MM)) : launch<KK, kPolNtLoad, 2, 512>(params(r, bytes, MM)); }; \
      if (g == 2) f = [&, bytes, ntStore](int r) { ntStore ? launch<KK, kPolNt, 1, 1024>(params(r, bytes, MM)) : launch<KK, kPolNtLoad, 1, 1024>(params(r, bytes, MM)); }; \
      vs.push_back({nm, KK, MM, bytes, f, g == 0 ? -1 : ref, {}});                                              \
    }                                                                                                            \
  }
  GEO(2, 2) GEO(1, 2) GEO(2, 1)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {
    std::vector<char> ref(2 * sizes[1]), got(2 * sizes[1]);
    for (size_t i = 0; i < vs.size(); i++) {
      std::vector<char>& out = vs[i].twin < 0 ? ref : got;
      for (int d = 0; d < vs[i].m; d++) CK(hipMemset(base[0].dst[d], 0, vs[i].bytes));
      vs[i].run(0);
      for (int d = 0; d < vs[i].m; d++)
        CK(hipMemcpy(out.data() + d * vs[i].bytes, base[0].dst[d], vs[i].bytes, hipMemcpyDeviceToHost));
      if (vs[i].twin >= 0 && memcmp(ref.data(), got.data(), vs[i].m * vs[i].bytes) != 0)
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
  printf("fp32 sum: GB/s of (K+M) x buffer, median (best) of %d blocks of %d launches; vs = median vs U4 B256\n", iters, BLK);
  double refMed = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double alg = (double)(v.k + v.m) * v.bytes;
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    if (v.twin < 0) refMed = med;
    printf("%-28s %8.1f us  %6.0f (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6, alg / mn / 1e6,
           (refMed / med - 1) * 100);
  }
  return 0;
}
