// C4's cost model: time of a K = 4, M = 1 reduce-copy against its size, through the product ABI
// (nexrReduceCopy: production policy and shape per size), int32 min and int8 max, 16-256 MiB per
// buffer, three rotating buffer sets (tuning harness). Prints, per size, the per-launch
// time of back-to-back launches (events around a block of 8) and of single launches (events around
// each one alone), then a least-squares fit time = a + bytes / rate over the sizes of each policy
// regime. Run under `rocprofv3 --kernel-trace --stats` for the kernels' own durations; NEXR_POLICY=1
// or 3 forces a cache policy (nexr_api.cpp pickPolicy) to compare regimes at one size.
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/c4_fit.cpp -Lnex-nccl_amd -lnexr -Wl,-rpath,'$ORIGIN/../nex-nccl_amd' -o tools/c4_fit
//   ./tools/c4_fit [blocks]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "../include/nexr.h"
#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));               \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)
#define CN(x)                                                       \
  do {                                                              \
    nexrResult_t r_ = (x);                                          \
    if (r_ != nexrSuccess) {                                        \
      printf("%s:%d nexr error %d\n", __FILE__, __LINE__, (int)r_); \
      exit(1);                                                      \
    }                                                               \
  } while (0)

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

struct Pt {
  double bytes, us;
};
static void fit(const char* what, const std::vector<Pt>& pts) {
  if (pts.size() < 2) return;
  double sx = 0, sy = 0, sxx = 0, sxy = 0;
  for (const Pt& p : pts) sx += p.bytes, sy += p.us, sxx += p.bytes * p.bytes, sxy += p.bytes * p.us;
  const double n = (double)pts.size();
  const double slope = (n * sxy - sx * sy) / (n * sxx - sx * sx), icpt = (sy - slope * sx) / n;
  double worst = 0;
  for (const Pt& p : pts) worst = std::max(worst, std::abs(p.us - (icpt + slope * p.bytes)));
  printf("  fit %-34s %zu sizes: %.2f us fixed + streaming at %.0f GB/s (%.4f of 8 TB/s); max residual %.2f us\n", what,
         pts.size(), icpt, 1e-3 / slope, 1e-3 / slope / 8000.0, worst);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 12;
  const int K = 4, R = 3, BLK = 8;
  const size_t mibs[] = {16, 24, 32, 48, 64, 80, 96, 100, 104, 112, 128, 160, 192, 256};
  struct Ty {
    const char* name;
    int dt;
    uint64_t arg;
  } types[] = {{"int32 min", nexrInt32, 0}, {"int8 max", nexrInt8, 1}};
  const char* pol = getenv("NEXR_POLICY");
  printf("K = 4, M = 1 through nexrReduceCopy%s%s; per-launch us (median of %d blocks): back-to-back blocks of %d,\n"
         "and single launches bracketed alone; streamed = 5 x buffer; policy by pickPolicy: plain < 64 MiB streamed,\n"
         "nt loads < 512 MiB, nt loads + stores from 512 MiB\n\n",
         pol ? ", NEXR_POLICY=" : "", pol ? pol : "", blocks, BLK);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const size_t maxBytes = mibs[sizeof mibs / sizeof mibs[0] - 1] << 20;
  std::vector<char*> buf(R * (K + 1));
  for (auto& q : buf) {
    CK(hipMalloc((void**)&q, maxBytes));
  }
  for (size_t i = 0; i < buf.size(); i++) fill_bits<<<4096, 256, 0, s>>>((uint32_t*)buf[i], maxBytes / 4, 77 + i);
  CK(hipStreamSynchronize(s));
  for (const Ty& t : types) {
    printf("%s\n  %8s %10s %12s %8s %12s %8s %s\n", t.name, "MiB/buf", "streamed", "b2b us", "frac", "single us", "frac",
           "policy");
    std::vector<Pt> regime[3];
    for (size_t mib : mibs) {
      const size_t bytes = mib << 20, esz = t.dt == nexrInt8 ? 1 : 4, n = bytes / esz;
      const double alg = (double)(K + 1) * bytes;
      auto call = [&](int r) {
        const void* srcs[4];
        for (int k = 0; k < K; k++) srcs[k] = buf[r * (K + 1) + k];
        void* dsts[1] = {buf[r * (K + 1) + K]};
        CN(nexrReduceCopy(K, srcs, 1, dsts, n, t.dt, nexrDevMinMax, t.arg, 0, nullptr, 0, s));
      };
      for (int w = 0; w < 2 * R; w++) call(w % R);
      CK(hipStreamSynchronize(s));
      std::vector<double> b2b, one;
      for (int it = 0; it < blocks; it++) {
        CK(hipEventRecord(e0, s));
        for (int b = 0; b < BLK; b++) call((it + b) % R);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        b2b.push_back(ms * 1e3 / BLK);
        CK(hipEventRecord(e0, s));
        call((it + 1) % R);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        one.push_back(ms * 1e3);
      }
      const double mb = median(b2b), mo = median(one);
      const size_t streamed = (K + 1) * mib;
      const int p = pol ? atoi(pol) : (streamed >= 512 ? 3 : streamed >= 64 ? 1 : 0);
      printf("  %8zu %10zu %12.2f %8.4f %12.2f %8.4f %s\n", mib, streamed, mb, alg / mb / 1e3 / 8000.0, mo,
             alg / mo / 1e3 / 8000.0, p == 3 ? "nt loads + stores" : p == 1 ? "nt loads" : "plain");
      regime[p == 3 ? 2 : p].push_back({alg, mb});
    }
    fit("(plain, back-to-back)", regime[0]);
    fit("(nt loads, back-to-back)", regime[1]);
    fit("(nt loads + stores, back-to-back)", regime[2]);
    printf("\n");
  }
  for (auto q : buf) CK(hipFree(q));
  return 0;
}
