// C4's 8-bit fold against the workgroup shape (tuning harness, not product code; VERDICT r03 "next" #3).
//
// profiles/r04e_fold8_cost_stats.txt puts int8 min/max at +0.7-0.8 % over int32 of the same op (prod at
// +0.1 %) over six same-box measurements, with the fold at its VALU floor (3K - 1 packed-16-bit
// instructions per dword). The one lever that does not change the instruction count is how the trip's
// 1024 packs are spread: U packs per lane x B lanes (U x B = 1024). More, shorter lanes (U = 1, B = 1024)
// halve each lane's fold and give the SIMD twice the waves to hide it behind; fewer, longer ones (U = 4,
// B = 256) put more loads in flight per lane. Production C4 is U = 2, B = 512. Every shape of every op
// is byte-checked against production, and timed beside int32 max (the control: a 1-instruction fold)
// and the uint32 sum of the same shape, interleaved in blocks over 3 rotating buffer sets.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=0 tools/geom8_ab.hip -o tools/geom8_ab
//   ./tools/geom8_ab <blocks>
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

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed, uint32_t mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31)) & mask;  // mask keeps floats finite (exponent bit cleared)
  }
}

template <int D, int OP, int U>
void launch(const RCParams& p, int grid) {
  reduce_copy_kernel<D, OP, 4, kPolNtLoad, U, kTripPacks / U, false><<<grid, kTripPacks / U>>>(p);
}

struct Var {
  std::string name;
  int cfg;  // index into the op table: which RCParams set (redArg, nElts) it runs on
  int u;
  std::function<void(const RCParams&, int)> run;
};

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 30;
  const size_t bytes = 64u << 20;
  const int R = 3, BLK = 6, K = 4;
  // ops: int8 min, int8 max, int8 prod, int32 max (control), uint32 sum (floor)
  const char* opn[] = {"int8 min", "int8 max", "int8 prod", "int32 max", "u32 sum"};
  const int esz[] = {1, 1, 1, 4, 4};
  const uint64_t redArg[] = {0x80, 0x7f, 0, 0x7fffffffull, 0};
  std::vector<Var> vs;
#define ADD(i, D, OP)                                                                                             \
  vs.push_back({std::string(opn[i]) + " U1 B1024", i, 1, [](const RCParams& p, int g) { launch<D, OP, 1>(p, g); }}); \
  vs.push_back({std::string(opn[i]) + " U2 B512", i, 2, [](const RCParams& p, int g) { launch<D, OP, 2>(p, g); }});  \
  vs.push_back({std::string(opn[i]) + " U4 B256", i, 4, [](const RCParams& p, int g) { launch<D, OP, 4>(p, g); }});
  ADD(0, nexrInt8, nexrDevMinMax)
  ADD(1, nexrInt8, nexrDevMinMax)
  ADD(2, nexrInt8, nexrDevProd)
  ADD(3, nexrInt32, nexrDevMinMax)
  ADD(4, nexrUint32, nexrDevSum)
#undef ADD
  // buffers: 3 rotating sets of K sources + 1 destination per variant family share the sources
  std::vector<std::vector<char*>> srcs(R, std::vector<char*>(K));
  std::vector<char*> dsts(R);
  for (int r = 0; r < R; r++) {
    for (int s = 0; s < K; s++) {
      CK(hipMalloc((void**)&srcs[r][s], bytes));
      fill_bits<<<2048, 256>>>((uint32_t*)srcs[r][s], bytes / 4, 7000 + r * 16 + s, 0xffffffffu);
    }
    CK(hipMalloc((void**)&dsts[r], bytes));
  }
  std::vector<std::vector<RCParams>> ps(5, std::vector<RCParams>(R));
  for (int i = 0; i < 5; i++)
    for (int r = 0; r < R; r++) {
      RCParams& p = ps[i][r];
      std::memset((void*)&p, 0, sizeof(p));
      for (int s = 0; s < K; s++) p.src[s] = srcs[r][s];
      p.dst[0] = dsts[r];
      p.nDsts = 1;
      p.nPacks = bytes / 16;
      p.nElts = bytes / esz[i];
      p.head = 0;
      p.redArg = redArg[i];
    }
  const int grid = (int)(bytes / 16 / kTripPacks);
  // What the kernels and their one-shot grid assume, checked on the host before any launch.
  for (int i = 0; i < 5; i++)
    for (int r = 0; r < R; r++) {
      const RCParams& p = ps[i][r];
      if (p.nElts * (uint64_t)esz[i] != p.nPacks * 16 || p.nPacks != (uint64_t)grid * kTripPacks || K > NEXR_MAX_SRCS) {
        fprintf(stderr, "bad parameters for %s\n", opn[i]);
        return 2;
      }
    }
  CK(hipDeviceSynchronize());
  // byte check: every shape against U = 2 (production) of the same op, on set 0
  {
    std::vector<char> ref(bytes), got(bytes);
    for (size_t v = 0; v < vs.size(); v++) {
      if (vs[v].u != 2) continue;
      CK(hipMemset(dsts[0], 0, bytes));
      vs[v].run(ps[vs[v].cfg][0], grid);
      CK(hipMemcpy(ref.data(), dsts[0], bytes, hipMemcpyDeviceToHost));
      for (size_t w = 0; w < vs.size(); w++) {
        if (vs[w].cfg != vs[v].cfg || w == v) continue;
        CK(hipMemset(dsts[0], 0, bytes));
        vs[w].run(ps[vs[w].cfg][0], grid);
        CK(hipMemcpy(got.data(), dsts[0], bytes, hipMemcpyDeviceToHost));
        printf("%-20s bytes %s %s\n", vs[w].name.c_str(), memcmp(ref.data(), got.data(), bytes) ? "MISMATCH" : "match",
               vs[v].name.c_str());
      }
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> us(vs.size());
  for (size_t v = 0; v < vs.size(); v++)
    for (int w = 0; w < 2; w++) vs[v].run(ps[vs[v].cfg][w % R], grid);
  for (int it = 0; it < blocks; it++) {
    for (size_t vi = 0; vi < vs.size(); vi++) {
      const size_t v = (it % 2) ? vs.size() - 1 - vi : vi;  // alternate the order every block
      vs[v].run(ps[vs[v].cfg][(it + BLK - 1) % R], grid);
      CK(hipEventRecord(e0));
      for (int bb = 0; bb < BLK; bb++) vs[v].run(ps[vs[v].cfg][(it + bb) % R], grid);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      us[v].push_back(ms * 1e3f / BLK);
    }
    if (it % 10 == 9) {
      printf("block %d done\n", it + 1);
      fflush(stdout);
    }
  }
  std::vector<double> med(vs.size());
  for (size_t v = 0; v < vs.size(); v++) {
    std::vector<float> s = us[v];
    std::sort(s.begin(), s.end());
    med[v] = s[s.size() / 2];
  }
  const double alg = (double)(K + 1) * bytes;
  printf("\nbuffer = 64 MiB, K = 4, M = 1, nt loads; median (mean) us of %d blocks of %d launches over %d rotating sets,\n"
         "interleaved; fraction of 8 TB/s; ratios to the uint32 sum of the same shape, to int32 max (the control) of the\n"
         "same shape, and to production (U2 B512) of the same op\n",
         blocks, BLK, R);
  for (size_t v = 0; v < vs.size(); v++) {
    double mean = 0;
    for (float x : us[v]) mean += x;
    mean /= us[v].size();
    size_t u32 = 0, ctl = 0, prod = 0;
    for (size_t w = 0; w < vs.size(); w++) {
      if (vs[w].cfg == 4 && vs[w].u == vs[v].u) u32 = w;
      if (vs[w].cfg == 3 && vs[w].u == vs[v].u) ctl = w;
      if (vs[w].cfg == vs[v].cfg && vs[w].u == 2) prod = w;
    }
    printf("  %-20s %8.2f (%8.2f) us  %.4f  over u32 %.4f  over int32 max %.4f  over U2 B512 %.4f\n", vs[v].name.c_str(),
           med[v], mean, alg / med[v] / 1e3 / 8000.0, med[v] / med[u32], med[v] / med[ctl], med[v] / med[prod]);
  }
  for (int r = 0; r < R; r++) {
    for (char* q : srcs[r]) CK(hipFree(q));
    CK(hipFree(dsts[r]));
  }
  return 0;
}
