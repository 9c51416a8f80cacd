// The 8-bit fold's cost at C4 (tuning harness, not product code; VERDICT r03 "next" #3).
//
// C4's int8 min / max / prod ran 0.6-2.7 % slower than a uint32 sum of the same bytes on the same
// buffers (BENCH_r03 `kernel_over_u32_sum` 1.006 / 1.027 / 1.018; int32 1.000-1.008). The fold's
// VALU count is already at the packed-16-bit floor (ISA of reduce_copy_kernel<0,2,4,1,2,512>: one
// v_pk_lshlrev_b16 per source dword to put the even bytes in the high halves, two v_pk_{min,max}_i16
// per dword per step, one v_perm_b32 per dword to join: 11 VALU per dword at K = 4, against 3 v_add_u32
// for the uint32 sum), so what is left to try is WHEN that work runs. Production loads source-major
// (every source's pack u = 0, then u = 1) and stores both packs after both folds; the variants here
// load pack-major (pack 0 of every source, then pack 1) and store each pack as soon as it is folded,
// so pack 0's fold and stores overlap pack 1's loads. Every variant is checked byte for byte against
// production, and every configuration is timed beside the uint32 sum of the same bytes on the same
// three rotating buffer sets, interleaved in blocks (the bench's `kernel_over_u32_sum`).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=0 tools/fold8_ab.hip -o tools/fold8_ab
//   ./tools/fold8_ab <MiB per buffer> <blocks>
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
    p[i] = (uint32_t)(z ^ (z >> 31));
  }
}

// Pack-major trip: pack u of every source is loaded before pack u + 1 of any, and each pack is stored
// right after its fold. One trip per workgroup (the one-shot grid; sizes here are whole trips).
template <int D, int OP, int K, int POL, bool IsMin, int U, int B>
__global__ __launch_bounds__(B) void pack_major(RCParams p) {
  Fold<D, OP, K, IsMin> f(p);
  const uint64_t off = ((uint64_t)blockIdx.x * (B * U) + threadIdx.x) * 16;
  u32x4 in[U][K];
#pragma unroll
  for (int u = 0; u < U; u++)
#pragma unroll
    for (int s = 0; s < K; s++) in[u][s] = ld16<POL>(p.src[s] + off + u * B * 16);
#pragma unroll
  for (int u = 0; u < U; u++) st16<POL>(p.dst[0] + off + u * B * 16, f.run(in[u]));
}

template <int D, int OP, int K, int POL, int U, int B>
void launch_pm(const RCParams& p, uint64_t nPacks) {
  if (OP == nexrDevMinMax && (p.redArg & 1) == 0)
    pack_major<D, OP, K, POL, true, U, B><<<(int)(nPacks / (U * B)), B>>>(p);
  else
    pack_major<D, OP, K, POL, false, U, B><<<(int)(nPacks / (U * B)), B>>>(p);
}

struct Var {
  std::string name;
  int cfg;     // which configuration (rows of the summary)
  bool base;   // the production kernel of the configuration (the byte reference)
  bool u32;    // the uint32 sum of the same bytes
  std::function<void(int)> run;
  std::vector<float> us;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 64) << 20;
  const int blocks = argc > 2 ? atoi(argv[2]) : 12;
  constexpr int K = 4;
  const int R = 3;
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
    p.nPacks = bytes / 16;
  }
  CK(hipDeviceSynchronize());
  const uint64_t P = bytes / 16;
  auto params = [&](int r, int dt, uint64_t arg) {
    RCParams q = ps[r];
    q.nElts = bytes / (dt == nexrInt32 || dt == nexrUint32 ? 4 : 1);
    q.redArg = arg;
    return q;
  };
  std::vector<Var> vs;
  const char* cfgs[] = {"int8 min", "int8 max", "int8 prod", "int32 min", "int32 max", "int32 prod"};
  // production (U2 B512, nt loads: C4's geometry and policy), then the pack-major variants
#define CFG(I, DT, OP, ARG)                                                                                       \
  vs.push_back({"production U2 B512", I, true, false, [&](int r) {                                              \
                  reduce_copy_kernel<DT, OP, K, kPolNtLoad><<<(int)(P / 1024), block_for(DT, K, kPolNtLoad)>>>( \
                      params(r, DT, ARG));                                                                      \
                }, {}});                                                                                        \
  vs.push_back({"pack-major U2 B512", I, false, false,                                                          \
                [&](int r) { launch_pm<DT, OP, K, kPolNtLoad, 2, 512>(params(r, DT, ARG), P); }, {}});          \
  vs.push_back({"pack-major U4 B256", I, false, false,                                                          \
                [&](int r) { launch_pm<DT, OP, K, kPolNtLoad, 4, 256>(params(r, DT, ARG), P); }, {}});          \
  vs.push_back({"u32 sum production", I, false, true, [&](int r) {                                              \
                  reduce_copy_kernel<nexrUint32, nexrDevSum, K, kPolNtLoad>                                     \
                      <<<(int)(P / 1024), block_for(nexrUint32, K, kPolNtLoad)>>>(params(r, nexrUint32, 0));    \
                }, {}});                                                                                        \
  vs.push_back({"u32 sum pack-major U2 B512", I, false, true,                                                   \
                [&](int r) { launch_pm<nexrUint32, nexrDevSum, K, kPolNtLoad, 2, 512>(params(r, nexrUint32, 0), P); }, {}});
  CFG(0, nexrInt8, nexrDevMinMax, 0x80)
  CFG(1, nexrInt8, nexrDevMinMax, 0x7f)
  CFG(2, nexrInt8, nexrDevProd, 0)
  CFG(3, nexrInt32, nexrDevMinMax, 0x80000000ull)
  CFG(4, nexrInt32, nexrDevMinMax, 0x7fffffffull)
  CFG(5, nexrInt32, nexrDevProd, 0)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {  // every variant against the production kernel of its configuration (or the uint32 production)
    std::vector<char> ref(bytes), got(bytes);
    const Var* base = nullptr;
    const Var* ubase = nullptr;
    for (auto& v : vs) {
      if (v.base) base = &v;
      if (v.u32 && v.name == "u32 sum production") ubase = &v;
      const Var* b = v.u32 ? ubase : base;
      if (b == &v) continue;
      b->run(0);
      CK(hipMemcpy(ref.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      CK(hipMemset(ps[0].dst[0], 0, bytes));
      v.run(0);
      CK(hipMemcpy(got.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      printf("%s %s: %s\n", cfgs[v.cfg], v.name.c_str(), memcmp(ref.data(), got.data(), bytes) ? "MISMATCH" : "bytes match");
    }
  }
  const int BLK = 6;  // launches per timed block, rotating over the R sets
  for (int it = 0; it < blocks; it++)
    for (auto& v : vs) {
      v.run((it + BLK - 1) % R);
      CK(hipEventRecord(e0));
      for (int bb = 0; bb < BLK; bb++) v.run((it + bb) % R);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.us.push_back(ms * 1e3f / BLK);
    }
  const double alg = (double)(K + 1) * bytes;
  printf("\nbuffer = %zu MiB, K = 4, M = 1; median (mean) us of %d blocks of %d launches over %d rotating sets; "
         "GB/s and fraction of 8 TB/s from the median\n",
         bytes >> 20, blocks, BLK, R);
  for (int c = 0; c < 6; c++) {
    double u32med = 0;
    for (auto& v : vs)
      if (v.cfg == c && v.u32 && v.name == "u32 sum production") {
        std::vector<float> s = v.us;
        std::sort(s.begin(), s.end());
        u32med = s[s.size() / 2];
      }
    printf("%s\n", cfgs[c]);
    for (auto& v : vs) {
      if (v.cfg != c) continue;
      std::vector<float> s = v.us;
      std::sort(s.begin(), s.end());
      double med = s[s.size() / 2], mean = 0;
      for (float x : s) mean += x;
      mean /= s.size();
      printf("  %-28s %8.2f (%8.2f) us  %6.0f GB/s  %.4f  over u32 sum %.4f\n", v.name.c_str(), med, mean,
             alg / med / 1e3, alg / med / 1e3 / 8000.0, med / u32med);
    }
  }
  return 0;
}
