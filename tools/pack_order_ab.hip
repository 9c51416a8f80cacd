// Load / store order inside a trip, A/B on the production kernel (tuning harness, not product code;
// VERDICT r03 "next" #3).
//
// reduce_copy_kernel<..., PM> (nexr_kernels.hip body()): PM = false is the round-1..3 order — every
// source's pack u = 0 is loaded, then u = 1, ..., and every pack is stored after the last fold, so the
// first fold waits for almost all of the lane's K x U loads. PM = true loads pack by pack and stores
// each pack right after its fold, so pack 0 folds and leaves while pack 1's loads still arrive. The
// same loads are in flight either way; only their order and the stores' timing differ. With U = 1
// (the 16-bit K = 8 geometry, K = 4 beyond 512 MiB) the two are the same code.
// tools/fold8_ab.hip measured a stand-alone pack-major trip on C4 (int8 min/max/prod 1.001-0.989 of
// a uint32 sum instead of 1.006-1.007; profiles/r04a_fold8_ab.txt); this runs the production
// kernel itself, both orders, on every geometry where U > 1, every variant byte-checked against
// production, beside the uint32 sum of the same bytes, interleaved in blocks on 3 rotating sets.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=0 tools/pack_order_ab.hip -o tools/pack_order_ab
//   ./tools/pack_order_ab <blocks>
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

struct Cfg {
  const char* name;
  int esz;  // element size of the configuration's datatype
  int k, m;
  size_t bytes;
  uint32_t mask;
  std::function<void(const RCParams&, int, bool)> run;  // (params, grid, pack-major)
  std::function<void(const RCParams&, int)> u32;
};

template <int D, int OP, int K, int POL>
void launch(const RCParams& p, int grid, bool pm) {
  constexpr int U = unroll_for(D, K, POL), B = block_for(D, K, POL);
  if (pm) reduce_copy_kernel<D, OP, K, POL, U, B, true><<<grid, B>>>(p);
  else reduce_copy_kernel<D, OP, K, POL, U, B, false><<<grid, B>>>(p);
}

template <int K, int POL>
void launch_u32(const RCParams& p, int grid) {
  reduce_copy_kernel<nexrUint32, nexrDevSum, K, POL><<<grid, block_for(nexrUint32, K, POL)>>>(p);
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 10;
  const uint32_t all = 0xffffffffu, fin = 0xbfffffffu;  // fin: fp32/bf16 exponents below all-ones
  std::vector<Cfg> cfgs = {
      {"C2 fp32 sum K=2 256MiB (nt/nt, U4 B256)", 4, 2, 1, 256u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrFloat32, nexrDevSum, 2, kPolNt>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<2, kPolNt>(p, g); }},
      {"C4 int8 min K=4 64MiB (nt load, U2 B512)", 1, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt8, nexrDevMinMax, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"C4 int8 max K=4 64MiB", 1, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt8, nexrDevMinMax, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"C4 int8 prod K=4 64MiB", 1, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt8, nexrDevProd, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"C4 int32 min K=4 64MiB", 4, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt32, nexrDevMinMax, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"C4 int32 max K=4 64MiB", 4, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt32, nexrDevMinMax, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"C4 int32 prod K=4 64MiB", 4, 4, 1, 64u << 20, all,
       [](const RCParams& p, int g, bool pm) { launch<nexrInt32, nexrDevProd, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"bf16 sum K=4 64MiB (U2 B512)", 2, 4, 1, 64u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrBfloat16, nexrDevSum, 4, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<4, kPolNtLoad>(p, g); }},
      {"fp32 sum K=3 64MiB (U4 B256)", 4, 3, 1, 64u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrFloat32, nexrDevSum, 3, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<3, kPolNtLoad>(p, g); }},
      {"fp32 sum K=2 M=2 64MiB (recvReduceCopySend)", 4, 2, 2, 64u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrFloat32, nexrDevSum, 2, kPolNtLoad>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<2, kPolNtLoad>(p, g); }},
      {"fp32 sum K=2 16MiB (plain, a ring slice's regime)", 4, 2, 1, 16u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrFloat32, nexrDevSum, 2, kPolPlain>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<2, kPolPlain>(p, g); }},
      {"fp16 sum K=2 256MiB (nt/nt, U4 B256)", 2, 2, 1, 256u << 20, fin,
       [](const RCParams& p, int g, bool pm) { launch<nexrFloat16, nexrDevSum, 2, kPolNt>(p, g, pm); },
       [](const RCParams& p, int g) { launch_u32<2, kPolNt>(p, g); }},
  };
  const uint64_t redArgs[] = {0, 0x80, 0x7f, 0, 0x80000000ull, 0x7fffffffull, 0, 0, 0, 0, 0, 0};
  const int R = 3, BLK = 6;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("production (PM=0: source-major loads, stores after the last fold) vs pack-major (PM=1); median (mean) us\n"
         "of %d blocks of %d launches over %d rotating sets, interleaved; fraction of 8 TB/s from the median;\n"
         "u32 = a uint32 sum of the same bytes (the bench's kernel_over_u32_sum floor)\n\n", blocks, BLK, R);
  for (size_t c = 0; c < cfgs.size(); c++) {
    const Cfg& cf = cfgs[c];
    std::vector<RCParams> ps(R);
    std::vector<char*> owned;
    for (int r = 0; r < R; r++) {
      RCParams& p = ps[r];
      std::memset((void*)&p, 0, sizeof(p));
      for (int s = 0; s < cf.k; s++) {
        char* q;
        CK(hipMalloc((void**)&q, cf.bytes));
        fill_bits<<<2048, 256>>>((uint32_t*)q, cf.bytes / 4, 1000 + c * 64 + r * 16 + s, cf.mask);
        p.src[s] = q;
        owned.push_back(q);
      }
      for (int d = 0; d < cf.m; d++) {
        CK(hipMalloc((void**)&p.dst[d], cf.bytes));
        owned.push_back(p.dst[d]);
      }
      p.nDsts = cf.m;
      p.nPacks = cf.bytes / 16;
      p.nElts = cf.bytes / cf.esz;  // the whole buffer is packed body: no head, no tail
      p.head = 0;
      p.redArg = redArgs[c];
    }
    // What the kernel and its one-shot grid assume, checked on the host before any launch.
    for (int r = 0; r < R; r++) {
      const RCParams& p = ps[r];
      if (p.nElts * (uint64_t)cf.esz != p.nPacks * 16 || p.head != 0 || p.nPacks % kTripPacks != 0 ||
          p.nDsts != cf.m || cf.k > NEXR_MAX_SRCS || cf.m > NEXR_MAX_DSTS) {
        fprintf(stderr, "bad parameters for %s\n", cf.name);
        return 2;
      }
      for (int s = 0; s < cf.k; s++)
        if (!p.src[s]) return 2;
      for (int d = 0; d < cf.m; d++)
        if (!p.dst[d]) return 2;
    }
    CK(hipDeviceSynchronize());
    const int grid = (int)(cf.bytes / 16 / kTripPacks);
    // byte check: PM=1 against PM=0 on set 0 (every destination)
    {
      std::vector<char> ref(cf.bytes), got(cf.bytes);
      bool ok = true;
      cf.run(ps[0], grid, false);
      CK(hipDeviceSynchronize());
      std::vector<std::vector<char>> refs(cf.m, std::vector<char>(cf.bytes));
      for (int d = 0; d < cf.m; d++) CK(hipMemcpy(refs[d].data(), ps[0].dst[d], cf.bytes, hipMemcpyDeviceToHost));
      for (int d = 0; d < cf.m; d++) CK(hipMemset(ps[0].dst[d], 0, cf.bytes));
      cf.run(ps[0], grid, true);
      CK(hipDeviceSynchronize());
      for (int d = 0; d < cf.m; d++) {
        CK(hipMemcpy(got.data(), ps[0].dst[d], cf.bytes, hipMemcpyDeviceToHost));
        ok = ok && memcmp(refs[d].data(), got.data(), cf.bytes) == 0;
      }
      printf("%s\n  pack-major bytes %s production's\n", cf.name, ok ? "match" : "MISMATCH");
    }
    RCParams pu[3];
    for (int r = 0; r < R; r++) {
      pu[r] = ps[r];
      pu[r].redArg = 0;
      pu[r].nElts = cf.bytes / 4;
    }
    std::vector<std::function<void(int)>> vs = {[&](int r) { cf.run(ps[r], grid, false); },
                                                 [&](int r) { cf.run(ps[r], grid, true); },
                                                 [&](int r) { cf.u32(pu[r], grid); }};
    const char* names[] = {"production (PM=0)", "pack-major (PM=1)", "u32 sum (production)"};
    std::vector<std::vector<float>> us(vs.size());
    for (auto& v : vs)
      for (int w = 0; w < 2; w++) v(w % R);
    for (int it = 0; it < blocks; it++)
      for (size_t vi = 0; vi < vs.size(); vi++) {
        const size_t v = (it % 2) ? vs.size() - 1 - vi : vi;  // alternate the order every block
        vs[v]((it + BLK - 1) % R);
        CK(hipEventRecord(e0));
        for (int bb = 0; bb < BLK; bb++) vs[v]((it + bb) % R);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        us[v].push_back(ms * 1e3f / BLK);
      }
    const double alg = (double)(cf.k + cf.m) * cf.bytes;
    std::vector<double> med(vs.size());
    for (size_t v = 0; v < vs.size(); v++) {
      std::vector<float> s = us[v];
      std::sort(s.begin(), s.end());
      med[v] = s[s.size() / 2];
    }
    for (size_t v = 0; v < vs.size(); v++) {
      double mean = 0;
      for (float x : us[v]) mean += x;
      mean /= us[v].size();
      printf("  %-22s %8.2f (%8.2f) us  %6.0f GB/s  %.4f  over u32 %.4f  over production %.4f\n", names[v], med[v], mean,
             alg / med[v] / 1e3, alg / med[v] / 1e3 / 8000.0, med[v] / med[2], med[v] / med[0]);
    }
    for (char* q : owned) CK(hipFree(q));
  }
  return 0;
}
