// Is the 8-bit K = 4 reduce-copy ALU-bound anywhere? (tuning harness, not product code)
//
// C4's int8 min/max/prod ran 2-4 % below the int32 ones on the same bytes (64 MiB per buffer, K = 4,
// same geometry). The 8-bit fold splits every source into even/odd 16-bit lanes, folds with packed
// 16-bit ops and joins with v_perm (Fold8, nexr_types.hpp): ~15 VALU ops per dword against 3 for
// int32. First run (profiles/r02_alu_probe_k4.log): int8 min 53.9 us at U4 B256, 52.7-52.9 at
// U2 B512 (= int32 min at U4 B256), 56.8-57.1 at U1 B1024; an XOR fold (no split/join) 52.2 — the
// fold's latency shows, and twice the waves per workgroup hide it. This version sweeps 8-bit sum / min /
// max / prod at K = 2, 4, 8 and int32 min / prod at K = 4, U4 B256 against U2 B512 (the same 16 KiB
// trip; each U2 variant checked byte for byte against its U4 twin), plus the XOR-fold floor
// (profiles/r02_alu_probe_8bit_sweep.log). tools/geom_sweep.hip then covers every datatype and K.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=0 tools/alu_probe.hip -o tools/alu_probe
//   ./tools/alu_probe <MiB per buffer> <iters>
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

template <int K, int U, int B>
__global__ __launch_bounds__(B) void k_xor(RCParams p) {
  const uint64_t base = (uint64_t)blockIdx.x * B * U * 16;
  u32x4 in[U][K];
#pragma unroll
  for (int s = 0; s < K; s++)
#pragma unroll
    for (int u = 0; u < U; u++) in[u][s] = ld16<kPolNtLoad>(p.src[s] + base + (threadIdx.x + u * B) * 16);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 r = in[u][0];
#pragma unroll
    for (int s = 1; s < K; s++) r ^= in[u][s];
    st16<kPolNtLoad>(p.dst[0] + base + (threadIdx.x + u * B) * 16, r);
  }
}

struct Var {
  std::string name;
  std::function<void(int)> run;
  bool check;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 64) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  constexpr int K = 8;  // buffers allocated for the largest fan-in swept
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
    q.nElts = bytes / (dt == nexrInt32 ? 4 : 1);  // (K is the kernel's template argument)
    q.redArg = arg;
    return q;
  };
  const uint64_t minArg8 = 0x80, minArg32 = 0x80000000ull;  // hostToDevRedOp: signed min xormask
  std::vector<Var> vs;
  // (dt, op, K) x {U4 B256 (production for 8-bit today), U2 B512}: checked byte for byte against each other
#define GEO(DT, OP, KK, ARG, NAME)                                                                                 \
  vs.push_back({std::string(NAME " K" #KK " U4 B256"), [&](int r) {                                                \
                  reduce_copy_kernel<DT, OP, KK, kPolNtLoad, 4, 256><<<(int)(P / 1024), 256>>>(params(r, DT, ARG)); \
                }, false, {}});                                                                                     \
  vs.push_back({std::string(NAME " K" #KK " U2 B512"), [&](int r) {                                                \
                  reduce_copy_kernel<DT, OP, KK, kPolNtLoad, 2, 512><<<(int)(P / 1024), 512>>>(params(r, DT, ARG)); \
                }, true, {}});
  GEO(nexrInt8, nexrDevMinMax, 4, minArg8, "int8 min")
  GEO(nexrInt8, nexrDevMinMax, 4, minArg8 ^ 0xff, "int8 max")
  GEO(nexrInt8, nexrDevProd, 4, 0, "int8 prod")
  GEO(nexrInt8, nexrDevSum, 4, 0, "int8 sum")
  GEO(nexrUint8, nexrDevMinMax, 4, 0, "uint8 min")
  GEO(nexrInt8, nexrDevMinMax, 2, minArg8, "int8 min")
  GEO(nexrInt8, nexrDevSum, 2, 0, "int8 sum")
  GEO(nexrInt8, nexrDevMinMax, 8, minArg8, "int8 min")
  GEO(nexrInt8, nexrDevProd, 8, 0, "int8 prod")
  GEO(nexrInt8, nexrDevSum, 8, 0, "int8 sum")
  GEO(nexrInt32, nexrDevMinMax, 4, minArg32, "int32 min")
  GEO(nexrInt32, nexrDevProd, 4, 0, "int32 prod")
  vs.push_back({"xor fold K4 U4 B256", [&](int r) { k_xor<4, 4, 256><<<(int)(P / 1024), 256>>>(ps[r]); }, false, {}});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {  // every U2 B512 variant against the U4 B256 variant of the same (dt, op, K) just before it
    std::vector<char> ref(bytes), got(bytes);
    for (size_t i = 1; i < vs.size(); i++) {
      if (!vs[i].check) continue;
      vs[i - 1].run(0);
      CK(hipMemcpy(ref.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      CK(hipMemset(ps[0].dst[0], 0, bytes));
      vs[i].run(0);
      CK(hipMemcpy(got.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      if (memcmp(ref.data(), got.data(), bytes) != 0) printf("MISMATCH: %s\n", vs[i].name.c_str());
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
  printf("buffer=%zu MiB, GB/s of (K+1) x buffer (median / best of %d blocks of %d launches)\n", bytes >> 20,
         iters, BLK);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const int kk = v.name[v.name.find(" K") + 2] - '0';
    const double alg = (double)(kk + 1) * bytes;
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-34s med %8.2f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6);
  }
  return 0;
}
