// Workgroups per CU, swept with an LDS reservation (tuning harness, not product code).
//
// tools/body_ab.hip (profiles/r05a_body_ab.txt) found the 16-bit K = 8 kernels 2-2.5 % faster held
// to one 1024-lane workgroup per CU than at the two that their round-5 register count allows, with
// the same code. Every trip of every configuration keeps K x U 16-B loads per lane in flight, so a
// CU's bytes in flight are (workgroups per CU) x (lanes per workgroup) x K x U x 16: this sweeps that
// count for each bench configuration and workgroup shape by launching the production kernel with a
// dynamic LDS reservation of 160 KiB / n (rounded), which admits n workgroups per CU and changes
// nothing in the code. Every variant is byte-checked against the configuration's production launch.
// Blocks of launches over three rotating buffer sets, interleaved, order alternated.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=6 tools/occupancy_ab.hip -o tools/occupancy_ab
//   ./tools/occupancy_ab <blocks>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// Round 5's bfloat16 fold, kept verbatim here as the A/B baseline of the round-6 one (group "bf16cvt"):
// integer RNE with a NaN select after every step (nexr_types.hpp at 3c2cdf3).
constexpr int kBf16IntRne = 100;
namespace nexr {
template <> struct Ty<kBf16IntRne> {
  using V = u16x8;
  static constexpr int EPP = 8;
  static constexpr bool kIsInt = false;
  static constexpr bool kCanon = false;
  __device__ static f32x8 widen(V x) { return bc<f32x8>(__builtin_convertvector(x, u32x8) << 16); }
  __device__ static V narrow(f32x8 f) {
    u32x8 u = bc<u32x8>(f);
    u32x8 r = (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
    i32x8 isnan = (u & 0x7fffffffu) > 0x7f800000u;
    r = isnan ? (u32x8)0x7fffu : r;
    return __builtin_convertvector(r, V);
  }
  __device__ static V add(V a, V b) { return narrow(widen(a) + widen(b)); }
  __device__ static V mul(V a, V b) { return narrow(widen(a) * widen(b)); }
  __device__ static V vmin(V c, V v) {
    f32x8 fc = widen(c), fv = widen(v);
    return narrow(fv < fc ? fv : fc);
  }
  __device__ static V vmax(V c, V v) {
    f32x8 fc = widen(c), fv = widen(v);
    return narrow(fv > fc ? fv : fc);
  }
  __device__ static V splat(uint64_t raw) { return (V)((uint16_t)raw); }
  __device__ static V canon(V x) { return x; }
  __device__ static V divide(V x, uint64_t) { return x; }
};
}  // namespace nexr

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed, uint32_t mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31)) & mask;
  }
}

constexpr int kLdsPerCu = 160 * 1024;
// Dynamic LDS that admits exactly n workgroups per CU (0: no reservation).
int lds_for(int n) {
  if (n <= 0) return 0;
  const int hi = kLdsPerCu / n, lo = kLdsPerCu / (n + 1);
  return ((lo + hi) / 2) & ~1023;
}

struct Var {
  std::string name;
  const void* fn;
  int block;
  int wgs;  // target workgroups per CU (0 = as the registers allow)
  int esz;
  int trip;  // packs per workgroup trip (U x B)
  uint64_t redArg;
  int k;  // the fan-in the kernel was compiled for: must equal the configuration's source count
  unsigned grid = 0;  // workgroups of the launch (0: one-shot, one per trip); fewer: the kernel grid-strides
};
struct Cfg {
  const char* name;
  int k;
  size_t bytes;
  uint32_t mask;
  std::vector<Var> vars;
  int m = 1;  // destinations (all written; the byte check reads the first)
};

template <int D, int OP, int K, int POL, bool IsMin, int U, int B>
Var var(const char* geom, int wgs, uint64_t redArg = 0) {
  char buf[128];
  snprintf(buf, sizeof buf, "%s, %d WG/CU%s", geom, wgs > 0 ? wgs : 0, wgs > 0 ? "" : " (registers)");
  return Var{buf, (const void*)&reduce_copy_kernel<D, OP, K, POL, IsMin, U, B>, B, wgs, 16 / Ty<D>::EPP, U * B, redArg, K};
}

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 10;
  // group "bench" (default): the bench configurations; "wide": fan-in 6 and 8 of every element size,
  // production geometry against one 1024-lane workgroup per CU
  const std::string group = argc > 2 ? argv[2] : "bench";
  const uint32_t all = 0xffffffffu, fin = 0x3bff3bffu;
  std::vector<Cfg> cfgs;
  if (group == "wide") {
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"fp32 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1),
                       var<D, OP, K, P, false, 1, 1024>("U1 B1024", 0), var<D, OP, K, P, false, 2, 512>("U2 B512", 2)}});
    }
    {
      constexpr int D = nexrUint32, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"uint32 sum K=8 256 MiB (nt/nt)", K, 256u << 20, all,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1)}});
    }
    {
      constexpr int D = nexrFloat64, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"fp64 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1)}});
    }
    {
      constexpr int D = nexrInt8, OP = nexrDevMinMax, K = 8, P = kPolNt;
      cfgs.push_back({"int8 max K=8 256 MiB (nt/nt)", K, 256u << 20, all,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0, 0x7f),
                       var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1, 0x7f)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 6, P = kPolNt;
      cfgs.push_back({"fp32 sum K=6 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1),
                       var<D, OP, K, P, false, 2, 512>("U2 B512", 2)}});
    }
    {
      constexpr int D = nexrFloat16, OP = nexrDevSum, K = 6, P = kPolNt;
      cfgs.push_back({"fp16 sum K=6 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 8, P = kPolNtLoad;
      cfgs.push_back({"fp32 sum K=8 32 MiB (nt loads)", K, 32u << 20, fin,
                      {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1)}});
    }
  }
  if (group == "k8shape") {  // the 16-bit K = 8 workgroup shape at one and more workgroups per CU
    constexpr int D = nexrFloat16, OP = nexrDevSum, K = 8, P = kPolNt;
    cfgs.push_back({"fp16 sum K=8 256 MiB (nt/nt): workgroup shape x workgroups per CU", K, 256u << 20, fin,
                    {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 1),
                     var<D, OP, K, P, false, 1, 512>("U1 B512", 2), var<D, OP, K, P, false, 1, 512>("U1 B512", 3),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 1), var<D, OP, K, P, false, 1, 256>("U1 B256", 2),
                     var<D, OP, K, P, false, 1, 256>("U1 B256", 4), var<D, OP, K, P, false, 1, 256>("U1 B256", 6),
                     var<D, OP, K, P, false, 2, 256>("U2 B256", 2), var<D, OP, K, P, false, 1, 768>("U1 B768", 1)}});
    constexpr int D2 = nexrFloat32, K2 = 2;
    cfgs.push_back({"fp32 sum K=2 256 MiB (nt/nt): workgroup shape x workgroups per CU", K2, 256u << 20, fin,
                    {var<D2, OP, K2, P, false, 4, 256>("U4 B256", 0), var<D2, OP, K2, P, false, 2, 1024>("U2 B1024", 2),
                     var<D2, OP, K2, P, false, 4, 1024>("U4 B1024", 1), var<D2, OP, K2, P, false, 4, 512>("U4 B512", 2),
                     var<D2, OP, K2, P, false, 8, 256>("U8 B256", 0), var<D2, OP, K2, P, false, 8, 256>("U8 B256", 4)}});
  }
  if (group == "c4pol") {  // C4's 64 MiB buffers (320 MiB streamed) under the nt-store policy too
    {
      constexpr int D = nexrInt8, OP = nexrDevMinMax, K = 4;
      cfgs.push_back({"C4 int8 max K=4 64 MiB: nt loads (production) vs nt loads + stores", K, 64u << 20, all,
                      {var<D, OP, K, kPolNtLoad, false, 2, 512>("nt-ld U2 B512", 0, 0x7f),
                       var<D, OP, K, kPolNt, false, 2, 512>("nt-st U2 B512", 0, 0x7f),
                       var<D, OP, K, kPolNt, false, 1, 1024>("nt-st U1 B1024", 1, 0x7f),
                       var<D, OP, K, kPolNt, false, 1, 512>("nt-st U1 B512", 2, 0x7f),
                       var<D, OP, K, kPolNt, false, 4, 256>("nt-st U4 B256", 0, 0x7f),
                       var<D, OP, K, kPolPlain, false, 2, 512>("plain U2 B512", 0, 0x7f)}});
    }
    {
      constexpr int D = nexrInt32, OP = nexrDevMinMax, K = 4;
      cfgs.push_back({"C4 int32 min K=4 64 MiB: nt loads (production) vs nt loads + stores", K, 64u << 20, all,
                      {var<D, OP, K, kPolNtLoad, true, 2, 512>("nt-ld U2 B512", 0, 0x80000000ull),
                       var<D, OP, K, kPolNt, true, 2, 512>("nt-st U2 B512", 0, 0x80000000ull),
                       var<D, OP, K, kPolNt, true, 1, 1024>("nt-st U1 B1024", 1, 0x80000000ull),
                       var<D, OP, K, kPolNt, true, 1, 512>("nt-st U1 B512", 2, 0x80000000ull)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 2;
      cfgs.push_back({"fp32 sum K=2 64 MiB (192 MiB streamed): plain vs nt loads vs nt loads + stores", K, 64u << 20, fin,
                      {var<D, OP, K, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, K, kPolNt, false, 4, 256>("nt-st U4 B256", 0),
                       var<D, OP, K, kPolPlain, false, 4, 256>("plain U4 B256", 0)}});
    }
  }
  if (group == "ntstore") {  // where the nt-store policy starts to pay, by fan-in and size
    constexpr int D = nexrFloat32, OP = nexrDevSum;
    for (int mib : {16, 32, 64, 128}) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=2 %d MiB (%d MiB streamed)", mib, 3 * mib);
      cfgs.push_back({name, 2, (size_t)mib << 20, fin,
                      {var<D, OP, 2, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, 2, kPolNt, false, 4, 256>("nt-st U4 B256", 0),
                       var<D, OP, 2, kPolPlain, false, 4, 256>("plain U4 B256", 0)}});
    }
    for (int mib : {16, 48}) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=8 %d MiB (%d MiB streamed)", mib, 9 * mib);
      cfgs.push_back({name, 8, (size_t)mib << 20, fin,
                      {var<D, OP, 8, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, 8, kPolNt, false, 1, 512>("nt-st U1 B512", 1),
                       var<D, OP, 8, kPolNtLoad, false, 1, 512>("nt-ld U1 B512", 1)}});
    }
    {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=3 64 MiB (256 MiB streamed)");
      cfgs.push_back({name, 3, 64u << 20, fin,
                      {var<D, OP, 3, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, 3, kPolNt, false, 4, 256>("nt-st U4 B256", 0)}});
    }
  }
  if (group == "ntstore2") {  // the policy edge for K = 1 copies and K = 2, M = 2 ring steps (96-512 MiB streamed)
    constexpr int D = nexrFloat32, OP = nexrDevSum;
    for (int mib : {32, 48, 64, 128, 192, 255}) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 copy K=1 M=1 %d MiB (%d MiB streamed)", mib, 2 * mib);
      cfgs.push_back({name, 1, (size_t)mib << 20, fin,
                      {var<D, OP, 1, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, 1, kPolNt, false, 4, 256>("nt-st U4 B256", 0),
                       var<D, OP, 1, kPolPlain, false, 4, 256>("plain U4 B256", 0)}});
    }
    for (int mib : {16, 24, 32, 64, 96, 127}) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=2 M=2 %d MiB (%d MiB streamed)", mib, 4 * mib);
      cfgs.push_back({name, 2, (size_t)mib << 20, fin,
                      {var<D, OP, 2, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, 2, kPolNt, false, 4, 256>("nt-st U4 B256", 0),
                       var<D, OP, 2, kPolPlain, false, 4, 256>("plain U4 B256", 0)}, 2});
    }
  }
  if (group == "ntstore3") {  // the tree schedule's other shapes: K = 1 with M = 3-4, K = 3-4 with M = 2
    constexpr int D = nexrFloat32, OP = nexrDevSum;
    struct KM { int k, m, mib; };
    const bool wideM = argc > 3 && std::string(argv[3]) == "m5";  // M = 5-8 (ntstore3 m5)
    const std::vector<KM> shapes = wideM ? std::vector<KM>{KM{1, 5, 16}, KM{1, 5, 48}, KM{1, 8, 12}, KM{1, 8, 32},
                                                           KM{2, 6, 12}, KM{2, 6, 36}, KM{3, 5, 12}, KM{3, 5, 32}}
                                         : std::vector<KM>{KM{1, 3, 24}, KM{1, 3, 64}, KM{1, 4, 20}, KM{1, 4, 60}, KM{3, 2, 20},
                                                           KM{3, 2, 60}, KM{3, 1, 32}, KM{4, 2, 16}, KM{4, 2, 48}};
    for (KM c : shapes) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=%d M=%d %d MiB (%d MiB streamed)", c.k, c.m, c.mib, (c.k + c.m) * c.mib);
      std::vector<Var> v;
#define NT3(K)                                                                                           \
  v = {var<D, OP, K, kPolNtLoad, false, unroll_for(D, K, kPolNtLoad), block_for(D, K, kPolNtLoad)>("nt-ld", 0), \
       var<D, OP, K, kPolNt, false, unroll_for(D, K, kPolNt), block_for(D, K, kPolNt)>("nt-st", lds_for(D, K, kPolNt) ? 1 : 0), \
       var<D, OP, K, kPolPlain, false, 4, 256>("plain", 0)};
      if (c.k == 1) { NT3(1) } else if (c.k == 2) { NT3(2) } else if (c.k == 3) { NT3(3) } else { NT3(4) }
#undef NT3
      cfgs.push_back({name, c.k, (size_t)c.mib << 20, fin, v, c.m});
    }
  }
  if (group == "ntstore4") {  // round 6: K = 2 with M = 7-8, K = 3 with M = 6-8 at 100-510 MiB streamed,
                               // and K = 5-8 (M = 1) just below the 512 MiB nt-store threshold
    constexpr int D = nexrFloat32, OP = nexrDevSum;
    struct KM { int k, m, mib; };
    const std::vector<KM> shapes = {KM{2, 7, 12}, KM{2, 7, 32}, KM{2, 7, 56}, KM{2, 8, 12}, KM{2, 8, 30}, KM{2, 8, 50},
                                    KM{3, 6, 12}, KM{3, 6, 32}, KM{3, 6, 56}, KM{3, 7, 11}, KM{3, 7, 30},
                                    KM{3, 7, 50}, KM{3, 8, 10}, KM{3, 8, 26}, KM{3, 8, 46}, KM{5, 1, 80},
                                    KM{5, 1, 85}, KM{6, 1, 69}, KM{6, 1, 73}, KM{8, 1, 53}, KM{8, 1, 56}};
    for (KM c : shapes) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=%d M=%d %d MiB (%d MiB streamed)", c.k, c.m, c.mib, (c.k + c.m) * c.mib);
      std::vector<Var> v;
#define NT4(K)                                                                                           \
  v = {var<D, OP, K, kPolNtLoad, false, unroll_for(D, K, kPolNtLoad), block_for(D, K, kPolNtLoad)>("nt-ld", 0), \
       var<D, OP, K, kPolNt, false, unroll_for(D, K, kPolNt), block_for(D, K, kPolNt)>("nt-st", lds_for(D, K, kPolNt) ? 1 : 0)};
      if (c.k == 2) { NT4(2) } else if (c.k == 3) { NT4(3) } else if (c.k == 5) { NT4(5) } else if (c.k == 6) { NT4(6) } else { NT4(8) }
#undef NT4
      cfgs.push_back({name, c.k, (size_t)c.mib << 20, fin, v, c.m});
    }
  }
  if (group == "c3pol") {  // C3 (K = 8, 256 MiB per buffer, 2.25 GiB streamed) and C2: nt stores or nt loads only
    {
      constexpr int D = nexrFloat16, OP = nexrDevSum, K = 8;
      cfgs.push_back({"C3 fp16 sum K=8 256 MiB: nt loads + stores (production) vs nt loads only", K, 256u << 20, fin,
                      {var<D, OP, K, kPolNt, false, 1, 512>("nt-st U1 B512", 1), var<D, OP, K, kPolNtLoad, false, 1, 512>("nt-ld U1 B512", 1),
                       var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 1),
                       var<D, OP, K, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0)}});
    }
    {
      constexpr int D = nexrBfloat16, OP = nexrDevSum, K = 8;
      cfgs.push_back({"C3 bf16 sum K=8 256 MiB: nt loads + stores (production) vs nt loads only", K, 256u << 20, fin,
                      {var<D, OP, K, kPolNt, false, 1, 1024>("nt-st U1 B1024", 1),
                       var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 1),
                       var<D, OP, K, kPolNtLoad, false, 1, 512>("nt-ld U1 B512", 1)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 2;
      cfgs.push_back({"C2 fp32 sum K=2 256 MiB: nt loads + stores (production) vs nt loads only vs plain", K, 256u << 20, fin,
                      {var<D, OP, K, kPolNt, false, 4, 256>("nt-st U4 B256", 0),
                       var<D, OP, K, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, K, kPolPlain, false, 4, 256>("plain U4 B256", 0)}});
    }
  }
  if (group == "k8mid") {  // 16-bit K = 8 below the nt-store policy: production 1 x 1024 at one workgroup per CU
    constexpr int OP = nexrDevSum, K = 8;
    for (int mib : {4, 16, 48}) {
      char* name = new char[96];
      snprintf(name, 96, "fp16 sum K=8 %d MiB (%d MiB streamed)", mib, 9 * mib);
      constexpr int D = nexrFloat16;
      if (mib == 4)
        cfgs.push_back({name, K, (size_t)mib << 20, fin,
                        {var<D, OP, K, kPolPlain, false, 1, 1024>("plain U1 B1024", 1), var<D, OP, K, kPolPlain, false, 4, 256>("plain U4 B256", 0),
                         var<D, OP, K, kPolPlain, false, 1, 512>("plain U1 B512", 1), var<D, OP, K, kPolPlain, false, 1, 1024>("plain U1 B1024", 0)}});
      else
        cfgs.push_back({name, K, (size_t)mib << 20, fin,
                        {var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 1), var<D, OP, K, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                         var<D, OP, K, kPolNtLoad, false, 1, 512>("nt-ld U1 B512", 1), var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 0),
                         var<D, OP, K, kPolNt, false, 1, 512>("nt-st U1 B512", 1)}});
    }
    for (int mib : {16, 48}) {
      char* name = new char[96];
      snprintf(name, 96, "bf16 sum K=8 %d MiB (%d MiB streamed)", mib, 9 * mib);
      constexpr int D = nexrBfloat16;
      cfgs.push_back({name, K, (size_t)mib << 20, fin,
                      {var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 1), var<D, OP, K, kPolNtLoad, false, 4, 256>("nt-ld U4 B256", 0),
                       var<D, OP, K, kPolNtLoad, false, 1, 1024>("nt-ld U1 B1024", 0), var<D, OP, K, kPolNt, false, 1, 1024>("nt-st U1 B1024", 1)}});
    }
  }
  if (group == "k35") {  // K = 3 and K = 5 under the nt-store policy (default 4 x 256): one workgroup per CU?
    constexpr int D = nexrFloat32, OP = nexrDevSum, P = kPolNt;
    cfgs.push_back({"fp32 sum K=3 256 MiB (1 GiB streamed, nt/nt)", 3, 256u << 20, fin,
                    {var<D, OP, 3, P, false, 4, 256>("U4 B256", 0), var<D, OP, 3, P, false, 1, 1024>("U1 B1024", 1),
                     var<D, OP, 3, P, false, 2, 512>("U2 B512", 1), var<D, OP, 3, P, false, 1, 512>("U1 B512", 1),
                     var<D, OP, 3, P, false, 1, 1024>("U1 B1024", 0), var<D, OP, 3, P, false, 4, 256>("U4 B256", 2)}});
    cfgs.push_back({"fp32 sum K=5 256 MiB (1.5 GiB streamed, nt/nt)", 5, 256u << 20, fin,
                    {var<D, OP, 5, P, false, 4, 256>("U4 B256", 0), var<D, OP, 5, P, false, 1, 1024>("U1 B1024", 1),
                     var<D, OP, 5, P, false, 1, 512>("U1 B512", 1), var<D, OP, 5, P, false, 1, 1024>("U1 B1024", 0),
                     var<D, OP, 5, P, false, 4, 256>("U4 B256", 2)}});
    constexpr int D2 = nexrBfloat16;
    cfgs.push_back({"bf16 sum K=5 256 MiB (1.5 GiB streamed, nt/nt)", 5, 256u << 20, fin,
                    {var<D2, OP, 5, P, false, 4, 256>("U4 B256", 0), var<D2, OP, 5, P, false, 1, 1024>("U1 B1024", 1),
                     var<D2, OP, 5, P, false, 1, 512>("U1 B512", 1)}});
  }
  if (group == "k3m") {  // K = 3 with 2-5 destinations under nt stores (96-512 MiB streamed): 4 x 256 or 1 x 1024 at one per CU
    constexpr int D = nexrFloat32, OP = nexrDevSum, P = kPolNt;
    struct KM { int m, mib; };
    for (KM c : {KM{2, 20}, KM{2, 60}, KM{5, 12}, KM{5, 32}}) {
      char* name = new char[96];
      snprintf(name, 96, "fp32 sum K=3 M=%d %d MiB (%d MiB streamed, nt/nt)", c.m, c.mib, (3 + c.m) * c.mib);
      cfgs.push_back({name, 3, (size_t)c.mib << 20, fin,
                      {var<D, OP, 3, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, 3, P, false, 4, 256>("U4 B256", 0),
                       var<D, OP, 3, P, false, 2, 512>("U2 B512", 1)}, c.m});
    }
  }
  if (group == "c4sizes") {  // C4's shape by buffer size: is 64 MiB short enough to pay a ramp / tail?
    constexpr int D = nexrInt32, OP = nexrDevMinMax, K = 4;
    for (int mib : {16, 32, 64, 96, 100}) {
      char* name = new char[96];
      snprintf(name, 96, "int32 min K=4 %d MiB (%d MiB streamed)", mib, 5 * mib);
      cfgs.push_back({name, K, (size_t)mib << 20, all,
                      {var<D, OP, K, kPolNtLoad, true, 2, 512>("nt-ld U2 B512", 0, 0x80000000ull),
                       var<D, OP, K, kPolNtLoad, true, 4, 256>("nt-ld U4 B256", 0, 0x80000000ull),
                       var<D, OP, K, kPolNt, true, 1, 1024>("nt-st U1 B1024", 1, 0x80000000ull)}});
    }
  }
  if (group == "c4types") {  // K = 4 under nt loads (C4's regime), 64 MiB: 2 x 512 against 4 x 256, by type
    constexpr int K = 4, P = kPolNtLoad;
#define C4T(D, OP, ISMIN, ARG, NAME, MASK)                                                                  \
  cfgs.push_back({NAME " K=4 64 MiB (nt loads)", K, 64u << 20, MASK,                                        \
                  {var<D, OP, K, P, ISMIN, 2, 512>("U2 B512", 0, ARG), var<D, OP, K, P, ISMIN, 4, 256>("U4 B256", 0, ARG), \
                   var<D, OP, K, P, ISMIN, 4, 256>("U4 B256", 4, ARG)}});
    C4T(nexrInt8, nexrDevMinMax, false, 0x7f, "int8 max", all)
    C4T(nexrInt8, nexrDevMinMax, true, 0x80, "int8 min", all)
    C4T(nexrInt8, nexrDevProd, false, 0, "int8 prod", all)
    C4T(nexrInt32, nexrDevMinMax, true, 0x80000000ull, "int32 min", all)
    C4T(nexrInt32, nexrDevProd, false, 0, "int32 prod", all)
    C4T(nexrFloat32, nexrDevSum, false, 0, "fp32 sum", fin)
    C4T(nexrBfloat16, nexrDevSum, false, 0, "bf16 sum", fin)
    C4T(nexrFloat16, nexrDevSum, false, 0, "fp16 sum", fin)
    C4T(nexrUint64, nexrDevSum, false, 0, "uint64 sum", all)
#undef C4T
  }
  if (group == "k8lanes") {  // lanes per CU at K >= 6: one workgroup of B lanes (U = 1) per CU
    {
      constexpr int D = nexrFloat16, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"fp16 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 1),
                       var<D, OP, K, P, false, 1, 256>("U1 B256", 1), var<D, OP, K, P, false, 1, 384>("U1 B384", 1),
                       var<D, OP, K, P, false, 1, 640>("U1 B640", 1), var<D, OP, K, P, false, 2, 256>("U2 B256", 1),
                       var<D, OP, K, P, false, 1, 128>("U1 B128", 2), var<D, OP, K, P, false, 1, 128>("U1 B128", 4)}});
    }
    {
      constexpr int D = nexrBfloat16, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"bf16 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 1),
                       var<D, OP, K, P, false, 1, 256>("U1 B256", 1)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 8, P = kPolNt;
      cfgs.push_back({"fp32 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 1),
                       var<D, OP, K, P, false, 1, 256>("U1 B256", 1)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 6, P = kPolNt;
      cfgs.push_back({"fp32 sum K=6 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 1),
                       var<D, OP, K, P, false, 1, 256>("U1 B256", 1)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K = 4, P = kPolNt;
      cfgs.push_back({"fp32 sum K=4 256 MiB (nt/nt)", K, 256u << 20, fin,
                      {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1),
                       var<D, OP, K, P, false, 1, 512>("U1 B512", 1), var<D, OP, K, P, false, 1, 512>("U1 B512", 2)}});
    }
    {
      constexpr int D = nexrInt8, OP = nexrDevMinMax, K = 4, P = kPolNtLoad;
      cfgs.push_back({"C4 int8 max K=4 64 MiB (nt loads)", K, 64u << 20, all,
                      {var<D, OP, K, P, false, 2, 512>("U2 B512", 0, 0x7f), var<D, OP, K, P, false, 1, 512>("U1 B512", 1, 0x7f),
                       var<D, OP, K, P, false, 1, 512>("U1 B512", 2, 0x7f), var<D, OP, K, P, false, 2, 512>("U2 B512", 2, 0x7f)}});
    }
  }
  if (group == "bf16cvt") {  // round 6: bf16 through v_cvt_pk_bf16_f32 + one final NaN canonicalisation
    constexpr int D = nexrBfloat16, D0 = kBf16IntRne, OP = nexrDevSum, K = 8, P = kPolNt;
    cfgs.push_back({"C3 bf16 sum K=8 256 MiB (nt/nt): hardware cvt (hw) vs round-5 integer RNE (int), lanes per CU", K,
                    256u << 20, fin,
                    {var<D0, OP, K, P, false, 1, 1024>("int U1 B1024", 1), var<D, OP, K, P, false, 1, 1024>("hw U1 B1024", 1),
                     var<D, OP, K, P, false, 1, 512>("hw U1 B512", 1), var<D, OP, K, P, false, 1, 512>("hw U1 B512", 2),
                     var<D0, OP, K, P, false, 1, 512>("int U1 B512", 2), var<D, OP, K, P, false, 2, 512>("hw U2 B512", 1),
                     var<D, OP, K, P, false, 1, 256>("hw U1 B256", 4)}});
    constexpr int F = nexrFloat16;
    cfgs.push_back({"C3 fp16 sum K=8 256 MiB (nt/nt): production and 2 x 512 per CU", K, 256u << 20, fin,
                    {var<F, OP, K, P, false, 1, 512>("U1 B512", 1), var<F, OP, K, P, false, 1, 512>("U1 B512", 2),
                     var<F, OP, K, P, false, 1, 256>("U1 B256", 4)}});
    constexpr int W = nexrUint32;
    cfgs.push_back({"uint32 sum K=8 256 MiB (nt/nt): the same bytes, bare stream", K, 256u << 20, all,
                    {var<W, OP, K, P, false, 1, 512>("U1 B512", 1), var<W, OP, K, P, false, 1, 512>("U1 B512", 2),
                     var<W, OP, K, P, false, 1, 1024>("U1 B1024", 1)}});
    constexpr int D4 = nexrFloat32, K4 = 4;
    cfgs.push_back({"fp32 sum K=4 256 MiB (nt/nt): 1 x 1024 (production) vs 2 x 512 per CU", K4, 256u << 20, fin,
                    {var<D4, OP, K4, P, false, 1, 1024>("U1 B1024", 1), var<D4, OP, K4, P, false, 1, 512>("U1 B512", 2),
                     var<D4, OP, K4, P, false, 2, 512>("U2 B512", 1)}});
    cfgs.push_back({"bf16 sum K=4 256 MiB (nt/nt): 1 x 1024 (production) vs 2 x 512 per CU", K4, 256u << 20, fin,
                    {var<D, OP, K4, P, false, 1, 1024>("hw U1 B1024", 1), var<D, OP, K4, P, false, 1, 512>("hw U1 B512", 2),
                     var<D0, OP, K4, P, false, 1, 1024>("int U1 B1024", 1)}});
  }
  if (group == "c4grid") {  // round 6: C4's ~3.6 us per launch inside the kernel: one-shot grid vs a grid-strided one
    constexpr int K = 4, P = kPolNtLoad;
    auto capped = [](Var v, unsigned grid) {
      v.grid = grid;
      v.name += ", grid " + std::to_string(grid);
      return v;
    };
    {
      constexpr int D = nexrInt32, OP = nexrDevMinMax;
      const Var one = var<D, OP, K, P, true, 4, 256>("U4 B256", 0, 0x80000000ull);
      cfgs.push_back({"C4 int32 min K=4 64 MiB (nt loads): one-shot 4096 workgroups vs grid-strided", K, 64u << 20, all,
                      {one, capped(one, 2048), capped(one, 1024), capped(one, 3072), var<D, OP, K, P, true, 2, 256>("U2 B256", 0, 0x80000000ull),
                       var<D, OP, K, P, true, 8, 256>("U8 B256", 0, 0x80000000ull)}});
    }
    {
      constexpr int D = nexrInt8, OP = nexrDevMinMax;
      const Var one = var<D, OP, K, P, false, 2, 512>("U2 B512", 0, 0x7f);
      cfgs.push_back({"C4 int8 max K=4 64 MiB (nt loads): one-shot 4096 workgroups vs grid-strided", K, 64u << 20, all,
                      {one, capped(one, 1024), capped(one, 512), capped(one, 2048), var<D, OP, K, P, false, 1, 512>("U1 B512", 0, 0x7f),
                       var<D, OP, K, P, false, 4, 512>("U4 B512", 0, 0x7f)}});
    }
    {
      constexpr int D = nexrFloat32, OP = nexrDevSum, K2 = 2;
      const Var one = var<D, OP, K2, kPolNt, false, 4, 256>("U4 B256", 0);
      cfgs.push_back({"C2 fp32 sum K=2 256 MiB (nt/nt): one-shot 16384 workgroups vs grid-strided", K2, 256u << 20, fin,
                      {one, capped(one, 2048), capped(one, 4096), capped(one, 8192)}});
    }
  }
  if (group == "k45") {  // round 6: K = 4-5 under nt stores, 1 x 1024 at one per CU (production) vs 1 x 512 at two
    constexpr int P = kPolNt;
#define K45(D, OP, K, ISMIN, ARG, NAME, MASK)                                                                \
  cfgs.push_back({NAME " K=" #K " 256 MiB (nt/nt)", K, 256u << 20, MASK,                                     \
                  {var<D, OP, K, P, ISMIN, 1, 1024>("U1 B1024", 1, ARG), var<D, OP, K, P, ISMIN, 1, 512>("U1 B512", 2, ARG), \
                   var<D, OP, K, P, ISMIN, 1, 1024>("U1 B1024", 1, ARG)}});
    K45(nexrFloat32, nexrDevSum, 4, false, 0, "fp32 sum", fin)
    K45(nexrBfloat16, nexrDevSum, 4, false, 0, "bf16 sum", fin)
    K45(nexrInt8, nexrDevMinMax, 4, false, 0x7f, "int8 max", all)
    K45(nexrInt32, nexrDevMinMax, 4, true, 0x80000000ull, "int32 min", all)
    K45(nexrFloat64, nexrDevSum, 4, false, 0, "fp64 sum", fin)
    K45(nexrFloat32, nexrDevSum, 5, false, 0, "fp32 sum", fin)
    K45(nexrBfloat16, nexrDevSum, 5, false, 0, "bf16 sum", fin)
    K45(nexrUint8, nexrDevProd, 5, false, 0, "uint8 prod", all)
#undef K45
  }
  if (group == "bench") {
  {
    constexpr int D = nexrFloat32, OP = nexrDevSum, K = 2, P = kPolNt;
    cfgs.push_back({"C2 fp32 sum K=2 256 MiB (nt/nt)", K, 256u << 20, fin,
                    {var<D, OP, K, P, false, 4, 256>("U4 B256", 0), var<D, OP, K, P, false, 4, 256>("U4 B256", 6),
                     var<D, OP, K, P, false, 4, 256>("U4 B256", 5), var<D, OP, K, P, false, 4, 256>("U4 B256", 4),
                     var<D, OP, K, P, false, 4, 256>("U4 B256", 3), var<D, OP, K, P, false, 4, 256>("U4 B256", 2),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 0), var<D, OP, K, P, false, 2, 512>("U2 B512", 2)}});
  }
  {
    constexpr int D = nexrFloat16, OP = nexrDevSum, K = 8, P = kPolNt;
    cfgs.push_back({"C3 fp16 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                    {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 0), var<D, OP, K, P, false, 2, 512>("U2 B512", 3),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 2), var<D, OP, K, P, false, 4, 256>("U4 B256", 0),
                     var<D, OP, K, P, false, 4, 256>("U4 B256", 6), var<D, OP, K, P, false, 4, 256>("U4 B256", 4)}});
  }
  {
    constexpr int D = nexrBfloat16, OP = nexrDevSum, K = 8, P = kPolNt;
    cfgs.push_back({"C3 bf16 sum K=8 256 MiB (nt/nt)", K, 256u << 20, fin,
                    {var<D, OP, K, P, false, 1, 1024>("U1 B1024", 0), var<D, OP, K, P, false, 1, 1024>("U1 B1024", 1),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 2), var<D, OP, K, P, false, 4, 256>("U4 B256", 4)}});
  }
  {
    constexpr int D = nexrInt8, OP = nexrDevMinMax, K = 4, P = kPolNtLoad;
    cfgs.push_back({"C4 int8 max K=4 64 MiB (nt loads)", K, 64u << 20, all,
                    {var<D, OP, K, P, false, 2, 512>("U2 B512", 0, 0x7f), var<D, OP, K, P, false, 2, 512>("U2 B512", 3, 0x7f),
                     var<D, OP, K, P, false, 2, 512>("U2 B512", 2, 0x7f), var<D, OP, K, P, false, 2, 512>("U2 B512", 1, 0x7f),
                     var<D, OP, K, P, false, 4, 256>("U4 B256", 0, 0x7f), var<D, OP, K, P, false, 4, 256>("U4 B256", 4, 0x7f)}});
  }
  {
    constexpr int D = nexrInt32, OP = nexrDevMinMax, K = 4, P = kPolNtLoad;
    cfgs.push_back({"C4 int32 min K=4 64 MiB (nt loads)", K, 64u << 20, all,
                    {var<D, OP, K, P, true, 2, 512>("U2 B512", 0, 0x80000000ull),
                     var<D, OP, K, P, true, 2, 512>("U2 B512", 3, 0x80000000ull),
                     var<D, OP, K, P, true, 2, 512>("U2 B512", 2, 0x80000000ull),
                     var<D, OP, K, P, true, 2, 512>("U2 B512", 1, 0x80000000ull)}});
  }
  }
  const int R = 3, BLK = 6;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("median (mean) us of %d blocks of %d launches over %d rotating sets, interleaved; fraction of 8 TB/s\n"
         "from the median; 'vs first' = median over the first variant's (production) median; in flight = bytes of\n"
         "loads outstanding per CU when every admitted lane has issued its trip\n\n", blocks, BLK, R);
  for (size_t c = 0; c < cfgs.size(); c++) {
    Cfg& cf = cfgs[c];
    std::vector<RCParams> base(R);
    std::vector<char*> owned;
    for (int r = 0; r < R; r++) {
      RCParams& p = base[r];
      std::memset((void*)&p, 0, sizeof(p));
      for (int s = 0; s < cf.k; s++) {
        char* q;
        CK(hipMalloc((void**)&q, cf.bytes));
        fill_bits<<<2048, 256>>>((uint32_t*)q, cf.bytes / 4, 2000 + c * 64 + r * 16 + s, cf.mask);
        p.src[s] = q;
        owned.push_back(q);
      }
      for (int d = 0; d < cf.m; d++) {
        CK(hipMalloc((void**)&p.dst[d], cf.bytes));
        owned.push_back(p.dst[d]);
      }
      p.nDsts = cf.m;
      p.nPacks = cf.bytes / 16;
      p.head = 0;
    }
    for (Var& v : cf.vars) {
      const int lds = lds_for(v.wgs);
      if (lds > 64 * 1024) CK(hipFuncSetAttribute(v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    }
    auto params = [&](const Var& v, int r) {
      RCParams p = base[r];
      p.nElts = cf.bytes / v.esz;
      p.redArg = v.redArg;
      return p;
    };
    for (const Var& v : cf.vars) {
      const RCParams p = params(v, 0);
      if (p.nElts * (uint64_t)v.esz != p.nPacks * 16 || p.nPacks % kTripPacks != 0 || cf.k > NEXR_MAX_SRCS ||
          cf.m < 1 || cf.m > NEXR_MAX_DSTS || v.k != cf.k) {
        fprintf(stderr, "bad parameters for %s / %s\n", cf.name, v.name.c_str());
        return 2;
      }
    }
    CK(hipDeviceSynchronize());
    // one-shot grid: one workgroup per trip of the variant's own size
    auto launch = [&](size_t vi, int r) {
      const Var& v = cf.vars[vi];
      RCParams p = params(v, r);
      void* args[] = {&p};
      const unsigned grid = v.grid ? v.grid : (unsigned)(cf.bytes / 16 / v.trip);
      CK(hipLaunchKernel(v.fn, dim3(grid), dim3(v.block), args, lds_for(v.wgs), nullptr));
    };
    printf("%s\n", cf.name);
    {  // bytes of every variant against the first (production) launch, set 0
      std::vector<char> ref(cf.bytes), got(cf.bytes);
      for (size_t vi = 0; vi < cf.vars.size(); vi++) {
        CK(hipMemset(base[0].dst[0], 0x5a, cf.bytes));
        launch(vi, 0);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(vi ? got.data() : ref.data(), base[0].dst[0], cf.bytes, hipMemcpyDeviceToHost));
        if (vi && memcmp(ref.data(), got.data(), cf.bytes) != 0) printf("  MISMATCH: %s\n", cf.vars[vi].name.c_str());
      }
    }
    std::vector<std::vector<float>> us(cf.vars.size());
    for (size_t vi = 0; vi < cf.vars.size(); vi++)
      for (int w = 0; w < 2; w++) launch(vi, w % R);
    for (int it = 0; it < blocks; it++)
      for (size_t k = 0; k < cf.vars.size(); k++) {
        const size_t vi = (it % 2) ? cf.vars.size() - 1 - k : k;
        launch(vi, (it + BLK - 1) % R);
        CK(hipEventRecord(e0));
        for (int bb = 0; bb < BLK; bb++) launch(vi, (it + bb) % R);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        us[vi].push_back(ms * 1e3f / BLK);
      }
    const double alg = (double)(cf.k + cf.m) * cf.bytes;
    double med0 = 0;
    for (size_t vi = 0; vi < cf.vars.size(); vi++) {
      std::vector<float> s = us[vi];
      std::sort(s.begin(), s.end());
      const double med = s[s.size() / 2];
      double mean = 0;
      for (float x : us[vi]) mean += x;
      mean /= us[vi].size();
      if (vi == 0) med0 = med;
      printf("  %-30s lds %6d  %8.2f (%8.2f) us  %6.0f GB/s  %.4f  vs first %.4f\n", cf.vars[vi].name.c_str(),
             lds_for(cf.vars[vi].wgs), med, mean, alg / med / 1e3, alg / med / 1e3 / 8000.0, med / med0);
    }
    for (char* q : owned) CK(hipFree(q));
  }
  return 0;
}
