// The round-5 kernel body against the round-4 one (tuning harness, not product code; VERDICT r04
// "next" #1 and #3).
//
// Round 5 changed three things in nexr_kernels.hip body():
//   - every buffer address is a workgroup-uniform base plus the lane's 32-bit offset, and only the
//     first destination is unrolled (further ones in a rolled loop): a lane no longer holds a 64-bit
//     pointer per buffer, so the 16-bit K = 8 kernels drop from 68 / 86 VGPRs to 42 / 56 and run two
//     1024-lane workgroups per CU instead of one;
//   - MinMax is two kernels (min, max) picked on the host, not one kernel with a runtime branch;
//   - the edge elements use rolled byte loops (code size only).
// This harness times the production kernel of this tree against a verbatim copy of the round-4
// body (`body_r04`, with its runtime min/max branch), byte-checks every variant against round 4,
// and adds: the new body held to one workgroup per CU by an LDS reservation (is it the occupancy?),
// the bf16 kernels on the same bytes, and a uint32 sum of the same bytes at the configuration's own
// geometry. Blocks of launches over three rotating buffer sets, interleaved, order alternated.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=6 tools/body_ab.hip -o tools/body_ab
//   ./tools/body_ab <blocks>
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

// ---- the round-4 body, verbatim but for its names (git show 39c5664:nex-nccl_amd/csrc/nexr_kernels.hip)
template <int D, int OP, int K, bool IsMin>
__device__ __forceinline__ void do_element_r04(const char* const (&src)[K], char* const (&dst)[NEXR_MAX_DSTS],
                                               int nDsts, const Fold<D, OP, K, IsMin>& f, uint64_t i) {
  constexpr int esz = 16 / Ty<D>::EPP;
  u32x4 in[K];
#pragma unroll
  for (int s = 0; s < K; s++) {
    in[s] = (u32x4)0u;
    __builtin_memcpy(&in[s], src[s] + i * esz, esz);
  }
  u32x4 out = f.run(in);
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++)
    if (d < nDsts) __builtin_memcpy(dst[d] + i * esz, &out, esz);
}

template <int D, int OP, int K, int POL, bool IsMin, int U, int B>
__device__ __forceinline__ void body_r04(const RCParams& p, uint64_t bid, uint64_t nblk) {
  using T = Ty<D>;
  constexpr int esz = 16 / T::EPP;
  Fold<D, OP, K, IsMin> f(p);
  if constexpr (OP == nexrDevPreMulSum) {
    if (p.prePtr) {
      uint64_t raw = 0;
      __builtin_memcpy(&raw, p.prePtr, esz);
      f.factor[0] = T::splat(raw);
    }
  }
  const char* src[K];
#pragma unroll
  for (int s = 0; s < K; s++) src[s] = p.src[s];
  char* dst[NEXR_MAX_DSTS];
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++) dst[d] = p.dst[d];
  const int nDsts = p.nDsts;
  const uint64_t gid = bid * B + threadIdx.x;
  const uint64_t nthreads = nblk * B;
  const uint64_t bodyElts = p.nPacks * T::EPP;
  const uint64_t head = p.head;
  const uint64_t tail = p.nElts - head - bodyElts;
  if (gid < head + tail) {
    const uint64_t e = gid < head ? gid : head + bodyElts + (gid - head);
    do_element_r04<D, OP, K, IsMin>(src, dst, nDsts, f, e);
  }
#pragma unroll
  for (int s = 0; s < K; s++) src[s] += head * esz;
#pragma unroll
  for (int d = 0; d < NEXR_MAX_DSTS; d++) dst[d] += head * esz;
  const uint64_t nPacks = p.nPacks;
  const uint64_t nFull = nPacks / (B * U);
  uint64_t g = bid;
  for (; g < nFull; g += nblk) {
    const uint64_t off = (g * (B * U) + threadIdx.x) * 16;
    u32x4 in[U][K];
#pragma unroll
    for (int s = 0; s < K; s++)
#pragma unroll
      for (int u = 0; u < U; u++) in[u][s] = ld16<POL>(src[s] + off + u * B * 16);
    u32x4 out[U];
#pragma unroll
    for (int u = 0; u < U; u++) out[u] = f.run(in[u]);
#pragma unroll
    for (int d = 0; d < NEXR_MAX_DSTS; d++) {
      if (d < nDsts) {
#pragma unroll
        for (int u = 0; u < U; u++) st16<POL>(dst[d] + off + u * B * 16, out[u]);
      }
    }
  }
  for (uint64_t j = nFull * (B * U) + gid; j < nPacks; j += nthreads) {
    u32x4 in[K];
#pragma unroll
    for (int s = 0; s < K; s++) in[s] = ld16<POL>(src[s] + j * 16);
    u32x4 out = f.run(in);
#pragma unroll
    for (int d = 0; d < NEXR_MAX_DSTS; d++)
      if (d < nDsts) st16<POL>(dst[d] + j * 16, out);
  }
}

template <int D, int OP, int K, int POL, int U = unroll_for(D, K, POL), int B = block_for(D, K, POL)>
__global__ __launch_bounds__(B) void r04_kernel(RCParams p) {
  if constexpr (OP == nexrDevMinMax) {
    if ((p.redArg & 1) == 0) body_r04<D, OP, K, POL, true, U, B>(p, blockIdx.x, gridDim.x);
    else body_r04<D, OP, K, POL, false, U, B>(p, blockIdx.x, gridDim.x);
  } else {
    body_r04<D, OP, K, POL, false, U, B>(p, blockIdx.x, gridDim.x);
  }
}

// The round-5 body with 96 KiB of LDS reserved per workgroup: at most one 1024-lane workgroup per CU,
// as the round-4 register count gave the 16-bit K = 8 kernels.
template <int D, int OP, int K, int POL, bool IsMin, int U = unroll_for(D, K, POL), int B = block_for(D, K, POL)>
__global__ __launch_bounds__(B) void one_wg_kernel(RCParams p) {
  __shared__ uint32_t pad[96 * 1024 / 4];
  if (p.nDsts < 0) pad[threadIdx.x] = 0;  // never true: keeps the reservation
  body<D, OP, K, POL, IsMin, U, B>(p, blockIdx.x, gridDim.x);
}

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed, uint32_t mask) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31)) & mask;
  }
}

struct Var {
  std::string name;
  int group;  // variants of one group must write identical bytes; the first of a group is its reference
  int esz;    // element size the variant's parameters are built for
  uint64_t redArg;
  std::function<void(const RCParams&, int)> run;
};
struct Cfg {
  const char* name;
  int k;
  size_t bytes;
  uint32_t mask;
  std::vector<Var> vars;
};

#define L(...) [](const RCParams& p, int g) { __VA_ARGS__<<<g, kBlk>>>(p); }

int main(int argc, char** argv) {
  const int blocks = argc > 1 ? atoi(argv[1]) : 10;
  const uint32_t all = 0xffffffffu, fin = 0x3bff3bffu;  // fin: finite values for every float type
  std::vector<Cfg> cfgs;
  {
    constexpr int D = nexrFloat32, K = 2, P = kPolNt, U = 4, kBlk = 256;
    cfgs.push_back({"C2 fp32 sum K=2 256 MiB (nt/nt, U4 B256)", K, 256u << 20, fin,
                    {{"r04 body", 0, 4, 0, L(r04_kernel<D, nexrDevSum, K, P>)},
                     {"r05 body (production)", 0, 4, 0, L(reduce_copy_kernel<D, nexrDevSum, K, P>)},
                     {"u32 sum, r05 body", 1, 4, 0, L(reduce_copy_kernel<nexrUint32, nexrDevSum, K, P, false, U, kBlk>)},
                     {"u32 sum, r04 body", 1, 4, 0, L(r04_kernel<nexrUint32, nexrDevSum, K, P, U, kBlk>)}}});
  }
  {
    constexpr int K = 8, P = kPolNt, U = 1, kBlk = 1024;
    cfgs.push_back(
        {"C3 fp16/bf16 sum K=8 256 MiB (nt/nt, U1 B1024)", K, 256u << 20, fin,
         {{"f16 r04 body", 0, 2, 0, L(r04_kernel<nexrFloat16, nexrDevSum, K, P>)},
          {"f16 r05 body (production)", 0, 2, 0, L(reduce_copy_kernel<nexrFloat16, nexrDevSum, K, P>)},
          {"f16 r05 body, 1 WG/CU", 0, 2, 0, L(one_wg_kernel<nexrFloat16, nexrDevSum, K, P, false>)},
          {"bf16 r04 body", 1, 2, 0, L(r04_kernel<nexrBfloat16, nexrDevSum, K, P>)},
          {"bf16 r05 body (production)", 1, 2, 0, L(reduce_copy_kernel<nexrBfloat16, nexrDevSum, K, P>)},
          {"bf16 r05 body, 1 WG/CU", 1, 2, 0, L(one_wg_kernel<nexrBfloat16, nexrDevSum, K, P, false>)},
          {"u32 sum U1 B1024, r05 body", 2, 4, 0, L(reduce_copy_kernel<nexrUint32, nexrDevSum, K, P, false, U, kBlk>)},
          {"u32 sum U1 B1024, r04 body", 2, 4, 0, L(r04_kernel<nexrUint32, nexrDevSum, K, P, U, kBlk>)}}});
  }
  {
    constexpr int K = 4, P = kPolNtLoad, U = 2, kBlk = 512;
    cfgs.push_back(
        {"C4 int8 K=4 64 MiB (nt loads, U2 B512)", K, 64u << 20, all,
         {{"i8 max r04 body", 0, 1, 0x7f, L(r04_kernel<nexrInt8, nexrDevMinMax, K, P>)},
          {"i8 max r05 (own kernel)", 0, 1, 0x7f, L(reduce_copy_kernel<nexrInt8, nexrDevMinMax, K, P, false>)},
          {"i8 min r04 body", 1, 1, 0x80, L(r04_kernel<nexrInt8, nexrDevMinMax, K, P>)},
          {"i8 min r05 (own kernel)", 1, 1, 0x80, L(reduce_copy_kernel<nexrInt8, nexrDevMinMax, K, P, true>)},
          {"i8 prod r04 body", 2, 1, 0, L(r04_kernel<nexrInt8, nexrDevProd, K, P>)},
          {"i8 prod r05", 2, 1, 0, L(reduce_copy_kernel<nexrInt8, nexrDevProd, K, P>)},
          {"u32 sum, r05 body", 3, 4, 0, L(reduce_copy_kernel<nexrUint32, nexrDevSum, K, P, false, U, kBlk>)}}});
  }
  {
    constexpr int K = 4, P = kPolNtLoad, kBlk = 512;
    cfgs.push_back({"C4 int32 K=4 64 MiB (nt loads, U2 B512)", K, 64u << 20, all,
                    {{"i32 max r04 body", 0, 4, 0x7fffffff, L(r04_kernel<nexrInt32, nexrDevMinMax, K, P>)},
                     {"i32 max r05", 0, 4, 0x7fffffff, L(reduce_copy_kernel<nexrInt32, nexrDevMinMax, K, P, false>)},
                     {"i32 min r04 body", 1, 4, 0x80000000ull, L(r04_kernel<nexrInt32, nexrDevMinMax, K, P>)},
                     {"i32 min r05", 1, 4, 0x80000000ull, L(reduce_copy_kernel<nexrInt32, nexrDevMinMax, K, P, true>)},
                     {"i32 prod r04 body", 2, 4, 0, L(r04_kernel<nexrInt32, nexrDevProd, K, P>)},
                     {"i32 prod r05", 2, 4, 0, L(reduce_copy_kernel<nexrInt32, nexrDevProd, K, P>)}}});
  }
  {
    constexpr int D = nexrFloat32, K = 2, P = kPolPlain, kBlk = 256;
    cfgs.push_back({"fp32 sum K=2 M=2 16 MiB (plain: a ring step's recvReduceCopySend)", K, 16u << 20, fin,
                    {{"r04 body", 0, 4, 0, L(r04_kernel<D, nexrDevSum, K, P>)},
                     {"r05 body (production)", 0, 4, 0, L(reduce_copy_kernel<D, nexrDevSum, K, P>)}}});
  }
  const int R = 3, BLK = 6;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("median (mean) us of %d blocks of %d launches over %d rotating sets, interleaved; fraction of 8 TB/s\n"
         "from the median; 'vs first' = median over the first variant's median\n\n", blocks, BLK, R);
  for (size_t c = 0; c < cfgs.size(); c++) {
    Cfg& cf = cfgs[c];
    const int m = (c == cfgs.size() - 1) ? 2 : 1;
    std::vector<RCParams> base(R);
    std::vector<char*> owned;
    for (int r = 0; r < R; r++) {
      RCParams& p = base[r];
      std::memset((void*)&p, 0, sizeof(p));
      for (int s = 0; s < cf.k; s++) {
        char* q;
        CK(hipMalloc((void**)&q, cf.bytes));
        fill_bits<<<2048, 256>>>((uint32_t*)q, cf.bytes / 4, 1000 + c * 64 + r * 16 + s, cf.mask);
        p.src[s] = q;
        owned.push_back(q);
      }
      for (int d = 0; d < m; d++) {
        CK(hipMalloc((void**)&p.dst[d], cf.bytes));
        owned.push_back(p.dst[d]);
      }
      p.nDsts = m;
      p.nPacks = cf.bytes / 16;
      p.head = 0;
    }
    // per-variant parameters (element count and op argument); the host checks what the one-shot grid
    // and the kernels assume before any launch
    auto params = [&](const Var& v, int r) {
      RCParams p = base[r];
      p.nElts = cf.bytes / v.esz;
      p.redArg = v.redArg;
      return p;
    };
    for (int r = 0; r < R; r++)
      for (const Var& v : cf.vars) {
        const RCParams p = params(v, r);
        if (p.nElts * (uint64_t)v.esz != p.nPacks * 16 || p.nPacks % kTripPacks != 0 || cf.k > NEXR_MAX_SRCS) {
          fprintf(stderr, "bad parameters for %s / %s\n", cf.name, v.name.c_str());
          return 2;
        }
      }
    CK(hipDeviceSynchronize());
    const int grid = (int)(cf.bytes / 16 / kTripPacks);
    printf("%s\n", cf.name);
    {  // byte check on set 0, every destination, against the first variant of the group
      std::vector<std::vector<std::vector<char>>> ref(cf.vars.size());
      std::vector<char> got(cf.bytes);
      for (size_t vi = 0; vi < cf.vars.size(); vi++) {
        const Var& v = cf.vars[vi];
        for (int d = 0; d < m; d++) CK(hipMemset(base[0].dst[d], 0x5a, cf.bytes));
        v.run(params(v, 0), grid);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        size_t first = vi;
        for (size_t w = 0; w < vi; w++)
          if (cf.vars[w].group == v.group) {
            first = w;
            break;
          }
        bool ok = true;
        for (int d = 0; d < m; d++) {
          CK(hipMemcpy(got.data(), base[0].dst[d], cf.bytes, hipMemcpyDeviceToHost));
          if (first == vi) ref[vi].push_back(got);
          else ok = ok && memcmp(ref[first][d].data(), got.data(), cf.bytes) == 0;
        }
        if (first != vi)
          printf("  %-30s bytes %s %s\n", v.name.c_str(), ok ? "match" : "MISMATCH", cf.vars[first].name.c_str());
      }
    }
    std::vector<std::vector<float>> us(cf.vars.size());
    auto launch = [&](size_t vi, int r) { cf.vars[vi].run(params(cf.vars[vi], r), grid); };
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
    const double alg = (double)(cf.k + m) * cf.bytes;
    double med0 = 0;
    for (size_t vi = 0; vi < cf.vars.size(); vi++) {
      std::vector<float> s = us[vi];
      std::sort(s.begin(), s.end());
      const double med = s[s.size() / 2];
      double mean = 0;
      for (float x : us[vi]) mean += x;
      mean /= us[vi].size();
      if (vi == 0) med0 = med;
      printf("  %-30s %8.2f (%8.2f) us  %6.0f GB/s  %.4f  vs first %.4f\n", cf.vars[vi].name.c_str(), med, mean,
             alg / med / 1e3, alg / med / 1e3 / 8000.0, med / med0);
    }
    for (char* q : owned) CK(hipFree(q));
  }
  return 0;
}
