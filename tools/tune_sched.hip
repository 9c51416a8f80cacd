// Work-schedule probe for the reduce-copy body (tuning harness, not product code): does the
// blockIdx -> trip mapping or a persistent, software-pipelined loop move the K-read + 1-write
// stream rate past what the one-shot grid reaches? Same per-trip access shape and arithmetic as
// the production kernel (nexr_kernels.hip is included; Fold/ld16/st16 are reused).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 -DTK_K=2 \
//         tools/tune_sched.hip -o tools/tune_sched_dt7_k2
//   ./tools/tune_sched_dt7_k2 <MiB per buffer> <iters>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#ifndef TK_K
#define TK_K 2
#endif

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
    // keep values small and finite for every float type: sign + low mantissa bits only
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0x83ff83ffu;
  }
}

template <int D, int K, int U, int POL>
struct Trip {
  __device__ static void load(const RCParams& p, uint64_t t, u32x4 (&in)[U][K]) {
    const uint64_t off = (t * (kBlock * U) + threadIdx.x) * 16;
#pragma unroll
    for (int s = 0; s < K; s++)
#pragma unroll
      for (int u = 0; u < U; u++) in[u][s] = ld16<POL>(p.src[s] + off + u * kBlock * 16);
  }
  __device__ static void finish(const RCParams& p, const Fold<D, 0, K, false>& f, uint64_t t,
                                const u32x4 (&in)[U][K]) {
    const uint64_t off = (t * (kBlock * U) + threadIdx.x) * 16;
#pragma unroll
    for (int u = 0; u < U; u++) st16<POL>(p.dst[0] + off + u * kBlock * 16, f.run(in[u]));
  }
};

// MODE 0: one-shot, XCD-contiguous (workgroups of XCD x = blockIdx % 8 take the x-th eighth)
// MODE 1: persistent, grid-stride over trips
// MODE 2: persistent, contiguous range per workgroup
// MODE 3: persistent, grid-stride, next trip's loads issued before this trip's stores
// MODE 4: persistent, contiguous range, pipelined like 3
// MODE 5: persistent, grid-stride within the XCD's eighth, pipelined
template <int D, int K, int U, int POL, int MODE>
__global__ __launch_bounds__(kBlock) void k_sched(RCParams p, uint64_t nTrips) {
  using TR = Trip<D, K, U, POL>;
  Fold<D, 0, K, false> f(p);
  const uint64_t b = blockIdx.x, G = gridDim.x;
  u32x4 cur[U][K];
  if constexpr (MODE == 0) {
    const uint64_t per = G / 8, t = (b & 7) * per + (b >> 3);
    if (t >= nTrips) return;
    TR::load(p, t, cur);
    TR::finish(p, f, t, cur);
  } else if constexpr (MODE == 1) {
    for (uint64_t t = b; t < nTrips; t += G) {
      TR::load(p, t, cur);
      TR::finish(p, f, t, cur);
    }
  } else if constexpr (MODE == 2) {
    const uint64_t t0 = nTrips * b / G, t1 = nTrips * (b + 1) / G;
    for (uint64_t t = t0; t < t1; t++) {
      TR::load(p, t, cur);
      TR::finish(p, f, t, cur);
    }
  } else {
    uint64_t t, end, step;
    if constexpr (MODE == 3) {
      t = b; end = nTrips; step = G;
    } else if constexpr (MODE == 4) {
      t = nTrips * b / G; end = nTrips * (b + 1) / G; step = 1;
    } else {
      const uint64_t per = nTrips / 8, gx = G / 8;
      t = (b & 7) * per + (b >> 3); end = (b & 7) * per + per; step = gx;
    }
    if (t >= end) return;
    TR::load(p, t, cur);
    for (;;) {
      const uint64_t nt = t + step;
      if (nt < end) {
        u32x4 nxt[U][K];
        TR::load(p, nt, nxt);
        TR::finish(p, f, t, cur);
#pragma unroll
        for (int u = 0; u < U; u++)
#pragma unroll
          for (int s = 0; s < K; s++) cur[u][s] = nxt[u][s];
        t = nt;
      } else {
        TR::finish(p, f, t, cur);
        break;
      }
    }
  }
}

struct Var {
  std::string name;
  std::function<void(int)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 10;
  constexpr int D = NEXR_DT, K = TK_K;
  constexpr int esz = 16 / Ty<D>::EPP;
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
    p.nElts = bytes / esz;
    p.nPacks = bytes / 16;
  }
  CK(hipDeviceSynchronize());
  int nCU = 0;
  CK(hipDeviceGetAttribute(&nCU, hipDeviceAttributeMultiprocessorCount, 0));
  const double alg = (double)(K + 1) * bytes;
  std::vector<Var> vs;
  const uint64_t P = bytes / 16;
  vs.push_back({"production one-shot U4", [&](int r) {
                  reduce_copy_kernel<D, 0, K, kPolNt, 4, kBlock><<<(int)(P / 1024), kBlock>>>(ps[r]);
                }, {}});
  const char* mode = getenv("TUNE_MODE");
  if (mode && strcmp(mode, "geom") == 0) {
    // Geometry grid of the production kernel: U packs per lane x B threads per workgroup, one-shot
    // grid, optionally capped to `occ` workgroups per CU through dynamic LDS.
#define VG(U, B, OCC)                                                                                   \
  {                                                                                                     \
    const size_t lds = (OCC) ? 163840 / (OCC) - 256 : 0;                                                \
    if (lds)                                                                                            \
      CK(hipFuncSetAttribute((const void*)&reduce_copy_kernel<D, 0, K, kPolNt, U, B>,                    \
                             hipFuncAttributeMaxDynamicSharedMemorySize, 163840));                      \
    vs.push_back({"U" #U " B" #B " occ<=" #OCC, [&, lds](int r) {                                       \
                    reduce_copy_kernel<D, 0, K, kPolNt, U, B><<<(int)(P / ((U) * (B))), B, lds>>>(ps[r]); \
                  }, {}});                                                                              \
  }
    VG(4, 256, 0) VG(4, 256, 2) VG(4, 256, 1) VG(2, 256, 0) VG(2, 512, 0) VG(2, 512, 1) VG(1, 1024, 0)
    VG(1, 1024, 1) VG(1, 512, 0) VG(2, 1024, 0) VG(4, 512, 0) VG(4, 512, 1)
  } else {
  CK(hipFuncSetAttribute((const void*)&reduce_copy_kernel<D, 0, K, kPolNt, 4, kBlock>,
                         hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
  // Occupancy cap through dynamic LDS: at most `occ` workgroups (= waves per SIMD) per CU.
  for (int occ : {1, 2, 3, 4, 5, 6}) {
    const size_t lds = 163840 / occ - 256;
    vs.push_back({"production one-shot U4 occ<=" + std::to_string(occ), [&, lds](int r) {
                    reduce_copy_kernel<D, 0, K, kPolNt, 4, kBlock><<<(int)(P / 1024), kBlock, lds>>>(ps[r]);
                  }, {}});
  }
#define VS(MODE, U, G, LABEL)                                                                     \
  vs.push_back({std::string(LABEL) + " U" #U " grid=" + std::to_string(G), [&, g = (int)(G)](int r) { \
                  k_sched<D, K, U, kPolNt, MODE><<<g, kBlock>>>(ps[r], P / (kBlock * U));         \
                }, {}});
  VS(0, 4, P / 1024, "xcd-contig one-shot")
  VS(0, 2, P / 512, "xcd-contig one-shot")
  VS(1, 4, nCU * 8, "persist stride")
  VS(1, 4, nCU * 4, "persist stride")
  VS(3, 4, nCU * 4, "persist stride pipe")
  VS(3, 2, nCU * 8, "persist stride pipe")
  VS(5, 2, nCU * 8, "persist xcd pipe")
  VS(5, 4, nCU * 4, "persist xcd pipe")
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  const int BLK = 10;
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
  // Every variant must produce the production kernel's bytes.
  {
    std::vector<char> ref(bytes), got(bytes);
    reduce_copy_kernel<D, 0, K, kPolNt, 4, kBlock><<<(int)(P / 1024), kBlock>>>(ps[0]);
    CK(hipMemcpy(ref.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
    for (size_t i = 1; i < vs.size(); i++) {
      CK(hipMemset(ps[0].dst[0], 0, bytes));
      vs[i].run(0);
      CK(hipMemcpy(got.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      if (memcmp(ref.data(), got.data(), bytes) != 0) printf("MISMATCH: %s\n", vs[i].name.c_str());
    }
  }
  printf("dt=%d K=%d buffer=%zu MiB CUs=%d alg bytes=%.0f\n", D, K, bytes >> 20, nCU, alg);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s med %8.1f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, alg / med / 1e6, alg / mn / 1e6);
  }
  return 0;
}
