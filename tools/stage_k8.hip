// Read/write phase-separation probe for the K = 8 reduce-copy (tuning harness, not product code).
//
// Question (VERDICT r1 "next" #6): the 8-read + 1-write mix runs at ~6.1 TB/s while 8 reads alone
// run at ~6.8 TB/s (profiles/r01_streams.log). Does separating the reads and the writes in time
// help? Every variant here keeps the production arithmetic (Ty<D>, reduce_step from
// nexr_types.hpp) and is checked byte-for-byte against the production kernel's output.
//
//   production   the shipped one-shot kernel at its shipped geometry (unroll_for / block_for)
//   seq-oneshot  one trip per workgroup, sources read ONE AT A TIME (depth-2 register prefetch:
//                src s+1 in flight while src s is folded), then the trip's stores: at any moment
//                a workgroup has at most two source streams open instead of K
//   seq-persist  the same trip body in a persistent grid (W workgroups per CU) striding over trips
//                in lock-step: workgroups that start together stay roughly in phase, so chip-wide
//                the reads of a trip window come in source order and the window's stores arrive as
//                one burst after its last source (read and write phases separated without a barrier)
//   lds-persist  persistent grid, every source streamed into an LDS ring with global_load_lds
//                (no VGPR cost per byte in flight, 3 sources in flight), folded from LDS into
//                registers, stores as one burst at the end of the trip
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=9 -DTK_K=8 \
//         tools/stage_k8.hip -o tools/stage_k8_dt9
//   ./tools/stage_k8_dt9 <MiB per buffer> <iters>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#ifndef TK_K
#define TK_K 8
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
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0x83ff83ffu;  // small finite values for every float type
  }
}

template <int D>
__device__ __forceinline__ u32x4 finish_pack(typename Ty<D>::V acc) {
  if constexpr (D == nexrFloat16) acc = Ty<D>::canon(acc);
  return bc<u32x4>(acc);
}

// One trip (B lanes x T packs of every buffer) with sources read one at a time, src s+1's loads in
// flight while src s is folded. sched_barrier keeps the compiler from hoisting every load up front
// (which would turn this back into the production all-sources-at-once schedule).
template <int D, int K, int T, int B, int POL>
__device__ __forceinline__ void seq_trip(const RCParams& p, uint64_t trip) {
  using V = typename Ty<D>::V;
  const uint64_t off = (trip * (uint64_t)(B * T) + threadIdx.x) * 16;
  u32x4 buf[2][T];
  V acc[T];
#pragma unroll
  for (int u = 0; u < T; u++) buf[0][u] = ld16<POL>(p.src[0] + off + u * B * 16);
#pragma unroll
  for (int u = 0; u < T; u++) buf[1][u] = ld16<POL>(p.src[1] + off + u * B * 16);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < T; u++) acc[u] = bc<V>(buf[0][u]);
#pragma unroll
  for (int s = 1; s < K; s++) {
    if (s + 1 < K) {
#pragma unroll
      for (int u = 0; u < T; u++) buf[(s + 1) & 1][u] = ld16<POL>(p.src[s + 1] + off + u * B * 16);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < T; u++) acc[u] = reduce_step<D, nexrDevSum, false>(acc[u], bc<V>(buf[s & 1][u]));
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int u = 0; u < T; u++) st16<POL>(p.dst[0] + off + u * B * 16, finish_pack<D>(acc[u]));
}

template <int D, int K, int T, int B, int POL>
__global__ __launch_bounds__(B) void k_seq_oneshot(RCParams p) {
  seq_trip<D, K, T, B, POL>(p, blockIdx.x);
}

template <int D, int K, int T, int B, int POL>
__global__ __launch_bounds__(B) void k_seq_persist(RCParams p, uint64_t nTrips) {
  for (uint64_t t = blockIdx.x; t < nTrips; t += gridDim.x) seq_trip<D, K, T, B, POL>(p, t);
}

// s_waitcnt vmcnt(N) with expcnt/lgkmcnt left at their maxima (gfx9 encoding: vmcnt[3:0] and
// vmcnt[5:4] at bits 15:14, expcnt 6:4, lgkmcnt 11:8). After unrolling, n is a constant and the
// switch folds to one instruction.
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 0xf) | ((N >> 4) << 14) | 0x0f70);
}
__device__ __forceinline__ void wait_vm_rt(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 6: wait_vm<6>(); break;
    case 8: wait_vm<8>(); break;
    case 12: wait_vm<12>(); break;
    case 16: wait_vm<16>(); break;
    default: wait_vm<0>(); break;
  }
}

// LDS ring: NB slots of one source's trip tile (B lanes x T packs x 16 B). Each lane's
// global_load_lds_dwordx4 writes 16 B, and the LDS image is lane-linear per
// wave-instruction (base + lane*16), so lane l of wave w, pack u lands at
// slot + u*B*16 + w*64*16 + l*16, i.e. exactly at its own (u, threadIdx) position: every lane reads
// back only what it loaded itself, so no workgroup barrier is needed, only the wave's vmcnt.
template <int D, int K, int T, int B, int POL, int NB>
__global__ __launch_bounds__(B) void k_lds_persist(RCParams p, uint64_t nTrips) {
  using V = typename Ty<D>::V;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int kSlot = B * T * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr unsigned aux = (POL & kPolNtLoad) ? 2u : 0u;  // nt bit of the cache-policy operand
  for (uint64_t t = blockIdx.x; t < nTrips; t += gridDim.x) {
    const uint64_t off = (t * (uint64_t)(B * T) + threadIdx.x) * 16;
    auto issue = [&](int s) {
#pragma unroll
      for (int u = 0; u < T; u++) {
        char* dstLds = lds + (s % NB) * kSlot + u * B * 16 + wave * 64 * 16;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(p.src[s] + off + u * B * 16),
                                         (void __attribute__((address_space(3)))*)dstLds, 16, 0, aux);
      }
    };
#pragma unroll
    for (int s = 0; s < NB - 1 && s < K; s++) issue(s);
    V acc[T];
#pragma unroll
    for (int s = 0; s < K; s++) {
      if (s + NB - 1 < K) issue(s + NB - 1);
      // wait for source s: the loads issued after it may stay in flight
      wait_vm_rt((s + NB - 1 < K ? NB - 1 : K - 1 - s) * T);
#pragma unroll
      for (int u = 0; u < T; u++) {
        const u32x4 x = *(const u32x4*)(lds + (s % NB) * kSlot + u * B * 16 + threadIdx.x * 16);
        acc[u] = s == 0 ? bc<V>(x) : reduce_step<D, nexrDevSum, false>(acc[u], bc<V>(x));
      }
    }
#pragma unroll
    for (int u = 0; u < T; u++) st16<POL>(p.dst[0] + off + u * B * 16, finish_pack<D>(acc[u]));
  }
}

struct Var {
  std::string name;
  std::function<void(int)> run;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  const int iters = argc > 2 ? atoi(argv[2]) : 8;
  constexpr int D = NEXR_DT, K = TK_K;
  constexpr int esz = 16 / Ty<D>::EPP;
  const int R = 2;
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
  const uint64_t P = bytes / 16;
  constexpr int PU = unroll_for(D, K, kPolNt), PB = block_for(D, K, kPolNt);
  std::vector<Var> vs;
  vs.push_back({"production U" + std::to_string(PU) + " B" + std::to_string(PB),
                [&](int r) { reduce_copy_kernel<D, 0, K, kPolNt, PU, PB><<<(int)(P / (PU * PB)), PB>>>(ps[r]); }, {}});
#define V1(T, B, POL)                                                                                \
  vs.push_back({"seq-oneshot T" #T " B" #B " pol" #POL,                                              \
                [&](int r) { k_seq_oneshot<D, K, T, B, POL><<<(int)(P / ((T) * (B))), B>>>(ps[r]); }, {}});
#define V2(T, B, W, POL)                                                                                   \
  vs.push_back({"seq-persist T" #T " B" #B " W" #W " pol" #POL, [&](int r) {                               \
                  k_seq_persist<D, K, T, B, POL><<<nCU * (W), B>>>(ps[r], P / ((T) * (B)));               \
                }, {}});
#define V3(T, B, W, NB)                                                                                     \
  {                                                                                                         \
    const size_t lds = (size_t)(NB) * (B) * (T) * 16;                                                       \
    CK(hipFuncSetAttribute((const void*)&k_lds_persist<D, K, T, B, kPolNt, NB>,                             \
                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                          \
    vs.push_back({"lds-persist T" #T " B" #B " W" #W " NB" #NB, [&, lds](int r) {                           \
                    k_lds_persist<D, K, T, B, kPolNt, NB><<<nCU * (W), B, lds>>>(ps[r], P / ((T) * (B))); \
                  }, {}});                                                                                  \
  }
  V1(1, 1024, 3) V1(2, 512, 3) V1(4, 256, 3) V1(4, 512, 3)
  V2(4, 256, 4, 3) V2(4, 256, 8, 3) V2(4, 512, 2, 3) V2(4, 512, 4, 3) V2(2, 1024, 2, 3) V2(8, 256, 2, 3)
  V2(8, 256, 4, 3) V2(4, 1024, 1, 3) V2(4, 512, 4, 1)
  V3(2, 256, 4, 3) V3(4, 256, 2, 3) V3(2, 512, 2, 3) V3(4, 512, 1, 3) V3(2, 1024, 1, 3)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  // Every variant must produce the production kernel's bytes (checked before timing).
  {
    std::vector<char> ref(bytes), got(bytes);
    vs[0].run(0);
    CK(hipMemcpy(ref.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
    for (size_t i = 1; i < vs.size(); i++) {
      CK(hipMemset(ps[0].dst[0], 0, bytes));
      vs[i].run(0);
      CK(hipMemcpy(got.data(), ps[0].dst[0], bytes, hipMemcpyDeviceToHost));
      if (memcmp(ref.data(), got.data(), bytes) != 0) printf("MISMATCH: %s\n", vs[i].name.c_str());
    }
  }
  const int BLK = 6;
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
  printf("dt=%d K=%d buffer=%zu MiB CUs=%d alg bytes=%.0f\n", D, K, bytes >> 20, nCU, alg);
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-36s med %8.1f us  %7.0f GB/s  (best %7.0f)\n", v.name.c_str(), med * 1e3, alg / med / 1e6, alg / mn / 1e6);
  }
  return 0;
}
