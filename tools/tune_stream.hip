// Streaming-geometry sweep for the K=2 fp32 sum reduce-copy (tuning harness, not product code).
// Builds standalone: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/tune_stream.hip -o tools/tune_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include <functional>
#include <string>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <int POL> __device__ __forceinline__ f4 ld(const f4* p) {
  if constexpr (POL & 1) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int POL> __device__ __forceinline__ void st(f4* p, f4 v) {
  if constexpr (POL & 2) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// grid-stride: each iteration a block covers blockDim*U consecutive packs
template <int U, int POL>
__global__ __launch_bounds__(256) void k_gs(const f4* __restrict__ a, const f4* __restrict__ b, f4* __restrict__ o, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  size_t stride = (size_t)gridDim.x * 256 * U;
  for (; i + (U - 1) * 256 < n; i += stride) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ld<POL>(a + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = ld<POL>(b + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) st<POL>(o + i + u * 256, x[u] + y[u]);
  }
  for (; i < n; i += 256) { o[i] = a[i] + b[i]; }
}

// contiguous: block owns one contiguous chunk
template <int U, int POL>
__global__ __launch_bounds__(256) void k_ct(const f4* __restrict__ a, const f4* __restrict__ b, f4* __restrict__ o, size_t n, size_t chunk) {
  size_t beg = (size_t)blockIdx.x * chunk;
  size_t end = beg + chunk < n ? beg + chunk : n;
  size_t i = beg + threadIdx.x;
  for (; i + (U - 1) * 256 < end; i += 256 * U) {
    f4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ld<POL>(a + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) y[u] = ld<POL>(b + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) st<POL>(o + i + u * 256, x[u] + y[u]);
  }
  for (; i < end; i += 256) o[i] = a[i] + b[i];
}

template <int U, int POL>
__global__ __launch_bounds__(256) void k_copy(const f4* __restrict__ a, f4* __restrict__ o, size_t n) {
  size_t i = (size_t)blockIdx.x * 256 * U + threadIdx.x;
  size_t stride = (size_t)gridDim.x * 256 * U;
  for (; i + (U - 1) * 256 < n; i += stride) {
    f4 x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ld<POL>(a + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) st<POL>(o + i + u * 256, x[u]);
  }
  for (; i < n; i += 256) o[i] = a[i];
}

struct Var { std::string name; double bytes; std::function<void(int)> run; std::vector<float> ms; };

int main(int argc, char** argv) {
  size_t bytes = (argc > 1 ? atol(argv[1]) : 256) << 20;
  int iters = argc > 2 ? atoi(argv[2]) : 20;
  size_t n = bytes / 16;
  const int R = 3;
  f4 *A[R], *B[R], *O[R];
  for (int r = 0; r < R; r++) {
    CK(hipMalloc(&A[r], bytes)); CK(hipMalloc(&B[r], bytes)); CK(hipMalloc(&O[r], bytes));
    CK(hipMemset(A[r], 0x3c, bytes)); CK(hipMemset(B[r], 0x3d, bytes)); CK(hipMemset(O[r], 0, bytes));
  }
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  printf("CUs=%d buffer=%zu MiB iters=%d\n", ncu, bytes >> 20, iters);
  std::vector<Var> vs;
  double b3 = 3.0 * bytes, b2 = 2.0 * bytes;
#define GS(U, POL, G) vs.push_back({"gs U=" #U " pol=" #POL " grid=" + std::to_string(G), b3, [=](int r) { k_gs<U, POL><<<G, 256>>>(A[r], B[r], O[r], n); }, {}});
#define CT(U, POL, G) vs.push_back({"ct U=" #U " pol=" #POL " grid=" + std::to_string(G), b3, [=](int r) { size_t ch = ((n + G - 1) / G + 255) / 256 * 256; k_ct<U, POL><<<G, 256>>>(A[r], B[r], O[r], n, ch); }, {}});
#define CP(U, POL, G) vs.push_back({"copy U=" #U " pol=" #POL " grid=" + std::to_string(G), b2, [=](int r) { k_copy<U, POL><<<G, 256>>>(A[r], O[r], n); }, {}});
  int full2 = (int)(n / (256 * 2)), full4 = (int)(n / (256 * 4)), full8 = (int)(n / (256 * 8));
  CP(4, 0, 2048) CP(4, 3, 2048)
  GS(1, 0, 2048) GS(2, 0, 2048) GS(4, 0, 2048) GS(8, 0, 2048)
  GS(4, 0, 1024) GS(4, 0, 4096) GS(4, 0, 8192) GS(2, 0, 4096)
  GS(4, 1, 2048) GS(4, 2, 2048) GS(4, 3, 2048) GS(2, 3, 4096) GS(8, 3, 1024)
  GS(4, 0, full4) GS(2, 0, full2) GS(8, 0, full8) GS(4, 3, full4) GS(4, 2, full4)
  CT(4, 0, 1024) CT(4, 0, 2048) CT(4, 3, 2048) CT(8, 3, 1024) CT(4, 2, 4096)
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (auto& v : vs) for (int w = 0; w < 3; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  for (int it = 0; it < iters; it++)
    for (auto& v : vs) {
      int r = it % R;
      CK(hipEventRecord(e0)); v.run(r); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); v.ms.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    printf("%-34s med %8.1f us  %7.0f GB/s  (best %7.0f GB/s)\n", v.name.c_str(), med * 1e3, v.bytes / med / 1e6, v.bytes / mn / 1e6);
  }
  // correctness spot-check of last reduce
  return 0;
}
