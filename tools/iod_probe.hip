// I/O-die locality probe (tuning harness, not product code). tools/numa_probe.hip found that an HBM
// line's latency depends on which half of the XCDs reads it: ~700 cycles from one group of four
// XCDs, ~1,000 from the other, alternating every 8 KiB of address with the phase flipping every
// 2 MiB (virtual address bit 13 XOR bit 21 predicted the faster group for 99.95 % of 4 KiB chunks).
// Question here: does it matter for BANDWIDTH? A streaming read (and a copy) over one buffer in
// three modes, the same bytes each:
//   mode 0  any: workgroup b takes granules b, b + grid, ... of the whole buffer
//   mode 1  side-matched: workgroups on XCC group g (XCC id / 4) take only granules with
//           bit13 ^ bit21 == g
//   mode 2  side-crossed: group g takes the granules with bit13 ^ bit21 != g
// Every mode is checked: the read returns the same checksum, the copy the same bytes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/iod_probe.hip -o tools/iod_probe
//   ./tools/iod_probe <MiB> <iters>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int kB = 256;            // lanes per workgroup
constexpr size_t kGran = 8192;     // bytes per granule: 256 lanes x 2 x 16 B

__device__ __forceinline__ int side_of(uintptr_t a) { return (int)(((a >> 13) ^ (a >> 21)) & 1); }

// The j-th granule of side s in a buffer whose base is 2 MiB aligned: granule g = 2j + (s ^ bit8(2j)).
__device__ __forceinline__ size_t granule_of_side(size_t j, int s, int baseSide) {
  const size_t g2 = 2 * j;
  return g2 + (size_t)((s ^ baseSide ^ (int)((g2 >> 8) & 1)) & 1);
}

// Static work split, for speed only: blocks are dealt round-robin over the 8 XCDs, so block b's rank
// among the blocks of its XCC group is (b / 8) * 4 + (XCC id mod 4). If that placement did not hold,
// granules would be skipped or repeated, and the checksum / copy check below would say so.
template <bool Copy>
__global__ __launch_bounds__(kB) void stream(const char* __restrict__ src, char* __restrict__ dst, size_t nGran,
                                             int mode, u32x4* sink) {
  uint32_t id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
  const int group = (int)((id & 0xf) >> 2);
  const int mySide = mode == 1 ? group : 1 - group;
  const int baseSide = side_of((uintptr_t)src);
  const size_t perSide = nGran / 2;
  const size_t rank = mode == 0 ? blockIdx.x : (blockIdx.x / 8) * 4 + (id & 3);
  const size_t stride = mode == 0 ? gridDim.x : gridDim.x / 2;
  const size_t n = mode == 0 ? nGran : perSide;
  u32x4 acc = (u32x4)0u;
  for (size_t j = rank; j < n; j += stride) {
    const size_t g = mode == 0 ? j : granule_of_side(j, mySide, baseSide);
    const size_t off = g * kGran + threadIdx.x * 16;
    const u32x4 a = __builtin_nontemporal_load((const u32x4*)(src + off));
    const u32x4 b = __builtin_nontemporal_load((const u32x4*)(src + off + kB * 16));
    if constexpr (Copy) {
      __builtin_nontemporal_store(a, (u32x4*)(dst + off));
      __builtin_nontemporal_store(b, (u32x4*)(dst + off + kB * 16));
    } else {
      acc ^= a ^ b;
    }
  }
  if constexpr (!Copy) sink[blockIdx.x * kB + threadIdx.x] = acc;
}

__global__ void fill(uint32_t* p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (uint32_t)(i * 2654435761u);
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? atoll(argv[1]) : 1024;
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  const size_t bytes = mib << 20;
  const size_t nGran = bytes / kGran;
  char *src, *dst, *dst2;
  u32x4* sink;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&dst2, bytes));
  CK(hipMalloc(&sink, (size_t)grid * kB * sizeof(u32x4)));
  fill<<<4096, 256>>>((uint32_t*)src, bytes / 4);
  CK(hipDeviceSynchronize());
  printf("# src %p dst %p, %zu MiB, grid %d x %d, sides of bases: src %d dst %d\n", (void*)src, (void*)dst, mib, grid,
         kB, (int)((((uintptr_t)src >> 13) ^ ((uintptr_t)src >> 21)) & 1),
         (int)((((uintptr_t)dst >> 13) ^ ((uintptr_t)dst >> 21)) & 1));
  if ((uintptr_t)src % (2u << 20) || (uintptr_t)dst % (2u << 20) || bytes % (2u << 20)) {
    fprintf(stderr, "needs 2 MiB aligned buffers and sizes\n");
    return 1;
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<u32x4> ref, got((size_t)grid * kB);
  auto xorall = [&](const std::vector<u32x4>& v) {
    u32x4 x = (u32x4)0u;
    for (auto& s : v) x ^= s;
    return x;
  };
  const char* names[3] = {"any", "side_matched", "side_crossed"};
  for (int copy = 0; copy < 2; copy++) {
    for (int round = 0; round < 3; round++) {
      for (int mode = 0; mode < 3; mode++) {
        float best = 1e30f, sum = 0;
        for (int it = 0; it < iters; it++) {
          CK(hipEventRecord(e0));
          if (copy)
            stream<true><<<grid, kB>>>(src, mode == 0 ? dst2 : dst, nGran, mode, sink);
          else
            stream<false><<<grid, kB>>>(src, nullptr, nGran, mode, sink);
          CK(hipEventRecord(e1));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          best = std::min(best, ms);
          sum += ms;
        }
        const double moved = (double)bytes * (copy ? 2 : 1);
        bool ok = true;
        if (!copy) {
          CK(hipMemcpy(got.data(), sink, got.size() * sizeof(u32x4), hipMemcpyDeviceToHost));
          u32x4 x = xorall(got);
          if (mode == 0 && round == 0) ref = {x};
          ok = x[0] == ref[0][0] && x[1] == ref[0][1] && x[2] == ref[0][2] && x[3] == ref[0][3];
        } else if (mode != 0) {
          std::vector<uint32_t> a(bytes / 4), b(bytes / 4);
          CK(hipMemcpy(a.data(), dst, bytes, hipMemcpyDeviceToHost));
          CK(hipMemcpy(b.data(), dst2, bytes, hipMemcpyDeviceToHost));
          ok = a == b;
        }
        printf("%s %-13s round %d: mean %.1f us, best %.1f us, %.0f GB/s (best %.0f) %s\n", copy ? "copy" : "read",
               names[mode], round, sum / iters * 1e3, best * 1e3, moved / (sum / iters) / 1e6, moved / best / 1e6,
               ok ? "ok" : "MISMATCH");
        fflush(stdout);
      }
    }
  }
  return 0;
}
