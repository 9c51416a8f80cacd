// LL / LL128 step kernels under different wire cache bits and sub-tile counts (tuning harness, not
// product code). Built once per variant, with the production kernels of nexr_ll.hip and macro
// overrides of their tuning constants:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_LL_LOAD_BITS=17 \
//         -DNEXR_LL_STORE_BITS=17 -DNEXR_LL_U=4 tools/ll_bits.hip -o tools/ll_bits_v
//   rocprofv3 --kernel-trace --stats -- ./tools/ll_bits_v        (kernel durations)
// fp32 sum; shapes send (src -> wire), recvReduceSend (src + wire -> wire) and recvReduceCopySend
// (+ dst) at 32 KiB, 576 KiB, 4 MiB and 64 MiB of data; every launch's outputs are compared with the
// first variant's (the production bits) by the caller through the printed checksums.
#include "../nex-nccl_amd/csrc/nexr_ll.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
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

__global__ void fill(float* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (float)((i * 2654435761u + seed) % 2001) - 1000.0f;
}

__global__ void checksum(const uint32_t* p, size_t n, unsigned long long* out) {
  unsigned long long s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    s += (unsigned long long)p[i] * (i % 977 + 1);
  atomicAdd(out, s);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  const size_t sizes[] = {32768, 589824, 4u << 20, 64u << 20};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  unsigned long long* cs;
  CK(hipMalloc((void**)&cs, 8));
  for (size_t n : sizes) {
    const size_t ne = n / 4;
    float *src, *dst;
    char *wIn, *wOut, *w128In, *w128Out;
    const size_t llWire = 2 * n + 64, ll128Wire = (n + 1919) / 1920 * 2048 + 64;
    CK(hipMalloc((void**)&src, n));
    CK(hipMalloc((void**)&dst, n));
    CK(hipMalloc((void**)&wIn, llWire));
    CK(hipMalloc((void**)&wOut, llWire));
    CK(hipMalloc((void**)&w128In, ll128Wire));
    CK(hipMalloc((void**)&w128Out, ll128Wire));
    fill<<<256, 256, 0, st>>>(src, ne, 7);
    const int reps_n = n >= (64u << 20) ? 20 : reps;
    for (int proto = 0; proto < 2; proto++) {
      for (int shape = -1; shape < 3; shape++) {  // -1: the wire-filling send with flag 5
        LLParams a;
        LL128Params b;
        memset(&a, 0, sizeof(a));
        memset(&b, 0, sizeof(b));
        a.nElts = b.nElts = ne;
        a.timeoutTicks = b.timeoutTicks = 100000000ull;
        a.src = b.src = (const char*)src;
        a.srcIsInput = b.srcIsInput = 1;
        a.nSend = b.nSend = 1;
        if (shape < 0) {
          a.send[0] = wIn, a.sendFlag[0] = 5;
          b.send[0] = w128In, b.sendFlag[0] = 5;
        } else {
          a.send[0] = wOut, a.sendFlag[0] = 6;
          b.send[0] = w128Out, b.sendFlag[0] = 6;
          if (shape >= 1) {
            a.nRecv = b.nRecv = 1;
            a.recv[0] = wIn, a.recvFlag[0] = 5;
            b.recv[0] = w128In, b.recvFlag[0] = 5;
          }
          if (shape == 2) a.dst = b.dst = (char*)dst;
        }
        const uint64_t grid = proto == 0 ? ((n + 7) / 8 + kLLTileLines - 1) / kLLTileLines
                                         : ((n + 1919) / 1920 * 128 + kLL128TileUnits - 1) / kLL128TileUnits;
        const int times = shape < 0 ? 1 : reps_n;
        for (int r = 0; r < times; r++) {
          if (proto == 0) CK(launch_ll(nexrFloat32, a, nexrDevSum, (int)grid, st));
          else CK(launch_ll128(nexrFloat32, b, nexrDevSum, (int)grid, st));
        }
        if (shape >= 0) {
          CK(hipMemsetAsync(cs, 0, 8, st));
          checksum<<<256, 256, 0, st>>>((const uint32_t*)(proto == 0 ? wOut : w128Out),
                                        (proto == 0 ? 2 * n : (n + 1919) / 1920 * 2048) / 4, cs);
          unsigned long long h;
          CK(hipMemcpyAsync(&h, cs, 8, hipMemcpyDeviceToHost, st));
          CK(hipStreamSynchronize(st));
          printf("proto=%s shape=%d bytes=%zu launches=%d checksum=%llu\n", proto ? "ll128" : "ll", shape, n, times,
                 h);
        }
      }
    }
    CK(hipStreamSynchronize(st));
    CK(hipFree(src));
    CK(hipFree(dst));
    CK(hipFree(wIn));
    CK(hipFree(wOut));
    CK(hipFree(w128In));
    CK(hipFree(w128Out));
  }
  printf("U=%d load_bits=%d store_bits=%d\n", kLLU, kLoadBits, kStoreBits);
  return 0;
}
