// Memory-locality probe (tuning harness, not product code): does the HBM latency a workgroup sees
// depend on which XCD it runs on and where the line sits, in a way the virtual address predicts?
//
// MI355X puts its 8 XCDs and 8 HBM3E stacks on two I/O dies; with memory interleaved over all stacks
// (NPS1) half of every stream crosses between the dies. If the stack of a 4 KiB chunk could be read
// off its virtual address (bits below the 2 MiB page), a reduce-copy could give each XCD the chunks
// behind its own die. This probe measures it: 32 workgroups, one lane each, read one 128-B line of
// every 4 KiB chunk of a never-touched region with one dependent, timed, non-temporal load at a time;
// every line is read exactly once chip-wide, so every load misses the L2 and the Infinity Cache.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/numa_probe.hip -o tools/numa_probe
//   ./tools/numa_probe <MiB probed> > out.csv      (columns: wg, xcc, chunk, cycles)
#include <hip/hip_runtime.h>

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

constexpr int kWGs = 32;  // one 128-B line of every 4 KiB chunk per workgroup

// laneStride is 0 at run time: every lane of the wave loads the same line (one request), and the
// address is not provably uniform, so the load stays a vector load (not the scalar cache).
__global__ __launch_bounds__(64) void probe(const uint32_t* __restrict__ base, int nChunks, uint32_t* lat,
                                            uint32_t* xcc, uint32_t* sink, int laneStride) {
  const int w = blockIdx.x;
  uint32_t id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
  if (threadIdx.x == 0) xcc[w] = id & 0xf;
  uint32_t acc = 0;
  for (int c = 0; c < nChunks; c++) {
    // the line (w) of chunk c, offset by the previous value (always 0) so the loads stay dependent
    const uint32_t* p = base + ((size_t)c * 4096 + (size_t)w * 128) / 4 + (acc & 1) + threadIdx.x * laneStride;
    const uint64_t t0 = clock64();
    const uint32_t v = __builtin_nontemporal_load(p);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t t1 = clock64();
    acc += v;
    if (threadIdx.x == 0) lat[(size_t)w * nChunks + c] = (uint32_t)(t1 - t0);
  }
  if (threadIdx.x == 0) sink[w] = acc;
}

int main(int argc, char** argv) {
  const int mib = argc > 1 ? atoi(argv[1]) : 8;
  const int nChunks = mib * 256;
  const size_t bytes = (size_t)mib << 20;
  uint32_t *buf, *lat, *xcc, *sink, *flush;
  CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0, bytes));
  const size_t flushBytes = (size_t)1 << 30;  // push the memset's lines out of the Infinity Cache
  CK(hipMalloc(&flush, flushBytes));
  CK(hipMemset(flush, 1, flushBytes));
  CK(hipMalloc(&lat, (size_t)kWGs * nChunks * 4));
  CK(hipMalloc(&xcc, kWGs * 4));
  CK(hipMalloc(&sink, kWGs * 4));
  CK(hipDeviceSynchronize());
  probe<<<kWGs, 64>>>(buf, nChunks, lat, xcc, sink, argc > 2 ? atoi(argv[2]) : 0);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> h((size_t)kWGs * nChunks), hx(kWGs);
  CK(hipMemcpy(h.data(), lat, h.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hx.data(), xcc, kWGs * 4, hipMemcpyDeviceToHost));
  printf("# base %p\nwg,xcc,chunk,cycles\n", (void*)buf);
  for (int w = 0; w < kWGs; w++)
    for (int c = 0; c < nChunks; c++) printf("%d,%u,%d,%u\n", w, hx[w], c, h[(size_t)w * nChunks + c]);
  return 0;
}
