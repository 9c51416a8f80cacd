// Small reduce-copies (the slices an emulated collective step moves, 128 KiB - 4 MiB per buffer):
// workgroup geometry vs launch-to-completion latency, one launch + stream synchronisation at a time
// as a ring step issues it. Production kernel template (nexr_kernels.hip included directly).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 tools/small_geom.hip -o xbin/small_geom
//   ./xbin/small_geom <iters>
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <algorithm>
#include <vector>

using namespace nexr;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 300;
  constexpr int D = nexrFloat32, K = 2, OP = nexrDevSum;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  char* base;
  const size_t maxBytes = 4 << 20;
  CK(hipMalloc((void**)&base, 3 * maxBytes));
  CK(hipMemset(base, 0, 3 * maxBytes));
  for (size_t bytes : {128u << 10, 512u << 10, 1u << 20, 2u << 20, 4u << 20}) {
    RCParams p;
    std::memset((void*)&p, 0, sizeof(p));
    p.src[0] = base;
    p.src[1] = base + maxBytes;
    p.dst[0] = base + 2 * maxBytes;
    p.nDsts = 1;
    p.nElts = bytes / 4;
    p.nPacks = bytes / 16;
    const int P = (int)(bytes / 16);
    struct Var {
      std::string name;
      std::function<void()> run;
    };
    std::vector<Var> vs = {
        {"U=4 B=256 (16 KiB trips)", [&] { reduce_copy_kernel<D, OP, K, 0, 4, 256><<<P / 1024, 256, 0, s>>>(p); }},
        {"U=2 B=256 (8 KiB trips)", [&] { reduce_copy_kernel<D, OP, K, 0, 2, 256><<<P / 512, 256, 0, s>>>(p); }},
        {"U=1 B=256 (4 KiB trips)", [&] { reduce_copy_kernel<D, OP, K, 0, 1, 256><<<P / 256, 256, 0, s>>>(p); }},
        {"U=1 B=128 (2 KiB trips)", [&] { reduce_copy_kernel<D, OP, K, 0, 1, 128><<<P / 128, 128, 0, s>>>(p); }},
        {"U=1 B=64 (1 KiB trips)", [&] { reduce_copy_kernel<D, OP, K, 0, 1, 64><<<P / 64, 64, 0, s>>>(p); }},
    };
    for (auto& v : vs) {  // warm up
      for (int i = 0; i < 20; i++) v.run();
      CK(hipStreamSynchronize(s));
    }
    std::vector<std::vector<double>> us(vs.size());
    for (int it = 0; it < iters; it++)
      for (size_t k = 0; k < vs.size(); k++) {
        auto t0 = std::chrono::steady_clock::now();
        vs[k].run();
        CK(hipStreamSynchronize(s));
        us[k].push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
      }
    printf("bytes/buffer %zu KiB: launch + sync, median us\n", bytes >> 10);
    for (size_t k = 0; k < vs.size(); k++) {
      std::sort(us[k].begin(), us[k].end());
      printf("  %-26s %7.2f\n", vs[k].name.c_str(), us[k][us[k].size() / 2]);
    }
  }
  return 0;
}
