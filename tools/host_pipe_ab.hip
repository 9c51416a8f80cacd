// Zero-copy launches on pinned host memory: the production kernel against a software-pipelined
// variant (tuning harness, not product code; DESIGN §6.4 / §8.2, C1's host_registered leg).
//
// A launch that touches host memory runs 32 workgroups (NEXR_HOST_GRID), each looping over trips of
// the production shape. Every trip reads all its sources, then writes its destinations, and the 32
// workgroups start together, so at C1's step sizes (1-2 MiB per buffer, a few trips per workgroup) the
// PCIe reads and writes of one launch alternate instead of overlapping (45-50 GB/s of the ~114 GB/s
// the two link directions carry, profiles/r05f_zero_copy_grid.txt). The pipelined variant issues the
// loads of a workgroup's next trip before the fold and stores of the current one, so both directions
// stay busy. This times both (fp32 sum, the ring's step shapes K1M1 / K2M1 / K2M2) on buffers from
// hipHostMalloc(Mapped | Portable) as nexrHostMemAlloc allocates them, byte-checks every variant
// against the production kernel, and reports: kernels back to back on one stream, launch +
// hipStreamSynchronize per call (a ring step), and two streams at once (C1's two rank threads).
// Result (profiles/r05y_host_pipe_ab_not_kept.txt): the pipelined variant is within +-5 % of
// production at every size and grid; zero-copy traffic tops out at 56-64 GB/s (1-2 MiB per buffer)
// and 74-84 GB/s (16 MiB) whatever the access order. Not kept.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=7 tools/host_pipe_ab.hip -o tools/host_pipe_ab
//   ./tools/host_pipe_ab [reps]
#include "../nex-nccl_amd/csrc/nexr_kernels.hip"

#include <algorithm>
#include <chrono>
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

// Full trips only (the harness's sizes are whole trips): load trip g+nblk, fold and store trip g.
template <int D, int OP, int K, int U, int B>
__global__ __launch_bounds__(B) void pipe_kernel(RCParams p) {
  Fold<D, OP, K, false> f(p);
#pragma unroll
  for (int s = 0; s < K; s++) asm volatile("" ::"s"(p.src[s]));
  asm volatile("" ::"s"(p.dst[0]));
  const int nDsts = p.nDsts;
  const uint64_t nFull = p.nPacks / (B * U);
  constexpr uint64_t kTrip = (uint64_t)B * U * 16;
  const uint32_t lane = threadIdx.x * 16u;
  const uint64_t nblk = gridDim.x;
  uint64_t g = blockIdx.x;
  u32x4 cur[U][K];
  auto load = [&](u32x4(&v)[U][K], uint64_t t) {
    const uint64_t tb = t * kTrip;
#pragma unroll
    for (int s = 0; s < K; s++) {
      const char* base = (const char*)uniform64((uint64_t)(p.src[s] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) v[u][s] = ld16<kPolPlain>(base + (uint32_t)(lane + u * B * 16));
    }
  };
  if (g < nFull) load(cur, g);
  for (; g < nFull; g += nblk) {
    u32x4 nxt[U][K];
    const bool more = g + nblk < nFull;
    if (more) load(nxt, g + nblk);
    u32x4 out[U];
#pragma unroll
    for (int u = 0; u < U; u++) out[u] = f.run(cur[u]);
    const uint64_t tb = g * kTrip;
    {
      char* base = (char*)uniform64((uint64_t)(p.dst[0] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) st16<kPolPlain>(base + (uint32_t)(lane + u * B * 16), out[u]);
    }
#pragma unroll 1
    for (int d = 1; d < nDsts; d++) {
      char* base = (char*)uniform64((uint64_t)(p.dst[d] + tb));
#pragma unroll
      for (int u = 0; u < U; u++) st16<kPolPlain>(base + (uint32_t)(lane + u * B * 16), out[u]);
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < U; u++)
#pragma unroll
        for (int s = 0; s < K; s++) cur[u][s] = nxt[u][s];
    }
  }
}

struct Var {
  std::string name;
  int tripPacks;  // packs per trip (U x B): the grid is capped by the number of trips
  int grid;
  std::function<void(const RCParams&, int, hipStream_t)> run;
};

template <int K>
static std::vector<Var> variants() {
  constexpr int D = nexrFloat32, OP = nexrDevSum;
  std::vector<Var> v;
  auto prod = [](const RCParams& p, int g, hipStream_t s) {
    reduce_copy_kernel<D, OP, K, kPolPlain><<<g, block_for(D, K, kPolPlain), 0, s>>>(p);
  };
  v.push_back({"production 4x256, 32 WG", kTripPacks, 32, prod});
  v.push_back({"production 4x256, 64 WG", kTripPacks, 64, prod});
#define PV(U, B, G)                                                                                   \
  v.push_back({"pipelined " #U "x" #B ", " #G " WG", U * B, G,                                        \
               [](const RCParams& p, int g, hipStream_t s) { pipe_kernel<D, OP, K, U, B><<<g, B, 0, s>>>(p); }})
  PV(1, 256, 32);
  PV(1, 256, 64);
  PV(1, 256, 128);
  PV(2, 256, 32);
  PV(2, 256, 64);
  PV(4, 256, 32);
  PV(1, 512, 32);
#undef PV
  return v;
}

static double median(std::vector<double> x) {
  std::sort(x.begin(), x.end());
  return x[x.size() / 2];
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 9;
  const size_t maxBytes = 16u << 20;
  // two buffer sets (one per stream), 4 buffers each, pinned and device-mapped like nexrHostMemAlloc
  char* host[2][4];
  for (int r = 0; r < 2; r++)
    for (int b = 0; b < 4; b++) {
      CK(hipHostMalloc((void**)&host[r][b], maxBytes, hipHostMallocMapped | hipHostMallocPortable));
      uint32_t x = 12345u + 77u * (r * 4 + b);
      uint32_t* w = (uint32_t*)host[r][b];
      for (size_t i = 0; i < maxBytes / 4; i++) {
        x = x * 1664525u + 1013904223u;
        w[i] = (x >> 9) | 0x3f800000u;  // floats in [1, 2)
      }
    }
  hipStream_t st[2];
  for (int r = 0; r < 2; r++) CK(hipStreamCreateWithFlags(&st[r], hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("fp32 sum on hipHostMalloc'd buffers; GB/s = (K+M) x bytes per buffer moved over PCIe per call;\n"
         "'serial': median us per kernel of %d back-to-back launches on one stream; 'sync': launch +\n"
         "hipStreamSynchronize per call; 'two streams': two calls at once on two buffer sets (aggregate)\n\n", 8);
  struct ShapeKM {
    const char* name;
    int k, m;
  };
  const ShapeKM shapes[] = {{"copy K1 M1", 1, 1}, {"reduce K2 M1", 2, 1}, {"recvReduceCopySend K2 M2", 2, 2}};
  const size_t sizes[] = {256u << 10, 1u << 20, 2u << 20, 4u << 20, 16u << 20};
  std::vector<char> ref(maxBytes), got(maxBytes);
  for (const ShapeKM& sh : shapes) {
    std::vector<Var> vars = sh.k == 1 ? variants<1>() : variants<2>();
    for (size_t bytes : sizes) {
      printf("%s, %zu KiB per buffer\n", sh.name, bytes >> 10);
      RCParams base[2];
      for (int r = 0; r < 2; r++) {
        RCParams& p = base[r];
        std::memset((void*)&p, 0, sizeof(p));
        for (int s = 0; s < sh.k; s++) p.src[s] = host[r][s];
        for (int d = 0; d < sh.m; d++) p.dst[d] = host[r][2 + d];
        p.nDsts = sh.m;
        p.nElts = bytes / 4;
        p.nPacks = bytes / 16;
        p.head = 0;
      }
      for (size_t vi = 0; vi < vars.size(); vi++) {
        const Var& v = vars[vi];
        if (bytes / 16 % v.tripPacks != 0 || bytes > maxBytes) {
          fprintf(stderr, "bad size for %s\n", v.name.c_str());
          return 2;
        }
        const int grid = std::min<int>(v.grid, (int)(bytes / 16 / v.tripPacks));
        // byte check (set 0, every destination) against the first variant
        bool ok = true;
        for (int d = 0; d < sh.m; d++) memset(base[0].dst[d], 0x5a, bytes);
        v.run(base[0], grid, st[0]);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(st[0]));
        for (int d = 0; d < sh.m; d++) {
          if (vi == 0 && d == 0) memcpy(ref.data(), base[0].dst[0], bytes);
          ok = ok && memcmp(ref.data(), base[0].dst[d], bytes) == 0;
        }
        std::vector<double> serial, sync, two;
        for (int it = 0; it < reps; it++) {
          const int n = 8;
          CK(hipEventRecord(e0, st[0]));
          for (int i = 0; i < n; i++) v.run(base[0], grid, st[0]);
          CK(hipEventRecord(e1, st[0]));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          serial.push_back(ms * 1e3 / n);
          auto t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < n; i++) {
            v.run(base[0], grid, st[0]);
            CK(hipStreamSynchronize(st[0]));
          }
          sync.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n);
          t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < n; i++) {
            v.run(base[0], grid, st[0]);
            v.run(base[1], grid, st[1]);
          }
          CK(hipStreamSynchronize(st[0]));
          CK(hipStreamSynchronize(st[1]));
          two.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n);
        }
        const double moved = (double)(sh.k + sh.m) * bytes;
        const double a = median(serial), b = median(sync), c = median(two);
        printf("  %-28s %-8s serial %8.1f us %6.1f GB/s | sync %8.1f us %6.1f GB/s | two streams %8.1f us %6.1f GB/s\n",
               v.name.c_str(), ok ? "exact" : "MISMATCH", a, moved / a / 1e3, b, moved / b / 1e3, c,
               2 * moved / c / 1e3);
        fflush(stdout);
      }
    }
  }
  return 0;
}
