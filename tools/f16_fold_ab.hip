// fp16 K = 8 fold through fp32 (tuning harness, not product code). On the same buffers the bf16 K = 8
// kernel runs 1-3 % ahead of the fp16 one (tools/k8_types_ab.py) although its fold costs more VALU
// work, and pacing the stores with s_sleep does not reproduce that (tools/pace_sweep.hip). This A/B
// gives the fp16 kernel a bf16-like fold: every step as half(float(acc) + float(v)) with explicit
// v_cvt_f32_f16 / v_add_f32 / v_cvt_f16_f32 (RNE), the same value as the production v_pk_add_f16
// (DESIGN §2), NaNs canonicalised at the end as production does. Outputs byte-checked against the
// production kernel; same geometry, policy and trip.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DNEXR_DT=6 tools/f16_fold_ab.hip \
//         -o tools/f16_fold_ab
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

__global__ void fill_bits(uint32_t* p, size_t n, uint64_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    p[i] = (uint32_t)(z ^ (z >> 31)) & 0x3bff3bffu;  // finite values for every float type
  }
}

constexpr int D = NEXR_DT;

typedef _Float16 hx2 __attribute__((ext_vector_type(2)));
typedef float fx2 __attribute__((ext_vector_type(2)));

// MODE 0: the production Fold; MODE 1: the fold through fp32, one rounding to half per step.
template <int MODE, int U = unroll_for(D, 8, kPolNt), int B = block_for(D, 8, kPolNt)>
__global__ __launch_bounds__(B) void fold_kernel(RCParams p) {
  constexpr int K = 8;
  Fold<D, nexrDevSum, K, false> f(p);
  const uint64_t off = ((uint64_t)blockIdx.x * (B * U) + threadIdx.x) * 16;
  u32x4 in[U][K];
#pragma unroll
  for (int s = 0; s < K; s++)
#pragma unroll
    for (int u = 0; u < U; u++) in[u][s] = ld16<kPolNt>(p.src[s] + off + u * B * 16);
  u32x4 out[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    if constexpr (MODE == 0) {
      out[u] = f.run(in[u]);
    } else {
      u32x4 acc = in[u][0];
#pragma unroll
      for (int s = 1; s < K; s++)
#pragma unroll
        for (int w = 0; w < 4; w++) {
          hx2 a = __builtin_bit_cast(hx2, acc[w]), v = __builtin_bit_cast(hx2, in[u][s][w]);
          fx2 fa = __builtin_convertvector(a, fx2), fv = __builtin_convertvector(v, fx2);
          asm volatile("" : "+v"(fa), "+v"(fv));  // keep the fp32 operands: no fold back to a half add
          fx2 r = fa + fv;
          asm volatile("" : "+v"(r));
          acc[w] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, hx2));
        }
      out[u] = bc<u32x4>(Ty<D>::canon(bc<typename Ty<D>::V>(acc)));
    }
  }
#pragma unroll
  for (int u = 0; u < U; u++) st16<kPolNt>(p.dst[0] + off + u * B * 16, out[u]);
}

struct Var {
  std::string name;
  int k;
  size_t bytes;
  std::function<void(int)> run;
  int ref;
  std::vector<float> ms;
};

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8;
  constexpr int esz = 16 / Ty<D>::EPP;
  const size_t maxBytes = 256u << 20;
  const int R = 3;
  std::vector<RCParams> base(R);
  for (int r = 0; r < R; r++) {
    std::memset((void*)&base[r], 0, sizeof(RCParams));
    for (int s = 0; s < 8; s++) {
      char* q;
      CK(hipMalloc((void**)&q, maxBytes));
      fill_bits<<<2048, 256>>>((uint32_t*)q, maxBytes / 4, 1000 + r * 16 + s);
      base[r].src[s] = q;
    }
    CK(hipMalloc((void**)&base[r].dst[0], maxBytes));
    base[r].nDsts = 1;
  }
  CK(hipDeviceSynchronize());
  auto params = [&](int r, size_t bytes) {
    RCParams q = base[r];
    q.nElts = bytes / esz;
    q.nPacks = bytes / 16;
    return q;
  };
  std::vector<Var> vs;
  const size_t BYTES = (size_t)256 << 20;
  const int grid = (int)(BYTES / 16 / (unroll_for(D, 8, kPolNt) * block_for(D, 8, kPolNt)));
  vs.push_back({"fp16 sum K8 256 MiB production fold", 8, BYTES,
                [=, &params](int r) { fold_kernel<0><<<grid, block_for(D, 8, kPolNt)>>>(params(r, BYTES)); }, -1, {}});
  vs.push_back({"fp16 sum K8 256 MiB fold through fp32", 8, BYTES,
                [=, &params](int r) { fold_kernel<1><<<grid, block_for(D, 8, kPolNt)>>>(params(r, BYTES)); }, 0, {}});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vs)
    for (int w = 0; w < 2; w++) v.run(w % R);
  CK(hipDeviceSynchronize());
  {
    std::vector<char> want(maxBytes), got(maxBytes);
    for (size_t i = 0; i < vs.size(); i++) {
      CK(hipMemset(base[0].dst[0], 0, vs[i].bytes));
      vs[i].run(0);
      CK(hipMemcpy(vs[i].ref < 0 ? want.data() : got.data(), base[0].dst[0], vs[i].bytes, hipMemcpyDeviceToHost));
      if (vs[i].ref >= 0 && memcmp(want.data(), got.data(), vs[i].bytes) != 0)
        printf("MISMATCH: %s\n", vs[i].name.c_str());
    }
  }
  const int BLK = 8;
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
  printf("dt=%d: median (best) of %d blocks of %d launches; vs = median vs production\n", D, iters, BLK);
  double refMed = 0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double alg = (double)(v.k + 1) * v.bytes;
    const float med = v.ms[v.ms.size() / 2], mn = v.ms[0];
    if (v.ref < 0) refMed = med;
    printf("%-36s %8.2f us  %6.0f GB/s (%6.0f)  vs %+5.1f %%\n", v.name.c_str(), med * 1e3, alg / med / 1e6,
           alg / mn / 1e6, (refMed / med - 1) * 100);
  }
  return 0;
}
