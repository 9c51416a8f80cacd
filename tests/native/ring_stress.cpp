// Host-only stress driver for the emulated ring (nexr_ring.cpp), built with sanitizers by
// tests/test_native_sanitizers.py: ThreadSanitizer for the FIFO head/tail protocol between rank
// threads, AddressSanitizer + UndefinedBehaviorSanitizer for the slicing arithmetic. Every
// reduceCopy / LL / LL128 step is served by the C oracle (no GPU involved). Integer sums are
// order-independent, so the expected result is plain arithmetic.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/nexr_ring.h"

extern "C" int oracle_reduce_copy_fn(int, const void* const*, int, void* const*, size_t, int, int, uint64_t, int,
                                     const uint64_t*, int, void*);
extern "C" int oracle_reduce_copy_ll_fn(const void*, int, int, const void* const*, const uint32_t*, void*, int,
                                        void* const*, const uint32_t*, size_t, int, int, uint64_t, int, uint32_t*,
                                        uint32_t, void*);
extern "C" int oracle_reduce_copy_ll128_fn(const void*, int, int, const void* const*, const uint64_t*, void*, int,
                                           void* const*, const uint64_t*, size_t, int, int, uint64_t, int, uint32_t*,
                                           uint32_t, void*);

int main() {
  int failures = 0;
  const int protos[3] = {nexrRingProtoSimple, nexrRingProtoLL, nexrRingProtoLL128};
  const size_t buffs[3] = {8 * 4096, 8 * 1024 * 16, 8 * 2048 * 2};
  for (int pi = 0; pi < 3; pi++) {
    for (int n = 2; n <= 6; n += 2) {
      nexrRingConfig cfg = {};
      cfg.nRanks = n;
      cfg.buffBytes = buffs[pi];
      cfg.memMode = nexrRingHostMemory;
      cfg.fn = (nexrReduceCopyFn)oracle_reduce_copy_fn;
      cfg.llFn = (nexrReduceCopyLLFn)oracle_reduce_copy_ll_fn;
      cfg.ll128Fn = (nexrReduceCopyLL128Fn)oracle_reduce_copy_ll128_fn;
      cfg.timeoutMs = 60000;
      cfg.protocol = protos[pi];
      nexrRingComm_t comm;
      if (nexrRingCommCreate(&comm, &cfg) != nexrSuccess) { printf("create failed\n"); return 2; }
      for (int iter = 0; iter < 3; iter++) {
        const size_t count = 10007 + 1000 * iter;
        std::vector<std::vector<uint32_t>> in(n, std::vector<uint32_t>(count)), out(n, std::vector<uint32_t>(count));
        std::vector<const void*> s(n);
        std::vector<void*> r(n);
        for (int k = 0; k < n; k++) {
          for (size_t i = 0; i < count; i++) in[k][i] = (uint32_t)(i * 2654435761u + k * 40503u + iter);
          s[k] = in[k].data();
          r[k] = out[k].data();
        }
        if (nexrRingAllReduce(comm, s.data(), r.data(), count, nexrUint32, nexrSum) != nexrSuccess) {
          printf("allreduce failed proto %d n %d\n", protos[pi], n);
          return 2;
        }
        for (int k = 0; k < n; k++)
          for (size_t i = 0; i < count; i++) {
            uint32_t e = 0;
            for (int j = 0; j < n; j++) e += in[j][i];
            if (out[k][i] != e) { failures++; break; }
          }
      }
      nexrRingCommDestroy(comm);
    }
  }
  printf("ring_stress failures=%d\n", failures);
  return failures ? 1 : 0;
}
