// Host-only stress driver for the emulated collectives (nexr_ring.cpp), built with sanitizers by
// tests/test_native_sanitizers.py: ThreadSanitizer for the FIFO head/tail protocol between rank
// threads (and between the two halves of a tree rank), AddressSanitizer + UndefinedBehaviorSanitizer
// for the slicing and chunking arithmetic. Every reduceCopy / LL / LL128 step is served by the C
// oracle (no GPU involved). Integer sums are order-independent, so the expected result of every
// collective is plain arithmetic.
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
  auto fail = [&](const char* what, int proto, int n) {
    printf("%s failed proto %d n %d\n", what, proto, n);
    failures++;
  };
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
      cfg.treeRanksPerNode = n == 4 ? 2 : 1;  // 4 ranks: 2 nodes of 2 (arity-3 heads); else a btree
      cfg.nChannels = n == 4 ? 3 : 2;          // concurrent channels (their own threads and links)
      nexrRingComm_t comm;
      if (nexrRingCommCreate(&comm, &cfg) != nexrSuccess) { printf("create failed\n"); return 2; }
      for (int iter = 0; iter < 3; iter++) {
        const size_t count = 10007 + 1000 * iter;
        const int root = iter % n;
        std::vector<std::vector<uint32_t>> in(n, std::vector<uint32_t>(count * n)), out(n);
        std::vector<const void*> s(n);
        std::vector<void*> r(n);
        for (int k = 0; k < n; k++) {
          for (size_t i = 0; i < count * n; i++) in[k][i] = (uint32_t)(i * 2654435761u + k * 40503u + iter);
          s[k] = in[k].data();
        }
        auto reset = [&] {
          for (int k = 0; k < n; k++) {
            out[k].assign(count * n, 0xdeadbeefu);
            r[k] = out[k].data();
          }
        };
        auto sum = [&](size_t i) {
          uint32_t e = 0;
          for (int j = 0; j < n; j++) e += in[j][i];
          return e;
        };
        // all-reduce, ring and tree
        for (int tree = 0; tree < 2; tree++) {
          reset();
          nexrResult_t rc = tree ? nexrTreeAllReduce(comm, s.data(), r.data(), count, nexrUint32, nexrSum)
                                 : nexrRingAllReduce(comm, s.data(), r.data(), count, nexrUint32, nexrSum);
          if (rc != nexrSuccess) { fail(tree ? "tree allreduce" : "allreduce", protos[pi], n); return 2; }
          for (int k = 0; k < n; k++)
            for (size_t i = 0; i < count; i++)
              if (out[k][i] != sum(i)) { fail(tree ? "tree allreduce value" : "allreduce value", protos[pi], n); break; }
        }
        // reduce-scatter: rank k gets the sum of segment k
        reset();
        if (nexrRingReduceScatter(comm, s.data(), r.data(), count, nexrUint32, nexrSum) != nexrSuccess) {
          fail("reducescatter", protos[pi], n);
          return 2;
        }
        for (int k = 0; k < n; k++)
          for (size_t i = 0; i < count; i++)
            if (out[k][i] != sum(k * count + i)) { fail("reducescatter value", protos[pi], n); break; }
        // all-gather of each rank's first `count` elements
        reset();
        if (nexrRingAllGather(comm, s.data(), r.data(), count, nexrUint32) != nexrSuccess) {
          fail("allgather", protos[pi], n);
          return 2;
        }
        for (int k = 0; k < n; k++)
          for (int j = 0; j < n; j++)
            for (size_t i = 0; i < count; i++)
              if (out[k][j * count + i] != in[j][i]) { fail("allgather value", protos[pi], n); j = n; break; }
        // reduce and broadcast to/from a rotating root
        reset();
        if (nexrRingReduce(comm, s.data(), r.data(), count, nexrUint32, nexrSum, root) != nexrSuccess) {
          fail("reduce", protos[pi], n);
          return 2;
        }
        for (size_t i = 0; i < count; i++)
          if (out[root][i] != sum(i)) { fail("reduce value", protos[pi], n); break; }
        reset();
        if (nexrRingBroadcast(comm, s.data(), r.data(), count, nexrUint32, root) != nexrSuccess) {
          fail("broadcast", protos[pi], n);
          return 2;
        }
        for (int k = 0; k < n; k++)
          for (size_t i = 0; i < count; i++)
            if (out[k][i] != in[root][i]) { fail("broadcast value", protos[pi], n); break; }
      }
      nexrRingCommDestroy(comm);
    }
  }
  printf("ring_stress failures=%d\n", failures);
  return failures ? 1 : 0;
}
