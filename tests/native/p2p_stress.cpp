// Host-only stress driver for ncclSend / ncclRecv between thread ranks (nexr_p2p.cpp, the extras
// library's nexrSendRecv), built with sanitizers by tests/test_native_sanitizers.py beside
// ring_stress.cpp: ThreadSanitizer for the send and recv halves of a rank running at once on their
// own threads over the shared connection-index-1 FIFO counters, AddressSanitizer +
// UndefinedBehaviorSanitizer for the chunking arithmetic (SIMPLE chunks, LL lines for messages of at
// most 16 KiB, self-sends, ranks with no send or no recv). Every step is served by the C oracle (no
// GPU involved); the expected bytes are the peer's input.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/nexr_extras.h"

extern "C" int oracle_reduce_copy_fn(int, const void* const*, int, void* const*, size_t, int, int, uint64_t, int,
                                     const uint64_t*, int, void*);
extern "C" int oracle_reduce_copy_ll_fn(const void*, int, int, const void* const*, const uint32_t*, void*, int,
                                        void* const*, const uint32_t*, size_t, int, int, uint64_t, int, uint32_t*,
                                        uint32_t, void*);

int main() {
  int failures = 0;
  for (int n = 2; n <= 6; n += 2) {
    for (int withLL = 0; withLL <= 1; withLL++) {
      nexrRingConfig cfg = {};
      cfg.nRanks = n;
      cfg.buffBytes = 8 * 32768;  // 32 KiB P2P chunks: a 200 KB message wraps the 8-slot FIFO
      cfg.memMode = nexrRingHostMemory;
      cfg.fn = (nexrReduceCopyFn)oracle_reduce_copy_fn;
      cfg.llFn = withLL ? (nexrReduceCopyLLFn)oracle_reduce_copy_ll_fn : nullptr;
      cfg.timeoutMs = 60000;
      cfg.protocol = nexrRingProtoSimple;
      nexrRingComm_t comm;
      if (nexrRingCommCreate(&comm, &cfg) != nexrSuccess) {
        printf("create failed\n");
        return 2;
      }
      const size_t sizes[4] = {4096, 16384, 200004, 1 << 20};  // LL-sized, the LL limit, ragged, many wraps
      for (int it = 0; it < 8; it++) {
        const size_t bytes = sizes[it % 4];
        const int shift = it % n;  // 0: every rank sends to itself (one copy)
        std::vector<std::vector<uint8_t>> in(n, std::vector<uint8_t>(bytes)), out(n, std::vector<uint8_t>(bytes));
        std::vector<const void*> s(n);
        std::vector<void*> r(n);
        std::vector<int> sp(n), rp(n);
        for (int k = 0; k < n; k++) {
          for (size_t i = 0; i < bytes; i++) in[k][i] = (uint8_t)(i * 131u + k * 17u + it);
          for (size_t i = 0; i < bytes; i++) out[k][i] = 0xa5;
          s[k] = in[k].data();
          r[k] = out[k].data();
          sp[k] = (k + shift) % n;
          rp[k] = (k - shift + n) % n;
        }
        if (it == 5) {  // rank 0 sends nothing and the rank that would receive from it receives nothing
          sp[0] = -1;
          rp[shift % n] = -1;
        }
        if (nexrSendRecv(comm, s.data(), sp.data(), r.data(), rp.data(), bytes) != nexrSuccess) {
          printf("sendrecv failed n %d ll %d it %d\n", n, withLL, it);
          failures++;
          break;
        }
        for (int k = 0; k < n; k++) {
          if (rp[k] < 0) {
            for (size_t i = 0; i < bytes; i++)
              if (out[k][i] != 0xa5) {
                printf("rank %d wrote without a recv n %d it %d\n", k, n, it);
                failures++;
                break;
              }
            continue;
          }
          for (size_t i = 0; i < bytes; i++)
            if (out[k][i] != in[rp[k]][i]) {
              printf("sendrecv value n %d ll %d it %d rank %d byte %zu\n", n, withLL, it, k, i);
              failures++;
              break;
            }
        }
      }
      nexrRingCommDestroy(comm);
    }
  }
  printf("p2p_stress failures=%d\n", failures);
  return failures ? 1 : 0;
}
