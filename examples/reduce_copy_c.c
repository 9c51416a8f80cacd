/*
 * reduce_copy_c.c — the drop-in boundary driven from plain C (C11, gcc), as the fork's host code
 * would: no HIP headers, no C++, only include/nexr.h and include/nexr_ring.h.
 *
 *   1. nexrReduceCopyHost on malloc'd (pageable) host buffers, the fork's emulated "device" memory:
 *      fp32 sum K=2 and int8 max K=4 against a plain C loop;
 *   2. BASELINE configs[0]: ncclAllReduce of 4 MiB of fp32 per rank over 2 emulated ranks
 *      (nexrRingCommCreate + nexrRingAllReduce, host memory, every ring step on the MI355X).
 *
 *   gcc -std=c11 -O2 -Iinclude examples/reduce_copy_c.c -Lnex-nccl_amd -lnexr_ring -lnexr \
 *       -Wl,-rpath,$PWD/nex-nccl_amd -o xbin/reduce_copy_c && ./xbin/reduce_copy_c
 * Prints "reduce_copy_c ok" and exits 0, or names the first mismatch and exits 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "nexr.h"
#include "nexr_ring.h"

static int fail(const char* what, long i) {
  printf("reduce_copy_c MISMATCH %s at %ld\n", what, i);
  return 1;
}

int main(void) {
  /* 1a. fp32 sum, K = 2, M = 1 (integer-valued, so any fold order is exact) */
  const size_t n = 3000017;
  float* a = malloc(n * sizeof(float));
  float* b = malloc(n * sizeof(float));
  float* o = malloc(n * sizeof(float));
  for (size_t i = 0; i < n; i++) {
    a[i] = (float)(i % 1000);
    b[i] = (float)((i * 7) % 1000) - 500.0f;
  }
  const void* srcs[2] = {a, b};
  void* dsts[1] = {o};
  nexrResult_t r = nexrReduceCopyHost(2, srcs, 1, dsts, n, nexrFloat32, nexrDevSum, 0, 0, NULL, 0, NULL);
  if (r != nexrSuccess) {
    printf("nexrReduceCopyHost: %d (hip %d)\n", (int)r, nexrGetLastHipError());
    return 1;
  }
  for (size_t i = 0; i < n; i++)
    if (o[i] != a[i] + b[i]) return fail("fp32 sum", (long)i);

  /* 1b. int8 max, K = 4, M = 2: the MinMax argument from the reference's encoder */
  const size_t m = 1000003;
  int8_t* s8[4];
  for (int k = 0; k < 4; k++) {
    s8[k] = malloc(m);
    for (size_t i = 0; i < m; i++) s8[k][i] = (int8_t)((i * (2 * k + 3) + 17 * k) & 0xff);
  }
  int8_t* d8[2] = {malloc(m), malloc(m)};
  nexrDevRedOpFull full;
  if (nexrHostToDevRedOp(&full, nexrMax, nexrInt8, 4) != nexrSuccess) return fail("encode max", 0);
  const void* s8v[4] = {s8[0], s8[1], s8[2], s8[3]};
  void* d8v[2] = {d8[0], d8[1]};
  r = nexrReduceCopyHost(4, s8v, 2, d8v, m, nexrInt8, full.op, full.scalarArg, 0, NULL, 0, NULL);
  if (r != nexrSuccess) return fail("int8 max call", (long)r);
  for (size_t i = 0; i < m; i++) {
    int8_t e = s8[0][i];
    for (int k = 1; k < 4; k++) e = s8[k][i] > e ? s8[k][i] : e;
    if (d8[0][i] != e || d8[1][i] != e) return fail("int8 max", (long)i);
  }

  /* 2. C1: 2 emulated ranks, ring all-reduce of 4 MiB fp32 each, host memory */
  const size_t count = 1 << 20;
  float* in[2];
  float* out[2];
  for (int k = 0; k < 2; k++) {
    in[k] = malloc(count * sizeof(float));
    out[k] = malloc(count * sizeof(float));
    for (size_t i = 0; i < count; i++) in[k][i] = (float)((i + 31 * k) % 4096);
  }
  nexrRingConfig cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.nRanks = 2;
  cfg.memMode = nexrRingHostMemory;
  nexrRingComm_t comm;
  if ((r = nexrRingCommCreate(&comm, &cfg)) != nexrSuccess) return fail("comm create", (long)r);
  const void* sb[2] = {in[0], in[1]};
  void* rb[2] = {out[0], out[1]};
  if ((r = nexrRingAllReduce(comm, sb, rb, count, nexrFloat32, nexrSum)) != nexrSuccess) return fail("allreduce", (long)r);
  nexrRingCommDestroy(comm);
  for (int k = 0; k < 2; k++)
    for (size_t i = 0; i < count; i++)
      if (out[k][i] != in[0][i] + in[1][i]) return fail("C1 all-reduce", (long)i);

  printf("reduce_copy_c ok\n");
  return 0;
}
