/*
 * ll_steps_c.c — a run of LL steps with the protocol's credits on the device, from plain C
 * (nexrReduceCopyLLSteps, include/nexr.h; reference src/device/prims_ll.h:55-83 and :249-318), as a
 * fork whose Primitives<..., ProtoLL> loop hands its LLGenericOp calls to the ABI would drive it.
 *
 * Two "ranks" on one GPU, each on a stream with a hardware queue of its own (hipExtStreamCreateWithCUMask,
 * every CU in the mask): rank A sends `steps` steps of its input through an 8-slot FIFO (send), rank B
 * receives each one and writes peer + its own input to its output (recvReduceCopy). The FIFO's head
 * words (NEXR_LL_HEAD_BYTES) sit behind its slots in the same zeroed allocation. With more steps than
 * slots every slot is rewritten only after B's credit for it came back. Device memory and streams come
 * from the HIP runtime's C API; the ABI itself is include/nexr.h only.
 *
 *   gcc -std=c11 -O2 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include examples/ll_steps_c.c \
 *       -Lnex-nccl_amd -lnexr -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/nex-nccl_amd \
 *       -Wl,-rpath,/opt/rocm/lib -o xbin/ll_steps_c
 *   ./xbin/ll_steps_c [steps = 40] [slot KiB = 64]
 *
 * Inputs are integer-valued, so the fp32 sums are exact; prints "ll_steps_c ok" and exits 0, or names
 * the first mismatch or error and exits 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "nexr.h"

#define CHECK_HIP(x)                                                     \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      printf("ll_steps_c HIP error %d at line %d\n", (int)e_, __LINE__); \
      return 1;                                                          \
    }                                                                    \
  } while (0)

#define SLOTS 8

int main(int argc, char** argv) {
  const int steps = argc > 1 ? atoi(argv[1]) : 40;
  const size_t slot = (argc > 2 ? (size_t)strtoul(argv[2], NULL, 10) : 64) << 10;
  const size_t per = slot / 2 / sizeof(float); /* fp32 elements per step: 8 data bytes per 16-B line */
  const size_t n = per * (size_t)steps;
  if (steps < 1 || slot < 4096 || slot % 16) {
    printf("ll_steps_c bad arguments\n");
    return 1;
  }
  float* ha = malloc(n * sizeof(float));
  float* hb = malloc(n * sizeof(float));
  float* ho = malloc(n * sizeof(float));
  for (size_t i = 0; i < n; i++) {
    ha[i] = (float)(i % 1000);
    hb[i] = (float)((i * 7) % 1000) - 500.0f;
  }
  hipDeviceProp_t prop;
  CHECK_HIP(hipGetDeviceProperties(&prop, 0));
  uint32_t mask[64];
  const int words = (prop.multiProcessorCount + 31) / 32;
  for (int i = 0; i < words; i++) mask[i] = 0xffffffffu;
  if (prop.multiProcessorCount % 32) mask[words - 1] = (1u << (prop.multiProcessorCount % 32)) - 1;
  hipStream_t sa, sb;
  CHECK_HIP(hipExtStreamCreateWithCUMask(&sa, (uint32_t)words, mask));
  CHECK_HIP(hipExtStreamCreateWithCUMask(&sb, (uint32_t)words, mask));
  float *da, *db, *dout;
  char* fifo;
  uint32_t* status;
  CHECK_HIP(hipMalloc((void**)&da, n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&db, n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&dout, n * sizeof(float)));
  CHECK_HIP(hipMalloc((void**)&fifo, slot * SLOTS + NEXR_LL_HEAD_BYTES));
  CHECK_HIP(hipMemset(fifo, 0, slot * SLOTS + NEXR_LL_HEAD_BYTES));
  CHECK_HIP(hipHostMalloc((void**)&status, 2 * sizeof(uint32_t), hipHostMallocMapped));
  status[0] = status[1] = 0;
  CHECK_HIP(hipMemcpy(da, ha, n * sizeof(float), hipMemcpyHostToDevice));
  CHECK_HIP(hipMemcpy(db, hb, n * sizeof(float), hipMemcpyHostToDevice));
  uint64_t* head = (uint64_t*)(fifo + slot * SLOTS);

  nexrLLStep* sendSteps = calloc((size_t)steps, sizeof(nexrLLStep));
  nexrLLStep* recvSteps = calloc((size_t)steps, sizeof(nexrLLStep));
  for (int k = 0; k < steps; k++) {
    sendSteps[k].srcBuf = 0, sendSteps[k].dstBuf = -1, sendSteps[k].srcIx = (int64_t)per * k;
    sendSteps[k].nElts = (uint32_t)per, sendSteps[k].send = 1;
    recvSteps[k].srcBuf = 0, recvSteps[k].dstBuf = 1, recvSteps[k].srcIx = (int64_t)per * k;
    recvSteps[k].dstIx = (int64_t)per * k, recvSteps[k].nElts = (uint32_t)per, recvSteps[k].recv = 1;
  }
  nexrLLConnSet a, b;
  memset(&a, 0, sizeof(a));
  memset(&b, 0, sizeof(b));
  a.input = da, a.nSend = 1, a.sendFifo[0] = fifo, a.sendHead[0] = head, a.sendStep[0] = 0;
  a.slotBytes = slot, a.nSlots = SLOTS;
  b.input = db, b.output = dout, b.nRecv = 1, b.recvFifo[0] = fifo, b.recvHead[0] = head, b.recvStep[0] = 0;
  b.slotBytes = slot, b.nSlots = SLOTS;
  /* the receiver first: its run polls the slots while the sender's is still being queued */
  nexrResult_t r = nexrReduceCopyLLSteps(&b, recvSteps, steps, nexrFloat32, nexrDevSum, 0, &status[1], 2000000,
                                         (nexrStream_t)sb);
  if (r == nexrSuccess)
    r = nexrReduceCopyLLSteps(&a, sendSteps, steps, nexrFloat32, nexrDevSum, 0, &status[0], 2000000,
                              (nexrStream_t)sa);
  if (r != nexrSuccess) {
    printf("ll_steps_c nexrReduceCopyLLSteps: %s\n", nexrGetErrorString(r));
    return 1;
  }
  CHECK_HIP(hipDeviceSynchronize());
  if (status[0] || status[1]) {
    printf("ll_steps_c status %u %u (a line or a credit never came)\n", status[0], status[1]);
    return 1;
  }
  CHECK_HIP(hipMemcpy(ho, dout, n * sizeof(float), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++)
    if (ho[i] != ha[i] + hb[i]) {
      printf("ll_steps_c MISMATCH at %zu: %f != %f\n", i, (double)ho[i], (double)(ha[i] + hb[i]));
      return 1;
    }
  printf("ll_steps_c ok: %d steps of %zu KiB slots through %d slots\n", steps, slot >> 10, SLOTS);
  free(sendSteps), free(recvSteps), free(ha), free(hb), free(ho);
  hipFree(da), hipFree(db), hipFree(dout), hipFree(fifo), hipHostFree(status);
  hipStreamDestroy(sa), hipStreamDestroy(sb);
  return 0;
}
