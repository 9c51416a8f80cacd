/*
 * multi_device_c.c — BASELINE configs[4] (C5) from plain C: one independent fp32 sum, K = 2, M = 1
 * reduce-copy of `MiB` MiB per buffer on every visible GPU, all from one host call to
 * nexrReduceCopyMultiDevice (a host thread, a stream and a start barrier per device,
 * no collective, no peer access). Device memory comes from the HIP runtime's C API; the ABI itself
 * is include/nexr.h only.
 *
 *   gcc -std=c11 -O2 -D__HIP_PLATFORM_AMD__ -Iinclude -I/opt/rocm/include examples/multi_device_c.c \
 *       -Lnex-nccl_amd -lnexr -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/nex-nccl_amd \
 *       -Wl,-rpath,/opt/rocm/lib -o xbin/multi_device_c
 *   ./xbin/multi_device_c [MiB per buffer = 256] [reps = 20] [works per device = 1]
 *
 * Each device's inputs are integer-valued (every fold order is exact) and distinct per device; after
 * the timed call every output is copied back and checked element by element against a + b. Prints
 * one line per device and an aggregate line ("multi_device_c ok ... GB/s"), exits 0; on a mismatch
 * or error it names it and exits 1.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "nexr.h"

#define CHECK_HIP(x)                                                        \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      printf("multi_device_c HIP error %d at line %d\n", (int)e_, __LINE__); \
      return 1;                                                             \
    }                                                                       \
  } while (0)

static float in_a(size_t i, int w) { return (float)((i + 101u * (unsigned)w) % 4096u); }
static float in_b(size_t i, int w) { return (float)((i * 7u + 13u * (unsigned)w) % 2048u) - 1024.0f; }

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)strtoul(argv[1], NULL, 10) : 256;
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int perDev = argc > 3 ? atoi(argv[3]) : 1;
  int nDev = 0;
  CHECK_HIP(hipGetDeviceCount(&nDev));
  const int nWorks = nDev * perDev;
  if (mib == 0 || reps < 1 || perDev < 1 || nWorks < 1 || nWorks > NEXR_MAX_MULTI_DEVICE_WORKS) {
    printf("multi_device_c bad arguments (devices %d)\n", nDev);
    return 1;
  }
  const size_t n = (mib << 20) / sizeof(float);
  float* host = malloc(n * sizeof(float));
  float* hostB = malloc(n * sizeof(float));
  nexrReduceCopyWork* works = calloc((size_t)nWorks, sizeof(nexrReduceCopyWork));
  int* devices = calloc((size_t)nWorks, sizeof(int));
  float** bufs = calloc((size_t)nWorks * 3, sizeof(float*));
  if (!host || !hostB || !works || !devices || !bufs) {
    printf("multi_device_c out of host memory\n");
    return 1;
  }
  for (int w = 0; w < nWorks; w++) {
    devices[w] = w % nDev;
    CHECK_HIP(hipSetDevice(devices[w]));
    for (int b = 0; b < 3; b++) CHECK_HIP(hipMalloc((void**)&bufs[3 * w + b], n * sizeof(float)));
    for (size_t i = 0; i < n; i++) {
      host[i] = in_a(i, w);
      hostB[i] = in_b(i, w);
    }
    CHECK_HIP(hipMemcpy(bufs[3 * w], host, n * sizeof(float), hipMemcpyHostToDevice));
    CHECK_HIP(hipMemcpy(bufs[3 * w + 1], hostB, n * sizeof(float), hipMemcpyHostToDevice));
    CHECK_HIP(hipMemset(bufs[3 * w + 2], 0xff, n * sizeof(float)));
    works[w].nSrcs = 2;
    works[w].nDsts = 1;
    works[w].srcs[0] = bufs[3 * w];
    works[w].srcs[1] = bufs[3 * w + 1];
    works[w].dsts[0] = bufs[3 * w + 2];
    works[w].nElts = n;
  }
  /* one untimed call (first-launch costs), then the timed one */
  double seconds = 0.0;
  nexrResult_t r = nexrReduceCopyMultiDevice(works, devices, nWorks, nexrFloat32, nexrDevSum, 1, NULL);
  if (r == nexrSuccess) r = nexrReduceCopyMultiDevice(works, devices, nWorks, nexrFloat32, nexrDevSum, reps, &seconds);
  if (r != nexrSuccess) {
    printf("multi_device_c nexrReduceCopyMultiDevice: %d (hip %d)\n", (int)r, nexrGetLastHipError());
    return 1;
  }
  for (int w = 0; w < nWorks; w++) {
    CHECK_HIP(hipSetDevice(devices[w]));
    CHECK_HIP(hipMemcpy(host, bufs[3 * w + 2], n * sizeof(float), hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; i++)
      if (host[i] != in_a(i, w) + in_b(i, w)) {
        printf("multi_device_c MISMATCH work %d (device %d) at %zu: %g\n", w, devices[w], i, (double)host[i]);
        return 1;
      }
    for (int b = 0; b < 3; b++) CHECK_HIP(hipFree(bufs[3 * w + b]));
  }
  const double bytes = 3.0 * (double)n * sizeof(float) * reps * nWorks;
  printf("multi_device_c ok devices=%d works=%d MiB=%zu reps=%d seconds=%.6f aggregate_GBps=%.1f\n", nDev, nWorks,
         mib, reps, seconds, bytes / seconds / 1e9);
  free(host);
  free(hostB);
  free(works);
  free(devices);
  free(bufs);
  return 0;
}
