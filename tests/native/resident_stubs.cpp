// Host-only stand-ins for the device-resident kernels' entry points (nex-nccl_amd/csrc/nexr_resident.hip),
// so that the sanitizer build of the emulated collectives (g++, no device code) links. The stress
// driver never calls the resident collectives; if it did, they would fail with an invalid value.
#include "../../nex-nccl_amd/csrc/nexr_resident.h"

namespace nexr {
#define NEXR_STUB(dt)                                                                                  \
  hipError_t launch_resident_dt##dt(int, const ResParams&, int, hipStream_t) { return hipErrorInvalidValue; } \
  hipError_t resident_blocks_per_cu_dt##dt(int, uint64_t, int, int*) { return hipErrorInvalidValue; }
NEXR_STUB(0) NEXR_STUB(1) NEXR_STUB(2) NEXR_STUB(3) NEXR_STUB(4)
NEXR_STUB(5) NEXR_STUB(6) NEXR_STUB(7) NEXR_STUB(8) NEXR_STUB(9)
#undef NEXR_STUB
}  // namespace nexr
