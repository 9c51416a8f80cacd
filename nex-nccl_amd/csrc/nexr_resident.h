// nexr_resident.h — the device-resident ring all-reduce (nexr_resident.hip), shared with its host
// side in nexr_ring.cpp. Not installed; not part of the ABI (include/nexr_ring.h declares the entry
// point, nexrRingAllReduceResident).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace nexr {

constexpr int kResMaxRanks = 16;   // ranks one communicator may have for the resident path
constexpr int kResMaxParts = 64;   // channel parts (MAXCHANNELS)
constexpr int kResMaxTeam = 128;   // workgroups per (rank, channel)
constexpr int kResCtrBytes = 256;  // one (channel, rank, team member) record: tail line + head line
constexpr int kResHeadOff = 128;   // byte offset of the head word in a record

// One (channel, rank) of the ring, static for the communicator. Record (ch, r, g) of a device's
// counter block sits at ((ch * nRanks + r) * kResMaxTeam + g) * kResCtrBytes: `tail` (written by the
// sender r-1 once slice data has landed in r's FIFO) at +0 and `head` (written by r once a slot is
// consumed, the sender's credit) at +kResHeadOff.
struct ResConn {
  char* recvFifo;  // the FIFO this rank receives into (its own device)
  char* sendFifo;  // the next rank's receive FIFO (peer memory when on another GPU)
  char* recvCtr;   // record (ch, r, 0) on this rank's device
  char* sendCtr;   // record (ch, r + 1, 0) on the next rank's device
};

struct ResParams {
  const ResConn* conns;  // [ch * nRanks + r], in the launching device's memory
  const char* input[kResMaxRanks];
  char* output[kResMaxRanks];
  int64_t partOffset[kResMaxParts], partCount[kResMaxParts];
  int partChannel[kResMaxParts];
  int rankOf[kResMaxRanks];  // workgroup group li = blockIdx.x / (nParts * team) runs rank rankOf[li]
  int64_t chunkCount;        // elements per ring chunk (calcCollChunking)
  int64_t stepElems;         // elements per FIFO step
  uint64_t stepBytes;
  uint64_t redArg;           // op argument; also the pre-op scalar (Primitives' redOpArgs[0])
  uint32_t* status;          // this device's status word (pinned host memory): 1 = a wait timed out
  uint64_t timeoutTicks;     // s_memrealtime ticks (100 MHz)
  int stepPerSlice, slicePerChunk;  // StepPerSlice / SlicePerChunk of the ring (collectives.h:17-18)
  int nRanks, nParts, team;
};
static_assert(sizeof(ResParams) <= 4000, "resident parameters must fit the kernel-argument segment");

// Launches grid = (ranks on this device) * nParts * team workgroups. Returns hipErrorInvalidValue for
// a datatype/op the kernel does not have.
hipError_t launch_resident(int dt, int devOp, const ResParams& p, int grid, hipStream_t s);

}  // namespace nexr
