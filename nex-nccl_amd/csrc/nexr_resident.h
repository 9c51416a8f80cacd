// nexr_resident.h — the device-resident ring collectives (nexr_resident.hip), shared with its host
// side in nexr_resident_host.cpp. Part of the opt-in extras library (libnexr_extras.so); not installed,
// not part of the ABI (include/nexr_extras.h declares the entry points, nexr*Resident).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace nexr {

constexpr int kResMaxRanks = 16;   // ranks one communicator may have for the resident path
constexpr int kResMaxParts = 64;   // channel parts (MAXCHANNELS)
constexpr int kResMaxTeam = 128;   // workgroups per (rank, channel)
constexpr int kResCtrBytes = 256;  // one (channel, rank, team member) record: tail line + head line
constexpr int kResHeadOff = 128;   // byte offset of the head word in a record
static_assert((size_t)kResMaxTeam * kResCtrBytes == 128 * 256, "process ranks reserve this much behind each FIFO");

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

enum { kResAllReduce = 0, kResReduceScatter = 1, kResAllGather = 2, kResReduce = 3, kResBroadcast = 4,
       kResTreeAllReduce = 5 };

// One (channel, rank) of the tree all-reduce (runTreeSplit), static for the communicator. Connection
// up[r] carries r -> parent(r) (its FIFO and records on the parent's GPU), down[r] parent(r) -> r (on
// r's GPU); the record pointers are member 0's, member g's at + g * kResCtrBytes.
struct ResTreeConn {
  char* upRecvFifo[3];  // up[child i]: the children's partial results arrive here
  char* upRecvCtr[3];
  char* upSendFifo;     // up[r], on the parent (unused at the root)
  char* upSendCtr;
  char* downRecvFifo;   // down[r] (unused at the root)
  char* downRecvCtr;
  char* downSendFifo[3];  // down[child i], on the child
  char* downSendCtr[3];
  int nDown;            // children, packed first (setTreeDown)
  int root;
};

struct ResParams {
  const ResConn* conns;  // [ch * nRanks + r], in the launching device's memory
  const ResTreeConn* tree;  // [ch * nRanks + r], kResTreeAllReduce only
  const char* input[kResMaxRanks];
  char* output[kResMaxRanks];
  int64_t partOffset[kResMaxParts], partCount[kResMaxParts];
  int partChannel[kResMaxParts];
  int rankOf[kResMaxRanks];  // workgroup group li = blockIdx.x / (nParts * team) runs rank rankOf[li]
  int64_t chunkCount;        // elements per ring chunk (calcCollChunking)
  int64_t stepElems;         // elements per FIFO step
  uint64_t stepBytes;
  uint64_t redArg;           // op argument; also the pre-op scalar (Primitives' redOpArgs[0])
  uint32_t* status;          // this device's status word (pinned host memory): 1 = a wait timed out,
                             // 2 = the host aborted the call (another GPU's launch failed)
  uint64_t timeoutTicks;     // s_memrealtime ticks (100 MHz)
  int64_t count;             // ReduceScatter recvcount / AllGather sendcount (rank segment stride)
  int stepPerSlice, slicePerChunk;  // ProtoSimple<SlicePerChunk, StepPerSlice> (collectives.h:16-25)
  int coll, root;            // kRes*; root of Reduce / Broadcast
  int nRanks, nParts, team;
};
static_assert(sizeof(ResParams) <= 4000, "resident parameters must fit the kernel-argument segment");

// Launches grid = (ranks on this device) * nParts * team workgroups (x 2 roles for the tree); one entry point per datatype,
// defined in the object compiled with -DNEXR_DT=<dt>. hipErrorInvalidValue for an op the datatype
// does not have.
#define NEXR_DECLARE_RESIDENT(dt)                                                                \
  hipError_t launch_resident_dt##dt(int devOp, const ResParams& p, int grid, hipStream_t s); \
  hipError_t resident_blocks_per_cu_dt##dt(int devOp, uint64_t redArg, int coll, int* blocks);
NEXR_DECLARE_RESIDENT(0) NEXR_DECLARE_RESIDENT(1) NEXR_DECLARE_RESIDENT(2) NEXR_DECLARE_RESIDENT(3)
NEXR_DECLARE_RESIDENT(4) NEXR_DECLARE_RESIDENT(5) NEXR_DECLARE_RESIDENT(6) NEXR_DECLARE_RESIDENT(7)
NEXR_DECLARE_RESIDENT(8) NEXR_DECLARE_RESIDENT(9)
#undef NEXR_DECLARE_RESIDENT
inline hipError_t launch_resident(int dt, int devOp, const ResParams& p, int grid, hipStream_t s) {
  switch (dt) {
    case 0: return launch_resident_dt0(devOp, p, grid, s);
    case 1: return launch_resident_dt1(devOp, p, grid, s);
    case 2: return launch_resident_dt2(devOp, p, grid, s);
    case 3: return launch_resident_dt3(devOp, p, grid, s);
    case 4: return launch_resident_dt4(devOp, p, grid, s);
    case 5: return launch_resident_dt5(devOp, p, grid, s);
    case 6: return launch_resident_dt6(devOp, p, grid, s);
    case 7: return launch_resident_dt7(devOp, p, grid, s);
    case 8: return launch_resident_dt8(devOp, p, grid, s);
    case 9: return launch_resident_dt9(devOp, p, grid, s);
  }
  return hipErrorInvalidValue;
}
// Workgroups of the (datatype, op) kernel one CU holds at once (hipOccupancyMaxActiveBlocksPerMultiprocessor):
// a device's grid must fit in this times its CUs, since a rank's workgroups wait on each other.
inline hipError_t resident_blocks_per_cu(int dt, int devOp, uint64_t redArg, int coll, int* blocks) {
  switch (dt) {
    case 0: return resident_blocks_per_cu_dt0(devOp, redArg, coll, blocks);
    case 1: return resident_blocks_per_cu_dt1(devOp, redArg, coll, blocks);
    case 2: return resident_blocks_per_cu_dt2(devOp, redArg, coll, blocks);
    case 3: return resident_blocks_per_cu_dt3(devOp, redArg, coll, blocks);
    case 4: return resident_blocks_per_cu_dt4(devOp, redArg, coll, blocks);
    case 5: return resident_blocks_per_cu_dt5(devOp, redArg, coll, blocks);
    case 6: return resident_blocks_per_cu_dt6(devOp, redArg, coll, blocks);
    case 7: return resident_blocks_per_cu_dt7(devOp, redArg, coll, blocks);
    case 8: return resident_blocks_per_cu_dt8(devOp, redArg, coll, blocks);
    case 9: return resident_blocks_per_cu_dt9(devOp, redArg, coll, blocks);
  }
  return hipErrorInvalidValue;
}

}  // namespace nexr
