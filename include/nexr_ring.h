/*
 * nexr_ring.h — CPU-emulated collectives that drive the reduce-copy ABI (include/nexr.h) from the
 * reference's own schedules: the caller side of the drop-in boundary.
 *
 * It restates, on host threads (one per emulated rank, two for a non-root tree rank, 1 channel):
 *   - runRing for ncclAllReduce (reference src/device/all_reduce.h:12-84), ncclReduceScatter
 *     (reduce_scatter.h:12-52), ncclAllGather (all_gather.h:12-66), ncclReduce (reduce.h:12-50) and
 *     ncclBroadcast (broadcast.h:12-58),
 *   - runTreeSplit for the tree ncclAllReduce (all_reduce.h:150-230) over the reference's tree
 *     topology: an intra-node chain (graph/connect.cc:51-61) whose node heads are joined by the
 *     double binary tree (graph/trees.cc:31-109, connect.cc:95-163),
 *   - Primitives::genericOp slicing and the reduceCopy call sites (src/device/prims_simple.h:190-330,
 *     directSend/directRecvReduceDirectSend/directRecvReduceCopyDirectSend/directRecvCopyDirectSend/
 *     directRecv :897-976),
 *   - the FIFO credit protocol of waitPeer/postPeer (prims_simple.h:111-188): NCCL_STEPS = 8 slots of
 *     buffBytes/8 per connection, head/tail step counters, StepPerSlice = 2, SlicePerChunk = 2
 *     (src/include/collectives.h:17-18),
 *   - or, with protocol = LL, LLGenericOp's one-step-per-call credits and line flags
 *     NCCL_LL_FLAG(step+1) (src/device/prims_ll.h:55-93, :218-283; chunk = stepSize/2,
 *     src/enqueue.cc:1997); with LL128, GenericOp's steps and 64-bit line flags step+1
 *     (src/device/prims_ll128.h:55-85, :294-331; chunk = stepSize*15/16, enqueue.cc:1998),
 *   - the host chunking for ring SIMPLE (src/enqueue.cc:1993-1996: chunkSize = stepSize * 4),
 *   - ncclLaunchOneRank for nRanks == 1 (src/device/onerank.cc:48-83),
 *   - op encoding through nexrHostToDevRedOp (src/enqueue.cc:2185-2278).
 * Every reduceCopy site calls a nexrReduceCopyFn — nexrReduceCopyHost (host memory) or
 * nexrReduceCopy + a wait for the step's completion (device memory) by default.
 *
 * Library: libnexr_ring.so (links libnexr.so). The schedules beyond SURVEY §8's rows — ncclSend /
 * ncclRecv and the device-resident forms — are declared in nexr_extras.h and built only into the
 * opt-in libnexr_extras.so (a superset of libnexr_ring.so; `make EXTRAS=1`).
 */
#ifndef NEXR_RING_H_
#define NEXR_RING_H_

#include "nexr.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Same signature as nexrReduceCopy / nexrReduceCopyHost. */
typedef nexrResult_t (*nexrReduceCopyFn)(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                         size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                                         int nPreOpSrcs, const uint64_t* preOpArgs, int postOp,
                                         nexrStream_t stream);

/* Same signature as nexrReduceCopyLL. */
typedef nexrResult_t (*nexrReduceCopyLLFn)(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                                           const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                                           const uint32_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                           uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                           nexrStream_t stream);

/* Same signature as nexrReduceCopyLL128. */
typedef nexrResult_t (*nexrReduceCopyLL128Fn)(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                                              const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                                              const uint64_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                              uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                              nexrStream_t stream);

typedef enum { nexrRingHostMemory = 0, nexrRingDeviceMemory = 1 } nexrRingMemMode_t;
/* The two protocols the emulated ring restates (the reference's NCCL_PROTO_SIMPLE / NCCL_PROTO_LL).
 * Numbered so that a zero-initialised config selects SIMPLE. */
typedef enum { nexrRingProtoSimple = 0, nexrRingProtoLL = 1, nexrRingProtoLL128 = 2 } nexrRingProto_t;

typedef struct {
  int nRanks;          /* emulated ranks (threads), >= 1 */
  size_t buffBytes;    /* per-connection buffer (NCCL_BUFFSIZE); 0 = the protocol default: 4 MiB
                          SIMPLE, 512 KiB LL, 4,915,200 B LL128 (src/init.cc:618-631) */
  int memMode;         /* nexrRingMemMode_t: where user buffers and FIFOs live */
  nexrReduceCopyFn fn; /* SIMPLE: NULL = nexrReduceCopyHost (host) / nexrReduceCopy (device) */
  int timeoutMs;       /* spin-wait bound per FIFO wait; 0 = 60000 */
  int protocol;        /* nexrRingProto_t (0 = SIMPLE) */
  nexrReduceCopyLLFn llFn; /* LL: NULL = nexrReduceCopyLL (device memory mode only) */
  nexrReduceCopyLL128Fn ll128Fn; /* LL128: NULL = nexrReduceCopyLL128 (device memory mode only) */
  int treeRanksPerNode; /* tree topology: ranks per emulated node (0 = all ranks on one node, i.e. a
                           chain); must divide nRanks. Node heads form the double binary tree */
  int treeIndex;        /* which tree of the double binary tree: 0 (the btree) or 1 (mirror/shift) */
  int nChannels;        /* channels (0 = 1, at most 64): every collective is split over them as the
                           reference's planner splits it (src/enqueue.cc:539-690); each channel has
                           its own links, FIFOs, streams and host threads and they run concurrently.
                           Like the reference's duplicated channels (graph/connect.cc:146-160), the
                           upper half of 2 or more channels uses the other tree of the double binary
                           tree. Send/Recv (extras) always uses channel 0 */
} nexrRingConfig;

typedef struct nexrRingComm* nexrRingComm_t;

/* Device mode: rank r uses HIP device r % deviceCount; FIFOs live on the receiving rank's device. */
NEXR_API nexrResult_t nexrRingCommCreate(nexrRingComm_t* comm, const nexrRingConfig* config);

/* ncclAllReduce over all emulated ranks at once: sendbuffs[r] / recvbuffs[r] are rank r's buffers
 * (host or device memory per memMode; in-place allowed). op is an ncclRedOp_t built-in. */
NEXR_API nexrResult_t nexrRingAllReduce(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op);

/* ncclReduceScatter: rank r's sendbuffs[r] holds nRanks*recvcount elements; recvbuffs[r] receives the
 * reduction of every rank's segment r (recvcount elements). */
NEXR_API nexrResult_t nexrRingReduceScatter(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                            size_t recvcount, int datatype, int op);

/* ncclAllGather: recvbuffs[r] (nRanks*sendcount elements) receives every rank's sendbuff in rank order;
 * in place when sendbuffs[r] == recvbuffs[r] + r*sendcount elements. */
NEXR_API nexrResult_t nexrRingAllGather(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t sendcount, int datatype);

/* ncclReduce: recvbuffs[root] receives the reduction; other ranks' recvbuffs are not touched (may be NULL). */
NEXR_API nexrResult_t nexrRingReduce(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                     size_t count, int datatype, int op, int root);

/* ncclBroadcast: every recvbuffs[r] receives sendbuffs[root] (other ranks' sendbuffs may be NULL). */
NEXR_API nexrResult_t nexrRingBroadcast(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int root);

/* ncclAllReduce with NCCL_ALGO_TREE: runTreeSplit over the topology of config->treeRanksPerNode /
 * treeIndex. The reduce-up and broadcast-down halves of a non-root rank run on two threads, as the
 * reference splits a block's threads between them. */
NEXR_API nexrResult_t nexrTreeAllReduce(nexrRingComm_t comm, const void* const* sendbuffs, void* const* recvbuffs,
                                        size_t count, int datatype, int op);

/* The tree links of `rank` in this communicator's topology: *up (-1 at the root) and down[0..2]
 * (-1 when absent, children packed first as setTreeDown does). */
NEXR_API nexrResult_t nexrTreeTopology(nexrRingComm_t comm, int rank, int* up, int* down);

/* How this communicator's rank threads wait for each device step before posting it (*word = 1: a
 * hipStreamWriteValue32 completion word the thread spins on; 0: hipStreamSynchronize). The word is
 * the default only when every rank runs on the same GPU; when the ranks span GPUs (thread ranks on
 * several devices, or process ranks whose published GPUs differ) the default is the
 * synchronisation. NEXR_STEP_WAIT=word / sync, read once per process, forces either. */
NEXR_API nexrResult_t nexrRingCommGetStepWait(nexrRingComm_t comm, int* word);

/* How the last thread-rank ring collective on this communicator ran its LL steps. *queued = 2: runs
 * on the device (nexrReduceCopyLLSteps), up to 96 steps per launch, the peers' data found by the
 * kernel's flag poll (prims_ll.h:38-93) and the slot credits by its poll of the receivers' head words in
 * device memory (waitSend / postRecv, :55-83), no host wait until the collective's end (the default
 * where 1 is possible and the communicator uses the library's own LL kernels; NEXR_LL_RUN=0 falls back
 * to 1). 1: queued, each step's kernel on the rank's stream with no host wait after it, the slots a
 * step read released once a completion ticket behind it lands (one per NEXR_LL_TICKET_EVERY steps,
 * default 4). 0: host-sequenced (SIMPLE, LL128, ranks on several GPUs, host memory, NEXR_LL_ASYNC=0,
 * or more rank streams on a GPU than it has hardware queues beside the default stream's). */
NEXR_API nexrResult_t nexrRingCommGetQueued(nexrRingComm_t comm, int* queued);

NEXR_API nexrResult_t nexrRingCommDestroy(nexrRingComm_t comm);

/*
 * Process ranks over peer memory (the §8(f) xGMI ring step): one process per GPU, each process one
 * rank of the same ring schedule. Like the reference's P2P transport in write mode
 * (src/transport/p2p.cc:231-240, :299, :402, :514-515, :542-543): every rank allocates the FIFO it
 * receives into, exports it with hipIpcGetMemHandle, and maps the next rank's FIFO with
 * hipIpcOpenMemHandle; its reduce-copy kernels write straight into that peer FIFO (over xGMI when
 * the ranks drive different GPUs). Step counters and the rendezvous live in a POSIX shared-memory
 * segment `shmName` (single node): every rank passes the same fresh name ("/name", no other '/');
 * the last rank to destroy its communicator unlinks it. Create blocks until all nRanks joined
 * (bounded by timeoutMs). Every rank must then issue the same sequence of nexrPeerRingAllReduce
 * calls (same count, datatype, op). Buffers are device memory on `device`. Destroy with
 * nexrRingCommDestroy.
 */
typedef struct {
  int nRanks;
  int rank;
  int device;          /* HIP device of this rank's buffers and kernels */
  size_t buffBytes;    /* 0 = the protocol default (as nexrRingConfig) */
  int protocol;        /* nexrRingProto_t */
  int timeoutMs;       /* rendezvous and per-wait bound; 0 = 60000 */
  const char* shmName; /* shared by all ranks of this communicator */
} nexrPeerRingConfig;

NEXR_API nexrResult_t nexrPeerRingCommCreate(nexrRingComm_t* comm, const nexrPeerRingConfig* config);

/* ncclAllReduce for this process's rank (sendbuff/recvbuff on config->device; in-place allowed). */
NEXR_API nexrResult_t nexrPeerRingAllReduce(nexrRingComm_t comm, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int op);

/* The other ring collectives for this process's rank, arguments as in the thread-rank versions. */
NEXR_API nexrResult_t nexrPeerRingReduceScatter(nexrRingComm_t comm, const void* sendbuff, void* recvbuff,
                                                size_t recvcount, int datatype, int op);
NEXR_API nexrResult_t nexrPeerRingAllGather(nexrRingComm_t comm, const void* sendbuff, void* recvbuff,
                                            size_t sendcount, int datatype);
NEXR_API nexrResult_t nexrPeerRingReduce(nexrRingComm_t comm, const void* sendbuff, void* recvbuff, size_t count,
                                         int datatype, int op, int root);
NEXR_API nexrResult_t nexrPeerRingBroadcast(nexrRingComm_t comm, const void* sendbuff, void* recvbuff, size_t count,
                                            int datatype, int root);

#ifdef __cplusplus
}
#endif

#endif /* NEXR_RING_H_ */
