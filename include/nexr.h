/*
 * nexr.h — C ABI of the MI355X-native reduce-copy primitive.
 *
 * This is the drop-in boundary for the one hot path of MJChku/nex-nccl this project rebuilds:
 * the element-wise K-source / M-destination reduce-copy that every collective's payload goes
 * through (reference: src/device/common_kernel.h:269-349 `reduceCopy`, inner loop
 * `reduceCopyPacks` :32-267, element arithmetic src/device/reduce_kernel.h:427-592).
 *
 * Plain C: pointers, sizes and integer enums only. Every enum value is numerically identical to
 * the reference so a caller can pass its own ncclDataType_t / ncclDevRedOp_t / ncclResult_t
 * values straight through.
 *
 * Ownership and ordering (reference src/enqueue.cc:1543-1640, src/device/onerank.cc:48-83):
 *   - the caller owns every buffer; nothing is allocated or freed inside a hot call;
 *   - device calls are stream-ordered and asynchronous on the given HIP stream (NULL = the
 *     default stream of the current device); they never synchronise the host;
 *   - calls are safe concurrently on different devices / streams (no global mutable state apart
 *     from the process-wide reduction semantics below, set before the first call: tuning knobs are
 *     read from the environment once; host staging resources are pooled per device);
 *   - errors are returned, never aborted on.
 */
#ifndef NEXR_H_
#define NEXR_H_

#include <stddef.h>
#include <stdint.h>
#ifndef __cplusplus
#include <stdbool.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define NEXR_API __attribute__((visibility("default")))

#define NEXR_VERSION_MAJOR 0
#define NEXR_VERSION_MINOR 3
#define NEXR_VERSION_PATCH 0

/* Maximum fan-in / fan-out of one call: srcs[]/dsts[] hold NCCL_MAX_ARITY+1 = 8 entries
 * (reference src/device/common.h:101-102, src/include/device.h:816,:842-846). */
#define NEXR_MAX_SRCS 8
#define NEXR_MAX_DSTS 8

/* Result codes — identical to ncclResult_t (reference src/nccl.h.in:40-48). */
typedef enum {
  nexrSuccess = 0,
  nexrUnhandledCudaError = 1, /* any hipError_t from the runtime */
  nexrSystemError = 2,
  nexrInternalError = 3,
  nexrInvalidArgument = 4,    /* bad K/M/dtype/op/null pointer/unsupported combination */
  nexrInvalidUsage = 5,
  nexrRemoteError = 6,
  nexrInProgress = 7,
  nexrNumResults = 8
} nexrResult_t;

/* Data types — identical to ncclDataType_t (reference src/nccl.h.in:278-290). */
typedef enum {
  nexrInt8 = 0, nexrChar = 0,
  nexrUint8 = 1,
  nexrInt32 = 2, nexrInt = 2,
  nexrUint32 = 3,
  nexrInt64 = 4,
  nexrUint64 = 5,
  nexrFloat16 = 6, nexrHalf = 6,
  nexrFloat32 = 7, nexrFloat = 7,
  nexrFloat64 = 8, nexrDouble = 8,
  nexrBfloat16 = 9,
  nexrFloat8e4m3 = 10, /* declared for enum parity; the fork never compiles its fp8 path
                          (reduce_kernel.h:17 guard), so calls return nexrInvalidArgument */
  nexrFloat8e5m2 = 11,
  nexrNumTypes = 12
} nexrDataType_t;

/* User-level reduction ops — identical to ncclRedOp_t (reference src/nccl.h.in:259-270). */
typedef enum { nexrSum = 0, nexrProd = 1, nexrMax = 2, nexrMin = 3, nexrAvg = 4, nexrNumOps = 5 } nexrRedOp_t;

/* Device reduction ops — identical to ncclDevRedOp_t (reference src/include/device.h:683-687). */
typedef enum {
  nexrDevSum = 0,
  nexrDevProd = 1,
  nexrDevMinMax = 2,     /* redOpArg bit 0: 0 = min, 1 = max (reduce_kernel.h:64) */
  nexrDevPreMulSum = 3,  /* preOp: x * scalar (scalar = raw bits of T in preOpArgs[s]) */
  nexrDevSumPostDiv = 4, /* integer types only; redOpArg = divisor<<1 | isSigned */
  nexrNumDevRedOps = 5
} nexrDevRedOp_t;

/* Byte-exact mirror of struct ncclDevRedOpFull (reference src/include/device.h:688-693):
 * two 4-byte enums at offsets 0 and 4, a one-byte bool at offset 8 (bytes 9-15 are padding the
 * library never reads), the 64-bit scalar at offset 16; sizeof == 24. tests/test_abi.py checks the
 * layout against a C restatement of the reference struct. */
typedef struct {
  int op;               /* nexrDevRedOp_t (ncclDevRedOp_t, an int-sized enum) */
  int proxyOp;          /* nexrRedOp_t the user asked for */
  bool scalarArgIsPtr;  /* scalarArg holds a device pointer to the scalar (onerank.cc:32-42) */
  uint64_t scalarArg;
} nexrDevRedOpFull;

typedef void* nexrStream_t; /* a hipStream_t; NULL = default stream */

/*
 * nexrReduceCopy — replaces the device primitive
 *   reduceCopy<Unroll,RedFn,T,0,MinSrcs,MaxSrcs,0,MinDsts,MaxDsts,PreOpSrcs>(
 *       thread, nThreads, redArg, preOpArgs, postOp, nSrcs, srcPtrs, nDsts, dstPtrs, nElts)
 * (reference src/device/common_kernel.h:331-349), called by genericOp at
 * src/device/prims_simple.h:264,:272,:282,:290 and by oneRankReduce at src/device/onerank.cc:43.
 *
 * For every element i in [0, nElts):
 *   acc = srcs[0][i]              (then acc = acc * preOpArgs[0]   if 0 < nPreOpSrcs, PreMulSum)
 *   for s in 1..nSrcs-1:
 *     v = srcs[s][i]              (then v   = v   * preOpArgs[s]   if s < nPreOpSrcs, PreMulSum)
 *     acc = reduce(acc, v)        (acc is the FIRST operand: reduce_kernel.h:152-168)
 *   if postOp: acc = acc / divisor                                  (SumPostDiv)
 *   dsts[d][i] = acc for every d
 * with the per-type scalar arithmetic of reduce_kernel.h:238-539 (real arithmetic, i.e. the
 * fork's SKIP_COMP at reduce_kernel.h:432 removed; Min/Max compared at the signedness of
 * `datatype`). Rounding to T after every step; integer sum/prod wrap modulo 2^bits.
 *
 * Device pointers; any alignment; dsts may alias srcs[0] exactly (in-place). nElts == 0 or
 * nDsts == 0 is a no-op (common_kernel.h:288-289). 1 <= nSrcs <= 8, 0 <= nDsts <= 8,
 * 0 <= nPreOpSrcs <= nSrcs, preOpArgs may be NULL when nPreOpSrcs == 0.
 */
NEXR_API nexrResult_t nexrReduceCopy(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                     size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                                     int nPreOpSrcs, const uint64_t* preOpArgs, int postOp,
                                     nexrStream_t stream);

/*
 * nexrReduceCopyBatch — many independent reduce-copies of one (datatype, devRedOp) in as few
 * launches as possible: the analogue of a kernel launch carrying a batch of works in its 4 KiB
 * argument block (reference src/include/device.h:1074-1098 ncclDevKernelArgs4K,
 * src/device/common.h:165-200 loadWorkBatchToShmem, :424-445 the per-block work loop). Each work
 * has exactly the semantics of one nexrReduceCopy call with its own fields. Works with the same
 * nSrcs share a launch (at most NEXR_MAX_BATCH_WORKS per launch); each work gets workgroups in
 * proportion to its size. Works run concurrently in no defined order, so no work's dsts may overlap
 * another work's srcs or dsts (in-place within one work is allowed). Every work is validated
 * before anything is launched: on an argument error nothing runs. Works with nElts == 0 or
 * nDsts == 0 are skipped. Small messages are launch-bound (~4 us per nexrReduceCopy call on
 * MI355X); a batch pays that once per launch.
 */
#define NEXR_MAX_BATCH_WORKS 14
typedef struct {
  int nSrcs;
  int nDsts;
  const void* srcs[NEXR_MAX_SRCS];
  void* dsts[NEXR_MAX_DSTS];
  size_t nElts;
  uint64_t redOpArg;
  int nPreOpSrcs;
  int postOp;
  uint64_t preOpArgs[NEXR_MAX_SRCS];
} nexrReduceCopyWork;

NEXR_API nexrResult_t nexrReduceCopyBatch(const nexrReduceCopyWork* works, int nWorks, int datatype, int devRedOp,
                                          nexrStream_t stream);

/*
 * nexrReduceCopyMultiDevice — independent reduce-copies on several GPUs of one node from one host
 * call: the independent-chunk sharding of SURVEY §8(e) (config C5) as a native host driver, with no
 * collective and no peer access. Work i runs on HIP device devices[i] (its buffers live there) on a
 * host thread of its own: hipSetDevice, a non-blocking stream of its own (checked out of a
 * process-wide per-device pool and handed back drained), a start barrier shared by all works, then `reps` reduce-copies (each exactly one nexrReduceCopy of work i) and
 * hipStreamSynchronize. Every work and device ordinal is validated before any thread starts; the
 * first error of any work is returned. When `seconds` is non-null it receives the wall time from the
 * barrier's release to the last device's completion. The caller's current device is unchanged. Works
 * must not overlap one another (in-place within one work is allowed). At most
 * NEXR_MAX_MULTI_DEVICE_WORKS works; several may name the same device.
 */
#define NEXR_MAX_MULTI_DEVICE_WORKS 64
NEXR_API nexrResult_t nexrReduceCopyMultiDevice(const nexrReduceCopyWork* works, const int* devices, int nWorks,
                                                int datatype, int devRedOp, int reps, double* seconds);

/*
 * nexrReduceCopyMultiDeviceSets — nexrReduceCopyMultiDevice with nSets rotating works per thread:
 * works[i * nSets + s] (s < nSets) all run on devices[i], and launch k (k < reps) of thread i is
 * work i * nSets + k mod nSets. With nSets buffer sets per GPU, consecutive launches never re-read
 * the previous launch's cache-resident bytes (the N = 1 bench's rotation, applied to C5). nSets = 1
 * is nexrReduceCopyMultiDevice. Validation, threads, streams, barrier and timing as above.
 */
#define NEXR_MAX_MULTI_DEVICE_SETS 8
NEXR_API nexrResult_t nexrReduceCopyMultiDeviceSets(const nexrReduceCopyWork* works, const int* devices, int nWorks,
                                                    int nSets, int datatype, int devRedOp, int reps, double* seconds);

/*
 * nexrReduceCopyHost — the same reduce-copy for buffers in HOST memory (the emulated
 * transport's staging FIFOs, reference src/include/device.h:753-771): copies the K inputs
 * host->device, runs nexrReduceCopy, copies the M outputs device->host, and synchronises the
 * stream before returning. Device scratch is a staging ring checked out of a process-wide,
 * per-device pool for the duration of the call and handed back at its end (grown on demand; the
 * only call that may allocate), so callers on short-lived threads reuse the same rings. When every buffer is pinned host memory (hipHostMalloc /
 * hipHostRegister / torch pin_memory) the kernel reads and writes it in place over PCIe (zero-copy,
 * both directions concurrently; NEXR_HOST_ZERO_COPY=0 disables). Otherwise the call stages through
 * device memory in chunks (NEXR_HOST_CHUNK_BYTES, default 8 MiB per buffer): chunk c is copied in
 * and reduced while chunk c-1 is copied out on a second stream.
 */
NEXR_API nexrResult_t nexrReduceCopyHost(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                         size_t nElts, int datatype, int devRedOp, uint64_t redOpArg,
                                         int nPreOpSrcs, const uint64_t* preOpArgs, int postOp,
                                         nexrStream_t stream);

/*
 * Host-memory registration — replaces ncclCommRegister / ncclCommDeregister (reference
 * src/nccl.h.in:243-246, src/register/register.cc:128-170) and ncclMemAlloc / ncclMemFree
 * (src/nccl.h.in:130-133, src/allocator.cc) for the fork's setting, where NEX "device memory" and
 * the transport's staging FIFOs are host memory.
 *   nexrHostRegister    page-locks and device-maps [buff, buff + size) (hipHostRegister, mapped +
 *                       portable) and records it in a process-wide cache sorted by address, like the
 *                       reference's regCache (register.cc:40-60). A range inside an entry already here
 *                       (registered, or from nexrHostMemAlloc) shares that entry (one more reference);
 *                       a range that partly overlaps one returns nexrInvalidUsage. Disjoint ranges that
 *                       share a page are separate entries (the runtime maps each; if it refused one,
 *                       nexrInvalidUsage). *handle is an opaque id that is never reused.
 *   nexrHostDeregister  drops one reference; the last one unregisters the range (NULL: no-op). A
 *                       handle with no reference left, or never issued, returns nexrInvalidUsage.
 *   nexrHostMemAlloc    pinned, device-mapped host memory (hipHostMalloc), recorded in the same cache.
 *   nexrHostMemFree     frees memory from nexrHostMemAlloc (NULL: no-op); nexrInvalidUsage while
 *                       registrations inside it remain (deregister them first).
 * nexrReduceCopyHost looks every buffer up in this cache first: a buffer wholly inside an entry is
 * read and written in place over PCIe with no runtime query. Other pinned memory (registered by the
 * caller directly) is still found with hipPointerGetAttributes on every call. Do not free or
 * unregister a range behind the library's back while it is registered here.
 */
NEXR_API nexrResult_t nexrHostRegister(void* buff, size_t size, void** handle);
NEXR_API nexrResult_t nexrHostDeregister(void* handle);
NEXR_API nexrResult_t nexrHostMemAlloc(void** ptr, size_t size);
NEXR_API nexrResult_t nexrHostMemFree(void* ptr);

/*
 * nexrGetHostPathStats — diagnostics: where nexrReduceCopyHost calls have spent host time since the
 * last reset (process-wide, every thread). calls / zeroCopyCalls: calls, and those whose every buffer
 * was pinned (one kernel over PCIe, no copies); registeredHits / pointerQueries: buffers classified
 * from the registration cache / by a runtime pointer query; classifyNs: classifying the buffers;
 * copyNs: host staging copies; launchNs: queuing kernels (and, on the runtime-copy pipeline, its
 * asynchronous copies); waitNs: waiting for the stream or a slot's kernel (kernel run time included).
 * reset != 0 zeroes the counters after reading them.
 */
typedef struct {
  uint64_t calls, zeroCopyCalls, registeredHits, pointerQueries;
  uint64_t classifyNs, copyNs, launchNs, waitNs;
} nexrHostPathStats;
NEXR_API nexrResult_t nexrGetHostPathStats(nexrHostPathStats* stats, int reset);

/*
 * nexrHostToDevRedOp — replaces hostToDevRedOp (reference src/enqueue.cc:2185-2278) for the
 * built-in ops: encodes (op, datatype, nRanks) into the device op and its 64-bit argument
 * (Min/Max xormask, Avg: integer nRanks<<1|signed or float 1/nRanks bit pattern).
 */
NEXR_API nexrResult_t nexrHostToDevRedOp(nexrDevRedOpFull* opFull, int op, int datatype, int nRanks);

/*
 * nexrLaunchOneRank — replaces ncclLaunchOneRank (reference src/device/onerank.cc:48-83,
 * declared src/include/device.h:1171): the nRanks == 1 all-reduce. Non-PreMulSum ops are a
 * stream-ordered copy (skipped when dst == src); PreMulSum runs a K=1 reduce-copy with the
 * scalar pre-op and postOp (onerank.cc:14-45), the scalar loaded from device memory when
 * redOp.scalarArgIsPtr.
 */
NEXR_API nexrResult_t nexrLaunchOneRank(void* dst, const void* src, size_t nElts, nexrDevRedOpFull redOp,
                                        int datatype, nexrStream_t stream);

/* One LL-protocol FIFO line — identical layout to union ncclLLFifoLine (reference
 * src/include/device.h:695-708): 8 data bytes split in two 32-bit halves, each followed by the
 * step flag; a line is valid when flag1 == flag2 == the expected flag. */
typedef struct {
  uint32_t data1, flag1, data2, flag2;
} nexrLLFifoLine;

/*
 * nexrReduceCopyLL — one step of the LL protocol's reduce-copy, LLGenericOp<RECV, SEND, SrcBuf,
 * DstBuf> (reference src/device/prims_ll.h:218-283), with the step's FIFO slots resolved by the
 * caller: recvLines[i] / sendLines[i] point at the peer's slot (recvPtr(i)/sendPtr(i), :38-41) and
 * recvFlags[i] / sendFlags[i] are NCCL_LL_FLAG(step+1) (:42-43). Per 8-byte data line:
 *   d = src (x redOpArg when srcIsInput and the op is PreMulSum: applyPreOp(redOp, ·))
 *   d = nRecv ? (src ? op(peer0, d) : peer0) : d;  d = op(peer_i, d) for i >= 1   (peer FIRST)
 *   d = postOp ? d / divisor : d                                                  (SumPostDiv)
 *   sendLines[i] = {lo32(d), flag_i, hi32(d), flag_i};  dst = d  (valid elements only)
 * Recv lines are polled until both flags match (system-scope loads), for at most timeoutUs
 * (0 = 1 s); a line that never becomes valid sets *status = 1 (status: optional device/host-mapped
 * word) and its outputs are left unwritten — the kernel never hangs. A poll that keeps failing also
 * reads *status every 64 tries and gives up when it is non-zero (another step timed out, or the
 * caller wrote it to abort: checkAbort, primitives.h:142-156). src/dst are any-aligned device
 * pointers (nullable: at least one input and one output); line buffers must be 16-B aligned.
 */
NEXR_API nexrResult_t nexrReduceCopyLL(const void* src, int srcIsInput, int nRecv, const void* const* recvLines,
                                       const uint32_t* recvFlags, void* dst, int nSend, void* const* sendLines,
                                       const uint32_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                       uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                       nexrStream_t stream);

/*
 * nexrReduceCopyLL128 — one step of the LL128 protocol's reduce-copy, GenericOp +
 * recvReduceSendCopy (reference src/device/prims_ll128.h:184-331), the step's slots resolved by the
 * caller (recvPtr(i)/sendPtr(i), flags = step+1 as 64-bit words, :45-50). Wire format: 2 KiB slices
 * of sixteen 128-B lines carrying 1920 data bytes; word 15 of every line is the flag; user 16-B
 * chunk ix = g*32 - 4*(g/2) + w - (g%2)*(w/8) of a slice sits at wire words 64g + 2w (+1) for
 * w % 8 != 7, and the w % 8 == 7 chunks are split over words 64g + 2w of g and g+1 (loadRegsBegin/
 * loadRegsFinish/storeRegs :86-174) — byte-identical to the reference's warp-32 layout. Arithmetic,
 * peer-first operand order, status/timeout and pointer rules as nexrReduceCopyLL; wire buffers must
 * be 16-B aligned and hold ceil(nElts*size/1920) slices.
 */
NEXR_API nexrResult_t nexrReduceCopyLL128(const void* src, int srcIsInput, int nRecv, const void* const* recvWire,
                                          const uint64_t* recvFlags, void* dst, int nSend, void* const* sendWire,
                                          const uint64_t* sendFlags, size_t nElts, int datatype, int devRedOp,
                                          uint64_t redOpArg, int postOp, uint32_t* status, uint32_t timeoutUs,
                                          nexrStream_t stream);

/*
 * nexrReduceCopyLLSteps — a run of LL steps of ONE Primitives (one rank's connections of one
 * channel) in as few launches as the steps allow, with the protocol's credits on the device: the
 * LLGenericOp calls of a schedule (reference src/device/prims_ll.h:249-318) together with their
 * waitSend / postRecv (:55-83), which the single-step nexrReduceCopyLL leaves to its caller.
 *
 * Every step of the run uses the same connections: nRecv receive FIFOs (steps with recv = 1 read all
 * of them, as LLGenericOp<RECV=1> does) and nSend send FIFOs, each nSlots (NCCL_STEPS) slots of
 * slotBytes. recvStep[i] / sendStep[i] are the connection's step counters at the first step of the
 * run (the flags follow: NCCL_LL_FLAG(step + 1), :42-43); each recv / send step advances them by one.
 * Credits live in device memory, one 8-byte word per wave at a 16-B stride, NEXR_LL_HEAD_BYTES per
 * connection (zeroed when the connection is made): the receiver stores its step count into its
 * connection's head words once it has read a step (postRecv), and a sender writes a slot only when
 * the head words of the connection it sends into show the step NCCL_STEPS earlier read (waitSend).
 * Both ends of a connection must therefore run their steps through this call (one wave of the
 * receiver's launch frees exactly the lines one wave of the sender's launch writes: both derive the
 * same grid from slotBytes). At the start of each launch the receiver stores recvStep into its
 * head words, so a connection may switch to this call after steps run by nexrReduceCopyLL once those
 * have completed.
 *
 * Element arithmetic, operand order, postOp, status and timeout as nexrReduceCopyLL, per step; user
 * offsets in elements of `datatype` (srcBuf / dstBuf: 0 input, 1 output, -1 none). The steps run as if
 * one at a time in order: where a step reads or writes user bytes an earlier step of the same launch
 * wrote or read at a different element position, the library starts a new launch. A step whose line
 * never arrives (or whose credit never comes) within timeoutUs sets *status = 1 and ends its
 * wave's run, and a non-zero *status ends the others' polls early (as nexrReduceCopyLL); the launch
 * never hangs. Launches are stream-ordered; the call returns after
 * queueing them. The runs on both ends of a connection must be able to run at once: streams on
 * hardware queues of their own (HIP shares its GPU_MAX_HW_QUEUES queues among streams and runs one
 * queue's kernels one after the other; a stream made by hipExtStreamCreateWithCUMask has its own), and
 * grids that fit the GPU together (one workgroup of 256 lanes per line tile of a slot, at most 64).
 */
#define NEXR_LL_STEPS_MAX_PEERS 3
#define NEXR_LL_HEAD_BYTES 4096
typedef struct {
  int64_t srcIx, dstIx; /* element offsets into the user buffer srcBuf / dstBuf */
  uint32_t nElts;       /* elements this step moves (0: the step only advances the counters) */
  uint8_t recv, send;   /* RECV / SEND of LLGenericOp */
  int8_t srcBuf, dstBuf;/* 0 input, 1 output, -1 none */
  uint8_t postOp;
  uint8_t pad[7];
} nexrLLStep;           /* 32 bytes */
typedef struct {
  const void* input;
  void* output;
  int nRecv, nSend;
  const void* recvFifo[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t* recvHead[NEXR_LL_STEPS_MAX_PEERS];       /* this rank's receive connections' head words */
  uint64_t recvStep[NEXR_LL_STEPS_MAX_PEERS];
  void* sendFifo[NEXR_LL_STEPS_MAX_PEERS];
  const uint64_t* sendHead[NEXR_LL_STEPS_MAX_PEERS]; /* the receivers' head words of the send connections */
  uint64_t sendStep[NEXR_LL_STEPS_MAX_PEERS];
  uint64_t slotBytes; /* bytes per FIFO slot, every connection (16-B multiple) */
  uint32_t nSlots;    /* NCCL_STEPS */
  uint32_t pad;
} nexrLLConnSet;
NEXR_API nexrResult_t nexrReduceCopyLLSteps(const nexrLLConnSet* conns, const nexrLLStep* steps, int nSteps,
                                            int datatype, int devRedOp, uint64_t redOpArg, uint32_t* status,
                                            uint32_t timeoutUs, nexrStream_t stream);

/*
 * Reduction semantics — which nex-nccl the library reproduces bit for bit. Process-wide, like an
 * NCCL parameter: the initial value comes from NEXR_SEMANTICS ("nccl", "fork" or "shipped"; default
 * "nccl"); nexrSetSemantics changes it for every later call (set it before the first call that
 * matters; calls already queued keep theirs). It applies to nexrReduceCopy, nexrReduceCopyBatch,
 * nexrReduceCopyMultiDevice, nexrReduceCopyHost, nexrLaunchOneRank, nexrReduceCopyLL and
 * nexrReduceCopyLL128, and so to every emulated collective built on them (include/nexr_ring.h).
 *   nexrSemanticsNccl     real arithmetic; Min/Max compared at the signedness of `datatype`
 *                         (upstream NCCL). The default.
 *   nexrSemanticsFork     the fork with SKIP_COMP removed: real arithmetic under the fork's own kernel
 *                         dispatch, where signed-integer Min/Max run on the unsigned kernel
 *                         (equivalent_primary, src/device/generate.py:128-136) whose FuncMinMax ignores
 *                         the sign xormask (reduce_kernel.h:59-65), so they compare as unsigned.
 *   nexrSemanticsShipped  the fork exactly as shipped: `#define SKIP_COMP` (reduce_kernel.h:432) makes
 *                         every ncclReduceScalar return its FIRST operand and the PreMulSum pre-op and
 *                         SumPostDiv post-op return their input (:434-539). reduceCopy then copies
 *                         srcs[0]'s bits to every destination; an LL / LL128 step (peer first) forwards
 *                         the last peer's data, or src when it has no peer.
 * Argument validation is the same in every mode.
 */
typedef enum {
  nexrSemanticsNccl = 0,
  nexrSemanticsFork = 1,
  nexrSemanticsShipped = 2,
  nexrNumSemantics = 3
} nexrSemantics_t;
NEXR_API nexrResult_t nexrSetSemantics(int semantics);
NEXR_API nexrResult_t nexrGetSemantics(int* semantics);

/*
 * nexrQueryLaunch — diagnostics: the launch nexrReduceCopy would make for these pointers and this
 * size (no GPU work, no device needed; the same validation as nexrReduceCopy with devRedOp = Sum). A
 * one-source call runs as a byte copy (the uint8 kernel), so its headElts and bodyPacks count bytes.
 * [0, headElts) and the tail are edge elements (headElts brings dsts[0] to a 128-B boundary when its
 * offset is a whole number of elements) and bodyPacks 16-B packs form the body, pack i being the 16
 * bytes at offset 16 i of every buffer. `unaligned` is 1 when the pointers share no 16-B phase: the
 * body then moves the misaligned buffers with unaligned 16-B accesses (ABI 0.2 dropped round 1's
 * always-zero `generic` field: `unaligned` now sits at offset 16). grid * block never exceeds 2^32 - 1 work items
 * (HIP's launch limit); larger calls grid-stride. policy: 0 plain, 1 non-temporal loads, 3
 * non-temporal loads and stores.
 */
typedef struct {
  uint32_t grid;
  int block;
  int packsPerLane;
  int policy;
  int unaligned;
  uint64_t headElts;
  uint64_t bodyPacks;
} nexrLaunchInfo;
NEXR_API nexrResult_t nexrQueryLaunch(int nSrcs, const void* const* srcs, int nDsts, void* const* dsts,
                                      size_t nElts, int datatype, nexrLaunchInfo* info);

/* Diagnostics: how many streams nexrReduceCopyMultiDevice and how many staging rings
 * nexrReduceCopyHost have created in this process so far (device rings of the chunk pipeline plus
 * pinned rings of the large-call copy-team path; all pooled and reused, so the counts stop growing
 * once the pools are warm). Either pointer may be NULL. */
NEXR_API nexrResult_t nexrGetPoolStats(uint64_t* multiDeviceStreams, uint64_t* hostStagingRings);

/* Bytes per element of a datatype (reference ncclTypeSize), 0 if unknown. */
NEXR_API size_t nexrTypeSize(int datatype);

/* Human-readable string for a result code (reference ncclGetErrorString). */
NEXR_API const char* nexrGetErrorString(nexrResult_t result);

/* Packed version: major*10000 + minor*100 + patch. */
NEXR_API int nexrGetVersion(void);

/* Last HIP error recorded by this thread inside the library (0 if none) — diagnostics only. */
NEXR_API int nexrGetLastHipError(void);

#ifdef __cplusplus
}
#endif

#endif /* NEXR_H_ */
