"""nex-nccl_amd — MI355X-native reduce-copy primitive (host-side mirror of the reference API).

The product is ``libnexr.so`` (C ABI, ``include/nexr.h``) built from ``csrc/`` for gfx950. This
module is the Python view of that boundary, mirroring the reference's operator interface for the
path: the device primitive ``reduceCopy`` (src/device/common_kernel.h:331-349), the one-rank
launcher ``ncclLaunchOneRank`` (src/device/onerank.cc:48-83) and the op encoder
``hostToDevRedOp`` (src/enqueue.cc:2185-2278). Same argument meaning, same integer enums and
result codes; failures raise :class:`NexrError` carrying the ``ncclResult_t``-compatible code.

There is no fallback: if ``libnexr.so`` is missing or fails to load, every call raises.
Import it with ``importlib.import_module("nex-nccl_amd")`` (the directory name has a hyphen).
"""
from __future__ import annotations

import ctypes
import enum
import os
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnexr.so")

MAX_SRCS = 8
MAX_DSTS = 8


class Result(enum.IntEnum):
    """ncclResult_t values (reference src/nccl.h.in:40-48)."""
    Success = 0
    UnhandledCudaError = 1
    SystemError = 2
    InternalError = 3
    InvalidArgument = 4
    InvalidUsage = 5
    RemoteError = 6
    InProgress = 7


class DataType(enum.IntEnum):
    """ncclDataType_t values (reference src/nccl.h.in:278-290)."""
    Int8 = 0
    Uint8 = 1
    Int32 = 2
    Uint32 = 3
    Int64 = 4
    Uint64 = 5
    Float16 = 6
    Float32 = 7
    Float64 = 8
    Bfloat16 = 9
    Float8e4m3 = 10
    Float8e5m2 = 11


class RedOp(enum.IntEnum):
    """ncclRedOp_t built-in values (reference src/nccl.h.in:259-270)."""
    Sum = 0
    Prod = 1
    Max = 2
    Min = 3
    Avg = 4


class DevRedOp(enum.IntEnum):
    """ncclDevRedOp_t values (reference src/include/device.h:683-687)."""
    Sum = 0
    Prod = 1
    MinMax = 2
    PreMulSum = 3
    SumPostDiv = 4


class Semantics(enum.IntEnum):
    """nexrSemantics_t (include/nexr.h): which nex-nccl the library reproduces bit for bit."""
    Nccl = 0     # real arithmetic, min/max at the datatype's signedness (default)
    Fork = 1     # the fork with SKIP_COMP removed: signed min/max on the unsigned kernel (generate.py:128-136)
    Shipped = 2  # the fork as shipped: SKIP_COMP (reduce_kernel.h:432), every reduce returns its first operand


TYPE_SIZE = {DataType.Int8: 1, DataType.Uint8: 1, DataType.Int32: 4, DataType.Uint32: 4,
             DataType.Int64: 8, DataType.Uint64: 8, DataType.Float16: 2, DataType.Float32: 4,
             DataType.Float64: 8, DataType.Bfloat16: 2, DataType.Float8e4m3: 1,
             DataType.Float8e5m2: 1}

# ABI symbols declared in include/nexr.h (checked by tests/test_abi.py)
ABI_SYMBOLS = ("nexrReduceCopy", "nexrReduceCopyBatch", "nexrReduceCopyMultiDevice", "nexrReduceCopyMultiDeviceSets",
               "nexrReduceCopyHost", "nexrHostToDevRedOp", "nexrLaunchOneRank",
               "nexrReduceCopyLL", "nexrReduceCopyLL128", "nexrReduceCopyLLSteps", "nexrQueryLaunch", "nexrGetPoolStats", "nexrTypeSize", "nexrGetErrorString", "nexrGetVersion",
               "nexrGetLastHipError", "nexrSetSemantics", "nexrGetSemantics", "nexrHostRegister", "nexrHostDeregister",
               "nexrHostMemAlloc", "nexrHostMemFree", "nexrGetHostPathStats")


class NexrError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = int(code)
        try:
            name = Result(self.code).name
        except ValueError:
            name = "Unknown"
        super().__init__(f"{what}: nexr result {self.code} ({name})" if what else f"nexr result {self.code} ({name})")


class DevRedOpFull(ctypes.Structure):
    """Byte-exact mirror of struct ncclDevRedOpFull (reference src/include/device.h:688-693): enum op
    at 0, enum proxyOp at 4, bool scalarArgIsPtr at 8 (9-15 padding), uint64 scalarArg at 16."""
    _fields_ = [("op", ctypes.c_int), ("proxyOp", ctypes.c_int), ("scalarArgIsPtr", ctypes.c_bool),
                ("scalarArg", ctypes.c_uint64)]


class LaunchInfo(ctypes.Structure):
    """Mirror of nexrLaunchInfo (include/nexr.h): what nexrQueryLaunch reports."""
    _fields_ = [("grid", ctypes.c_uint32), ("block", ctypes.c_int), ("packsPerLane", ctypes.c_int),
                ("policy", ctypes.c_int), ("unaligned", ctypes.c_int),
                ("headElts", ctypes.c_uint64),
                ("bodyPacks", ctypes.c_uint64)]


class HostPathStats(ctypes.Structure):
    """Mirror of nexrHostPathStats (include/nexr.h): nexrGetHostPathStats' counters."""
    _fields_ = [(f, ctypes.c_uint64) for f in ("calls", "zeroCopyCalls", "registeredHits", "pointerQueries",
                                               "classifyNs", "copyNs", "launchNs", "waitNs")]


MAX_BATCH_WORKS = 14  # NEXR_MAX_BATCH_WORKS


class ReduceCopyWork(ctypes.Structure):
    """Mirror of nexrReduceCopyWork (include/nexr.h): one reduce-copy of a batch."""
    _fields_ = [("nSrcs", ctypes.c_int), ("nDsts", ctypes.c_int), ("srcs", ctypes.c_void_p * 8),
                ("dsts", ctypes.c_void_p * 8), ("nElts", ctypes.c_size_t), ("redOpArg", ctypes.c_uint64),
                ("nPreOpSrcs", ctypes.c_int), ("postOp", ctypes.c_int), ("preOpArgs", ctypes.c_uint64 * 8)]


LL_STEPS_MAX_PEERS = 3  # NEXR_LL_STEPS_MAX_PEERS
LL_HEAD_BYTES = 4096   # NEXR_LL_HEAD_BYTES


class LLStep(ctypes.Structure):
    """Mirror of nexrLLStep (include/nexr.h): one LLGenericOp call of a run (32 bytes)."""
    _fields_ = [("srcIx", ctypes.c_int64), ("dstIx", ctypes.c_int64), ("nElts", ctypes.c_uint32),
                ("recv", ctypes.c_uint8), ("send", ctypes.c_uint8), ("srcBuf", ctypes.c_int8),
                ("dstBuf", ctypes.c_int8), ("postOp", ctypes.c_uint8), ("pad", ctypes.c_uint8 * 7)]


class LLConnSet(ctypes.Structure):
    """Mirror of nexrLLConnSet (include/nexr.h): the connections a run of LL steps uses."""
    _fields_ = [("input", ctypes.c_void_p), ("output", ctypes.c_void_p), ("nRecv", ctypes.c_int),
                ("nSend", ctypes.c_int), ("recvFifo", ctypes.c_void_p * 3), ("recvHead", ctypes.c_void_p * 3),
                ("recvStep", ctypes.c_uint64 * 3), ("sendFifo", ctypes.c_void_p * 3),
                ("sendHead", ctypes.c_void_p * 3), ("sendStep", ctypes.c_uint64 * 3),
                ("slotBytes", ctypes.c_uint64), ("nSlots", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


_lib = None


def hip_runtime() -> ctypes.CDLL:
    """The HIP runtime libnexr runs on (the one libamdhip64 mapped in this process, see lib()), for
    harness calls the ABI does not cover (hipDeviceEnablePeerAccess in tools/xgmi_probe.py)."""
    lib()
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln})
    if len(paths) != 1:
        raise NexrError(Result.InternalError, f"expected one HIP runtime in the process, found {paths}")
    return ctypes.CDLL(paths[0])


def _preload_hip_runtime() -> None:
    """One HIP runtime per process. torch ships its own libamdhip64 (soname libamdhip64.so.7, NEEDED
    by torch as "libamdhip64.so" through its RUNPATH), so loading libnexr first would map
    /opt/rocm's runtime and torch then a second one: torch's streams and allocations would be
    foreign handles to libnexr (hipErrorNoDevice / invalid handle at the first launch). When a
    runtime is already mapped (torch imported, or any other), libnexr's NEEDED libamdhip64.so.7
    resolves to it. Otherwise, if torch is installed, its runtime file is mapped here by path,
    without importing torch: libnexr then binds to it through the soname, and a later `import
    torch` finds that same file already mapped. Without torch, /opt/rocm's runtime serves."""
    with open("/proc/self/maps") as f:
        if any("libamdhip64" in ln for ln in f):
            return
    import importlib.util
    try:
        spec = importlib.util.find_spec("torch")
    except (ImportError, ValueError):
        spec = None
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        cand = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            return


def lib() -> ctypes.CDLL:
    """Load libnexr.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NexrError(Result.InternalError,
                        f"{LIB_PATH} not built (run __graft_entry__.build() or make -C nex-nccl_amd/csrc)")
    _preload_hip_runtime()
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, i32, sz = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_size_t
    P = ctypes.POINTER
    for name in ("nexrReduceCopy", "nexrReduceCopyHost"):
        f = getattr(L, name)
        f.argtypes = [i32, P(vp), i32, P(vp), sz, i32, i32, u64, i32, P(u64), i32, vp]
        f.restype = i32
    L.nexrReduceCopyBatch.argtypes = [P(ReduceCopyWork), i32, i32, i32, vp]
    L.nexrReduceCopyBatch.restype = i32
    L.nexrReduceCopyMultiDevice.argtypes = [P(ReduceCopyWork), P(i32), i32, i32, i32, i32, P(ctypes.c_double)]
    L.nexrReduceCopyMultiDevice.restype = i32
    L.nexrReduceCopyMultiDeviceSets.argtypes = [P(ReduceCopyWork), P(i32), i32, i32, i32, i32, i32, P(ctypes.c_double)]
    L.nexrReduceCopyMultiDeviceSets.restype = i32
    L.nexrHostToDevRedOp.argtypes = [P(DevRedOpFull), i32, i32, i32]
    L.nexrHostToDevRedOp.restype = i32
    L.nexrLaunchOneRank.argtypes = [vp, vp, sz, DevRedOpFull, i32, vp]
    L.nexrLaunchOneRank.restype = i32
    L.nexrQueryLaunch.argtypes = [i32, P(vp), i32, P(vp), sz, i32, P(LaunchInfo)]
    L.nexrQueryLaunch.restype = i32
    L.nexrGetPoolStats.argtypes = [P(u64), P(u64)]
    L.nexrGetPoolStats.restype = i32
    L.nexrSetSemantics.argtypes = [i32]
    L.nexrSetSemantics.restype = i32
    L.nexrGetSemantics.argtypes = [P(i32)]
    L.nexrGetSemantics.restype = i32
    L.nexrReduceCopyLL.argtypes = [vp, i32, i32, P(vp), P(ctypes.c_uint32), vp, i32, P(vp), P(ctypes.c_uint32), sz,
                                   i32, i32, u64, i32, vp, ctypes.c_uint32, vp]
    L.nexrReduceCopyLL.restype = i32
    L.nexrReduceCopyLL128.argtypes = [vp, i32, i32, P(vp), P(u64), vp, i32, P(vp), P(u64), sz,
                                      i32, i32, u64, i32, vp, ctypes.c_uint32, vp]
    L.nexrReduceCopyLL128.restype = i32
    L.nexrReduceCopyLLSteps.argtypes = [P(LLConnSet), P(LLStep), i32, i32, i32, u64, vp, ctypes.c_uint32, vp]
    L.nexrReduceCopyLLSteps.restype = i32
    L.nexrTypeSize.argtypes = [i32]
    L.nexrTypeSize.restype = sz
    L.nexrGetErrorString.argtypes = [i32]
    L.nexrGetErrorString.restype = ctypes.c_char_p
    L.nexrGetVersion.argtypes = []
    L.nexrGetVersion.restype = i32
    L.nexrGetLastHipError.argtypes = []
    L.nexrGetLastHipError.restype = i32
    L.nexrHostRegister.argtypes = [vp, sz, P(vp)]
    L.nexrHostRegister.restype = i32
    L.nexrHostDeregister.argtypes = [vp]
    L.nexrHostDeregister.restype = i32
    L.nexrHostMemAlloc.argtypes = [P(vp), sz]
    L.nexrHostMemAlloc.restype = i32
    L.nexrHostMemFree.argtypes = [vp]
    L.nexrHostMemFree.restype = i32
    L.nexrGetHostPathStats.argtypes = [P(HostPathStats), i32]
    L.nexrGetHostPathStats.restype = i32
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        extra = ""
        if rc == Result.UnhandledCudaError:
            extra = f" (hipError {lib().nexrGetLastHipError()})"
        raise NexrError(rc, what + extra)


def _ptr_array(ptrs: Sequence[int]):
    arr = (ctypes.c_void_p * max(1, len(ptrs)))()
    for i, p in enumerate(ptrs):
        arr[i] = ctypes.c_void_p(int(p)) if p else None
    return arr


def _u64_array(vals: Optional[Sequence[int]]):
    if not vals:
        return None
    arr = (ctypes.c_uint64 * len(vals))()
    for i, v in enumerate(vals):
        arr[i] = int(v) & 0xFFFFFFFFFFFFFFFF
    return arr


def reduce_copy_ptrs(srcs: Sequence[int], dsts: Sequence[int], n_elts: int, datatype: int, dev_red_op: int,
                     red_op_arg: int = 0, pre_op_args: Optional[Sequence[int]] = None, post_op: bool = False,
                     stream: int = 0, host: bool = False) -> None:
    """Raw-pointer reduce-copy through the C ABI (``nexrReduceCopy`` / ``nexrReduceCopyHost``).

    ``srcs``/``dsts`` are device addresses (host addresses when ``host=True``); ``stream`` is a
    hipStream_t handle (0 = default stream). Mirrors reduceCopy(…, redArg, preOpArgs, postOp,
    nSrcs, srcPtrs, nDsts, dstPtrs, nElts) (common_kernel.h:331-349)."""
    L = lib()
    pre = list(pre_op_args) if pre_op_args else []
    f = L.nexrReduceCopyHost if host else L.nexrReduceCopy
    rc = f(len(srcs), _ptr_array(srcs), len(dsts), _ptr_array(dsts), int(n_elts), int(datatype),
           int(dev_red_op), int(red_op_arg) & 0xFFFFFFFFFFFFFFFF, len(pre), _u64_array(pre),
           1 if post_op else 0, ctypes.c_void_p(int(stream)) if stream else None)
    _check(rc, "nexrReduceCopyHost" if host else "nexrReduceCopy")


def make_work(srcs: Sequence[int], dsts: Sequence[int], n_elts: int, red_op_arg: int = 0,
              pre_op_args: Optional[Sequence[int]] = None, post_op: bool = False) -> ReduceCopyWork:
    """One nexrReduceCopyWork from device addresses (raises on more than 8 srcs/dsts)."""
    pre = list(pre_op_args) if pre_op_args else []
    if len(srcs) > 8 or len(dsts) > 8 or len(pre) > 8:
        raise NexrError(Result.InvalidArgument, "at most 8 srcs, dsts and preOpArgs per work")
    w = ReduceCopyWork()
    w.nSrcs, w.nDsts, w.nElts = len(srcs), len(dsts), int(n_elts)
    for i, a in enumerate(srcs):
        w.srcs[i] = int(a)
    for i, a in enumerate(dsts):
        w.dsts[i] = int(a)
    w.redOpArg = int(red_op_arg) & 0xFFFFFFFFFFFFFFFF
    w.nPreOpSrcs = len(pre)
    for i, v in enumerate(pre):
        w.preOpArgs[i] = int(v) & 0xFFFFFFFFFFFFFFFF
    w.postOp = 1 if post_op else 0
    return w


def reduce_copy_batch(works: Sequence[ReduceCopyWork], datatype: int, dev_red_op: int, stream: int = 0) -> None:
    """``nexrReduceCopyBatch``: independent reduce-copies of one (datatype, op) in few launches."""
    arr = (ReduceCopyWork * max(1, len(works)))(*works)
    _check(lib().nexrReduceCopyBatch(arr, len(works), int(datatype), int(dev_red_op),
                                     ctypes.c_void_p(int(stream)) if stream else None), "nexrReduceCopyBatch")


def reduce_copy_multi_device(works: Sequence[ReduceCopyWork], devices: Sequence[int], datatype: int,
                             dev_red_op: int, reps: int = 1) -> float:
    """``nexrReduceCopyMultiDevice``: work i on GPU devices[i], one host thread and stream per work,
    a shared start barrier, `reps` launches each. Returns seconds from the barrier to the last
    device's completion."""
    if len(works) != len(devices):
        raise NexrError(Result.InvalidArgument, "one device per work")
    arr = (ReduceCopyWork * max(1, len(works)))(*works)
    dev = (ctypes.c_int * max(1, len(devices)))(*[int(d) for d in devices])
    secs = ctypes.c_double(0.0)
    _check(lib().nexrReduceCopyMultiDevice(arr, dev, len(works), int(datatype), int(dev_red_op), int(reps),
                                           ctypes.byref(secs)), "nexrReduceCopyMultiDevice")
    return secs.value


def reduce_copy_multi_device_sets(works_per_device: Sequence[Sequence[ReduceCopyWork]], devices: Sequence[int],
                                  datatype: int, dev_red_op: int, reps: int = 1) -> float:
    """``nexrReduceCopyMultiDeviceSets``: ``works_per_device[i]`` (the same number of works for every
    entry) are rotating sets on GPU devices[i]: launch k of its thread runs set k mod len. Returns
    seconds from the start barrier to the last device's completion."""
    if len(works_per_device) != len(devices) or not works_per_device:
        raise NexrError(Result.InvalidArgument, "one list of works per device")
    n_sets = len(works_per_device[0])
    if any(len(w) != n_sets for w in works_per_device):
        raise NexrError(Result.InvalidArgument, "the same number of sets on every device")
    flat = [w for ws in works_per_device for w in ws]
    arr = (ReduceCopyWork * max(1, len(flat)))(*flat)
    dev = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
    secs = ctypes.c_double(0.0)
    _check(lib().nexrReduceCopyMultiDeviceSets(arr, dev, len(devices), n_sets, int(datatype), int(dev_red_op),
                                               int(reps), ctypes.byref(secs)), "nexrReduceCopyMultiDeviceSets")
    return secs.value


def query_launch(srcs: Sequence[int], dsts: Sequence[int], n_elts: int, datatype: int) -> LaunchInfo:
    """nexrQueryLaunch: the grid, block, cache policy and edge/body split nexrReduceCopy would use
    (no device work)."""
    info = LaunchInfo()
    _check(lib().nexrQueryLaunch(len(srcs), _ptr_array(srcs), len(dsts), _ptr_array(dsts), int(n_elts),
                                 int(datatype), ctypes.byref(info)), "nexrQueryLaunch")
    return info


def pool_stats() -> tuple:
    """(streams created by nexrReduceCopyMultiDevice, staging rings created by nexrReduceCopyHost)."""
    a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(lib().nexrGetPoolStats(ctypes.byref(a), ctypes.byref(b)), "nexrGetPoolStats")
    return a.value, b.value


def host_register(addr: int, nbytes: int) -> int:
    """nexrHostRegister (ncclCommRegister's counterpart for host memory): page-lock and device-map
    [addr, addr + nbytes) and record it in libnexr's registration cache. Returns the handle."""
    h = ctypes.c_void_p()
    _check(lib().nexrHostRegister(ctypes.c_void_p(int(addr)), int(nbytes), ctypes.byref(h)), "nexrHostRegister")
    return int(h.value or 0)


def host_deregister(handle: int) -> None:
    """nexrHostDeregister: drop one reference to a registration (the last one unregisters)."""
    _check(lib().nexrHostDeregister(ctypes.c_void_p(int(handle)) if handle else None), "nexrHostDeregister")


def host_mem_alloc(nbytes: int) -> int:
    """nexrHostMemAlloc (ncclMemAlloc's counterpart): pinned, device-mapped host memory."""
    p = ctypes.c_void_p()
    _check(lib().nexrHostMemAlloc(ctypes.byref(p), int(nbytes)), "nexrHostMemAlloc")
    return int(p.value)


def host_mem_free(addr: int) -> None:
    _check(lib().nexrHostMemFree(ctypes.c_void_p(int(addr)) if addr else None), "nexrHostMemFree")


def host_path_stats(reset: bool = False) -> dict:
    """nexrGetHostPathStats: where nexrReduceCopyHost calls have spent host time (ns) since the last
    reset, with the counts of calls, zero-copy calls, cache hits and runtime pointer queries."""
    st = HostPathStats()
    _check(lib().nexrGetHostPathStats(ctypes.byref(st), 1 if reset else 0), "nexrGetHostPathStats")
    return {f: int(getattr(st, f)) for f, _ in HostPathStats._fields_}


def set_semantics(mode: int) -> None:
    """nexrSetSemantics: process-wide reduction semantics for every later call (Semantics)."""
    _check(lib().nexrSetSemantics(int(mode)), "nexrSetSemantics")


def get_semantics() -> int:
    v = ctypes.c_int(-1)
    _check(lib().nexrGetSemantics(ctypes.byref(v)), "nexrGetSemantics")
    return v.value


def host_to_dev_red_op(op: int, datatype: int, n_ranks: int = 1) -> DevRedOpFull:
    """hostToDevRedOp (reference src/enqueue.cc:2185-2278) for the built-in ops."""
    out = DevRedOpFull()
    _check(lib().nexrHostToDevRedOp(ctypes.byref(out), int(op), int(datatype), int(n_ranks)), "nexrHostToDevRedOp")
    return out


def launch_one_rank(dst: int, src: int, n_elts: int, red_op: DevRedOpFull, datatype: int, stream: int = 0) -> None:
    """ncclLaunchOneRank (reference src/device/onerank.cc:48-83)."""
    _check(lib().nexrLaunchOneRank(ctypes.c_void_p(int(dst)) if dst else None,
                                   ctypes.c_void_p(int(src)) if src else None, int(n_elts), red_op,
                                   int(datatype), ctypes.c_void_p(int(stream)) if stream else None),
           "nexrLaunchOneRank")


def reduce_copy_ll(src: int, recv_lines: Sequence[int], recv_flags: Sequence[int], dst: int,
                   send_lines: Sequence[int], send_flags: Sequence[int], n_elts: int, datatype: int,
                   dev_red_op: int, red_op_arg: int = 0, src_is_input: bool = True, post_op: bool = False,
                   status: int = 0, timeout_us: int = 0, stream: int = 0) -> None:
    """One LL-protocol step (LLGenericOp, reference src/device/prims_ll.h:218-283) on device pointers."""
    u32 = ctypes.c_uint32
    rf = (u32 * max(1, len(recv_flags)))(*[int(f) & 0xFFFFFFFF for f in recv_flags])
    sf = (u32 * max(1, len(send_flags)))(*[int(f) & 0xFFFFFFFF for f in send_flags])
    rc = lib().nexrReduceCopyLL(ctypes.c_void_p(int(src)) if src else None, 1 if src_is_input else 0,
                                len(recv_lines), _ptr_array(recv_lines), rf,
                                ctypes.c_void_p(int(dst)) if dst else None, len(send_lines), _ptr_array(send_lines),
                                sf, int(n_elts), int(datatype), int(dev_red_op), int(red_op_arg) & 0xFFFFFFFFFFFFFFFF,
                                1 if post_op else 0, ctypes.c_void_p(int(status)) if status else None,
                                int(timeout_us), ctypes.c_void_p(int(stream)) if stream else None)
    _check(rc, "nexrReduceCopyLL")


def reduce_copy_ll128(src: int, recv_wire: Sequence[int], recv_flags: Sequence[int], dst: int,
                      send_wire: Sequence[int], send_flags: Sequence[int], n_elts: int, datatype: int,
                      dev_red_op: int, red_op_arg: int = 0, src_is_input: bool = True, post_op: bool = False,
                      status: int = 0, timeout_us: int = 0, stream: int = 0) -> None:
    """One LL128-protocol step (prims_ll128.h:184-331) on device pointers."""
    rf = _u64_array(list(recv_flags)) if recv_flags else None
    sf = _u64_array(list(send_flags)) if send_flags else None
    rc = lib().nexrReduceCopyLL128(ctypes.c_void_p(int(src)) if src else None, 1 if src_is_input else 0,
                                   len(recv_wire), _ptr_array(recv_wire), rf,
                                   ctypes.c_void_p(int(dst)) if dst else None, len(send_wire), _ptr_array(send_wire),
                                   sf, int(n_elts), int(datatype), int(dev_red_op),
                                   int(red_op_arg) & 0xFFFFFFFFFFFFFFFF, 1 if post_op else 0,
                                   ctypes.c_void_p(int(status)) if status else None, int(timeout_us),
                                   ctypes.c_void_p(int(stream)) if stream else None)
    _check(rc, "nexrReduceCopyLL128")


def ll_step(src_buf: int = -1, src_ix: int = 0, dst_buf: int = -1, dst_ix: int = 0, n_elts: int = 0,
            recv: bool = False, send: bool = False, post_op: bool = False) -> LLStep:
    """One step of a run (buffers: 0 input, 1 output, -1 none)."""
    s = LLStep()
    s.srcIx, s.dstIx, s.nElts = int(src_ix), int(dst_ix), int(n_elts)
    s.recv, s.send, s.srcBuf, s.dstBuf, s.postOp = int(bool(recv)), int(bool(send)), int(src_buf), int(dst_buf), \
        int(bool(post_op))
    return s


def reduce_copy_ll_steps(input_ptr: int, output_ptr: int, recv: Sequence[tuple], send: Sequence[tuple],
                         slot_bytes: int, steps: Sequence[LLStep], datatype: int, dev_red_op: int,
                         red_op_arg: int = 0, n_slots: int = 8, status: int = 0, timeout_us: int = 0,
                         stream: int = 0) -> None:
    """A run of LL steps with device credits (nexrReduceCopyLLSteps, reference prims_ll.h:55-83 and
    :249-318). recv / send: (fifo pointer, head-words pointer, step counter) per connection."""
    cs = LLConnSet()
    cs.input, cs.output = int(input_ptr) or None, int(output_ptr) or None
    cs.nRecv, cs.nSend = len(recv), len(send)
    for i, (fifo, head, step) in enumerate(recv):
        cs.recvFifo[i], cs.recvHead[i], cs.recvStep[i] = int(fifo), int(head), int(step)
    for i, (fifo, head, step) in enumerate(send):
        cs.sendFifo[i], cs.sendHead[i], cs.sendStep[i] = int(fifo), int(head), int(step)
    cs.slotBytes, cs.nSlots = int(slot_bytes), int(n_slots)
    arr = (LLStep * max(1, len(steps)))(*steps)
    rc = lib().nexrReduceCopyLLSteps(ctypes.byref(cs), arr, len(steps), int(datatype), int(dev_red_op),
                                     int(red_op_arg) & 0xFFFFFFFFFFFFFFFF,
                                     ctypes.c_void_p(int(status)) if status else None, int(timeout_us),
                                     ctypes.c_void_p(int(stream)) if stream else None)
    _check(rc, "nexrReduceCopyLLSteps")


def version() -> int:
    return lib().nexrGetVersion()


# ---- torch convenience layer (device memory and streams only; the compute is libnexr) ----------
def torch_datatype(dtype) -> DataType:
    import torch
    m = {torch.int8: DataType.Int8, torch.uint8: DataType.Uint8, torch.int32: DataType.Int32,
         torch.int64: DataType.Int64, torch.float16: DataType.Float16, torch.float32: DataType.Float32,
         torch.float64: DataType.Float64, torch.bfloat16: DataType.Bfloat16}
    for name, dt in (("uint32", DataType.Uint32), ("uint64", DataType.Uint64)):
        t = getattr(torch, name, None)
        if t is not None:
            m[t] = dt
    if dtype not in m:
        raise NexrError(Result.InvalidArgument, f"unsupported torch dtype {dtype}")
    return m[dtype]


def reduce_copy(srcs, dsts, dev_red_op: int = DevRedOp.Sum, red_op_arg: int = 0,
                pre_op_args: Optional[Sequence[int]] = None, post_op: bool = False, datatype: Optional[int] = None,
                stream=None) -> None:
    """Reduce-copy over torch tensors on one device: every dst[i] = fold(srcs)[i].

    All tensors must be contiguous with the same element count. ``datatype`` defaults to the
    tensors' dtype (pass ``DataType.Uint32``/``Uint64`` explicitly for unsigned views of int32/int64
    storage). ``stream`` is a torch stream (default: the current stream)."""
    import torch
    if not srcs:
        raise NexrError(Result.InvalidArgument, "no sources")
    n = srcs[0].numel()
    for t in list(srcs) + list(dsts):
        if not t.is_contiguous() or t.numel() != n:
            raise NexrError(Result.InvalidArgument, "tensors must be contiguous and equally sized")
    dt = torch_datatype(srcs[0].dtype) if datatype is None else DataType(datatype)
    if stream is None and srcs[0].is_cuda:
        stream = torch.cuda.current_stream(srcs[0].device)
    handle = stream.cuda_stream if stream is not None else 0
    reduce_copy_ptrs([t.data_ptr() for t in srcs], [t.data_ptr() for t in dsts], n, dt, dev_red_op,
                     red_op_arg, pre_op_args, post_op, handle, host=not srcs[0].is_cuda)
