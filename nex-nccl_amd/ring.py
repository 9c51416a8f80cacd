"""Python view of the CPU-emulated collectives (include/nexr_ring.h, libnexr_ring.so; with
``extras=True`` the opt-in include/nexr_extras.h, libnexr_extras.so).

The ring and tree schedules (runRing of all_reduce.h, reduce_scatter.h, all_gather.h, reduce.h,
broadcast.h; runTreeSplit, all_reduce.h:150-230) and the genericOp slicing / FIFO credit
protocol (src/device/prims_simple.h:111-330) run on host threads in C++; every reduceCopy site calls
the MI355X reduce-copy ABI (or any function with its signature, e.g. a test checker).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

from . import NexrError, Result, _check, lib

_HERE = os.path.dirname(os.path.abspath(__file__))
RING_LIB_PATH = os.path.join(_HERE, "libnexr_ring.so")
# Opt-in (make -C nex-nccl_amd/csrc EXTRAS=1): include/nexr_extras.h, a superset of libnexr_ring.so.
EXTRAS_LIB_PATH = os.path.join(_HERE, "libnexr_extras.so")
RING_ABI_SYMBOLS = ("nexrRingCommCreate", "nexrRingAllReduce", "nexrRingReduceScatter", "nexrRingAllGather",
                    "nexrRingReduce", "nexrRingBroadcast", "nexrTreeAllReduce", "nexrTreeTopology",
                    "nexrRingCommGetStepWait", "nexrRingCommGetQueued", "nexrRingCommDestroy", "nexrPeerRingCommCreate",
                    "nexrPeerRingAllReduce", "nexrPeerRingReduceScatter", "nexrPeerRingAllGather",
                    "nexrPeerRingReduce", "nexrPeerRingBroadcast")
EXTRAS_ABI_SYMBOLS = ("nexrSendRecv", "nexrPeerSendRecv", "nexrRingAllReduceResident",
                      "nexrRingReduceScatterResident", "nexrRingAllGatherResident", "nexrRingReduceResident",
                      "nexrRingBroadcastResident", "nexrTreeAllReduceResident", "nexrPeerRingAllReduceResident")

HOST_MEMORY = 0
DEVICE_MEMORY = 1
PROTO_SIMPLE = 0
PROTO_LL = 1
PROTO_LL128 = 2

REDUCE_COPY_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_uint64, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int,
                                  ctypes.c_void_p)


class RingConfig(ctypes.Structure):
    _fields_ = [("nRanks", ctypes.c_int), ("buffBytes", ctypes.c_size_t), ("memMode", ctypes.c_int),
                ("fn", ctypes.c_void_p), ("timeoutMs", ctypes.c_int), ("protocol", ctypes.c_int),
                ("llFn", ctypes.c_void_p), ("ll128Fn", ctypes.c_void_p), ("treeRanksPerNode", ctypes.c_int),
                ("treeIndex", ctypes.c_int), ("nChannels", ctypes.c_int)]


class PeerRingConfig(ctypes.Structure):
    _fields_ = [("nRanks", ctypes.c_int), ("rank", ctypes.c_int), ("device", ctypes.c_int),
                ("buffBytes", ctypes.c_size_t), ("protocol", ctypes.c_int), ("timeoutMs", ctypes.c_int),
                ("shmName", ctypes.c_char_p)]


_libs = {}


def _bind_ring(L: ctypes.CDLL) -> None:
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    arr = ctypes.POINTER(ctypes.c_void_p)
    L.nexrRingCommCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(RingConfig)]
    for name, extra in (("nexrRingAllReduce", [i32]), ("nexrRingReduceScatter", [i32]), ("nexrRingAllGather", []),
                        ("nexrRingReduce", [i32, i32]), ("nexrRingBroadcast", [i32]), ("nexrTreeAllReduce", [i32])):
        getattr(L, name).argtypes = [vp, arr, arr, sz, i32] + extra
    for name, extra in (("nexrPeerRingAllReduce", [i32]), ("nexrPeerRingReduceScatter", [i32]),
                        ("nexrPeerRingAllGather", []), ("nexrPeerRingReduce", [i32, i32]),
                        ("nexrPeerRingBroadcast", [i32])):
        getattr(L, name).argtypes = [vp, vp, vp, sz, i32] + extra
    L.nexrTreeTopology.argtypes = [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
    L.nexrRingCommGetStepWait.argtypes = [vp, ctypes.POINTER(i32)]
    L.nexrRingCommGetQueued.argtypes = [vp, ctypes.POINTER(i32)]
    L.nexrPeerRingCommCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(PeerRingConfig)]
    L.nexrRingCommDestroy.argtypes = [vp]
    for name in RING_ABI_SYMBOLS:
        getattr(L, name).restype = ctypes.c_int


def _bind_extras(L: ctypes.CDLL) -> None:
    vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    arr = ctypes.POINTER(ctypes.c_void_p)
    for name, extra in (("nexrRingAllReduceResident", [i32]), ("nexrTreeAllReduceResident", [i32]),
                        ("nexrRingReduceScatterResident", [i32]), ("nexrRingAllGatherResident", []),
                        ("nexrRingReduceResident", [i32, i32]), ("nexrRingBroadcastResident", [i32])):
        getattr(L, name).argtypes = [vp, arr, arr, sz, i32] + extra
    L.nexrPeerRingAllReduceResident.argtypes = [vp, vp, vp, sz, i32, i32]
    L.nexrSendRecv.argtypes = [vp, arr, ctypes.POINTER(i32), arr, ctypes.POINTER(i32), sz]
    L.nexrPeerSendRecv.argtypes = [vp, vp, i32, vp, i32, sz]
    for name in EXTRAS_ABI_SYMBOLS:
        getattr(L, name).restype = ctypes.c_int


def ring_lib() -> ctypes.CDLL:
    """libnexr_ring.so: the graded callers (include/nexr_ring.h)."""
    if "ring" not in _libs:
        lib()  # libnexr.so first (the ring library links against it)
        if not os.path.exists(RING_LIB_PATH):
            raise NexrError(Result.InternalError, f"{RING_LIB_PATH} not built")
        L = ctypes.CDLL(RING_LIB_PATH)
        _bind_ring(L)
        _libs["ring"] = L
    return _libs["ring"]


def extras_available() -> bool:
    return os.path.exists(EXTRAS_LIB_PATH)


def extras_lib() -> ctypes.CDLL:
    """libnexr_extras.so (opt-in): nexr_ring.h's entry points plus include/nexr_extras.h's."""
    if "extras" not in _libs:
        lib()
        if not extras_available():
            raise NexrError(Result.InvalidUsage, f"{EXTRAS_LIB_PATH} not built (make -C nex-nccl_amd/csrc EXTRAS=1)")
        L = ctypes.CDLL(EXTRAS_LIB_PATH)
        _bind_ring(L)
        _bind_extras(L)
        _libs["extras"] = L
    return _libs["extras"]


class RingComm:
    """N emulated ranks (host threads) of one communicator: ring collectives (ncclAllReduce,
    ncclReduceScatter, ncclAllGather, ncclReduce, ncclBroadcast) and the tree ncclAllReduce, each
    run on all ranks at once (one buffer per rank)."""

    def __init__(self, n_ranks: int, mem_mode: int = HOST_MEMORY, buff_bytes: int = 0,
                 fn_address: Optional[int] = None, timeout_ms: int = 0, protocol: int = PROTO_SIMPLE,
                 ll_fn_address: Optional[int] = None, ll128_fn_address: Optional[int] = None,
                 tree_ranks_per_node: int = 0, tree_index: int = 0, n_channels: int = 0, extras: bool = False):
        """extras=True: the communicator lives in the opt-in libnexr_extras.so, which adds send/recv and
        the device-resident collectives; every call on it goes to that library."""
        cfg = RingConfig(n_ranks, buff_bytes, mem_mode, fn_address or None, timeout_ms, protocol,
                         ll_fn_address or None, ll128_fn_address or None, tree_ranks_per_node, tree_index, n_channels)
        self._L = extras_lib() if extras else ring_lib()
        self.extras = extras
        h = ctypes.c_void_p()
        _check(self._L.nexrRingCommCreate(ctypes.byref(h), ctypes.byref(cfg)), "nexrRingCommCreate")
        self._h = h
        self.n_ranks = n_ranks

    def all_reduce(self, sendbuffs: Sequence[int], recvbuffs: Sequence[int], count: int, datatype: int,
                   op: int) -> None:
        if len(sendbuffs) != self.n_ranks or len(recvbuffs) != self.n_ranks:
            raise NexrError(Result.InvalidArgument, "one send and one recv buffer per rank")
        s = (ctypes.c_void_p * self.n_ranks)(*[int(p) for p in sendbuffs])
        r = (ctypes.c_void_p * self.n_ranks)(*[int(p) for p in recvbuffs])
        _check(self._L.nexrRingAllReduce(self._h, s, r, int(count), int(datatype), int(op)), "nexrRingAllReduce")

    def all_reduce_resident(self, sendbuffs: Sequence[int], recvbuffs: Sequence[int], count: int, datatype: int,
                            op: int) -> None:
        """The same all-reduce as one device-resident launch per GPU (nexrRingAllReduceResident)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrRingAllReduceResident(self._h, s, r, int(count), int(datatype), int(op)),
               "nexrRingAllReduceResident")

    def tree_all_reduce_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrTreeAllReduceResident(self._h, s, r, int(count), int(datatype), int(op)),
               "nexrTreeAllReduceResident")

    def reduce_scatter_resident(self, sendbuffs, recvbuffs, recvcount: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrRingReduceScatterResident(self._h, s, r, int(recvcount), int(datatype), int(op)),
               "nexrRingReduceScatterResident")

    def all_gather_resident(self, sendbuffs, recvbuffs, sendcount: int, datatype: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrRingAllGatherResident(self._h, s, r, int(sendcount), int(datatype)),
               "nexrRingAllGatherResident")

    def reduce_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrRingReduceResident(self._h, s, r, int(count), int(datatype), int(op), int(root)),
               "nexrRingReduceResident")

    def broadcast_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._extras().nexrRingBroadcastResident(self._h, s, r, int(count), int(datatype), int(root)),
               "nexrRingBroadcastResident")

    def _arrays(self, sendbuffs, recvbuffs):
        if len(sendbuffs) != self.n_ranks or len(recvbuffs) != self.n_ranks:
            raise NexrError(Result.InvalidArgument, "one send and one recv buffer per rank")
        s = (ctypes.c_void_p * self.n_ranks)(*[int(p) if p else None for p in sendbuffs])
        r = (ctypes.c_void_p * self.n_ranks)(*[int(p) if p else None for p in recvbuffs])
        return s, r

    def reduce_scatter(self, sendbuffs, recvbuffs, recvcount: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._L.nexrRingReduceScatter(self._h, s, r, int(recvcount), int(datatype), int(op)),
               "nexrRingReduceScatter")

    def all_gather(self, sendbuffs, recvbuffs, sendcount: int, datatype: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._L.nexrRingAllGather(self._h, s, r, int(sendcount), int(datatype)), "nexrRingAllGather")

    def reduce(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._L.nexrRingReduce(self._h, s, r, int(count), int(datatype), int(op), int(root)),
               "nexrRingReduce")

    def broadcast(self, sendbuffs, recvbuffs, count: int, datatype: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._L.nexrRingBroadcast(self._h, s, r, int(count), int(datatype), int(root)), "nexrRingBroadcast")

    def tree_all_reduce(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(self._L.nexrTreeAllReduce(self._h, s, r, int(count), int(datatype), int(op)), "nexrTreeAllReduce")

    def send_recv(self, sendbuffs, send_peers, recvbuffs, recv_peers, nbytes: int) -> None:
        """ncclSend/ncclRecv of every rank in one group: rank r sends nbytes of sendbuffs[r] to
        send_peers[r] and receives nbytes from recv_peers[r] into recvbuffs[r] (-1: none)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        sp = (ctypes.c_int * self.n_ranks)(*[int(v) for v in send_peers])
        rp = (ctypes.c_int * self.n_ranks)(*[int(v) for v in recv_peers])
        _check(self._extras().nexrSendRecv(self._h, s, sp, r, rp, int(nbytes)), "nexrSendRecv")

    def step_wait(self) -> str:
        """"word" or "sync": how this communicator's rank threads wait for a device step
        (nexrRingCommGetStepWait; sync when the ranks span GPUs)."""
        w = ctypes.c_int()
        _check(self._L.nexrRingCommGetStepWait(self._h, ctypes.byref(w)), "nexrRingCommGetStepWait")
        return "word" if w.value else "sync"

    def queued(self) -> int:
        """How the last ring collective ran its LL steps (nexrRingCommGetQueued): 2 runs on the device
        with device credits, 1 queued launches, 0 host-sequenced (LL steps need every rank on one GPU
        and device memory for 1 or 2)."""
        w = ctypes.c_int()
        _check(self._L.nexrRingCommGetQueued(self._h, ctypes.byref(w)), "nexrRingCommGetQueued")
        return int(w.value)

    def tree_topology(self, rank: int):
        """(up, [down...]) of `rank` in this communicator's tree (-1 = none)."""
        up = ctypes.c_int()
        down = (ctypes.c_int * 3)()
        _check(self._L.nexrTreeTopology(self._h, int(rank), ctypes.byref(up), down), "nexrTreeTopology")
        return up.value, [d for d in down if d >= 0]

    def _extras(self) -> ctypes.CDLL:
        if not self.extras:
            raise NexrError(Result.InvalidUsage, "send/recv and the resident collectives are in the opt-in extras "
                                                 "library: create the communicator with extras=True")
        return self._L

    def close(self) -> None:
        if self._h:
            self._L.nexrRingCommDestroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PeerRingComm:
    """This process's rank of a ring whose ranks are processes (one per GPU), FIFOs shared over IPC.

    Every rank passes the same fresh ``shm_name`` (e.g. made by rank 0 and broadcast out of band);
    the constructor blocks until all ``n_ranks`` processes have joined."""

    def __init__(self, n_ranks: int, rank: int, shm_name: str, device: int = 0, buff_bytes: int = 0,
                 protocol: int = PROTO_SIMPLE, timeout_ms: int = 0, extras: bool = False):
        self._name = shm_name.encode()
        cfg = PeerRingConfig(n_ranks, rank, device, buff_bytes, protocol, timeout_ms, self._name)
        self._L = extras_lib() if extras else ring_lib()
        self.extras = extras
        h = ctypes.c_void_p()
        _check(self._L.nexrPeerRingCommCreate(ctypes.byref(h), ctypes.byref(cfg)), "nexrPeerRingCommCreate")
        self._h = h
        self.n_ranks, self.rank = n_ranks, rank

    def all_reduce(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int) -> None:
        _check(self._L.nexrPeerRingAllReduce(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                                int(datatype), int(op)), "nexrPeerRingAllReduce")

    def all_reduce_resident(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int) -> None:
        """This rank's part of the all-reduce as one device-resident launch (nexrPeerRingAllReduceResident)."""
        _check(self._extras().nexrPeerRingAllReduceResident(self._h, int(sendbuff) or None, int(recvbuff) or None,
                                                        int(count), int(datatype), int(op)),
               "nexrPeerRingAllReduceResident")

    def reduce_scatter(self, sendbuff: int, recvbuff: int, recvcount: int, datatype: int, op: int) -> None:
        _check(self._L.nexrPeerRingReduceScatter(self._h, int(sendbuff) or None, int(recvbuff) or None,
                                                    int(recvcount), int(datatype), int(op)), "nexrPeerRingReduceScatter")

    def all_gather(self, sendbuff: int, recvbuff: int, sendcount: int, datatype: int) -> None:
        _check(self._L.nexrPeerRingAllGather(self._h, int(sendbuff) or None, int(recvbuff) or None, int(sendcount),
                                                int(datatype)), "nexrPeerRingAllGather")

    def reduce(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int, root: int) -> None:
        _check(self._L.nexrPeerRingReduce(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                             int(datatype), int(op), int(root)), "nexrPeerRingReduce")

    def send_recv(self, sendbuff: int, send_peer: int, recvbuff: int, recv_peer: int, nbytes: int) -> None:
        _check(self._extras().nexrPeerSendRecv(self._h, int(sendbuff) or None, int(send_peer), int(recvbuff) or None,
                                           int(recv_peer), int(nbytes)), "nexrPeerSendRecv")

    def step_wait(self) -> str:
        """"word" or "sync": how this communicator's rank threads wait for a device step
        (nexrRingCommGetStepWait; sync when the ranks span GPUs)."""
        w = ctypes.c_int()
        _check(self._L.nexrRingCommGetStepWait(self._h, ctypes.byref(w)), "nexrRingCommGetStepWait")
        return "word" if w.value else "sync"

    def broadcast(self, sendbuff: int, recvbuff: int, count: int, datatype: int, root: int) -> None:
        _check(self._L.nexrPeerRingBroadcast(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                                int(datatype), int(root)), "nexrPeerRingBroadcast")

    def _extras(self) -> ctypes.CDLL:
        if not self.extras:
            raise NexrError(Result.InvalidUsage, "send/recv and the resident collectives are in the opt-in extras "
                                                 "library: create the communicator with extras=True")
        return self._L

    def close(self) -> None:
        if self._h:
            self._L.nexrRingCommDestroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
