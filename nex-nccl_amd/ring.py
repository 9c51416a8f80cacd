"""Python view of the CPU-emulated collectives (include/nexr_ring.h, libnexr_ring.so).

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
RING_ABI_SYMBOLS = ("nexrRingCommCreate", "nexrRingAllReduce", "nexrRingReduceScatter", "nexrRingAllGather",
                    "nexrRingReduce", "nexrRingBroadcast", "nexrTreeAllReduce", "nexrTreeTopology",
                    "nexrRingCommDestroy", "nexrPeerRingCommCreate", "nexrPeerRingAllReduce",
                    "nexrPeerRingReduceScatter", "nexrPeerRingAllGather", "nexrPeerRingReduce",
                    "nexrPeerRingBroadcast", "nexrPatReduceScatter", "nexrPatAllGather", "nexrPatSchedule",
                    "nexrSendRecv", "nexrPeerPatReduceScatter", "nexrPeerPatAllGather", "nexrPeerSendRecv",
                    "nexrRingAllReduceResident", "nexrRingReduceScatterResident", "nexrRingAllGatherResident",
                    "nexrRingReduceResident", "nexrRingBroadcastResident", "nexrTreeAllReduceResident",
                    "nexrPeerRingAllReduceResident")

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


_ring = None


def ring_lib() -> ctypes.CDLL:
    global _ring
    if _ring is None:
        lib()  # libnexr.so first (the ring library links against it)
        if not os.path.exists(RING_LIB_PATH):
            raise NexrError(Result.InternalError, f"{RING_LIB_PATH} not built")
        L = ctypes.CDLL(RING_LIB_PATH)
        L.nexrRingCommCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(RingConfig)]
        L.nexrRingCommCreate.restype = ctypes.c_int
        L.nexrRingAllReduce.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.nexrRingAllReduce.restype = ctypes.c_int
        L.nexrRingAllReduceResident.argtypes = L.nexrRingAllReduce.argtypes
        L.nexrRingAllReduceResident.restype = ctypes.c_int
        L.nexrTreeAllReduceResident.argtypes = L.nexrRingAllReduce.argtypes
        L.nexrTreeAllReduceResident.restype = ctypes.c_int
        L.nexrPeerRingAllReduceResident.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                    ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.nexrPeerRingAllReduceResident.restype = ctypes.c_int
        _arr, _i, _sz = ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_size_t
        for f, extra in ((L.nexrRingReduceScatterResident, [_i, _i]), (L.nexrRingAllGatherResident, [_i]),
                         (L.nexrRingReduceResident, [_i, _i, _i]), (L.nexrRingBroadcastResident, [_i, _i])):
            f.argtypes = [ctypes.c_void_p, _arr, _arr, _sz] + extra
            f.restype = ctypes.c_int
        vp, i32, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        arr = ctypes.POINTER(ctypes.c_void_p)
        for name, extra in (("nexrRingReduceScatter", [i32]), ("nexrRingAllGather", []), ("nexrRingReduce", [i32, i32]),
                            ("nexrRingBroadcast", [i32]), ("nexrTreeAllReduce", [i32]),
                            ("nexrPatReduceScatter", [i32]), ("nexrPatAllGather", [])):
            f = getattr(L, name)
            f.argtypes = [vp, arr, arr, sz, i32] + extra
            f.restype = ctypes.c_int
        L.nexrPeerSendRecv.argtypes = [vp, vp, i32, vp, i32, sz]
        L.nexrPeerSendRecv.restype = ctypes.c_int
        for name, extra in (("nexrPeerRingReduceScatter", [i32]), ("nexrPeerRingAllGather", []),
                            ("nexrPeerPatReduceScatter", [i32]), ("nexrPeerPatAllGather", []),
                            ("nexrPeerRingReduce", [i32, i32]), ("nexrPeerRingBroadcast", [i32])):
            f = getattr(L, name)
            f.argtypes = [vp, vp, vp, sz, i32] + extra
            f.restype = ctypes.c_int
        L.nexrSendRecv.argtypes = [vp, arr, ctypes.POINTER(i32), arr, ctypes.POINTER(i32), sz]
        L.nexrSendRecv.restype = ctypes.c_int
        L.nexrPatSchedule.argtypes = [i32, i32, i32, sz, i32, sz, ctypes.POINTER(ctypes.c_int64), sz,
                                      ctypes.POINTER(sz), ctypes.POINTER(i32)]
        L.nexrPatSchedule.restype = ctypes.c_int
        L.nexrTreeTopology.argtypes = [vp, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        L.nexrTreeTopology.restype = ctypes.c_int
        L.nexrPeerRingCommCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(PeerRingConfig)]
        L.nexrPeerRingCommCreate.restype = ctypes.c_int
        L.nexrPeerRingAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_int]
        L.nexrPeerRingAllReduce.restype = ctypes.c_int
        L.nexrRingCommDestroy.argtypes = [ctypes.c_void_p]
        L.nexrRingCommDestroy.restype = ctypes.c_int
        _ring = L
    return _ring


PAT_FIELDS = ("recvDim", "sendDim", "recvOffset", "sendOffset", "stepOffset", "postRecv", "postSend", "nelem",
              "last", "skipped", "inpIx", "outIx")


def pat_schedule(reduce_scatter: bool, n_ranks: int, rank: int, count: int, datatype: int, buff_bytes: int = 0):
    """The PAT step stream of one rank (nexrPatSchedule): (list of dicts with PAT_FIELDS, parallelFactor)."""
    L = ring_lib()
    n_ops = ctypes.c_size_t()
    pf = ctypes.c_int()
    _check(L.nexrPatSchedule(int(reduce_scatter), n_ranks, rank, count, datatype, buff_bytes, None, 0,
                             ctypes.byref(n_ops), ctypes.byref(pf)), "nexrPatSchedule")
    buf = (ctypes.c_int64 * (12 * n_ops.value))()
    _check(L.nexrPatSchedule(int(reduce_scatter), n_ranks, rank, count, datatype, buff_bytes, buf, n_ops.value,
                             ctypes.byref(n_ops), ctypes.byref(pf)), "nexrPatSchedule")
    vals = list(buf)
    return [dict(zip(PAT_FIELDS, vals[12 * i:12 * i + 12])) for i in range(n_ops.value)], pf.value


class RingComm:
    """N emulated ranks (host threads) of one communicator: ring collectives (ncclAllReduce,
    ncclReduceScatter, ncclAllGather, ncclReduce, ncclBroadcast) and the tree ncclAllReduce, each
    run on all ranks at once (one buffer per rank)."""

    def __init__(self, n_ranks: int, mem_mode: int = HOST_MEMORY, buff_bytes: int = 0,
                 fn_address: Optional[int] = None, timeout_ms: int = 0, protocol: int = PROTO_SIMPLE,
                 ll_fn_address: Optional[int] = None, ll128_fn_address: Optional[int] = None,
                 tree_ranks_per_node: int = 0, tree_index: int = 0, n_channels: int = 0):
        cfg = RingConfig(n_ranks, buff_bytes, mem_mode, fn_address or None, timeout_ms, protocol,
                         ll_fn_address or None, ll128_fn_address or None, tree_ranks_per_node, tree_index, n_channels)
        h = ctypes.c_void_p()
        _check(ring_lib().nexrRingCommCreate(ctypes.byref(h), ctypes.byref(cfg)), "nexrRingCommCreate")
        self._h = h
        self.n_ranks = n_ranks

    def all_reduce(self, sendbuffs: Sequence[int], recvbuffs: Sequence[int], count: int, datatype: int,
                   op: int) -> None:
        if len(sendbuffs) != self.n_ranks or len(recvbuffs) != self.n_ranks:
            raise NexrError(Result.InvalidArgument, "one send and one recv buffer per rank")
        s = (ctypes.c_void_p * self.n_ranks)(*[int(p) for p in sendbuffs])
        r = (ctypes.c_void_p * self.n_ranks)(*[int(p) for p in recvbuffs])
        _check(ring_lib().nexrRingAllReduce(self._h, s, r, int(count), int(datatype), int(op)), "nexrRingAllReduce")

    def all_reduce_resident(self, sendbuffs: Sequence[int], recvbuffs: Sequence[int], count: int, datatype: int,
                            op: int) -> None:
        """The same all-reduce as one device-resident launch per GPU (nexrRingAllReduceResident)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingAllReduceResident(self._h, s, r, int(count), int(datatype), int(op)),
               "nexrRingAllReduceResident")

    def tree_all_reduce_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrTreeAllReduceResident(self._h, s, r, int(count), int(datatype), int(op)),
               "nexrTreeAllReduceResident")

    def reduce_scatter_resident(self, sendbuffs, recvbuffs, recvcount: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingReduceScatterResident(self._h, s, r, int(recvcount), int(datatype), int(op)),
               "nexrRingReduceScatterResident")

    def all_gather_resident(self, sendbuffs, recvbuffs, sendcount: int, datatype: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingAllGatherResident(self._h, s, r, int(sendcount), int(datatype)),
               "nexrRingAllGatherResident")

    def reduce_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingReduceResident(self._h, s, r, int(count), int(datatype), int(op), int(root)),
               "nexrRingReduceResident")

    def broadcast_resident(self, sendbuffs, recvbuffs, count: int, datatype: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingBroadcastResident(self._h, s, r, int(count), int(datatype), int(root)),
               "nexrRingBroadcastResident")

    def _arrays(self, sendbuffs, recvbuffs):
        if len(sendbuffs) != self.n_ranks or len(recvbuffs) != self.n_ranks:
            raise NexrError(Result.InvalidArgument, "one send and one recv buffer per rank")
        s = (ctypes.c_void_p * self.n_ranks)(*[int(p) if p else None for p in sendbuffs])
        r = (ctypes.c_void_p * self.n_ranks)(*[int(p) if p else None for p in recvbuffs])
        return s, r

    def reduce_scatter(self, sendbuffs, recvbuffs, recvcount: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingReduceScatter(self._h, s, r, int(recvcount), int(datatype), int(op)),
               "nexrRingReduceScatter")

    def all_gather(self, sendbuffs, recvbuffs, sendcount: int, datatype: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingAllGather(self._h, s, r, int(sendcount), int(datatype)), "nexrRingAllGather")

    def reduce(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingReduce(self._h, s, r, int(count), int(datatype), int(op), int(root)),
               "nexrRingReduce")

    def broadcast(self, sendbuffs, recvbuffs, count: int, datatype: int, root: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrRingBroadcast(self._h, s, r, int(count), int(datatype), int(root)), "nexrRingBroadcast")

    def tree_all_reduce(self, sendbuffs, recvbuffs, count: int, datatype: int, op: int) -> None:
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrTreeAllReduce(self._h, s, r, int(count), int(datatype), int(op)), "nexrTreeAllReduce")

    def pat_reduce_scatter(self, sendbuffs, recvbuffs, recvcount: int, datatype: int, op: int) -> None:
        """ncclReduceScatter with NCCL_ALGO_PAT (SIMPLE)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrPatReduceScatter(self._h, s, r, int(recvcount), int(datatype), int(op)),
               "nexrPatReduceScatter")

    def pat_all_gather(self, sendbuffs, recvbuffs, sendcount: int, datatype: int) -> None:
        """ncclAllGather with NCCL_ALGO_PAT (SIMPLE)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        _check(ring_lib().nexrPatAllGather(self._h, s, r, int(sendcount), int(datatype)), "nexrPatAllGather")

    def send_recv(self, sendbuffs, send_peers, recvbuffs, recv_peers, nbytes: int) -> None:
        """ncclSend/ncclRecv of every rank in one group: rank r sends nbytes of sendbuffs[r] to
        send_peers[r] and receives nbytes from recv_peers[r] into recvbuffs[r] (-1: none)."""
        s, r = self._arrays(sendbuffs, recvbuffs)
        sp = (ctypes.c_int * self.n_ranks)(*[int(v) for v in send_peers])
        rp = (ctypes.c_int * self.n_ranks)(*[int(v) for v in recv_peers])
        _check(ring_lib().nexrSendRecv(self._h, s, sp, r, rp, int(nbytes)), "nexrSendRecv")

    def tree_topology(self, rank: int):
        """(up, [down...]) of `rank` in this communicator's tree (-1 = none)."""
        up = ctypes.c_int()
        down = (ctypes.c_int * 3)()
        _check(ring_lib().nexrTreeTopology(self._h, int(rank), ctypes.byref(up), down), "nexrTreeTopology")
        return up.value, [d for d in down if d >= 0]

    def close(self) -> None:
        if self._h:
            ring_lib().nexrRingCommDestroy(self._h)
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
                 protocol: int = PROTO_SIMPLE, timeout_ms: int = 0):
        self._name = shm_name.encode()
        cfg = PeerRingConfig(n_ranks, rank, device, buff_bytes, protocol, timeout_ms, self._name)
        h = ctypes.c_void_p()
        _check(ring_lib().nexrPeerRingCommCreate(ctypes.byref(h), ctypes.byref(cfg)), "nexrPeerRingCommCreate")
        self._h = h
        self.n_ranks, self.rank = n_ranks, rank

    def all_reduce(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int) -> None:
        _check(ring_lib().nexrPeerRingAllReduce(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                                int(datatype), int(op)), "nexrPeerRingAllReduce")

    def all_reduce_resident(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int) -> None:
        """This rank's part of the all-reduce as one device-resident launch (nexrPeerRingAllReduceResident)."""
        _check(ring_lib().nexrPeerRingAllReduceResident(self._h, int(sendbuff) or None, int(recvbuff) or None,
                                                        int(count), int(datatype), int(op)),
               "nexrPeerRingAllReduceResident")

    def reduce_scatter(self, sendbuff: int, recvbuff: int, recvcount: int, datatype: int, op: int) -> None:
        _check(ring_lib().nexrPeerRingReduceScatter(self._h, int(sendbuff) or None, int(recvbuff) or None,
                                                    int(recvcount), int(datatype), int(op)), "nexrPeerRingReduceScatter")

    def all_gather(self, sendbuff: int, recvbuff: int, sendcount: int, datatype: int) -> None:
        _check(ring_lib().nexrPeerRingAllGather(self._h, int(sendbuff) or None, int(recvbuff) or None, int(sendcount),
                                                int(datatype)), "nexrPeerRingAllGather")

    def reduce(self, sendbuff: int, recvbuff: int, count: int, datatype: int, op: int, root: int) -> None:
        _check(ring_lib().nexrPeerRingReduce(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                             int(datatype), int(op), int(root)), "nexrPeerRingReduce")

    def pat_reduce_scatter(self, sendbuff: int, recvbuff: int, recvcount: int, datatype: int, op: int) -> None:
        _check(ring_lib().nexrPeerPatReduceScatter(self._h, int(sendbuff) or None, int(recvbuff) or None,
                                                   int(recvcount), int(datatype), int(op)), "nexrPeerPatReduceScatter")

    def pat_all_gather(self, sendbuff: int, recvbuff: int, sendcount: int, datatype: int) -> None:
        _check(ring_lib().nexrPeerPatAllGather(self._h, int(sendbuff) or None, int(recvbuff) or None, int(sendcount),
                                               int(datatype)), "nexrPeerPatAllGather")

    def send_recv(self, sendbuff: int, send_peer: int, recvbuff: int, recv_peer: int, nbytes: int) -> None:
        _check(ring_lib().nexrPeerSendRecv(self._h, int(sendbuff) or None, int(send_peer), int(recvbuff) or None,
                                           int(recv_peer), int(nbytes)), "nexrPeerSendRecv")

    def broadcast(self, sendbuff: int, recvbuff: int, count: int, datatype: int, root: int) -> None:
        _check(ring_lib().nexrPeerRingBroadcast(self._h, int(sendbuff) or None, int(recvbuff) or None, int(count),
                                                int(datatype), int(root)), "nexrPeerRingBroadcast")

    def close(self) -> None:
        if self._h:
            ring_lib().nexrRingCommDestroy(self._h)
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
