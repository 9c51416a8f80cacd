"""TEST INFRASTRUCTURE ONLY — the reference's PAT ReduceScatter / AllGather, restated in Python.

PAT (NCCL_ALGO_PAT, "Parallel Aggregated Trees") is the third algorithm that calls reduceCopy for
ncclReduceScatter and ncclAllGather. A compute thread turns the collective into a stream of
ncclPatStep records (PatRSAlgorithm / PatAGAlgorithm, reference src/device/collectives.h:433-906);
parallelFactor worker groups consume them in lock-step batches (reduce_scatter.h:80-139,
all_gather.h:113-172, patBarrier over all NCCL_PAT_NWORKERS threads, prims_simple.h:76-78), each
running patReduce (prims_simple.h:992-1088) or patCopy (:1090-1183) with one reduceCopy per step.

This module restates the two generators from the reference text and runs every rank's batches on
an idealised machine: all ranks in one process, FIFOs without a slot limit (indexed by absolute
step, so no credits), data folded with the C oracle's reduce_copy. It is independent of
nex-nccl_amd/csrc/nexr_ring.cpp, whose 8-slot FIFOs, credits and host threads it checks.
"""
from __future__ import annotations

import numpy as np

from . import reduce_copy

NCCL_STEPS = 8             # src/include/device.h:649
PAT_NWORKERS = 512         # NCCL_PAT_NWORKERS, collectives.h:402
MAX_PARALLEL = PAT_NWORKERS // 32


def _log2_up(n):
    p = 0
    while (1 << p) < n:
        p += 1
    return p


def _ffs(i, mx):
    """firstBitSet (collectives.h:471-479)."""
    return (i & -i).bit_length() - 1 if i else mx


def chunk_count(n_ranks, count, esz, step_bytes, all_gather):
    """calcCollChunking for PAT on one channel (enqueue.cc:1993-1996, :2048-2051, grain :2062)."""
    chunk = step_bytes
    n_bytes = n_ranks * count * esz
    while chunk * (32 if all_gather else 16) > n_bytes and chunk > 65536:
        chunk //= 2
    return (chunk // 512 * 512) // esz


class _Geometry:
    def __init__(self, step_size, step_depth, max_pf, channel_size, esz, nranks):
        self.parallel_factor = max_pf
        self.agg_delta = self.nr_pow2 = 1 << _log2_up(nranks)
        self.agg_factor = 1
        while step_size // (channel_size * esz * self.agg_factor) >= 2 and self.agg_factor < nranks // 2:
            self.agg_factor *= 2
            self.agg_delta //= 2
        self.post_freq = self.agg_factor
        self.parallel_factor = min(self.parallel_factor, self.post_freq)
        d = step_depth
        while d > 1 and self.agg_factor < nranks // 2:
            d //= 2
            self.agg_factor *= 2
            self.agg_delta //= 2


def _step():
    return dict(recvDim=-1, sendDim=-1, recvOffset=-1, sendOffset=-1, stepOffset=0, postRecv=0, postSend=0,
                nelem=0, last=0, skipped=0, inpIx=0, outIx=0)


class RsPlan(_Geometry):
    """PatRSAlgorithm (collectives.h:434-684) over the channel part [offset, end) of `count`."""

    def __init__(self, chunk, esz, count, rank, nranks, offset=0, end=None):
        end = count if end is None else end
        super().__init__(chunk * esz, NCCL_STEPS, MAX_PARALLEL, end - offset, esz, nranks)
        self.offset, self.end, self.count, self.chunk = offset, end, count, chunk
        self.rank, self.n = rank, nranks
        self._reset()

    @staticmethod
    def _mirror_invert(i, mx):
        ret, mask, imask = 0, 1, mx // 2
        while mask < mx:
            if not i & mask:
                ret += imask
            mask <<= 1
            imask >>= 1
        return ret

    @staticmethod
    def _new_peer(i, pow2):
        return bin((i ^ (pow2 - 1)) + 1).count("1") == 1

    def _reset_a(self):
        self.a = 0
        self.send_skipped = self.step_offset = 0
        self.last_a = self.agg_factor
        if self.phase >= 2:
            self.last_a //= 2 * self.scale
        if self.phase == 4:
            self.last_a = 1

    def _reset(self):
        self.nelem = min(self.chunk, self.end - self.offset)
        self.phase, self.scale, self.as_ = 0, 1, self.agg_delta - 1
        self._reset_a()

    def next(self):
        ps = _step()
        ps["nelem"] = self.nelem
        ps["outIx"] = self.offset
        ps["stepOffset"] = self.step_offset
        a, last_a, pf, n, nel = self.a, self.last_a, self.post_freq, self.n, self.nelem
        flush = (a % pf) + 1 >= pf or a == last_a - 1
        skip = False
        if a >= last_a:
            skip = True
        elif self.phase == 0:
            s = self._mirror_invert(a, last_a) * self.agg_delta + self.as_
            skip = s >= n
            ps.update(inpIx=((self.rank + s) % n) * self.count + self.offset, recvDim=-1, sendDim=0, outIx=0,
                      recvOffset=-1, sendOffset=(a % pf) * nel, postSend=int(flush), postRecv=0)
        elif self.phase == 1:
            s = self._mirror_invert(a, last_a) * self.agg_delta + self.as_
            skip = s >= n
            rd = _ffs(s, self.nr_pow2)
            ps.update(recvDim=rd, sendOffset=(a % pf) * nel, recvOffset=(a % pf) * nel,
                      postSend=int(rd == 0 and flush), postRecv=int(flush))
            s -= 1 << rd
            ps["inpIx"] = ((self.rank + n + s) % n) * self.count + self.offset
            ps["sendDim"] = _ffs(s, self.nr_pow2) if s else -1
            if ps["sendDim"] == -1:
                ps["sendOffset"] = -1
            elif self.as_ - (1 << rd) == 0:
                if self._new_peer(a, self.agg_factor):
                    self.send_skipped = a
                    ps["stepOffset"] = self.step_offset = 0
                ps["sendOffset"] = ((a - self.send_skipped) % pf) * nel
            if s < n and skip:
                ps.update(recvDim=-1, recvOffset=-1, postRecv=0)
                skip = False
            if rd > 0 and ((a - self.send_skipped) % pf) + 1 >= pf and not skip:
                self.step_offset += 1
        elif self.phase == 2:
            s = (2 * self._mirror_invert(a, last_a) + 1) * self.scale * self.agg_delta + 1
            ps["postRecv"] = 0
            skip = s >= n
            ps["recvDim"] = 0
            ps["postSend"] = int(a == last_a - 1)
            s -= 1
            if s < n and skip:
                ps.update(recvDim=-1, recvOffset=-1)
                skip = False
            elif not skip:
                fo = a + self.agg_factor - self.agg_factor // self.scale
                ps["postRecv"] |= int((fo + 1) % pf == 0)
                ps["recvOffset"] = (fo % pf) * nel
            ps["inpIx"] = ((self.rank + n + s) % n) * self.count + self.offset
            ps["sendDim"] = _ffs(s, self.nr_pow2) if s else -1
            ps["postSend"] |= int((a + 1) % pf == 0)
            ps["sendOffset"] = (a % pf) * nel
        elif self.phase == 3:
            s = (2 * self._mirror_invert(a, last_a) + 1) * self.scale * self.agg_delta
            ps["postRecv"] = int(a == last_a - 1)
            skip = s >= n
            rd = _ffs(s, self.nr_pow2)
            ps.update(recvDim=rd, postSend=0)
            s -= 1 << rd
            ps["postRecv"] |= int((a + 1) % pf == 0)
            ps["recvOffset"] = (a % pf) * nel
            ps["inpIx"] = ((self.rank + n + s) % n) * self.count + self.offset
            ps["sendDim"] = _ffs(s, self.nr_pow2) if s else -1
            if s < n and skip:
                ps.update(recvDim=-1, recvOffset=-1, postRecv=0)
                skip = False
            if self._new_peer(a, self.agg_factor // (2 * self.scale)):
                self.send_skipped = a
                ps["stepOffset"] = self.step_offset = 0
            fo = a - self.send_skipped
            if (fo % pf) + 1 >= pf and not skip:
                self.step_offset += 1
            ps["sendOffset"] = (fo % pf) * nel if ps["sendDim"] >= 0 else -1
        elif self.phase == 4:
            ps.update(recvDim=0, sendDim=-1, inpIx=self.rank * self.count + self.offset,
                      recvOffset=((self.agg_factor - 1) % pf) * nel, sendOffset=-1, postRecv=1, postSend=0)
            self.offset += self.chunk
        self.a += 1
        if self.a >= self.last_a and self.a >= self.parallel_factor:
            p = self.phase
            if p == 1:
                self.as_ -= 1
            if p == 3:
                self.scale *= 2
            if p == 0:
                self.phase = (2 if self.agg_factor > 1 else 4) if self.as_ == 1 else 1
            elif p == 1:
                self.phase = 0 if self.as_ % 2 == 1 else 1
            elif p == 2:
                self.phase = 3
            elif p == 3:
                self.phase = 2 if self.scale < self.agg_factor else 4
            else:
                self.phase = 5
            if p == 4:
                if self.offset >= self.end:
                    ps["last"] = 2
                else:
                    self._reset()
            else:
                self._reset_a()
        elif self.phase == 4 and self.offset >= self.end:
            ps["last"] = 1
        ps["skipped"] = int(skip)
        return ps


class AgPlan(_Geometry):
    """PatAGAlgorithm (collectives.h:687-906) over the channel part [offset, end) of `count`."""

    def __init__(self, chunk, esz, count, rank, nranks, offset=0, end=None):
        end = count if end is None else end
        super().__init__(chunk * esz, NCCL_STEPS, MAX_PARALLEL, end - offset, esz, nranks)
        self.offset, self.end, self.count, self.chunk = offset, end, count, chunk
        self.rank, self.n = rank, nranks
        self.as_dim = _log2_up(self.agg_delta)
        self._reset()

    def _reset_a(self):
        self.a = 0
        self.last_a = self.agg_factor
        if self.phase >= 2:
            self.last_a //= 2 * self.scale

    def _reset(self):
        self.nelem = min(self.chunk, self.end - self.offset)
        self.scale = self.agg_factor // 2
        self.phase = 2 if self.scale else 1
        self.v = 0
        self.bit_count = [self.as_dim - i for i in range(self.as_dim)]
        self.bit_zero_step = [1] * self.as_dim
        self.as_ = self._next_as()
        self._reset_a()

    def _next_as(self):
        for d in range(self.as_dim):
            p = 1 << d
            self.bit_count[d] -= 1
            if self.bit_count[d] == 0:
                self.v ^= p
                self.bit_count[d] = p
                if not self.v & p:
                    self.bit_count[d] += _ffs(self.bit_zero_step[d], self.as_dim) - 1
                    if self.bit_count[d] == 0:
                        self.v ^= p
                        self.bit_count[d] = p
                    self.bit_zero_step[d] += 1
        return self.v

    def next(self):
        ps = _step()
        ps["nelem"] = self.nelem
        ps["inpIx"] = self.offset
        a, pf, n, nel, ad, as_ = self.a, self.post_freq, self.n, self.nelem, self.agg_delta, self.as_
        skip = False
        if a >= self.last_a:
            skip = True
        elif self.phase == 0:
            s = a * ad + as_
            skip = s >= n
            ps.update(outIx=((self.rank + s) % n) * self.count + self.offset, sendDim=-1, recvDim=0, inpIx=0,
                      sendOffset=-1, recvOffset=(a % pf) * nel, stepOffset=0,
                      postRecv=int(a % pf == pf - 1 or (a + 1) * ad + as_ >= n), postSend=0)
        elif self.phase == 1:
            s = a * ad + as_
            skip = s >= n
            sd = _ffs(s, self.nr_pow2)
            s -= 1 << sd
            ps.update(sendDim=sd, outIx=((self.rank + n + s) % n) * self.count + self.offset,
                      recvDim=_ffs(s, self.nr_pow2) if s else -1, sendOffset=(a % pf) * nel,
                      recvOffset=(a % pf) * nel, postSend=int(a % pf == pf - 1 or (a + 1) * ad + as_ >= n),
                      postRecv=int(sd == 0 and (a % pf == pf - 1 or (a + 1) * ad + as_ - 1 >= n)),
                      stepOffset=0 if sd == 0 else a // pf)
            if ps["recvDim"] == -1:
                ps.update(recvOffset=-1, postRecv=0)
            elif as_ - (1 << sd) == 0:
                fo = (a * ad) >> (ps["recvDim"] + 1)
                ps["recvOffset"] = (fo % pf) * nel
                ps["postRecv"] = int(sd == 0 and (fo % pf == pf - 1 or ((((fo + 1) * 2) + 1) << ps["recvDim"]) >= n))
                ps["stepOffset"] = 0 if sd == 0 else fo // pf
            if s < n and sd == 0 and skip:
                ps.update(sendDim=-1, sendOffset=-1, postSend=0)
                skip = False
        elif self.phase == 2:
            s = (2 * a + 1) * self.scale * ad
            ps["postSend"] = int(a % pf == pf - 1 or (2 * (a + 1) + 1) * self.scale * ad >= n)
            ps["postRecv"] = 0
            skip = s >= n
            sd = _ffs(s, self.nr_pow2)
            s -= 1 << sd
            ps.update(sendDim=sd, sendOffset=(a % pf) * nel, stepOffset=a // pf,
                      outIx=((self.rank + n + s) % n) * self.count + self.offset,
                      recvDim=_ffs(s, self.nr_pow2) if s else -1)
            if ps["recvDim"] == -1:
                ps["recvOffset"] = -1
            else:
                fo = (a * 2 * self.scale * ad) >> (ps["recvDim"] + 1)
                ps["recvOffset"] = (fo % pf) * nel
                ps["stepOffset"] = fo // pf
        self.a += 1
        if self.a >= self.last_a and self.a >= self.parallel_factor:
            p = self.phase
            if p == 2:
                self.scale //= 2
            if p == 2:
                self.phase = 2 if self.scale else 1
            elif p == 1:
                self.phase = 0 if self.as_ % 2 == 1 else 1
            else:
                self.phase = 1
            if p == 0 or (p == 1 and self.as_ % 2 == 0):
                self.as_ = self._next_as()
            if p == 0 and self.as_ == self.agg_delta // 2:
                self.offset += self.chunk
                if self.offset >= self.end:
                    ps["last"] = 2
                else:
                    self._reset()
            else:
                self._reset_a()
        elif (self.phase == 0 and self.as_ == 1 and self.offset + self.chunk >= self.end
              and self.a - 1 >= ((self.last_a - 1) // self.parallel_factor) * self.parallel_factor):
            ps["last"] = 1
        ps["skipped"] = int(skip)
        return ps


def schedule(reduce_scatter, n_ranks, rank, count, esz, step_bytes, offset=0, end=None):
    """Every ncclPatStep of one rank's compute thread for the part [offset, end), and parallelFactor."""
    end = count if end is None else end
    chunk = chunk_count(n_ranks, end - offset, esz, step_bytes, not reduce_scatter)
    plan = (RsPlan if reduce_scatter else AgPlan)(chunk, esz, count, rank, n_ranks, offset, end)
    ops = []
    while True:
        ops.append(plan.next())
        if ops[-1]["last"] == 2:
            return ops, plan.parallel_factor


def _simulate(reduce_scatter, inputs, outputs, esz, step_bytes, fold, n_channels=1):
    """Runs every channel's part: each channel has its own links (fresh FIFOs and counters)."""
    n = len(inputs)
    count = outputs[0].size // (1 if reduce_scatter else n)
    from .ring import channel_parts
    for _, lo, cnt in channel_parts(n_channels, count, esz, n):
        _simulate_part(reduce_scatter, inputs, outputs, esz, step_bytes, fold, lo, lo + cnt)


def _simulate_part(reduce_scatter, inputs, outputs, esz, step_bytes, fold, offset, end):
    """Runs every rank's batches; `fold(srcs, dsts)` performs one reduceCopy on numpy views."""
    n = len(inputs)
    count = outputs[0].size // (1 if reduce_scatter else n)
    step_elems = step_bytes // esz
    dt = inputs[0].dtype
    fifo = {}   # (from, to) -> {absolute step -> array of step_elems}
    tail = {}   # (from, to) -> steps published by the sender
    state = []
    for r in range(n):
        ops, pf = schedule(reduce_scatter, n, r, count, esz, step_bytes, offset, end)
        dims = [d for d in range(32) if (1 << d) < n]
        lo = {d: (r - (1 << d)) % n for d in dims}
        hi = {d: (r + (1 << d)) % n for d in dims}
        recv = {d: (lo[d], r) if reduce_scatter else (hi[d], r) for d in dims}
        send = {d: (r, hi[d]) if reduce_scatter else (r, lo[d]) for d in dims}
        state.append(dict(ops=ops, pf=pf, b=0, recv=recv, send=send, rstep={d: 0 for d in dims},
                          sstep={d: 0 for d in dims}, racc={d: 0 for d in dims}, sacc={d: 0 for d in dims}, lacc=0))

    def slot(conn, step):
        f = fifo.setdefault(conn, {})
        if step not in f:
            f[step] = np.zeros(step_elems, dtype=dt)
        return f[step]

    def ready(st, batch):
        for op in batch:
            if op["skipped"] or op["recvDim"] < 0:
                continue
            d = op["recvDim"]
            need = st["rstep"][d] + (0 if reduce_scatter else op["stepOffset"]) + 1
            if tail.get(st["recv"][d], 0) < need:
                return False
        return True

    def run_batch(r, st, batch):
        post_r, post_s, new_racc, new_sacc, new_lacc = set(), set(), {}, {}, st["lacc"]
        for op in batch:
            if op["skipped"]:
                continue
            nel = max(op["nelem"], 0)
            if reduce_scatter:
                srcs = []
                if op["recvDim"] >= 0:
                    d = op["recvDim"]
                    srcs.append(slot(st["recv"][d], st["rstep"][d])[op["recvOffset"]:op["recvOffset"] + nel])
                own = inputs[r][op["inpIx"]:op["inpIx"] + nel]
                if op["sendDim"] >= 0:
                    d = op["sendDim"]
                    s = st["sstep"][d] + op["stepOffset"]
                    dst = slot(st["send"][d], s)[op["sendOffset"]:op["sendOffset"] + nel]
                    mark = op["sendOffset"] + nel + s * step_elems
                    if st["sacc"][d] >= mark:
                        own = dst
                    new_sacc[d] = max(new_sacc.get(d, -1), mark)
                else:
                    dst = outputs[r][op["outIx"]:op["outIx"] + nel]
                    if st["lacc"] < op["outIx"] + nel:
                        new_lacc = max(new_lacc, op["outIx"] + nel)
                    else:
                        own = dst
                srcs.append(own)
                if nel:
                    fold(srcs, [dst])
            else:
                if op["recvDim"] >= 0:
                    d = op["recvDim"]
                    s = st["rstep"][d] + op["stepOffset"]
                    src = slot(st["recv"][d], s)[op["recvOffset"]:op["recvOffset"] + nel]
                    mark = op["recvOffset"] + nel + s * step_elems
                    out = outputs[r][op["outIx"]:op["outIx"] + nel] if st["racc"][d] < mark else None
                    new_racc[d] = max(new_racc.get(d, -1), mark)
                else:
                    src = inputs[r][op["inpIx"]:op["inpIx"] + nel]
                    if st["lacc"] < op["inpIx"] + nel:
                        out = outputs[r][op["outIx"]:op["outIx"] + nel]
                        new_lacc = max(new_lacc, op["inpIx"] + nel)
                    else:
                        out = None
                dsts = []
                if op["sendDim"] >= 0:
                    d = op["sendDim"]
                    dsts.append(slot(st["send"][d], st["sstep"][d])[op["sendOffset"]:op["sendOffset"] + nel])
                if out is not None and not np.shares_memory(out, src):
                    dsts.append(out)
                if nel and dsts:
                    fold([src], dsts)
            if op["postRecv"] and op["recvDim"] >= 0:
                post_r.add(op["recvDim"])
            if op["postSend"] and op["sendDim"] >= 0:
                post_s.add(op["sendDim"])
        st["lacc"] = new_lacc
        for d, v in new_racc.items():
            st["racc"][d] = max(st["racc"][d], v)
        for d, v in new_sacc.items():
            st["sacc"][d] = max(st["sacc"][d], v)
        for d in post_s:
            st["sstep"][d] += 1
            tail[st["send"][d]] = st["sstep"][d]
        for d in post_r:
            st["rstep"][d] += 1

    while True:
        progressed, done = False, True
        for r, st in enumerate(state):
            pf, ops = st["pf"], st["ops"]
            if st["b"] >= len(ops):
                continue
            done = False
            batch = ops[st["b"]:st["b"] + pf]
            if not ready(st, batch):
                continue
            run_batch(r, st, batch)
            st["b"] += pf
            progressed = True
            if any(op["last"] for op in batch):
                st["b"] = len(ops)
        if done:
            return
        if not progressed:
            raise RuntimeError("PAT schedule deadlocked")


def reduce_scatter_expected(inputs, datatype, dev_op, arg, step_bytes=(4 << 20) // NCCL_STEPS, n_channels=1):
    """Every rank's output of the PAT ncclReduceScatter (recvcount = input size / nRanks)."""
    n = len(inputs)
    esz = inputs[0].itemsize
    count = inputs[0].size // n
    outputs = [np.zeros(count, dtype=inputs[0].dtype) for _ in range(n)]

    def fold(srcs, dsts):
        # srcs = [received partial, own input or accumulator] (prims_simple.h:1028-1060)
        res = reduce_copy([np.array(s) for s in srcs], 1, datatype, dev_op, arg)[0]
        dsts[0][...] = res

    _simulate(True, inputs, outputs, esz, step_bytes, fold, n_channels)
    return outputs


def all_gather_expected(inputs, step_bytes=(4 << 20) // NCCL_STEPS, outputs=None, n_channels=1):
    """Every rank's output of the PAT ncclAllGather (inputs in place when `outputs` holds them)."""
    n = len(inputs)
    count = inputs[0].size
    if outputs is None:
        outputs = [np.zeros(count * n, dtype=inputs[0].dtype) for _ in range(n)]

    def fold(srcs, dsts):
        for d in dsts:
            d[...] = srcs[0]

    _simulate(False, inputs, outputs, inputs[0].itemsize, step_bytes, fold, n_channels)
    return outputs
