"""Child process of tests/test_host_paths_gpu.py: with the host-path knobs set in its environment
(NEXR_HOST_COPY_THREADS, NEXR_HOST_MT_MIN_BYTES, NEXR_HOST_MT_CHUNK_BYTES, NEXR_HOST_CHUNK_BYTES — read
once by the library), run nexrReduceCopyHost on pageable, pinned and mixed host buffers and compare
every output with the oracle. argv[1] names the path the knobs select, for the report."""
import importlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402
import oracle  # noqa: E402


def concurrent(nexr) -> int:
    """Eight host threads at once, each with its own pageable buffers: every call checks a staging
    ring out of the pool and returns it, so the pool ends with at most one ring per concurrent call."""
    import threading
    n = 2_000_003
    srcs = mg.gen_inputs(mg.F32, 3, n, 777, special=True)
    exp = oracle.reduce_copy(srcs, 1, mg.F32, mg.SUM, threads=8)[0]
    errors = []

    def call(t):
        try:
            torch.cuda.set_device(0)
            mine = [s.copy() for s in srcs]
            for _ in range(3):
                d = np.zeros_like(srcs[0])
                nexr.reduce_copy_ptrs([m.ctypes.data for m in mine], [d.ctypes.data], n, mg.F32, mg.SUM, host=True)
                if mg.canon_bytes(mg.F32, d) != mg.canon_bytes(mg.F32, exp):
                    errors.append(f"thread {t}: mismatch")
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append(repr(e))

    ths = [threading.Thread(target=call, args=(t,)) for t in range(8)]
    [t.start() for t in ths]
    [t.join(timeout=120) for t in ths]
    if any(t.is_alive() for t in ths) or errors:
        print("CONCURRENT FAILURE", errors[:3], flush=True)
        return 1
    streams, rings = nexr.pool_stats()
    if rings > 8:
        print(f"POOL: {rings} rings for 8 concurrent callers", flush=True)
        return 1
    print("host-path ok concurrent", (streams, rings), flush=True)
    return 0


def main() -> int:
    nexr = importlib.import_module("nex-nccl_amd")
    if len(sys.argv) > 2 and sys.argv[2] == "concurrent":
        return concurrent(nexr)
    # (datatype, op, K, M, n, pinned mask over [srcs..., dsts...], in place on src0)
    cases = [(mg.F32, mg.SUM, 2, 1, 3_000_017, 0, False), (mg.BF16, mg.SUM, 8, 1, 1_000_003, 0, False),
             (mg.I8, mg.MINMAX, 4, 2, 2_000_001, 0b000010, False), (mg.F16, mg.PROD, 3, 1, 777_777, 0b0101, False),
             (mg.U64, mg.SUM, 5, 3, 300_001, 0b10000001, False), (mg.I32, mg.SUMPOSTDIV, 2, 1, 1_234_567, 0, True),
             (mg.F64, mg.MINMAX, 1, 2, 99_999, 0b100, False), (mg.U8, mg.PREMULSUM, 3, 1, 5_000_011, 0b1000, True)]
    for dt, op, k, m, n, mask, inplace in cases:
        srcs = mg.gen_inputs(dt, k, n, 5151 + dt + k, special=True)
        arg = mg.minmax_arg(dt, dt != mg.U64) if op == mg.MINMAX else 0
        pre = None
        if op == mg.SUMPOSTDIV:
            arg = (3 << 1) | 1
        if op == mg.PREMULSUM:
            pre = [3] * k
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, pre_op_args=pre, post_op=op == mg.SUMPOSTDIV, threads=8)[0]
        keep, sp, dp, outs = [], [], [], []
        for i in range(k + (0 if inplace else m)):
            if mask >> i & 1:  # pinned: a page-locked byte tensor holding the buffer
                raw = (srcs[i].copy() if i < k else np.zeros_like(srcs[0])).view(np.uint8)
                t = torch.from_numpy(raw).pin_memory()
                keep.append(t)
                ptr, view = t.data_ptr(), (lambda t=t, dtp=srcs[0].dtype: t.numpy().view(dtp))
            else:
                a = srcs[i].copy() if i < k else np.zeros_like(srcs[0])
                keep.append(a)
                ptr, view = a.ctypes.data, (lambda a=a: a)
            (sp if i < k else dp).append(ptr)
            if i >= k:
                outs.append(view)
        if inplace:
            dtp = srcs[0].dtype
            dp, outs = [sp[0]], [(lambda v=keep[0]: v.numpy().view(dtp) if hasattr(v, "numpy") else v)]
        nexr.reduce_copy_ptrs(sp, dp, n, dt, op, arg, pre, op == mg.SUMPOSTDIV, host=True)
        for o in outs:
            if mg.canon_bytes(dt, o()) != mg.canon_bytes(dt, exp):
                print(f"MISMATCH dt={dt} op={op} k={k} m={m} n={n} mask={mask:b} inplace={inplace}", flush=True)
                return 1
    streams, rings = nexr.pool_stats()
    if rings > 1:  # sequential calls reuse one ring of the path (grown in place), never one per call
        print(f"POOL: {rings} staging rings created over {len(cases)} sequential calls", flush=True)
        return 1
    print("host-path ok", sys.argv[1] if len(sys.argv) > 1 else "", (streams, rings), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
