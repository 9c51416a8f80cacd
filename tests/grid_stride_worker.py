"""Child process of tests/test_grid_stride_gpu.py: with NEXR_GRID / NEXR_POLICY set in its
environment (read once by the library), run reduce-copies whose one-shot grid would be far larger
than the forced grid, so every workgroup strides over many trips, and compare with the oracle."""
import importlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, "golden")]

import torch  # noqa: E402

import make_golden as mg  # noqa: E402
import oracle  # noqa: E402


def main() -> int:
    nexr = importlib.import_module("nex-nccl_amd")
    cases = [(mg.F32, mg.SUM, 2, 1, 3_000_017), (mg.BF16, mg.SUM, 8, 1, 1_000_003), (mg.I8, mg.MINMAX, 4, 2, 2_000_001),
             (mg.F16, mg.PROD, 3, 1, 777_777), (mg.U64, mg.SUM, 5, 3, 300_001)]
    for dt, op, k, m, n in cases:
        srcs = mg.gen_inputs(dt, k, n, 4242 + dt, special=True)
        arg = mg.minmax_arg(dt, True) if op == mg.MINMAX else 0
        exp = oracle.reduce_copy(srcs, 1, dt, op, arg, threads=8)[0]
        ds = [torch.from_numpy(s.copy()).cuda() for s in srcs]
        out = [torch.zeros_like(ds[0]) for _ in range(m)]
        torch.cuda.synchronize()
        nexr.reduce_copy_ptrs([t.data_ptr() for t in ds], [t.data_ptr() for t in out], n, dt, op, arg)
        torch.cuda.synchronize()
        for o in out:
            if mg.canon_bytes(dt, o.cpu().numpy()) != mg.canon_bytes(dt, exp):
                print(f"MISMATCH dt={dt} op={op} k={k} n={n}", flush=True)
                return 1
    print("grid-stride ok", os.environ.get("NEXR_GRID"), os.environ.get("NEXR_POLICY"), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
