"""Child process of tests/test_reduce_copy_gpu.py::test_first_one_workgroup_per_cu_launch_inside_graph_capture:
the process's FIRST launch of a kernel that reserves LDS for one workgroup per CU (fp16 K = 8 under the
nt-store policy, forced by the parent with NEXR_POLICY=3; the launch also sets the kernel's dynamic-LDS
attribute once per device) happens inside a HIP graph capture; the graph is replayed on new data and
compared with the oracle bit for bit. The worker checks the launch shape before capturing."""
import importlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(HERE, "golden")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import make_golden as mg  # noqa: E402
import oracle  # noqa: E402


def main() -> int:
    nexr = importlib.import_module("nex-nccl_amd")
    n, k = 1_000_003, 8
    ins = [torch.zeros(n, dtype=torch.float16, device="cuda") for _ in range(k)]
    out = torch.zeros(n, dtype=torch.float16, device="cuda")
    info = nexr.query_launch([t.data_ptr() for t in ins], [out.data_ptr()], n, mg.F16)
    if (info.policy, info.block, info.packsPerLane) != (3, 512, 1):
        print(f"not the one-workgroup-per-CU shape: policy {info.policy} block {info.block}")
        return 1
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        nexr.reduce_copy_ptrs([t.data_ptr() for t in ins], [out.data_ptr()], n, mg.F16, mg.SUM, 0, None, False,
                              torch.cuda.current_stream().cuda_stream)
    for rep in range(3):
        srcs = mg.gen_inputs(mg.F16, k, n, 700 + rep, special=True)
        for t, s in zip(ins, srcs):
            t.copy_(torch.from_numpy(s.view(np.float16).copy()))
        g.replay()
        torch.cuda.synchronize()
        exp = oracle.reduce_copy(srcs, 1, mg.F16, mg.SUM, 0, threads=8)[0]
        if mg.canon_bytes(mg.F16, out.cpu().numpy().view(np.uint16)) != mg.canon_bytes(mg.F16, exp):
            print(f"replay {rep}: MISMATCH")
            return 1
    print("graph replays exact")
    return 0


if __name__ == "__main__":
    sys.exit(main())
