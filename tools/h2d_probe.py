"""PCIe probe: copy-engine H2D / D2H rates alone and together, and the zero-copy kernel path
(nexrReduceCopy reading/writing pinned host memory directly), for the C2 byte mix."""
import importlib, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
nexr = importlib.import_module("nex-nccl_amd")
MB = 1 << 20
n_bytes = 256 * MB
hs = [torch.empty(n_bytes, dtype=torch.uint8).pin_memory() for _ in range(3)]
for h in hs:
    h.random_(0, 255)
ds = [torch.empty(n_bytes, dtype=torch.uint8, device="cuda") for _ in range(3)]
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

def t(fn, reps=3):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps

def h2d2():
    with torch.cuda.stream(s1):
        ds[0].copy_(hs[0], non_blocking=True); ds[1].copy_(hs[1], non_blocking=True)
def d2h1():
    with torch.cuda.stream(s2):
        hs[2].copy_(ds[2], non_blocking=True)
def both():
    h2d2(); d2h1()
def h2d2_two_streams():
    with torch.cuda.stream(s1):
        ds[0].copy_(hs[0], non_blocking=True)
    with torch.cuda.stream(s2):
        ds[1].copy_(hs[1], non_blocking=True)
a = t(h2d2); print(f"H2D 512 MiB one stream      {a*1e3:7.2f} ms {512*MB/a/1e9:6.1f} GB/s")
a = t(h2d2_two_streams); print(f"H2D 2x256 MiB two streams   {a*1e3:7.2f} ms {512*MB/a/1e9:6.1f} GB/s")
a = t(d2h1); print(f"D2H 256 MiB                 {a*1e3:7.2f} ms {256*MB/a/1e9:6.1f} GB/s")
a = t(both); print(f"H2D 512 || D2H 256          {a*1e3:7.2f} ms {768*MB/a/1e9:6.1f} GB/s (bytes moved)")
n = n_bytes // 4
hs_f = [h.view(torch.float32) for h in hs]
for i in range(2):
    hs_f[i].uniform_(-1, 1)
def zc():
    nexr.reduce_copy_ptrs([hs[0].data_ptr(), hs[1].data_ptr()], [hs[2].data_ptr()], n, 7, 0,
                          stream=torch.cuda.current_stream().cuda_stream)
a = t(zc); print(f"zero-copy reduce K=2 M=1      {a*1e3:7.2f} ms {768*MB/a/1e9:6.1f} GB/s algorithmic")
ok = torch.equal(hs_f[2], hs_f[0] + hs_f[1]); print("zero-copy correct:", ok)
def staged():
    nexr.reduce_copy_ptrs([hs[0].data_ptr(), hs[1].data_ptr()], [hs[2].data_ptr()], n, 7, 0, host=True)
a = t(staged); print(f"staged pipeline K=2 M=1       {a*1e3:7.2f} ms {768*MB/a/1e9:6.1f} GB/s algorithmic")
for pol in ("0",):
    pass
