import importlib, sys, torch
sys.path.insert(0, "/root/repo")
nexr = importlib.import_module("nex-nccl_amd")
s = torch.cuda.current_stream()
n = 64 << 20  # fp32 elements = 256 MiB
rows = []
for name, (oa, ob, oo) in {"aligned": (0, 0, 0), "shared phase 4B": (4, 4, 4), "src1 +4B": (0, 4, 0),
                           "dst +4B": (0, 0, 4), "src1 +1B u8": (0, 1, 0)}.items():
    dt = 1 if "u8" in name else 7
    esz = 1 if dt == 1 else 4
    nn = n * 4 // esz
    sets = []
    for _ in range(3):
        a = torch.empty(nn * esz + 64, dtype=torch.uint8, device="cuda")
        b = torch.empty(nn * esz + 64, dtype=torch.uint8, device="cuda")
        o = torch.empty(nn * esz + 64, dtype=torch.uint8, device="cuda")
        a.random_(0, 100); b.random_(0, 100)
        sets.append((a.data_ptr() + oa, b.data_ptr() + ob, o.data_ptr() + oo, a, b, o))
    info = nexr.query_launch([sets[0][0], sets[0][1]], [sets[0][2]], nn, dt)
    def launch(i):
        x = sets[i % 3]
        nexr.reduce_copy_ptrs([x[0], x[1]], [x[2]], nn, dt, 0, 0, None, False, s.cuda_stream)
    for i in range(3): launch(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for i in range(20): launch(i)
    e1.record(s); e1.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"{name:<18} grid={info.grid} block={info.block} {us:8.1f} us {3*nn*esz/us/1e3:8.1f} GB/s", flush=True)
    del sets; torch.cuda.empty_cache()
