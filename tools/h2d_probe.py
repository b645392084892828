"""Host<->device copy rates on the GPU box: pageable vs
pinned, 1.6 GB (one C3 table).  python tools/h2d_probe.py"""
import time

import torch

n = 200_000_000  # int64 cells = 1.6 GB
dev = torch.device("cuda", 0)
d = torch.empty(n, dtype=torch.int64, device=dev)
for pinned in (False, True):
    h = torch.empty(n, dtype=torch.int64, pin_memory=pinned)
    h.fill_(1)
    for direction in ("H2D", "D2H"):
        for rep in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if direction == "H2D":
                d.copy_(h, non_blocking=pinned)
            else:
                h.copy_(d, non_blocking=pinned)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        print(f"{'pinned' if pinned else 'pageable':8s} {direction}: {n * 8 / dt / 1e9:6.1f} GB/s", flush=True)
    del h
t0 = time.perf_counter()
h = torch.empty(n, dtype=torch.int64)
h.fill_(1)
torch.cuda.synchronize()
t1 = time.perf_counter()
torch.cuda.cudart().cudaHostRegister(h.data_ptr(), n * 8, 0)
t2 = time.perf_counter()
d.copy_(h, non_blocking=True)
torch.cuda.synchronize()
t3 = time.perf_counter()
torch.cuda.cudart().cudaHostUnregister(h.data_ptr())
print(f"hostRegister 1.6 GB: {1e3 * (t2 - t1):.1f} ms, then H2D {n * 8 / (t3 - t2) / 1e9:.1f} GB/s", flush=True)
