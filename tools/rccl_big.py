"""RCCL point-to-point to self (one-rank nccl group) with large messages:
does a batch of isend / irecv pairs of 0.5-6 GiB arrive intact?

    python tools/rccl_big.py
"""
import os
import sys

import torch
import torch.distributed as dist


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29551")
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    ok = True
    for sizes in ([64 << 20], [128 << 20], [200 << 20], [255 << 20], [(256 << 20) + 8], [64 << 20] * 8,
                  [300 << 20, 200 << 20], [700 << 20]):  # int64 elements: 0.5 GiB ... 5.5 GiB per message
        xs = [torch.randint(-(1 << 62), 1 << 62, (n,), dtype=torch.int64, device=dev) for n in sizes]
        ys = [torch.empty_like(x) for x in xs]
        ops = [dist.P2POp(dist.irecv, y, 0) for y in ys] + [dist.P2POp(dist.isend, x, 0) for x in xs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        torch.cuda.synchronize()
        eq = [bool(torch.equal(x, y)) for x, y in zip(xs, ys)]
        gib = [round(x.numel() * 8 / 2 ** 30, 2) for x in xs]
        print(f"messages of {gib} GiB: equal {eq}", flush=True)
        ok &= all(eq)
        del xs, ys
    dist.destroy_process_group()
    print("PASS" if ok else "FAIL", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
