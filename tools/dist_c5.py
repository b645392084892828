"""BASELINE C5 (|R| = 1e8, |S| = 1e9, Zipf(0.9) over 1e8 keys, seeds 3 / 4,
WHERE col0 > 5000) through the multi-GPU driver smj/dist.py with W ranks
that all share cuda:0 (the exchange staged through gloo: RCCL needs one GPU
per rank).  Reports the per-rank loads, load_max_over_mean and the joined
row count, and checks the joined row count and an order-sensitive checksum
of the concatenated rank outputs against the single-call result of the
library's partitioned mode on the same tables.

    python tools/dist_c5.py [--ranks 8] [--scale 1.0] [-o profiles/r02_dist_c5.json]
"""
import argparse
import json
import os
import socket
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

SELECT = (0, 5000, 0, 5000)


def checksum(J):
    """Order-sensitive: sum over rows of (row index + 1) * (key ^ payR ^ payS), mod 2^64."""
    if J.shape[0] == 0:
        return 0
    idx = torch.arange(1, J.shape[0] + 1, device=J.device, dtype=torch.int64)
    v = J[:, 0] ^ J[:, 1] ^ J[:, 2]
    return int((idx * v).sum().item()) & ((1 << 64) - 1)


def worker(rank, world, port, nr, ns, out):
    from smj import dist as sdist
    from smj import ops
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    r0, r1 = nr * rank // world, nr * (rank + 1) // world
    s0, s1 = ns * rank // world, ns * (rank + 1) // world
    R = ops.gen_zipf(r1 - r0, row0=r0, seed=3, domain=100_000_000, theta=0.9, device="cuda:0")
    S = ops.gen_zipf(s1 - s0, row0=s0, seed=4, domain=100_000_000, theta=0.9, device="cuda:0")
    torch.cuda.synchronize()
    dist.barrier()
    stats = {}
    t0 = time.perf_counter()
    J = sdist.sort_merge_join(R, S, select=SELECT, keys=(0, 0), stats=stats)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"rank": rank, "rows_in": stats["rows_in"], "joined": int(J.shape[0]), "seconds": dt,
           "load_max_over_mean": stats["load_max_over_mean"], "stages": stats["stages"],
           "first_key": int(J[0, 0]) if J.shape[0] else None, "last_key": int(J[-1, 0]) if J.shape[0] else None}
    # the rank outputs concatenated in rank order = the global result: checksum pieces
    idx0 = torch.tensor([J.shape[0]], dtype=torch.int64)
    counts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(counts, idx0)
    base = sum(int(c) for c in counts[:rank])
    if J.shape[0]:
        idx = torch.arange(base + 1, base + 1 + J.shape[0], device=J.device, dtype=torch.int64)
        res["checksum_part"] = int((idx * (J[:, 0] ^ J[:, 1] ^ J[:, 2])).sum().item()) & ((1 << 64) - 1)
    else:
        res["checksum_part"] = 0
    with open(os.path.join(out, f"rank{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of C5's row counts")
    ap.add_argument("-o", default=os.path.join(REPO, "gpurun_out", "dist_c5.json"))
    a = ap.parse_args()
    nr, ns = int(1e8 * a.scale), int(1e9 * a.scale)
    tmp = os.path.join(REPO, "gpurun_out", "dist_c5_ranks")
    os.makedirs(tmp, exist_ok=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    t0 = time.perf_counter()
    mp.spawn(worker, args=(a.ranks, port, nr, ns, tmp), nprocs=a.ranks, join=True)
    wall = time.perf_counter() - t0
    ranks = [json.load(open(os.path.join(tmp, f"rank{r}.json"))) for r in range(a.ranks)]
    joined = sum(r["joined"] for r in ranks)
    csum = sum(r["checksum_part"] for r in ranks) & ((1 << 64) - 1)
    print(f"dist: {a.ranks} ranks, joined {joined}, load_max_over_mean {ranks[0]['load_max_over_mean']:.4f}",
          flush=True)
    # the single-call reference on the same tables (partitioned mode, one process)
    from smj import ops
    R = ops.gen_zipf(nr, seed=3, domain=100_000_000, theta=0.9, device="cuda:0")
    S = ops.gen_zipf(ns, seed=4, domain=100_000_000, theta=0.9, device="cuda:0")
    _, _, J = ops.sort_merge_join(R, S, 0, 0, (0, 5000), (0, 5000))
    ref_joined, ref_csum = int(J.shape[0]), checksum(J)
    out = {"workload": f"C5 x {a.scale}: |R| = {nr}, |S| = {ns}, Zipf(0.9) over 1e8 keys, seeds 3 / 4, "
                       f"WHERE col0 > 5000, {a.ranks} ranks of smj/dist.py sharing one MI355X (gloo exchange)",
           "ranks": ranks, "joined": joined, "checksum": csum,
           "single_call_joined": ref_joined, "single_call_checksum": ref_csum,
           "equal_to_single_call": joined == ref_joined and csum == ref_csum,
           "load_max_over_mean": ranks[0]["load_max_over_mean"],
           "rows_per_rank": [r["rows_in"][0] + r["rows_in"][1] for r in ranks], "wall_s": wall}
    with open(a.o, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "ranks"}), flush=True)
    assert out["equal_to_single_call"], "distributed result differs from the single-call result"


if __name__ == "__main__":
    main()
