"""Full-size parity of the distributed path on one GPU (RCCL loopback): the
joined rows of every smj.dist step equal the single-call result, bit for bit.

    python tools/loop_check.py [--workload c3|c4|c5] [--steps 3]

The single call (smj_dev_sort_merge_join, partitioned mode above 1.6e8 rows)
is itself parity-tested against the oracle (tests/test_gpu_*.py); this checks
that the range partition + RCCL exchange + per-stage pipeline reproduce it at
BASELINE sizes, on every step (the first one included)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from smj import dist as sdist  # noqa: E402
from smj import ops  # noqa: E402

SELECT = (0, 5000, 0, 5000)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--workload", default="c3", choices=["c3", "c4", "c5"])
    p.add_argument("--steps", type=int, default=3)
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    if a.workload == "c5":
        R = ops.gen_zipf(100_000_000, seed=3, domain=100_000_000, theta=0.9, device=dev)
        S = ops.gen_zipf(1_000_000_000, seed=4, domain=100_000_000, theta=0.9, device=dev)
    else:
        n = 100_000_000 if a.workload == "c3" else 1_000_000_000
        R = ops.gen_uniform(n, seed=1, key_range=3 * n, device=dev)
        S = ops.gen_uniform(n, seed=2, key_range=3 * n, device=dev)
    _, _, J0 = ops.sort_merge_join(R, S, 0, 0, (SELECT[0], SELECT[1]), (SELECT[2], SELECT[3]))
    torch.cuda.synchronize()
    print(f"{a.workload}: single call {J0.shape[0]} joined rows", flush=True)
    ok = True
    for i in range(a.steps):
        t0 = time.perf_counter()
        st = {}
        J = sdist.sort_merge_join(R, S, select=SELECT, keys=(0, 0), stats=st, loopback=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        same = J.shape == J0.shape and bool(torch.equal(J, J0))
        ok &= same
        print(f"step {i}: {J.shape[0]} rows, equal={same}, {dt * 1e3:.1f} ms, loads {st.get('loads')}", flush=True)
        del J
    dist.destroy_process_group()
    print("PASS" if ok else "FAIL", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
