"""Multi-GPU sort-merge-join: one process per GPU, range partition on the join
key + one all-to-all over RCCL/xGMI.

The reference partitions rows over DPUs and merges sorted runs through the
host in ceil(log2 D) rounds (app.c:155-218, :412-547), then splits the join
with host binary searches (app.c:585-633).  Here every rank starts with a
contiguous slice of R and of S (rank order = input order) and:

  1. splitters: every rank samples keys of its slices, one all_gather, and
     the same W-1 key splitters are chosen everywhere (key-only splitters:
     one key never spans two ranks);
  2. per table: a stable select + bucket scatter (one onesweep pass with the
     bucket as the digit), an all_to_all of the W bucket counts and one
     all_to_all_single of the rows -- received chunks land in SOURCE-RANK
     order, so equal keys keep their global input order;
  3. the fused local pipeline (smj_dev_sort_merge_join: MSD sample sort of
     the received R and S slices + zip join) with no select -- the partition
     step already applied the WHERE clause.

Concatenating the per-rank outputs in rank order is exactly cpu_app.c's
result (stable sort + zip join are per-key operations on disjoint key ranges).
The local operators come from an `ops` object: HipOps (the product path) or,
in the gloo CPU tests only, an oracle-backed stand-in.
"""
import torch
import torch.distributed as dist

from . import ops as hip_ops

INT64_MAX = (1 << 63) - 1


class HipOps:
    """The product operators: HIP kernels behind libsmj_hip.so."""
    sort_merge_join = staticmethod(hip_ops.sort_merge_join)
    partition_count = staticmethod(hip_ops.partition_count)
    partition_scatter = staticmethod(hip_ops.partition_scatter)


def _sample_keys(table, key_col, samples):
    n = table.shape[0]
    if n == 0:
        return table.new_empty((0,))
    idx = torch.linspace(0, n - 1, min(samples, n), device=table.device).round().long()
    return table[idx, key_col].contiguous()


def _wire_device(t, group=None):
    """Where collective buffers live: the tensor's own device under RCCL; the
    host under gloo (which moves CPU tensors only) -- used by the CPU tests and
    by the 2-rank-on-one-GPU test, never by the RCCL product path."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return t.device


def choose_splitters(tables_and_keys, world, group=None, samples=4096):
    """W-1 sorted key splitters, identical on every rank (one all_gather)."""
    local = torch.cat([_sample_keys(t, k, samples) for t, k in tables_and_keys])
    home = local.device
    dev = _wire_device(local, group)
    local = local.to(dev)
    # fixed-size exchange: pad with INT64_MAX and a count
    cnt = torch.tensor([local.numel()], dtype=torch.int64, device=dev)
    cap = len(tables_and_keys) * samples
    buf = torch.full((cap,), INT64_MAX, dtype=torch.int64, device=dev)
    buf[: local.numel()] = local
    all_cnt = [torch.empty_like(cnt) for _ in range(world)]
    all_buf = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(all_cnt, cnt, group=group)
    dist.all_gather(all_buf, buf, group=group)
    keys = torch.cat([b[: int(c.item())] for b, c in zip(all_buf, all_cnt)])
    if keys.numel() == 0:
        return torch.zeros(world - 1, dtype=torch.int64, device=home)
    keys = torch.sort(keys).values
    L = keys.numel()
    pos = torch.tensor([max((i + 1) * L // world - 1, 0) for i in range(world - 1)], device=dev)
    return keys[pos].contiguous().to(home)


def exchange_rows(send, counts, group=None):
    """all_to_all_single of bucket-contiguous rows; returns rows received in
    source-rank order."""
    home = send.device
    dev = _wire_device(send, group)
    send = send.to(dev)
    world = len(counts)
    send_counts = torch.tensor(counts, dtype=torch.int64, device=dev)
    recv_counts = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    rc = [int(x) for x in recv_counts.tolist()]
    recv = torch.empty((sum(rc), send.shape[1]), dtype=send.dtype, device=dev)
    dist.all_to_all_single(recv, send.contiguous(), output_split_sizes=rc, input_split_sizes=list(counts),
                           group=group)
    return recv.to(home)


def sort_merge_join(R, S, select=(0, 5000, 0, 5000), keys=(0, 0), group=None, ops=None, samples=4096,
                    timings=None):
    """The distributed pipeline; returns this rank's slice of the result (the
    global result is the concatenation over ranks in rank order)."""
    ops = ops or HipOps
    sc1, sv1, sc2, sv2 = select
    k1, k2 = keys
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if world == 1:
        return ops.sort_merge_join(R, S, k1, k2, (sc1, sv1), (sc2, sv2))[2]

    spl = choose_splitters([(R, k1), (S, k2)], world, group, samples)
    local = []
    for T, key, sc, sv in ((R, k1, sc1, sv1), (S, k2, sc2, sv2)):
        counts, _ = ops.partition_count(T, spl, key, sc, sv)
        send = ops.partition_scatter(T, spl, counts, key, sc, sv)
        local.append(exchange_rows(send, counts, group))
        del send
    return ops.sort_merge_join(local[0], local[1], k1, k2, None, None)[2]
