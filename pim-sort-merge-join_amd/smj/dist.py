"""Multi-GPU sort-merge-join: one process per GPU, range partition on the join
key + one all-to-all over RCCL/xGMI.

The reference partitions rows over DPUs and merges sorted runs through the
host in ceil(log2 D) rounds (app.c:155-218, :412-547), then splits the join
with host binary searches (app.c:585-633).  Here every rank starts with a
contiguous slice of R and of S (rank order = input order) and:

  1. splitters: every rank samples keys of its slices, one all_gather, and
     the same W-1 sample quantiles are chosen everywhere; each distinct
     splitter key u gets a single-key bucket (u-1, u] between the open
     ranges (a heavy key is a bucket of its own);
  2. per table: a stable select + bucket scatter (one pass with the bucket as
     the digit); one all_gather of every rank's bucket counts; the same W-1
     cuts are computed everywhere over the bucket-ordered sequence (R + S
     rows balanced per rank): at a bucket edge, or inside a single-key
     bucket at an OCCURRENCE index -- the same index for R and S, so the
     zip join's pairs (occurrence i of R with occurrence i of S) stay on one
     rank; each rank then sends contiguous slices of its bucket-ordered rows
     in one all_to_all_single -- received chunks land in SOURCE-RANK order,
     so equal keys keep their global input order;
  3. the fused local pipeline (smj_dev_sort_merge_join: MSD sample sort of
     the received R and S slices + zip join) with no select -- the partition
     step already applied the WHERE clause.

Stages (exchange / compute overlap): each rank's key range is cut into K
consecutive sub-ranges (W*K balanced segments instead of W).  Segment
d*K + k goes to rank d in stage k.  Stage k's rows travel as one batch of
point-to-point sends / receives (RCCL group over xGMI; received chunks
placed in source-rank order) while the local pipeline sorts and joins stage
k - 1's sub-range: sort and zip join are per-key operations, so the stage
outputs concatenated in stage order are the rank's slice of the result.
The cuts use R's exact counts and S's sample estimate, so they are known once
R is partitioned, and R's stage-0 rows travel while S is being partitioned (on
a side stream, so the transfers are not ordered behind it).

Concatenating the per-rank outputs in rank order is exactly cpu_app.c's
result (stable sort + zip join are per-key operations on disjoint key ranges).
The local operators come from an `ops` object: HipOps (the product path) or,
in the gloo CPU tests only, an oracle-backed stand-in.
"""
import os

import torch
import torch.distributed as dist

from . import ops as hip_ops

INT64_MIN = -(1 << 63)
INT64_MAX = (1 << 63) - 1
MAX_BOUNDS = 63  # smj_dev_partition*: <= 64 buckets
# Exchange stages K (key sub-ranges per rank whose exchange overlaps the
# previous one's sort + join).  One GPU (the RCCL loopback) measured best at
# K = 2 (profiles/r03/r03zg_loop_stages.txt: the self-copies share HBM with the
# pipeline, so more stages only add calls).  Across GPUs the exchange runs
# over xGMI, not HBM, and dominates: (W - 1) / W of 3.2 GB per C3 rank over
# W - 1 links of ~76 GB/s per direction (W = 8: ~5 ms, W = 2: ~21 ms, against
# ~5 ms of local compute), so the exposed part, ~T_x / K + max(T_x, T_c) (K -
# 1) / K + T_c / K, is smallest at the largest K the partition allows (4 at W
# = 8; stage_count).  A model, not a measurement: no 8-GPU node has run it.
_STAGES_ENV = os.environ.get("SMJ_DIST_STAGES")
DEFAULT_STAGES = int(_STAGES_ENV) if _STAGES_ENV else None


# Stage shares within a rank (SMJ_DIST_STAGE_FRAC, e.g. "0.35,0.65").  On one
# GPU (loopback) the exchange is shorter than the pipeline, so small first
# stages start the pipeline sooner while the larger later ones are in flight
# (two stages: exposed ~ X f0 + max(P f0, X (1 - f0)) + P (1 - f0), best at f0
# = X / (X + P) ~ 0.35 for X = 2.7, P = 5 ms).  Measured on one box
# (profiles/r04/r04i): 0.5/0.5 9.88-9.95 ms, 0.35/0.65 9.61-9.62, 0.25/0.75
# 9.89-9.92, three stages 0.15/0.3/0.55 9.38-9.49 (the default there).  Round 5,
# with S's partition on its own stream (profiles/r05/r05m, r05o: two rounds
# each on two boxes): K = 2 9.00 / 8.86 / 9.11 / 9.07, K = 3 9.06 / 8.96 / 9.11
# / 9.17, K = 4 9.22 / 9.20 / 9.46 / 9.26 ms -- two stages again; then with
# packed exchange rows (half the self-copy bytes, profiles/r05/r05zf) K = 1
# 8.14 / 8.23, K = 2 8.42 / 8.44, K = 3 9.57 / 9.77 ms: on one GPU the copy
# is now cheaper than a second pipeline call, so one stage.  Across GPUs the
# exchange dominates and the stages stay equal.
_FRAC_ENV = os.environ.get("SMJ_DIST_STAGE_FRAC")


def stage_fracs(world, K):
    if _FRAC_ENV:
        f = [float(x) for x in _FRAC_ENV.split(",")]
        if len(f) == K and all(x > 0 for x in f):
            return f
    if world == 1 and K == 2:
        return [0.35, 0.65]
    if world == 1 and K == 3:
        return [0.15, 0.3, 0.55]
    return None


def default_stages(world, rows=0):
    """rows: the larger table's rows on this rank.  One rank (the loopback):
    one stage while the tables fit one pipeline call, else three -- a single
    stage of C4's 1e9-row tables held every buffer at once and ran 459 ms
    against 90 (profiles/r05/r05zg).  More ranks: 4 (every rank alike)."""
    if DEFAULT_STAGES is not None:
        return DEFAULT_STAGES
    if world == 1:
        return 1 if rows <= PACK_MAX_ROWS else 3
    return 4
# loopback: a rank's own segment also travels through the point-to-point
# transport (send / receive to itself; RCCL only: gloo keeps the device copy)
# instead of a device copy, and one rank runs the whole distributed path: the
# RCCL exchange on a one-GPU box
LOOPBACK = os.environ.get("SMJ_DIST_LOOPBACK", "0") == "1"
# diagnostics: SMJ_DIST_TRACE=1 synchronises after every phase and prints its
# wall time (rank 0, stderr) -- it serialises the overlap, so never in a timed
# run; SMJ_DIST_TRACE=2 prints the host's progress without synchronising (where
# the host thread is when a run stalls)
TRACE_MODE = os.environ.get("SMJ_DIST_TRACE", "0")
TRACE = TRACE_MODE in ("1", "2")


_T_LAST = [0.0]  # the host time the previous traced call returned


class _Tracer:
    def __init__(self, on, rank):
        import time
        self.on, self.rank, self.time = on and rank == 0, rank, time
        self.t = self.time.perf_counter() if self.on else 0.0
        if self.on and _T_LAST[0]:
            import sys
            print(f"smj.dist trace: since the previous call returned: {(self.t - _T_LAST[0]) * 1e3:.2f} ms",
                  file=sys.stderr, flush=True)

    def end(self):
        if self.on:
            self("return")
            _T_LAST[0] = self.time.perf_counter()

    def __call__(self, what):
        if not self.on:
            return
        if TRACE_MODE == "1":
            torch.cuda.synchronize()
        t = self.time.perf_counter()
        import sys
        print(f"smj.dist trace: {what}: {(t - self.t) * 1e3:.2f} ms", file=sys.stderr, flush=True)
        self.t = t


# the per-stage pipelines in two halves on a side stream (SMJ_DIST_SPLIT=0:
# one blocking call per stage on the current stream, after the next stage's
# transfers are posted)
SPLIT_STAGES = os.environ.get("SMJ_DIST_SPLIT", "1") != "0"
_SPLIT_SIDE = {}  # device -> the stage pipelines' side stream


def _side_stream(device):
    s = _SPLIT_SIDE.get(str(device))
    if s is None:
        s = _SPLIT_SIDE[str(device)] = torch.cuda.Stream(device=device, priority=-1)  # like the compute stream
    return s


class HipOps:
    """The product operators: HIP kernels behind libsmj_hip.so."""
    sort_merge_join = staticmethod(hip_ops.sort_merge_join)
    partition = staticmethod(hip_ops.partition)
    partition_count = staticmethod(hip_ops.partition_count)
    partition_plan = staticmethod(hip_ops.partition_plan)    # asynchronous: counts stay on the device
    partition_apply = staticmethod(hip_ops.partition_apply)
    partition_regions = staticmethod(hip_ops.partition_regions)  # one read of the table (msd_part1_kernel)
    sort_merge_join_begin = staticmethod(hip_ops.sort_merge_join_begin)  # the pipeline enqueued; job.end(out) finishes it
    sort_merge_join_begin_pk = staticmethod(hip_ops.sort_merge_join_begin_pk)  # the same on packed exchange rows
    unpack_rows = staticmethod(hip_ops.unpack_rows)
    dist_sample = staticmethod(hip_ops.dist_sample)        # the splitter sample (smj_dev_dist_sample)
    dist_splitters = staticmethod(hip_ops.dist_splitters)  # the splitters from the gathered samples
    region_capacities = staticmethod(hip_ops.region_capacities)
    writes_into = True  # sort_merge_join(..., out=view) writes the joined rows there


_SAMPLE_IDX = {}


def sample_index(n, samples, device=None):
    """min(samples, n) row indices spread evenly over [0, n - 1], in exact
    int64 arithmetic (a float32 linspace rounds n - 1 up to n above 2^24 rows
    and would read past the table).  Cached per (n, samples, device): the
    same slices come back every step."""
    key = (n, samples, str(device))
    idx = _SAMPLE_IDX.get(key)
    if idx is None:
        k = min(samples, n)
        idx = torch.arange(k, dtype=torch.int64, device=device) * (n - 1) // max(k - 1, 1)
        if len(_SAMPLE_IDX) > 64:
            _SAMPLE_IDX.clear()
        _SAMPLE_IDX[key] = idx
    return idx


def _sample_keys(table, key_col, samples):
    n = table.shape[0]
    if n == 0:
        return table.new_empty((0,))
    return table[:, key_col].index_select(0, sample_index(n, samples, table.device))


def _wire_device(t, group=None):
    """Where collective buffers live: the tensor's own device under RCCL; the
    host under gloo (which moves CPU tensors only) -- used by the CPU tests and
    by the 2-rank-on-one-GPU test, never by the RCCL product path."""
    if t.is_cuda and dist.get_backend(group) == "gloo":
        return torch.device("cpu")
    return t.device


def seg_fracs(world, K, frac=None):
    """Cumulative fractions of the W*K - 1 segment boundaries: segment d*K + k
    (rank d, stage k) holds frac[k] / W of the rows (frac: the stage shares
    within a rank, equal by default)."""
    frac = frac or [1.0 / K] * K
    cum = [sum(frac[:k]) / sum(frac) for k in range(K)]
    return [(d + cum[k]) / world for d in range(world) for k in range(K)][1:]


_PINNED = {}  # (device, words) -> a pinned host buffer for _splitters_hip's one copy


def _splitters_hip(ops, tables_and_keys, world, group, samples, parts, own, fracs, est):
    """choose_splitters on the device, in four operations: the library's
    sample kernel, one all_gather_into_tensor, the library's order-statistic
    kernel, one device -> host copy (round 4's torch path took ~25 small
    launches and host gaps, ~0.6 ms of the loopback step; profiles/r05/r05p).
    Same samples, same positions, same splitters as the torch path."""
    (R, kR), (S, kS) = tables_and_keys
    H, stride = 5, 5 + 2 * samples
    dev = R.device
    buf = ops.dist_sample(R, S, kR, kS, samples)
    allx = torch.empty(world * stride + parts, dtype=torch.int64, device=dev)
    gathered = allx[:world * stride]
    dist.all_gather_into_tensor(gathered, buf, group=group)
    q20 = [int(round(f_ * (1 << 20))) for f_ in fracs] if fracs is not None else None
    ops.dist_splitters(gathered, world, stride, parts, q20, out=allx[world * stride:])
    key = (str(dev), allx.numel())
    host = _PINNED.get(key)
    if host is None:
        if len(_PINNED) > 8:
            _PINNED.clear()
        host = _PINNED[key] = torch.empty(allx.numel(), dtype=torch.int64, pin_memory=True)
    host.copy_(allx, non_blocking=True)
    torch.cuda.current_stream(dev).synchronize()
    got = host.numpy().copy()
    me = dist.get_rank(group)
    if own is not None:
        o = me * stride + H
        for x in range(2):
            c = int(got[me * stride + 1 + x])
            own.append(got[o: o + c])
            o += c
    if est is not None:
        est["all"] = got[:world * stride].reshape(world, stride)
        est["H"], est["nt"] = H, 2
    spl = got[world * stride: world * stride + parts - 1]
    if int(got[world * stride + parts - 1]) == 0:
        return [0] * (parts - 1)
    return [int(x) for x in spl]


def choose_splitters(tables_and_keys, world, group=None, samples=4096, parts=None, own=None, fracs=None,
                     est=None, ops=None):
    """parts - 1 (default W - 1) sorted key splitters, identical on every rank,
    as a host list: one all_gather of every rank's sample (a fixed-size buffer,
    padded with INT64_MAX, plus its valid count), the sort and the order
    statistics on the device, one device -> host copy of the result.  own (a
    list): gets this rank's sampled keys per table (host lists, from the same
    copy) -- partition_regions sizes its regions from them.  est (a dict):
    gets every rank's sampled keys per table and its table rows (host), from
    which any rank can estimate every bucket's global rows (estimate_counts)."""
    parts = parts or world
    home = tables_and_keys[0][0].device
    dev = _wire_device(tables_and_keys[0][0], group)
    if (ops is not None and hasattr(ops, "dist_splitters") and len(tables_and_keys) == 2 and dev.type == "cuda"
            and all(t.is_cuda for t, _ in tables_and_keys) and parts <= MAX_BOUNDS + 1):
        return _splitters_hip(ops, tables_and_keys, world, group, samples, parts, own, fracs, est)
    nt = len(tables_and_keys)
    cap = nt * samples
    H = 1 + 2 * nt  # header: [total samples, samples per table..., rows per table...]
    # [header, keys..., INT64_MAX pads]: the sampled keys are gathered straight
    # into their slice (on the wire device when the transport is gloo)
    buf = torch.full((cap + H,), INT64_MAX, dtype=torch.int64, device=home)
    at = H
    hdr = [0] * H
    for x, (t, k) in enumerate(tables_and_keys):
        n = t.shape[0]
        c = min(samples, n)
        hdr[1 + x], hdr[1 + nt + x] = c, n
        if n:
            idx = sample_index(n, samples, t.device)
            torch.index_select(t[:, k], 0, idx, out=buf[at: at + c])
            at += c
    hdr[0] = at - H
    buf[:H] = torch.tensor(hdr, dtype=torch.int64).to(home, non_blocking=True)
    buf = buf.to(dev)
    allb = torch.empty((world, cap + H), dtype=torch.int64, device=dev)
    dist.all_gather(list(allb.unbind(0)), buf, group=group)  # rows of allb (gloo has no all_gather_into_tensor)
    L = allb[:, 0].sum()
    # the pads sort last (a real INT64_MAX key sorts among them: the same value)
    keys = torch.sort(allb[:, H:].reshape(-1)).values
    if fracs is None:
        pos = (torch.arange(1, parts, dtype=torch.int64, device=dev) * L // parts - 1).clamp(min=0)
    else:  # boundary i at the cumulative fraction fracs[i] of the sample
        q = torch.tensor([int(round(f_ * (1 << 20))) for f_ in fracs], dtype=torch.int64, device=dev)
        pos = (q * L // (1 << 20) - 1).clamp(min=0)
    # one host copy, kept as a numpy array (a .tolist() of the ~8k sampled keys
    # cost ~0.3 ms of host time per step in the loopback trace, profiles/r04/r04j)
    parts_ = [keys[pos], L.view(1), buf[H:at]]
    if est is not None:
        parts_.append(allb.reshape(-1))
    got = torch.cat(parts_).cpu().numpy()
    if own is not None:
        o = parts
        for t, _ in tables_and_keys:
            c = min(samples, t.shape[0])
            own.append(got[o: o + c])
            o += c
    if est is not None:
        est["all"] = got[parts + (at - H):].reshape(world, cap + H)
        est["H"], est["nt"] = H, nt
    if int(got[parts - 1]) == 0:
        return [0] * (parts - 1)
    return [int(x) for x in got[:parts - 1]]


def estimate_counts(est, t, bounds):
    """Global rows per bucket of table t estimated from every rank's sample
    (each rank's samples of t weigh its rows / its sample count); identical on
    every rank.  Rows a WHERE clause drops are counted too (the sample ignores
    the select): an estimate for balancing cuts, never for correctness."""
    import numpy as np
    a, H, nt = est["all"], est["H"], est["nt"]
    nb = len(bounds) + 1
    tot = np.zeros(nb)
    bnd = np.asarray(bounds, dtype=np.int64)
    for r in range(a.shape[0]):
        c = [int(a[r, 1 + x]) for x in range(nt)]
        n = int(a[r, 1 + nt + t])
        if c[t] == 0:
            continue
        o = H + sum(c[:t])
        b = np.searchsorted(bnd, a[r, o: o + c[t]], side="left")
        tot += np.bincount(b, minlength=nb) * (n / c[t])
    return np.rint(tot).astype(np.int64).tolist()  # (round half to even, as round())


def bucket_bounds(spl):
    """Boundaries s for the partition kernels' bucket(k) = #{s < k}: every
    distinct splitter key u (spl: a host list) gets the single-key bucket
    (u-1, u].  Returns (s, single) with single[b] true when bucket b holds
    exactly one key value."""
    spl = [int(x) for x in (spl.tolist() if isinstance(spl, torch.Tensor) else spl)]
    s = []
    for u in sorted(set(spl)):
        if u > INT64_MIN and (not s or s[-1] < u - 1):
            s.append(u - 1)
        s.append(u)
    if len(s) > MAX_BOUNDS:  # too many ranks for single-key buckets: key-only splitters
        s = sorted(set(spl))
    single = [(b == 0 and bool(s) and s[0] == INT64_MIN) or (0 < b < len(s) and s[b] - s[b - 1] == 1)
              for b in range(len(s) + 1)]
    return s, single


def choose_cuts(GR, GS, single, world, fracs=None):
    """W-1 cuts (bucket, occurrence) over the global bucket-ordered sequence,
    balancing R + S rows per rank: rows of buckets < b go left, and of bucket
    b the occurrences < o (o = 0 unless b is a single-key bucket).  The same
    o applies to R and S.  Identical on every rank (pure function of the
    gathered counts)."""
    nb = len(GR)
    tot = [GR[b] + GS[b] for b in range(nb)]
    total = sum(tot)
    cuts, acc, b, prev = [], 0, 0, (0, 0)
    for d in range(1, world):
        target = total * (fracs[d - 1] if fracs else d / world)
        while b < nb and acc + tot[b] <= target:
            acc += tot[b]
            b += 1
        if b == nb:
            cut = (nb, 0)
        elif single[b]:
            need = target - acc  # smallest o with min(o, GR) + min(o, GS) >= need, or o - 1 if closer
            lo, hi = 0, max(GR[b], GS[b])
            while lo < hi:
                mid = (lo + hi) // 2
                if min(mid, GR[b]) + min(mid, GS[b]) >= need:
                    hi = mid
                else:
                    lo = mid + 1
            left = min(lo, GR[b]) + min(lo, GS[b])
            if lo > 0 and need - (min(lo - 1, GR[b]) + min(lo - 1, GS[b])) < left - need:
                lo -= 1
            cut = (b, lo)
        else:  # a multi-key bucket moves whole: the nearer edge
            cut = (b, 0) if target - acc <= acc + tot[b] - target else (b + 1, 0)
        cut = max(cut, prev)
        cuts.append(cut)
        prev = cut
    return cuts


def slice_counts(local, prefix, cuts, nb):
    """Rows of this rank's bucket-ordered buffer per destination rank: cut
    (b, o) sits after the local buckets < b and, of bucket b, the local rows
    whose global occurrence (prefix[b] = rows of bucket b on earlier ranks +
    local offset) is below o."""
    def pos(cut):
        b, o = cut
        p = sum(local[:b])
        if b < nb:
            p += min(max(o - prefix[b], 0), local[b])
        return p
    edges = [0] + [pos(c) for c in cuts] + [sum(local)]
    return [edges[d + 1] - edges[d] for d in range(len(edges) - 1)]


def slice_ranges(local, prefix, cuts, nb):
    """The rows of this rank's bucket-partitioned table per destination
    segment, as (bucket, lo, hi) local offset ranges: cut (b, o) splits bucket
    b at the local rows whose global occurrence (prefix[b] + local offset) is
    below o.  Every segment's ranges ascend in bucket order; their row counts
    are slice_counts(...)."""
    def at(cut):
        b, o = cut
        return (b, 0) if b >= nb else (b, min(max(o - prefix[b], 0), local[b]))
    edges = [(0, 0)] + [at(c) for c in cuts] + [(nb, 0)]
    out = []
    for d in range(len(edges) - 1):
        (b0, c0), (b1, c1) = edges[d], edges[d + 1]
        rs = []
        for b in range(b0, min(b1, nb - 1) + 1):
            lo = c0 if b == b0 else 0
            hi = c1 if b == b1 else local[b]
            if hi > lo:
                rs.append((b, lo, hi))
        out.append(rs)
    return out


def gather_counts(counts, world, group=None, device=None):
    """all_gather of this rank's integer vector (a list, or a device tensor
    that stays on the device until the one host copy of the gathered
    result); returns a world x len list."""
    if isinstance(counts, torch.Tensor):
        t = counts.to(device if device is not None else counts.device)
    else:
        t = torch.tensor(counts, dtype=torch.int64, device=device)
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=group)
    return torch.stack(out).tolist()


def stage_count(world, stages):
    """Stages K such that the W*K - 1 splitters, each with a single-key
    bucket, fit the partition kernel: 2 (W K - 1) <= MAX_BOUNDS."""
    k = max(1, int(stages))
    while k > 1 and 2 * (world * k - 1) > MAX_BOUNDS:
        k -= 1
    return k


class _Stage:
    """One stage's receives in flight: wait() returns the [R, S] rows of this
    rank's sub-range (None for a table not posted), chunks in source-rank
    order."""

    def __init__(self, works, recvs, home):
        self.works, self.recvs, self.home = works, recvs, home

    def wait(self):
        for w in self.works:
            w.wait()
        return [None if r is None else r.to(self.home) for r in self.recvs]


def _wait_all(pending):
    out = [None, None]
    for st in pending:
        for t, r in enumerate(st.wait()):
            if r is not None:
                out[t] = r
    return out


# RCCL point-to-point messages above ~2 GiB arrive corrupted (tools/rccl_big.py,
# profiles/r04/r04e: a 2.34 GiB send to self differs, 0.5 GiB is exact), so
# every (peer, bucket range) message is cut into pieces of at most this many
# bytes -- on both sides alike, in order
MAX_MSG_BYTES = int(os.environ.get("SMJ_DIST_MAX_MSG", str(512 << 20)))


def _pieces(lo, hi, cols):
    step = max(1, MAX_MSG_BYTES // (8 * cols))
    return [(a, min(hi, a + step)) for a in range(lo, hi, step)]


def post_stage(k, K, sends, regs, sl, rank, world, home, group=None, loopback=False):
    """Post stage k's exchange: segment d*K + k of every table goes to rank d.
    sl[t][r][j] = the (bucket, lo, hi) local row ranges of src rank r's table-t
    buffer in segment j (known on every rank from the gathered counts, so no
    count exchange is needed); regs[t][b] = where bucket b's rows start in
    this rank's buffer.  One message per (bucket range, peer): received ranges
    are placed in source-rank, then bucket order -- the global input order of
    the segment's rows.  sends are on the wire device (_wire_device), None for
    a table not posted in this call; received rows are returned on `home`."""
    p2p, recvs = [], []
    loopback = loopback and dist.get_backend(group) != "gloo"  # gloo pairs never connect a rank to itself
    me = rank * K + k
    for t, wire in enumerate(sends):
        if wire is None:
            recvs.append(None)
            continue
        rc = sum(hi - lo for r in range(world) for (_, lo, hi) in sl[t][r][me])
        recv = torch.empty((rc, wire.shape[1]), dtype=wire.dtype, device=wire.device)
        at = 0
        cols = wire.shape[1]
        for r in range(world):
            for b, lo, hi in sl[t][r][me]:
                c = hi - lo
                if r == rank and not loopback:
                    o = regs[t][b] + lo
                    recv[at: at + c].copy_(wire[o: o + c])
                else:
                    for a0, a1 in _pieces(at, at + c, cols):
                        p2p.append(dist.P2POp(dist.irecv, recv[a0: a1], r, group, tag=(t * 64 + b) * 64 + k))
                at += c
        for d in range(world):
            if d == rank and not loopback:
                continue
            for b, lo, hi in sl[t][rank][d * K + k]:
                o = regs[t][b] + lo
                for a0, a1 in _pieces(o, o + hi - lo, cols):
                    p2p.append(dist.P2POp(dist.isend, wire[a0: a1], d, group, tag=(t * 64 + b) * 64 + k))
        recvs.append(recv)
    works = dist.batch_isend_irecv(p2p) if p2p else []
    return _Stage(works, recvs, home)


def sort_merge_join(R, S, select=(0, 5000, 0, 5000), keys=(0, 0), group=None, ops=None, samples=4096,
                    stats=None, stages=None, loopback=None):
    """The distributed pipeline; returns this rank's slice of the result (the
    global result is the concatenation over ranks in rank order).  stats
    (optional dict) gets the rows this rank received per table and the
    max / mean load over ranks (load-balance report).  stages: key sub-ranges
    per rank whose exchange overlaps the previous one's sort + join
    (default SMJ_DIST_STAGES, else default_stages(W): 1 on one rank (3 for tables over 1.6e8 rows), 4 at
    W > 1, lowered by stage_count to what the partition fits; 1 = exchange
    everything, then compute).
    loopback (default SMJ_DIST_LOOPBACK=1): the rank's own segments also go
    through send / receive to itself, and a single rank takes the whole
    distributed path (exercises the RCCL transport on one GPU).
    The local pipeline has a fixed cost per call: 1e8 rows per table take
    6.03 ms in one call, 6.37 ms in 2 and 8.53 ms in 4 (tools/part_probe.py)."""
    ops = ops or HipOps
    sc1, sv1, sc2, sv2 = select
    k1, k2 = keys
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    # loopback needs a process group (a one-rank RCCL group sending to itself);
    # without one the single-rank call is the local pipeline
    loopback = (LOOPBACK if loopback is None else loopback) and dist.is_initialized()
    if world == 1 and not loopback:
        return ops.sort_merge_join(R, S, k1, k2, (sc1, sv1), (sc2, sv2))[2]
    if not R.is_cuda:
        return _sort_merge_join(R, S, sc1, sv1, sc2, sv2, k1, k2, group, ops, samples, stats, stages, loopback,
                                world, rank)
    # The local work runs on a high-priority stream of its own.  RCCL's
    # point-to-point kernels run on the process group's stream; HIP multiplexes
    # streams onto GPU_MAX_HW_QUEUES hardware queues, and a trace of the
    # one-GPU loopback (profiles/r03c_loopback_trace.txt) found RCCL's stream
    # and torch's default stream on the SAME queue: every exchange kernel then
    # ran between two pipeline kernels instead of beside them.
    caller = torch.cuda.current_stream(R.device)
    cs = _compute_stream(R.device)
    cs.wait_stream(caller)
    with torch.cuda.stream(cs):
        J = _sort_merge_join(R, S, sc1, sv1, sc2, sv2, k1, k2, group, ops, samples, stats, stages, loopback,
                             world, rank)
    caller.wait_stream(cs)
    J.record_stream(caller)
    return J


_STREAMS = {}


def _compute_stream(device):
    s = _STREAMS.get(device)
    if s is None:
        s = _STREAMS[device] = torch.cuda.Stream(device=device, priority=-1)
    return s


REGIONS = os.environ.get("SMJ_DIST_REGIONS", "1") != "0"  # 0: the counting partition (plan / apply), A/B
REGION_SCALE = float(os.environ.get("SMJ_DIST_REGION_SCALE", "1"))  # tests: < 1 forces the overflow fallback


# Packed exchange (round 5): a 2-column table's partitioned rows travel as one
# int64 word each -- (int32 key - key base) | (int32 other - other base) << 32
# (smj.h smj_dev_partition_regions_pk) -- so the partition writes, the
# exchange moves and the receiving pipeline's first pass reads half the
# bytes.  The key base is the middle of the gathered key sample of the table;
# the other column's base is 0 (row ids and payloads under 2^31 pack).  A row
# that does not fit sets a flag every rank sees in the gathered counts, and
# every rank then re-partitions that table unpacked (SMJ_DIST_PACK=0: never
# pack).
PACK = os.environ.get("SMJ_DIST_PACK", "1") != "0"
PACK_MAX_ROWS = 160_000_000  # smj_dev_sort_merge_join_begin_pk's limit per table; larger stages are unpacked first


def _key_range(est, t):
    """(min, max) of table t's sampled keys over every rank (the gathered
    sample buffers of choose_splitters), None without samples."""
    a, H, nt = est["all"], est["H"], est["nt"]
    lo, hi = None, None
    for r in range(a.shape[0]):
        c = [int(a[r, 1 + x]) for x in range(nt)]
        o = H + sum(c[:t])
        if c[t]:
            k = a[r, o: o + c[t]]
            lo = int(k.min()) if lo is None else min(lo, int(k.min()))
            hi = int(k.max()) if hi is None else max(hi, int(k.max()))
    return None if lo is None else (lo, hi)


def _key_base(est, t):
    """The middle of table t's sampled keys over every rank, 0 without samples."""
    r = _key_range(est, t)
    return 0 if r is None else (r[0] + r[1]) // 2


# A packed key is (int32)(key - base): with the base in the middle of the
# sampled keys, a sample spanning 2^31 or more already shows keys that cannot
# fit, and every call would pay a packed partition that is thrown away plus an
# unpacked re-partition.  Such tables are sent plain from the start,
# and a table whose packing failed on any rank is remembered (by tensor, shape
# and key column) so that the next calls on it do not try again.
PACK_SPAN = 1 << 31
_NOPACK = set()


def _pack_id(T, k):
    return (T.data_ptr(), tuple(T.shape), int(k)) if T.is_cuda else None


def _unpacked(ops, t, key, pack):
    return t if pack is None else ops.unpack_rows(t, key, pack)


def _partition(ops, T, bounds, cnt, own, k, sc, sv, pack=None):
    """This rank's table T partitioned by bucket.  With partition_regions (one
    read of T): bucket b's rows at region starts sized from T's sample `own`;
    else the counting partition (plan + apply: two reads), bucket-contiguous.
    cnt (device, nb + 1) gets the counts and the overflow flag.  Returns
    (buffer, region starts or None = contiguous)."""
    nb = len(bounds) + 1
    if REGIONS and hasattr(ops, "partition_regions"):
        reg, _ = ops.region_capacities(own, T.shape[0], bounds)
        if REGION_SCALE < 1.0:
            caps = [int(c * REGION_SCALE) for c in reg[nb:]]
            reg = [sum(caps[:b]) for b in range(nb)] + caps
        if pack is not None:
            return ops.partition_regions(T, bounds, reg, cnt, k, sc, sv, pack=pack), reg[:nb]
        return ops.partition_regions(T, bounds, reg, cnt, k, sc, sv), reg[:nb]
    cnt[nb:].zero_()
    plan = ops.partition_plan(T, bounds, cnt[:nb], k, sc, sv)
    return ops.partition_apply(T, bounds, plan, k, sc, sv), None


def _repartition(ops, T, bounds, k, sc, sv):
    """The counting partition of a table whose one-read partition overflowed a
    region (counts unchanged: the one-read pass counts every row)."""
    nb = len(bounds) + 1
    cnt = torch.empty(nb, dtype=torch.int64, device=T.device)
    plan = ops.partition_plan(T, bounds, cnt, k, sc, sv)
    return ops.partition_apply(T, bounds, plan, k, sc, sv)


_GATHER_SIDE = {}  # device -> the count gathers' host-copy stream
S_SIDE = os.environ.get("SMJ_DIST_S_SIDE", "1") != "0"
_S_SIDE = {}  # device -> the stream S's partition runs on


def _s_stream(device):
    s = _S_SIDE.get(str(device))
    if s is None:
        s = _S_SIDE[str(device)] = torch.cuda.Stream(device=device, priority=-1)
    return s


class _HostGather:
    """all_gather of a small int64 device vector (bucket counts + flag) whose
    host copy waits for the collective only -- not for work enqueued on the
    compute stream after it (the next table's partition).  Under gloo (CPU
    wire) it is the synchronous gather_counts."""

    def __init__(self, t, world, group):
        dev = _wire_device(t, group)
        self.res = None
        if dev.type == "cpu":
            self.res = gather_counts(t, world, group, dev)
            return
        self.outs = [torch.empty_like(t) for _ in range(world)]
        work = dist.all_gather(self.outs, t, group=group, async_op=True)  # ordered after t's producer
        side = _GATHER_SIDE.get(str(t.device))
        if side is None:
            side = _GATHER_SIDE[str(t.device)] = torch.cuda.Stream(device=t.device)
        with torch.cuda.stream(side):
            work.wait()
            self.host = torch.empty((world, t.numel()), dtype=t.dtype, pin_memory=True)
            self.host.copy_(torch.stack(self.outs), non_blocking=True)
            self.ev = torch.cuda.Event()
            self.ev.record(side)

    def result(self):
        if self.res is None:
            self.ev.synchronize()
            self.res = self.host.tolist()
            del self.outs
        return self.res


def _sort_merge_join(R, S, sc1, sv1, sc2, sv2, k1, k2, group, ops, samples, stats, stages, loopback, world, rank):
    K = stage_count(world, default_stages(world, max(R.shape[0], S.shape[0])) if stages is None else stages)
    nseg = world * K
    tr = _Tracer(TRACE and R.is_cuda, rank)

    own, est = [], {}
    fr = stage_fracs(world, K)
    fracs = seg_fracs(world, K, fr) if fr else None
    spl = choose_splitters([(R, k1), (S, k2)], world, group, samples, parts=nseg, own=own, fracs=fracs,
                           est=est, ops=ops)  # host sync 1
    tr("splitters")
    bounds, single = bucket_bounds(spl)
    nb = len(bounds) + 1
    tabs = [(R, k1, sc1, sv1), (S, k2, sc2, sv2)]
    wire = _wire_device(R, group)
    # R partitioned (one read) on the compute stream and its counts gathered
    # -- the host copy waits for that gather only.  S is partitioned on a side
    # stream (S_SIDE), so that R's stage-0 transfers, posted as soon as R's
    # counts are known, do not wait for it: the process group orders its
    # work after the CURRENT stream (R's partition only), and S's count gather
    # is issued after R's stage 0 from the side stream (waiting for S's
    # partition only).  The cuts come from R's exact counts and S's sample
    # estimate (any (bucket, occurrence) cut is valid: R and S apply the same
    # one).  Round 4 issued both partitions and both gathers on the compute
    # stream first, so the stage-0 transfers queued behind S's partition and
    # only the host's wait was removed; SMJ_DIST_S_SIDE=0 keeps
    # that order.
    cnt = [torch.empty(nb + 1, dtype=torch.int64, device=R.device) for _ in range(2)]
    cur = torch.cuda.current_stream(R.device) if R.is_cuda else None
    sside = _s_stream(R.device) if (R.is_cuda and S_SIDE) else None
    # packed exchange rows (PACK, above): the product operators on the device
    # with the RCCL wire, and 2-column tables
    can_pack = (PACK and REGIONS and R.is_cuda and wire.type == "cuda" and hasattr(ops, "unpack_rows")
                and hasattr(ops, "sort_merge_join_begin_pk"))
    if can_pack:
        # a stage over PACK_MAX_ROWS rows per table runs in the library's
        # partitioned mode, which reads plain rows: the received words would
        # need an unpack pass (C4 / C5 on one GPU), so such jobs send plain
        # rows -- judged from the tables' sizes (all ranks, from the sample
        # headers) and the largest stage share, with a margin
        smax = (max(fr) / sum(fr)) if fr else 1.0 / K
        a = est["all"]
        big = max(int(a[:, 1 + 2 + x].sum()) for x in range(2)) * smax / world * 1.25
        can_pack = big <= PACK_MAX_ROWS
    packs = []
    for x, (T, k) in enumerate(((R, k1), (S, k2))):
        kr = _key_range(est, x)
        ok = (can_pack and T.shape[1] == 2 and _pack_id(T, k) not in _NOPACK
              and (kr is None or kr[1] - kr[0] < PACK_SPAN))
        packs.append(((kr[0] + kr[1]) // 2 if kr else 0, 0) if ok else None)
    pack_fallbacks = 0
    tr("bounds, regions, key bases")
    part = [_partition(ops, R, bounds, cnt[0], own[0], k1, sc1, sv1, packs[0])]
    gR = _HostGather(cnt[0], world, group)
    tr("R partition + gather enqueued")
    if sside is not None:
        # after R's partition: the two calls share the library's partition
        # scratch (region words, look-back status words), so they must not run
        # at once -- only the process group's work is kept off S's partition
        # (r05a: concurrent partitions corrupted R's look-back, an illegal
        # address at C3); also orders everything before this step first
        sside.wait_stream(cur)
        with torch.cuda.stream(sside):
            part.append(_partition(ops, S, bounds, cnt[1], own[1], k2, sc2, sv2, packs[1]))
        gS = None
    else:
        part.append(_partition(ops, S, bounds, cnt[1], own[1], k2, sc2, sv2, packs[1]))
        gS = _HostGather(cnt[1], world, group)
    counts, sends, regs, sl = [None, None], [None, None], [None, None], [None, None]

    def finish(t, allc):  # this table's exact counts: overflow fix-up, send buffer, row ranges
        # flag word bit 1: a look-back timed out on that rank (a bug; its
        # prefixes, and with them every rank's cuts, would be wrong) -- every
        # rank sees every flag, so all raise together instead of hanging
        late = [r for r in range(world) if allc[r][nb] & 2]
        if late:
            raise RuntimeError(f"smj.dist: the partition's look-back timed out on rank(s) {late} (table {t})")
        counts[t] = [allc[r][:nb] for r in range(world)]
        buf, reg = part[t]
        if packs[t] is not None and any(allc[r][nb] & 5 for r in range(world)):
            # a row that did not pack (bit 2) or a region overflow (bit 0) on ANY
            # rank: every rank re-partitions this table unpacked, so that all
            # senders and receivers agree on its format
            T, k, sc, sv = tabs[t]
            buf, reg = _repartition(ops, T, bounds, k, sc, sv), None
            packs[t] = None
            nonlocal pack_fallbacks
            pack_fallbacks += 1
            if any(allc[r][nb] & 4 for r in range(world)) and _pack_id(T, k) is not None:
                _NOPACK.add(_pack_id(T, k))
        elif reg is not None and allc[rank][nb] & 1:  # a region overflowed: the counting partition
            T, k, sc, sv = tabs[t]
            buf, reg = _repartition(ops, T, bounds, k, sc, sv), None
        if reg is None:  # bucket-contiguous
            reg = [sum(counts[t][rank][:b]) for b in range(nb)]
        end = max([reg[b] + counts[t][rank][b] for b in range(nb)] + [0])
        sends[t] = buf[:end].to(wire)  # only the rows the regions hold (under gloo: a host copy)
        regs[t] = reg
        part[t] = None
        sl[t] = [slice_ranges(counts[t][r], [sum(counts[t][q][b] for q in range(r)) for b in range(nb)], cuts, nb)
                 for r in range(world)]

    tr("S partition enqueued")
    allcR = gR.result()  # host sync 2 (R's counts)
    tr("partition R + counts")
    GR = [sum(allcR[r][b] for r in range(world)) for b in range(nb)]
    GSe = estimate_counts(est, 1, bounds)
    cuts = choose_cuts(GR, GSe, single, nseg, fracs)
    finish(0, allcR)
    pending = [post_stage(0, K, [sends[0], None], regs, sl, rank, world, R.device, group, loopback)]  # R's stage 0
    if gS is None:
        with torch.cuda.stream(sside):
            gS = _HostGather(cnt[1], world, group)
    allcS = gS.result()  # host sync 3 (S's counts)
    if sside is not None:
        cur.wait_stream(sside)  # S's partition before anything that reads its buffer on the compute stream
    finish(1, allcS)
    tr("partition S + counts; R stage 0 posted")
    pending.append(post_stage(0, K, [None, sends[1]], regs, sl, rank, world, R.device, group, loopback))
    seg = [[[sum(hi - lo for (_, lo, hi) in sl[t][r][j]) for j in range(nseg)] for r in range(world)]
           for t in range(2)]
    rows_in = [sum(seg[t][r][rank * K + k] for r in range(world) for k in range(K)) for t in range(2)]
    bound = sum(min(sum(seg[0][r][rank * K + k] for r in range(world)),
                    sum(seg[1][r][rank * K + k] for r in range(world))) for k in range(K))
    into = getattr(ops, "writes_into", False)
    ncols = R.shape[1] + S.shape[1] - 1
    J = torch.empty((max(bound, 1), ncols), dtype=R.dtype, device=R.device) if into else None
    parts, at = [], 0
    tr("stage 0 posted")
    begin = getattr(ops, "sort_merge_join_begin", None) if into and R.is_cuda and SPLIT_STAGES else None
    side = _side_stream(R.device) if begin else None
    for k in range(K):
        Rk, Sk = _wait_all(pending)
        tr(f"stage {k} received")
        job = None
        if begin and Rk.shape[0] and Sk.shape[0]:
            # this stage's pipeline is enqueued before the next stage's
            # transfers are posted -- posting costs ~0.3 ms of host time per
            # stage (profiles/r04/r04y), which the GPU now spends sorting --
            # on a side stream: the process group orders its transfers after
            # the current stream's work, and they must not wait for the sort
            side.wait_stream(torch.cuda.current_stream())
            if packs[0] is None and packs[1] is None:
                job = begin(Rk, Sk, k1, k2, None, None, stream=side)
            else:
                with torch.cuda.stream(side):
                    if max(Rk.shape[0], Sk.shape[0]) > PACK_MAX_ROWS:  # the partitioned mode reads rows, not words
                        Rk, Sk = _unpacked(ops, Rk, k1, packs[0]), _unpacked(ops, Sk, k2, packs[1])
                        job = begin(Rk, Sk, k1, k2, None, None, stream=side)
                    else:
                        job = ops.sort_merge_join_begin_pk(Rk, Sk, k1, k2, packs[0], packs[1], stream=side)
            tr(f"stage {k} pipeline begun")
        if k + 1 < K:
            try:
                pending = [post_stage(k + 1, K, sends, regs, sl, rank, world, R.device, group, loopback)]
            except BaseException:
                if job is not None:  # the thread's pipeline scratch is the job's until it ends
                    job.end()
                raise
            tr(f"stage {k + 1} posted")
        if Rk.shape[0] == 0 or Sk.shape[0] == 0:
            continue
        if job is not None:
            b = min(Rk.shape[0], Sk.shape[0])
            got = job.end(out=J[at: at + b])[2]  # waits for the side stream
            torch.cuda.current_stream().wait_stream(side)
            at += got.shape[0]
            del job
        elif into:
            b = min(Rk.shape[0], Sk.shape[0])
            Rk, Sk = _unpacked(ops, Rk, k1, packs[0]), _unpacked(ops, Sk, k2, packs[1])
            got = ops.sort_merge_join(Rk, Sk, k1, k2, None, None, out=J[at: at + b])[2]
            at += got.shape[0]
        else:
            Rk, Sk = _unpacked(ops, Rk, k1, packs[0]), _unpacked(ops, Sk, k2, packs[1])
            parts.append(ops.sort_merge_join(Rk, Sk, k1, k2, None, None)[2])
        del Rk, Sk
        tr(f"stage {k} sorted + joined")
    del sends
    if stats is not None:  # every rank's load, from the gathered counts (no communication)
        loads = [sum(seg[t][r][d * K + k] for t in range(2) for r in range(world) for k in range(K))
                 for d in range(world)]
        mean = sum(loads) / world
        stats.update(rows_in=rows_in, loads=loads, load_max_over_mean=(max(loads) / mean) if mean else 1.0,
                     cuts=cuts, buckets=nb, stages=K, exchange_packed=[p is not None for p in packs],
                     pack_fallbacks=pack_fallbacks)
    tr.end()
    if into:
        return J[:at]
    if not parts:
        return R.new_empty((0, ncols))
    return torch.cat(parts) if len(parts) > 1 else parts[0]
