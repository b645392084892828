#!/usr/bin/env python3
"""bench.py -- MI355X sort-merge-join throughput (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one rank per GPU)

Workload (BASELINE.json configs[2], "C3"): per GPU |R| = |S| = 1e8 rows of
(int64 key, int64 payload), keys iid uniform in [1, 3n] (n = rows of the
whole job's table), payload = global row index, R seed 1 / S seed 2, the
reference's user.h WHERE col0 > 5000 and JOIN_KEY 0.  Inputs are generated
on the device and resident in HBM before timing.  One step = the whole hot
path: select + stable sort of R and of S, then the 1:1 zip join (N = 1);
for N > 1 the range partition + RCCL all-to-all exchange comes first and
per-GPU work is fixed (weak scaling: the N=8 job is 8e8 x 8e8); the
exchange runs in stages (key sub-ranges) overlapping the local sort + join
of the previous stage (smj/dist.py).

value = (|R| + |S| over all ranks) / max-over-ranks seconds per step.

--workload c4 / c5 times the other BASELINE tables: C4's 1e9 x 1e9 uniform
tables (configs[3]), C5's 1e8 x 1e9 Zipf(0.9) tables (configs[4]); --workload
c3w SURVEY 8(d)'s C3-wide stress input (C3's sizes, full-range signed int64
keys, S planted with R's keys in a random third of its rows, WHERE col0 >
INT64_MIN so that every row passes).  On one GPU
they run through the library's partitioned mode; under torchrun (or
--loopback) they are STRONG-scaled: the job's tables are fixed and rank r
generates its contiguous slice, global rows [r n / W, (r + 1) n / W) (row0 =
r n / W: the generators are functions of the global row, so the tables do not
depend on W), then the range partition + RCCL exchange of smj/dist.py.

Every line carries "verified" (after the timed steps, outside them): under
torchrun / --loopback each rank digests its slice of the joined rows at its
global position (smj_dev_digest, order-sensitive) and rank 0 compares them with
the single-GPU call on the whole job's tables; at N = 1 (every workload) the
timed step's sorted tables and joined rows are compared with the CPU port's
(oracle/cpu_mt.cpp on the full tables, the cpu_baseline_mt leg).  A mismatch prints the line with "verified": false and
exits 3 on every rank.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "pim-sort-merge-join_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from smj import ops  # noqa: E402
from smj import dist as sdist  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
SELECT = (0, 5000, 0, 5000)    # user.h SELECT_COL1/VAL1, SELECT_COL2/VAL2
SELECT_WIDE = (0, -(1 << 63), 0, -(1 << 63))  # C3-wide: WHERE col0 > INT64_MIN (~every row)
KEYS = (0, 0)                  # user.h JOIN_KEY1/2
METRIC = "joined rows/sec on |R|=|S|=1e8 int64-key tables; achieved HBM GB/s vs peak"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# stdout carries exactly one JSON line: the process's fd 1 points at stderr
# for the whole run (RCCL prints a version banner to stdout when its first
# communicator comes up), and the result goes to a private copy of the real
# stdout
_RESULT_FD = None


def _claim_stdout():
    global _RESULT_FD
    sys.stdout.flush()
    _RESULT_FD = os.dup(1)
    os.dup2(2, 1)


def emit(line):
    sys.stdout.flush()
    os.write(_RESULT_FD if _RESULT_FD is not None else 1, (json.dumps(line) + "\n").encode())


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=100_000_000, help="rows per table per GPU")
    p.add_argument("--workload", default="c3", choices=["c3", "c3w", "c4", "c5"],
                   help="c3 (default, the metric's config); c3w: C3-wide (full-range keys); "
                        "c4 / c5: BASELINE's 1e9-row tables on one GPU")
    p.add_argument("--key-range", type=int, default=0,
                   help="c3 / c4: keys iid uniform in [1, K] instead of [1, 3n] (a probe of other key densities)")
    p.add_argument("--cpu-sample", type=int, default=196608,
                   help="rows per table for the single-core cpu_app.c baseline (0 = skip)")
    p.add_argument("--cpu-mt", type=int, default=1,
                   help="time the multi-core CPU port (oracle/cpu_mt.cpp) on the full workload (0 = skip)")
    p.add_argument("--loopback", action="store_true",
                   help="N = 1 through the distributed path (smj.dist, RCCL process group of one rank, "
                        "own segments sent to itself): the multi-GPU pipeline's cost without cross-GPU traffic")
    p.add_argument("--verify", type=int, default=1,
                   help="after the timed steps, check the result: distributed / --loopback against the single-GPU "
                        "call on the whole job's tables (rank 0), N = 1 against the CPU port (--cpu-mt); "
                        "a mismatch exits 3 (0 = skip)")
    p.add_argument("--pmc", default=None,
                   help="committed rocprofv3 PMC traffic summary for the roofline 'traffic' field "
                        "(default: profiles/pmc_traffic.json for c3, profiles/pmc_traffic_<workload>.json otherwise)")
    a = p.parse_args()
    if a.pmc is None:
        a.pmc = os.path.join(REPO, "profiles", "pmc_traffic.json" if a.workload == "c3" else f"pmc_traffic_{a.workload}.json")
    return a


def workload_name(w, world, distributed):
    """config.workload: the BASELINE.json config the line measures."""
    if w in ("c3", "c3w"):
        head = ("C3 |R|=|S|=1e8 per GPU, (int64 key, int64 payload), WHERE col0 > 5000, JOIN_KEY 0" if w == "c3" else
                "C3-wide (SURVEY 8(d) stress input) |R|=|S|=1e8 per GPU, full-range signed int64 keys, S planted "
                "with R's keys in a random third of its rows, WHERE col0 > INT64_MIN, JOIN_KEY 0")
        return head + ("; range partition + RCCL exchange, weak scaling (|R|=|S|=%d x 1e8)" % world
                       if distributed else "")
    base = {"c4": "C4 (BASELINE configs[3]) 1B x 1B rows, uniform int64 keys in [1,3e9]",
            "c5": "C5 (BASELINE configs[4]) 100M x 1B rows, Zipf(0.9) keys over 1e8 values"}[w]
    if distributed:
        return base + ", WHERE col0 > 5000; range-partitioned across %d GPU%s via RCCL%s (strong scaling)" % (
            world, "s" if world > 1 else "", " loopback" if world == 1 else "")
    return base + ", WHERE col0 > 5000; ONE GPU (the library's partitioned mode)"


def step_single(R, S, bufs):
    """One pass of the hot path: the fused MSD pipeline (select + stable sort of
    R and S, 1:1 zip join; sorted tables and joined rows all written)."""
    Rs, Ss, J = ops.sort_merge_join(R, S, KEYS[0], KEYS[1], (SELECT[0], SELECT[1]), (SELECT[2], SELECT[3]),
                                    R_sorted=bufs["R"], S_sorted=bufs["S"], out=bufs["J"])
    return (Rs.shape[0], Ss.shape[0], J.shape[0])


MASK64 = (1 << 64) - 1


def verify_distributed(J, rank, world, dev, full_tables, wire=None):
    """Self-check of a distributed (or --loopback) result, after the timed
    steps: every rank digests its slice of the joined rows at its global
    position (smj_dev_digest: order-sensitive, position-mixed), the digests
    and row counts are gathered, and rank 0 runs the single-GPU call
    (smj_dev_sort_merge_join, the partitioned mode above 1.6e8 rows) on the
    whole job's tables -- full_tables() makes them -- and digests the same
    slices of its result.  Returns (ok on every rank, details on rank 0).
    The reference order is the one the reference's host builds by
    concatenating DPU outputs in DPU order (app.c:585-692).  wire: the
    device the gathers run on (cpu under gloo; default dev)."""
    t0 = time.perf_counter()
    wire = dev if wire is None else wire
    cnt = torch.tensor([J.shape[0]], dtype=torch.int64, device=wire)
    allc = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(allc, cnt)
    counts = [int(c.item()) for c in allc]
    offs = [sum(counts[:r]) for r in range(world)]
    d = ops.digest_async(J, offs[rank]).to(wire)
    alld = [torch.zeros_like(d) for _ in range(world)]
    dist.all_gather(alld, d)
    got = [int(x.item()) & MASK64 for x in alld]
    flag = torch.zeros(1, dtype=torch.int64, device=wire)
    info = None
    if rank == 0:
        torch.cuda.empty_cache()  # the distributed path's cached blocks, for the library's own allocations
        Rf, Sf = full_tables()
        log(f"[verify] reference call on {Rf.shape[0]} x {Sf.shape[0]} rows "
            f"(free {torch.cuda.mem_get_info()[0] / 2**30:.1f} GiB)")
        _, _, Jf = ops.sort_merge_join(Rf, Sf, KEYS[0], KEYS[1], (SELECT[0], SELECT[1]), (SELECT[2], SELECT[3]))
        log(f"[verify] reference call done: {Jf.shape[0]} joined rows")
        total = Jf.shape[0]
        ref = [ops.digest(Jf[offs[r]: offs[r] + counts[r]], offs[r]) if offs[r] + counts[r] <= total else None
               for r in range(world)]
        whole = ops.digest(Jf)
        bad = [r for r in range(world) if ref[r] != got[r]]
        ok = not bad and sum(counts) == total and (sum(got) & MASK64) == whole
        flag.fill_(1 if ok else 0)
        info = {"ok": ok, "against": "single-GPU smj_dev_sort_merge_join on the whole job's tables (rank 0)",
                "kind": "self-consistency: the distributed path against the same library's single-GPU call (they "
                        "share the sampler, heavy-key and packed pass-B kernels); that call is checked against the "
                        "CPU port by the N = 1 line (cpu_baseline_mt) and against the oracle by the GPU tests",
                "joined_rows": sum(counts), "reference_joined_rows": total, "digest": "%016x" % (sum(got) & MASK64),
                "reference_digest": "%016x" % whole, "mismatched_ranks": bad,
                "seconds": None}
        del Rf, Sf, Jf
        torch.cuda.empty_cache()
    dist.broadcast(flag, 0)
    if info is not None:
        info["seconds"] = round(time.perf_counter() - t0, 2)
    return bool(flag.item()), info


def main():
    global SELECT
    a = parse()
    if a.workload == "c3w":
        SELECT = SELECT_WIDE
    _claim_stdout()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        log(f"note: --gpus {a.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # SMJ_BENCH_REHEARSE=1: the N > 1 line rehearsed on fewer GPUs than ranks
    # (tests/test_gpu_bench.py on the one-GPU test box): ranks share the
    # visible GPUs, and the process group is gloo (RCCL takes one GPU per
    # rank) -- smj.dist then stages the exchange through host memory.  Never
    # a measurement: the line says so in config.parallelism.
    rehearse = os.environ.get("SMJ_BENCH_REHEARSE", "0") != "0"
    if rehearse:
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    backend = "gloo" if rehearse else "nccl"
    wire = torch.device("cpu") if backend == "gloo" else dev  # bench.py's own collectives
    if world > 1 or a.loopback:
        kw = {} if rehearse else {"device_id": dev}
        if world == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group(backend, rank=0, world_size=1, **kw)
        else:
            dist.init_process_group(backend, **kw)
    distributed = world > 1 or a.loopback

    n = a.rows
    strong = a.workload in ("c4", "c5")  # C4 / C5: the job's tables are fixed (BASELINE configs[3], [4])
    if a.workload in ("c3", "c3w"):
        NR = NS = n * world       # weak: n rows per table per GPU
    elif a.workload == "c4":
        NR = NS = 1_000_000_000
    else:
        NR, NS = 100_000_000, 1_000_000_000
    key_range = {"c5": 100_000_000, "c3w": None}.get(a.workload, a.key_range or 3 * NR)  # C5: the Zipf domain; c3w: 2^64

    def shard(N):  # this rank's contiguous slice of a table of N global rows
        if not strong:
            return rank * n, n
        r0 = N * rank // world
        return r0, N * (rank + 1) // world - r0

    (r0R, nr), (r0S, ns) = shard(NR), shard(NS)
    if a.workload == "c5":
        R = ops.gen_zipf(nr, row0=r0R, seed=3, domain=100_000_000, theta=0.9, device=dev)
        S = ops.gen_zipf(ns, row0=r0S, seed=4, domain=100_000_000, theta=0.9, device=dev)
    elif a.workload == "c3w":
        R = ops.gen_wide(nr, row0=r0R, seed=1, device=dev)
        S = ops.gen_wide(ns, row0=r0S, seed=2, plant_seed=1, plant_rows=NR, device=dev)
    else:
        R = ops.gen_uniform(nr, row0=r0R, seed=1, key_range=key_range, device=dev)
        S = ops.gen_uniform(ns, row0=r0S, seed=2, key_range=key_range, device=dev)
    if strong:
        n = NS  # rows per table of one single-GPU call (the PMC summary's key)
    bufs = None
    if not distributed:
        bufs = {"R": torch.empty_like(R), "S": torch.empty_like(S),
                "J": torch.empty((min(nr, ns), 3), dtype=torch.int64, device=dev)}
    torch.cuda.synchronize()

    lb = {}

    def step():
        if not distributed:
            return step_single(R, S, bufs)
        return sdist.sort_merge_join(R, S, select=SELECT, keys=KEYS, stats=lb, loopback=a.loopback)

    t_start = time.perf_counter()

    def progress(what):  # one stderr line per phase (rank 0): a long run shows where it is
        if rank == 0:
            log(f"[bench {time.perf_counter() - t_start:7.1f} s] {what}")

    progress(f"inputs ready ({nr} + {ns} rows on this rank)")
    for i in range(a.warmup):
        step()
        torch.cuda.synchronize()
        progress(f"warmup step {i + 1}/{a.warmup} done")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ms0 = torch.cuda.memory_stats(dev)
    t0 = time.perf_counter()
    res = None
    for i in range(a.steps):
        # the previous step's joined rows are dead before the next step runs:
        # holding them made every distributed step after the first allocate a
        # second output buffer (6 GB at C4) inside the timed region -- 0.1-0.5 s
        # on boxes whose driver was still returning an earlier process's memory
        # (profiles/r06/r06y5, r06z2)
        res = None
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    ms1 = torch.cuda.memory_stats(dev)
    # device allocations inside the timed steps (a cache miss of the torch
    # allocator maps fresh memory -- tens of ms per large buffer): logged, so
    # a slow run shows whether that is where its time went
    progress("allocator in the timed steps: " + ", ".join(
        f"{k} +{ms1.get(k, 0) - ms0.get(k, 0)}" for k in ("num_alloc_retries", "num_device_alloc", "num_device_free")))
    # the per-kernel breakdown (HIP events around every pipeline stage) from
    # separate steps after the timed ones: recording the events adds a little
    # host gap per stage, so they stay out of the timed steps
    psteps = max(1, min(a.steps, 5))
    ops.prof_enable(True)
    ops.prof_report()  # reset
    for i in range(psteps):
        step()
    torch.cuda.synchronize()
    ops.prof_enable(False)
    progress(f"{a.steps} timed + {psteps} profiled steps done ({dt / a.steps * 1e3:.3f} ms/step)")
    prof = ops.prof_report()
    # pass-B row layout of the last pipeline call (MsdPlan::packB: one 8-B word per
    # row when the payload fits int32 and the selected keys span < 2^32, else 16-B rows)
    packb = ops.msd_packb() if not distributed else None
    if world == 1:
        log(f"msd stats (single-key groups, LSD-fallback groups, mR, mS): {ops.msd_stats()}; "
            f"(groups, radix-tier, wide-tier, in-LDS LSD): {ops.msd_groups()}")

    joined = int(res[2]) if not distributed else int(res.shape[0])

    def full_tables():  # the whole job's tables (rank 0's verification call)
        if world == 1:
            return R, S
        if a.workload == "c5":
            return (ops.gen_zipf(NR, row0=0, seed=3, domain=100_000_000, theta=0.9, device=dev),
                    ops.gen_zipf(NS, row0=0, seed=4, domain=100_000_000, theta=0.9, device=dev))
        if a.workload == "c3w":
            return (ops.gen_wide(NR, row0=0, seed=1, device=dev),
                    ops.gen_wide(NS, row0=0, seed=2, plant_seed=1, plant_rows=NR, device=dev))
        return (ops.gen_uniform(NR, row0=0, seed=1, key_range=key_range, device=dev),
                ops.gen_uniform(NS, row0=0, seed=2, key_range=key_range, device=dev))

    verified, verification = None, None
    if distributed and a.verify:
        progress("verification: digests of every rank's slice, then the single-GPU call on rank 0")
        verified, verification = verify_distributed(res, rank, world, dev, full_tables, wire)
        if rank == 0:
            log(f"verification: {verification}")
    rank_rows = [nr + ns]  # every rank's generated input rows (R + S), rank order
    if world > 1:
        got = [torch.zeros(1, dtype=torch.int64, device=wire) for _ in range(world)]
        dist.all_gather(got, torch.tensor([nr + ns], dtype=torch.int64, device=wire))
        rank_rows = [int(g.item()) for g in got]
    t = torch.tensor([dt, float(joined)], dtype=torch.float64, device=wire)
    if world > 1:
        tt = t.clone()
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        joined = int(tt[1].item())
        dt = float(t[0].item())
    ms_step = dt / a.steps * 1e3
    rows_step = NR + NS  # the whole job's input rows per step
    value = rows_step / (dt / a.steps)

    # roofline of the dominant kernel: algorithmic bytes / its event time
    # (kernels with algorithmic bytes only: at small test sizes a fixed-cost
    # bookkeeping kernel can take the most time)
    dom = max((kv for kv in prof.items() if kv[1]["bytes"] > 0), key=lambda kv: kv[1]["ms"], default=(None, None))
    roof = None
    pmc = None
    from smj._lib import source_sha as _source_sha
    source_sha = _source_sha()
    # the PMC summary is per launch of ONE configuration (profiles/pmc_traffic.json:
    # the single-GPU C3 call): its bytes are attached only to a line timing the
    # same launches -- never to the dist / loopback stages (half-size launches)
    # or another workload
    if os.path.exists(a.pmc) and not distributed:
        with open(a.pmc) as f:
            pmc = json.load(f)
        if pmc.get("rows_per_table") != n or pmc.get("workload", "c3") != a.workload:
            pmc = None
        elif pmc.get("source_sha") != source_sha:
            # the summary was collected on another build of the library: its bytes
            # may describe kernels that no longer exist
            log(f"PMC summary {a.pmc}: source_sha {pmc.get('source_sha')} != this tree's {source_sha}: not attached")
            pmc = None
    if pmc and pmc.get("runs"):
        # ... and with the same launches per step (the partitioned mode's part
        # count changes them): a summary of other launches is not attached
        for name, d in prof.items():
            k = pmc.get("kernels", {}).get(name)
            if k and d["launches"] and k["launches"] * psteps != d["launches"] * pmc["runs"]:
                log(f"PMC summary {a.pmc}: {name} {k['launches']} launches in {pmc['runs']} steps, "
                    f"this run {d['launches']} in {psteps}: not attached")
                pmc = None
                break
    if dom[0]:
        name, d = dom
        ach = d["bytes"] / (d["ms"] * 1e-3) / 1e9
        traffic = None
        if pmc:
            k = pmc.get("kernels", {}).get(name)
            if k:
                traffic = k.get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "kernel": name, "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "alg_bytes_per_launch": d["bytes"] / max(d["launches"], 1),
                "avg_launch_ms": round(d["ms"] / max(d["launches"], 1), 4),
                "share_of_step": round(d["ms"] / psteps / ms_step, 3)}
    # SURVEY 8(d) sort-phase figure: bytes the sort passes FETCH (PMC FETCH_SIZE x 2,
    # profiles/pmc_traffic.json) per launch over their measured launch time
    sort_passes = None
    if pmc:
        sort_passes = {}
        for name in ("msd_part_a", "msd_part_b", "msd_final", "msd_final_tiers"):
            k, d = pmc.get("kernels", {}).get(name), prof.get(name)
            if k and d and d["launches"]:
                fetched = 2.0 * k["fetch_kib_raw"] * 1024
                gbs = fetched / (d["ms"] / d["launches"] * 1e-3) / 1e9
                sort_passes[name] = {"fetched_bytes_per_launch": round(fetched), "fetch_GBps": round(gbs, 1),
                                     "frac_of_peak": round(gbs / HBM_PEAK_GBS, 4)}
        # each pass writes what it reads and HBM's data bus carries both
        # directions: a pass can fetch at most half the peak
        sort_passes["read_ceiling_frac_of_peak"] = 0.5
        if any(v["frac_of_peak"] > 0.5 for v in sort_passes.values() if isinstance(v, dict)):
            log("PMC summary does not match the timed launches: traffic / sort_passes dropped")
            sort_passes = None
            if roof:
                roof["traffic"] = None
    # whole-pipeline roofline: 48 B per input row + 24 B per joined row
    b_alg = 48.0 * rows_step + 24.0 * joined
    pipe_gbs = b_alg / (dt / a.steps) / 1e9

    cpu = None
    if rank == 0 and world == 1 and a.cpu_sample > 0 and a.workload in ("c3", "c3w") and not distributed:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU baseline leg only
        m = min(a.cpu_sample, n)
        Rh = R[:m].cpu().numpy()
        Sh = S[:m].cpu().numpy()
        secs, jrows, kind = oracle.time_cpu_pipeline(Rh, Sh, SELECT, KEYS)
        # the reference sort is O(n^2) (cpu_app.c:172-202), so its
        # rows/s at the sample overstates it at C3 size; the full workload's
        # time extrapolated as (n / m)^2 from the measured sample
        full_s = secs * (n / m) ** 2
        cpu = {"value": round(2 * m / secs, 1), "unit": "rows/s", "cores": 1, "kind": kind,
               "sample": f"first {m} rows of R and of S of this workload "
                         f"({'keys in [1,%d]' % key_range if key_range else 'full-range int64 keys'}); "
                         f"cpu_app.c select + O(n^2) insertion sort + zip join, 1 thread, gcc -O2; "
                         f"{secs:.2f} s, {jrows} joined rows",
               "n2_extrapolation": {"rows_per_table": n, "seconds": round(full_s, 1), "days": round(full_s / 86400, 2),
                                    "value": round(2 * n / full_s, 3), "unit": "rows/s",
                                    "basis": f"measured {secs:.2f} s at {m} rows/table x ({n}/{m})^2"}}

    cpu_mt = None
    if rank == 0 and world == 1 and a.cpu_mt and not distributed:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # CPU baseline leg only
        # the host cores this process may use: the CPU share granted to this GPU's job
        # (OMP_NUM_THREADS on the GPU box), else every core the process is affine to
        usable = len(os.sched_getaffinity(0))
        threads = min(int(os.environ.get("OMP_NUM_THREADS", "0")) or usable, usable)
        secs, rows, outs = oracle.mt_pipeline(R.cpu().numpy(), S.cpu().numpy(), SELECT, KEYS, threads,
                                              outputs=True)
        cpu_mt = {"value": round(rows_step / secs, 1), "unit": "rows/s", "cores": threads, "kind": "port",
                  "sample": f"the full workload ({NR} x {NS} rows): oracle/cpu_mt.cpp, cpu_app.c's select + "
                            f"stable sort + zip join on {threads} threads (the host cores granted to this GPU's "
                            f"job; {usable} usable, {os.cpu_count()} in the node) (chunk sort + merge rounds), g++ -O3; "
                            f"{secs:.2f} s, {rows[2]} joined rows"}
        # the timed GPU step's outputs (last step: the same deterministic result)
        # against the CPU port's, by the order-sensitive digest (smj_dev_digest
        # on the device, its C restatement oracle.digest on the host)
        if a.verify:
            gpu_out = (bufs["R"][: res[0]], bufs["S"][: res[1]], bufs["J"][: res[2]])
            dg = [ops.digest(t) for t in gpu_out]
            dc = [oracle.digest(t) for t in outs]
            ok = tuple(res) == tuple(rows) and dg == dc
            verified = ok
            verification = {"ok": ok, "against": "oracle/cpu_mt.cpp on the full workload (sorted R, sorted S, "
                                                 "joined rows: row counts + order-sensitive digests)",
                            "kind": "independent: the CPU port of cpu_app.c's select + stable sort + zip join",
                            "rows": list(res), "cpu_rows": list(rows),
                            "digests": ["%016x" % x for x in dg], "cpu_digests": ["%016x" % x for x in dc]}
            log(f"verification: {verification}")
        del outs

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "rows/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None, "dtype": "int64",
            "data": {"c3w": "synthetic: splitmix64 full-range signed int64 keys, S planted with R's keys in a random "
                            "third of its rows (smj_dev_gen_wide), payload = global row index (generated on device)",
                     "c5": "synthetic: Zipf(0.9) keys over 1e8 values (smj_dev_gen_zipf), payload = global row index "
                           "(generated on device)"}.get(
                a.workload, "synthetic: splitmix64 keys iid uniform in [1,3n], payload = global row index "
                            "(generated on device)"),
            "config": {"workload": workload_name(a.workload, world, distributed),
                       "rows_per_table_per_gpu": [nr, ns], "rows_per_table_total": [NR, NS],
                       "rank_input_rows": rank_rows, "key_range": key_range,
                       "joined_rows": joined, "parallelism": f"range-partition x{world}" + (" (RCCL loopback)" if a.loopback else "")
                                      + (" (REHEARSAL: gloo, ranks sharing GPUs; not a measurement)" if rehearse else ""),
                       "load_max_over_mean": round(lb.get("load_max_over_mean", 1.0), 4),
                       "rank_rows_after_exchange": lb.get("loads"),
                       "exchange_stages": lb.get("stages", 0),
                       "select": list(SELECT),
                       "pass_b_layout": None if packb is None else ("packed 8-B words" if packb else "16-B rows"),
                       "source_sha": source_sha},
            "roofline": roof,
            "pipeline_roofline": {"alg_bytes_per_step": b_alg, "achieved": round(pipe_gbs, 1),
                                  "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                                  "frac": round(pipe_gbs / (HBM_PEAK_GBS * world), 4)},
            "kernels": {k: {"launches": v["launches"], "ms_per_step": round(v["ms"] / psteps, 4),
                            "GBps": round(v["bytes"] / max(v["ms"], 1e-9) / 1e6, 1)} for k, v in prof.items()},
            "cpu_baseline": cpu,
            "cpu_baseline_mt": cpu_mt,
            "sort_passes": sort_passes,
            "verified": verified,
            "verification": verification,
        }
        emit(line)
    if dist.is_initialized():
        dist.destroy_process_group()
    if verified is False:
        log("VERIFICATION FAILED: the result differs from the reference call")
        sys.exit(3)


if __name__ == "__main__":
    main()
