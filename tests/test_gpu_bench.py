"""bench.py's contract at small sizes on the test box's one GPU.

The driver runs `python bench.py` (N = 1) and, on an 8-GPU node, `torchrun
--nproc-per-node N bench.py --gpus N`.  The N > 1 code of bench.py (barriers,
max-over-ranks timing, the gathered row counts, the per-rank digests and rank
0's verification call) is rehearsed here with several ranks sharing cuda:0
under gloo (SMJ_BENCH_REHEARSE=1: RCCL takes one GPU per rank), so that the
first multi-GPU run is not the first time that code executes."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _run(cmd, env_extra=None, timeout=600):
    env = dict(os.environ)
    env.update(env_extra or {})
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-4000:]
    return _line(p.stdout)


@pytest.mark.gpu
def test_bench_single_gpu_line(pkg_built, oracle_built):
    """N = 1: one JSON line with the contract's fields, the CPU legs and a
    verified result (the timed step's outputs against oracle/cpu_mt.cpp)."""
    d = _run([sys.executable, "bench.py", "--rows", "2000000", "--steps", "3", "--warmup", "1",
              "--cpu-sample", "2048", "--cpu-mt", "1"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["value"] > 0
    assert d["roofline"]["bound"] == "hbm" and 0 < d["roofline"]["frac"] < 1
    assert d["cpu_baseline"]["cores"] == 1 and d["cpu_baseline_mt"]["cores"] >= 1
    assert d["verified"] is True, d["verification"]


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_bench_multi_rank_rehearsal(pkg_built, world):
    """N > 1 under torchrun: every rank generates its shard, the staged
    exchange runs, rank 0 prints one line whose value is the whole job's rows
    over the max-over-ranks time, and the distributed result is verified
    against rank 0's single-GPU call on the whole job's tables."""
    rows = 1_000_000
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
              "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py", "--gpus", str(world),
              "--rows", str(rows), "--steps", "2", "--warmup", "1"],
             {"SMJ_BENCH_REHEARSE": "1", "OMP_NUM_THREADS": "2"})
    assert d["n_gpus"] == world and d["scaling"] == "weak"
    assert d["config"]["rows_per_table_total"] == [rows * world, rows * world]
    assert d["config"]["rank_input_rows"] == [2 * rows] * world
    assert "REHEARSAL" in d["config"]["parallelism"]
    assert d["verified"] is True, d["verification"]
    assert d["verification"]["joined_rows"] == d["config"]["joined_rows"]
    assert abs(d["value"] - 2 * rows * world / (d["ms_per_step"] * 1e-3)) / d["value"] < 1e-3
