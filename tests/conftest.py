"""Shared pytest setup.

Markers:
  gpu  -- needs an MI355X (run with `-m gpu` on the GPU box); everything else
          runs on the CPU-only build container (`-m "not gpu"`).
"""
import gzip
import json
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "pim-sort-merge-join_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_dir(tmp_path_factory):
    """tests/golden with every *.gz fixture unpacked (session temp dir)."""
    d = tmp_path_factory.mktemp("golden")
    for name in os.listdir(GOLDEN):
        src = os.path.join(GOLDEN, name)
        if name.endswith(".gz"):
            with gzip.open(src, "rb") as g, open(d / name[:-3], "wb") as f:
                shutil.copyfileobj(g, f)
        elif os.path.isfile(src):
            shutil.copy(src, d / name)
    return d


def fixture_path(golden_dir, name):
    return str(golden_dir / (name[:-3] if name.endswith(".gz") else name))


def case_config(entry, defaults):
    cfg = entry["config"] or defaults
    sel = (cfg["SELECT_COL1"], cfg["SELECT_VAL1"], cfg["SELECT_COL2"], cfg["SELECT_VAL2"])
    keys = (cfg["JOIN_KEY1"], cfg["JOIN_KEY2"])
    return sel, keys


@pytest.fixture(scope="session")
def oracle_built():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    return True


@pytest.fixture(scope="session")
def pkg_built():
    """Build libsmj_hip.so / smj_app / libsmj_csv.so in-tree (hipcc, gfx950)."""
    subprocess.run(["make", "-s", "-j8", "-C", PKG], check=True, stdout=subprocess.DEVNULL)
    return True


@pytest.fixture(scope="session")
def gpu(pkg_built):
    import torch
    assert torch.cuda.is_available(), "gpu-marked test needs an MI355X"
    from smj import _lib
    lib = _lib.load(build_if_missing=False)
    return lib


@pytest.fixture(autouse=True)
def _gpu_memlog(request):
    """SMJ_TEST_MEMLOG=1: after each test, the device memory the library, torch
    and everything else hold (finding what keeps memory between tests)."""
    yield
    if os.environ.get("SMJ_TEST_MEMLOG") != "1":
        return
    import torch
    if not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    from smj import ops
    free, total = torch.cuda.mem_get_info()
    lib = ops.scratch_bytes()
    tor = torch.cuda.memory_reserved()
    print(f"\n[memlog] {request.node.name}: lib {lib / 2**30:.1f} GiB, torch reserved {tor / 2**30:.1f}, "
          f"free {free / 2**30:.1f}, other {(total - free - lib - tor) / 2**30:.1f}", flush=True)
