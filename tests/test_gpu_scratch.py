"""Library scratch: smj_trim / smj_set_scratch_limit (the reference's
per-phase dpu_free, app.c:307,402,503,761) and the partitioned mode's
fallback when its second scratch set cannot be had.  Every
result is compared with the CPU oracle."""
import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

from test_gpu_msd import dev, host, ref_pipeline, table  # noqa: E402

SEL = (0, 5000)


def _tables(n=300_000, seed=5):
    rng = np.random.default_rng(seed)
    return table(rng, n, 2, "uniform", 0, 0), table(rng, n, 2, "uniform", 0, 10 ** 9)


def _check(R, S, got):
    Rs, Ss, J = ref_pipeline(R, S, 0, 0, SEL, SEL)
    np.testing.assert_array_equal(host(got[0]), Rs.reshape(-1, 2))
    np.testing.assert_array_equal(host(got[1]), Ss.reshape(-1, 2))
    np.testing.assert_array_equal(host(got[2]), J.reshape(-1, 3))


def test_trim_returns_every_buffer(gpu, oracle_built):
    from smj import ops
    R, S = _tables()
    got = ops.sort_merge_join(dev(R), dev(S), 0, 0, SEL, SEL)
    torch.cuda.synchronize()
    assert ops.scratch_bytes() > 0
    ops.trim()
    assert ops.scratch_bytes() == 0
    _check(R, S, got)
    again = ops.sort_merge_join(dev(R), dev(S), 0, 0, SEL, SEL)  # scratch allocated afresh
    _check(R, S, again)


def test_trim_refused_while_a_job_is_open(gpu, oracle_built):
    from smj import _lib, ops
    R, S = _tables(200_000, 6)
    job = ops.sort_merge_join_begin(dev(R), dev(S), 0, 0, SEL, SEL)
    try:
        with pytest.raises(_lib.SmjError):
            ops.trim()
    finally:
        got = job.end()
    _check(R, S, got)
    ops.trim()


def test_scratch_limit_trims_after_each_call(gpu, oracle_built):
    from smj import ops
    R, S = _tables(250_000, 7)
    ops.set_scratch_limit(0)
    try:
        for _ in range(2):
            got = ops.sort_merge_join(dev(R), dev(S), 0, 0, SEL, SEL)
            assert ops.scratch_bytes() == 0
            _check(R, S, got)
    finally:
        ops.set_scratch_limit(-1)


@pytest.mark.parametrize("fail", [1, 2, 5])
def test_partitioned_mode_without_room_for_a_second_set(gpu, oracle_built, fail):
    """The overlapped partitioned mode (two parts in flight, two scratch sets):
    the front phase of part `fail` cannot get its scratch -- the part whose back
    is due finishes on its own set, the other set is released and the rest run
    one at a time.  Odd and even failing parts (either set), bit-exact."""
    from smj import _lib, ops
    lib = _lib.load()
    R, S = _tables(400_000, 8 + fail)
    ops.force_parts(6)
    try:
        ops.trim()  # both sets fresh
        lib.smj_debug_fail_front(fail)
        got = ops.sort_merge_join(dev(R), dev(S), 0, 0, SEL, SEL)
        torch.cuda.synchronize()
    finally:
        seq_from = lib.smj_debug_fail_front(-1)
        ops.force_parts(0)
    assert seq_from == fail
    _check(R, S, got)
