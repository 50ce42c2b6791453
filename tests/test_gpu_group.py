"""One caller, several devices (mmba.h ABI 9, SURVEY 8(b) "Threading"): a
Solver on ``Context.multi(devices)`` is frame-sharded over the devices and
driven from the calling thread -- the reference calls solveFrames once, on
Maya's main thread (adjust_base.cpp:1174-1183).  On a one-GPU box the device
is named N times, so the N shards run on device 0 through the same entry
(the in-process transport).

Bars: the group solve equals the explicitly threaded shards
(test_gpu_sharded.run_sharded, the one-process-per-GPU code path with its
all-gather hand-back) bit for bit; it matches the oracle at 1e-6 where the
sharded tests do; interrupts, plan reuse, measure, the outputs of a
device-resident solve and the problems that do not shard behave as the
unsharded plan does."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Context, Solver

from test_gpu_sharded import CASES, run_sharded

pytestmark = pytest.mark.gpu


def group_solve(prob, opt, n, **kw):
    ctx = Context.multi([0] * n)
    try:
        assert ctx.num_devices == n
        s = Solver(prob, opt, context=ctx)
        try:
            shards = s.num_shards
            out = s.solve(**kw)
        finally:
            s.close()
    finally:
        ctx.close()
    return out, shards


def unsharded(prob, opt, gpu_ctx, **kw):
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        return s.solve(**kw)
    finally:
        s.close()


@pytest.mark.parametrize("nshards", [2, 4, 8])
def test_group_equals_threaded_shards(nshards):
    """The C4 spec scene, first full step (2 evaluations): the group entry and
    the explicitly threaded shards run the same collectives on the same
    partition, so every output agrees bit for bit -- x from each shard's own
    parameters, fvec / errorDistanceList from each shard's own observations
    (group) against the all-gather hand-back (threads)."""
    prob = S.make_config(3, frames=20 * nshards, scale=0.002 * nshards)
    opt = S.config_options(prob, iterations=2)
    g, shards = group_solve(prob, opt, nshards)
    assert shards == nshards
    t = run_sharded(prob, opt, nshards)[0]
    np.testing.assert_array_equal(g.x, t.x)
    np.testing.assert_array_equal(g.fvec, t.fvec)
    np.testing.assert_array_equal(g.err_user, t.err_user)
    np.testing.assert_array_equal(g.err_dist, t.err_dist)
    np.testing.assert_array_equal(g.fnorm_trace, t.fnorm_trace)
    for k in ("reason_number", "iterations", "function_evals", "jacobian_evals",
              "error_final", "error_avg", "error_min", "error_max", "error_rms"):
        assert g.result[k] == t.result[k], k


@pytest.mark.parametrize("nshards", [2, 4, 8])
def test_group_first_step_matches_unsharded(nshards, gpu_ctx):
    """x after the first full LM step on the 6-frame C4 variant, group of
    nshards against the unsharded solve (the bar of
    test_gpu_sharded.test_sharded_ba_x_before_the_valley: 1e-6)."""
    prob = S.make_config(3, frames=20 * nshards, scale=0.002 * nshards, window=6,
                         depth=(4.0, 10.0))
    opt = S.config_options(prob, iterations=2)
    ref = unsharded(prob, opt, gpu_ctx)
    g, _ = group_solve(prob, opt, nshards)
    for k in ("reason_number", "iterations", "function_evals"):
        assert g.result[k] == ref.result[k], k
    np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-7)
    assert np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3)) <= 1e-6
    np.testing.assert_allclose(g.fvec, ref.fvec, rtol=0, atol=1e-6 * np.max(np.abs(ref.fvec)))


@pytest.mark.parametrize("nshards,wc", [(2, False), (4, False), (4, True)])
def test_group_fused_jacobian_shards(nshards, wc, gpu_ctx):
    """Shards of >= 256 camera-frames take the fused Jacobian + camera-frame
    normal-equation pass (k_jac_ne_u, the bench scene's path; the smaller
    sharded scenes take the split passes): 256 frames per shard at a fifth of
    the C4 bundle density, and the 6-frame variant (the partitioned band
    form).  First full step against the unsharded solve: every ||f|| at 1e-7
    and x at 1e-6 (the default whole-S form runs the unsharded solver on the
    all-reduced S); then the whole run's first five ||f|| at 1e-6 and the
    final cost at 1e-3 (a wrong block or a missing gradient term diverges at
    the first step: 1.2e9 against 476)."""
    kw = dict(window=6, depth=(4.0, 10.0)) if wc else {}
    prob = S.make_config(3, frames=256 * nshards, scale=0.1 * nshards, **kw)
    for it in (2, 60):
        opt = S.config_options(prob, iterations=it)
        ref = unsharded(prob, opt, gpu_ctx)
        g, shards = group_solve(prob, opt, nshards)
        assert shards == nshards
        if it == 2:
            np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-7)
            assert np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3)) <= 1e-6
        else:
            np.testing.assert_allclose(g.fnorm_trace[:5], ref.fnorm_trace[:5], rtol=1e-6)
            assert abs(g.result["error_final"] - ref.result["error_final"]) <= \
                1e-3 * ref.result["error_final"]


@pytest.mark.parametrize("idx,kw,nshards", CASES)
def test_group_matches_oracle(idx, kw, nshards, oracle):
    """The sharded oracle cases through the group entry: reason, counts,
    every ||f|| of the trace and x at 1e-6 against the oracle."""
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    xr, fr, eur, edr, rr, trr = oracle.solve(prob, opt)
    g, shards = group_solve(prob, opt, nshards)
    assert shards == nshards
    assert g.result["reason_number"] == rr.reason_number
    assert g.result["outer_iterations"] == rr.outer_iterations
    np.testing.assert_allclose(g.fnorm_trace, trr, rtol=1e-6, atol=1e-9 * trr[0])
    assert np.max(np.abs(g.x - xr) / np.maximum(np.abs(xr), 1e-3)) <= 1e-6
    np.testing.assert_allclose(g.err_dist, edr, rtol=0, atol=1e-4 * np.max(np.abs(edr)))


@pytest.mark.parametrize("after", [1, 2, 7, 40])
def test_group_interrupt(after, gpu_ctx):
    """The interrupt callback is polled on the calling thread only and its
    answer reaches every shard: the group stops where the unsharded solve
    stops (reason -1, the same evaluation counts)."""
    prob = S.make_config(1, frames=24, scale=0.05)
    opt = S.config_options(prob)

    def make():
        calls = [0]

        def cb():
            calls[0] += 1
            return calls[0] > after
        return cb, calls

    cb, calls_u = make()
    ref = unsharded(prob, opt, gpu_ctx, interrupt=cb)
    cb, calls_g = make()
    g, _ = group_solve(prob, opt, 2, interrupt=cb)
    assert calls_g[0] == calls_u[0]
    for k in ("reason_number", "iterations", "function_evals", "jacobian_evals",
              "user_interrupted"):
        assert g.result[k] == ref.result[k], k
    assert g.result["reason_number"] == -1


def test_group_reuse_measure_and_outputs(gpu_ctx):
    """Plan reuse through the group: two solves give the same bits; a
    device-resident solve's outputs fetched afterwards equal the solve's own
    hand-back; measure (at x0 and at the solution) equals the unsharded
    measure's residuals and statistics."""
    prob = S.make_config(1, frames=36, scale=0.05)
    opt = S.config_options(prob)
    ctx = Context.multi([0, 0, 0])
    try:
        s = Solver(prob, opt, context=ctx)
        try:
            a = s.solve()
            b = s.solve()
            np.testing.assert_array_equal(a.x, b.x)
            np.testing.assert_array_equal(a.fvec, b.fvec)
            c = s.solve(fetch=False)
            np.testing.assert_array_equal(c.x, a.x)
            f, eu, ed = s.outputs()
            np.testing.assert_array_equal(f, a.fvec)
            np.testing.assert_array_equal(eu, a.err_user)
            np.testing.assert_array_equal(ed, a.err_dist)
            mg = [s.measure(), s.measure(a.x)]
        finally:
            s.close()
    finally:
        ctx.close()
    u = Solver(prob, opt, context=gpu_ctx)
    try:
        mu = [u.measure(), u.measure(a.x)]
    finally:
        u.close()
    for (fg, eug, edg, stg), (fu, euu, edu, stu) in zip(mg, mu):
        np.testing.assert_array_equal(fg, fu)
        np.testing.assert_array_equal(eug, euu)
        np.testing.assert_array_equal(edg, edu)
        np.testing.assert_allclose(stg, stu, rtol=1e-13)


def test_group_replicated_problem(gpu_ctx):
    """A problem the frame partition cannot take (rolling shutter) is solved
    by the first device alone: one shard, the unsharded plan's bits."""
    prob = S.make_config(4, frames=12, scale=0.05, rolling_shutter=0.5)
    opt = S.config_options(prob, iterations=6)
    ref = unsharded(prob, opt, gpu_ctx)
    g, shards = group_solve(prob, opt, 2)
    assert shards == 1
    np.testing.assert_array_equal(g.x, ref.x)
    np.testing.assert_array_equal(g.fvec, ref.fvec)
    np.testing.assert_array_equal(g.fnorm_trace, ref.fnorm_trace)


def test_group_single_device_is_plain_plan(gpu_ctx):
    prob = S.make_config(1, frames=24, scale=0.05)
    opt = S.config_options(prob)
    ref = unsharded(prob, opt, gpu_ctx)
    g, shards = group_solve(prob, opt, 1)
    assert shards == 1
    np.testing.assert_array_equal(g.x, ref.x)
    np.testing.assert_array_equal(g.fvec, ref.fvec)


def test_group_refusals():
    with pytest.raises(MmbaError) as e:
        Context.multi([0, 99])
    assert e.value.code == abi.MMBA_ERR_INVALID
    prob = S.make_config(3, frames=40, scale=0.004)
    opt = S.config_options(prob, iterations=2)
    ctx = Context.multi([0, 0])
    try:
        s = Solver(prob, opt, context=ctx)
        try:
            with pytest.raises(MmbaError) as e:
                s.jacobian(prob.x0)
            assert e.value.code == abi.MMBA_ERR_UNSUPPORTED
            # the refusal leaves the group usable
            s.solve()
        finally:
            s.close()
    finally:
        ctx.close()


def _group_solver(prob, opt, n):
    ctx = Context.multi([0] * n)
    return ctx, Solver(prob, opt, context=ctx)


def test_group_shard_failure_releases_peers(paths):
    """a shard failing with an ordinary error (Invalid) in the
    middle of a solve, while its peer waits in a collective, releases the
    peer: the call returns the failing shard's code in bounded time and the
    group is unusable afterwards (MMBA_ERR_COMM), never a hang."""
    import time
    prob = S.make_config(1, frames=24, scale=0.05)
    opt = S.config_options(prob)
    ctx, s = _group_solver(prob, opt, 2)
    try:
        assert s.num_shards == 2
        paths(abi.PATH_FAULT_SHARD, 2)  # rank 1 fails at its first damped solve
        t0 = time.perf_counter()
        with pytest.raises(MmbaError) as e:
            s.solve()
        assert e.value.code == abi.MMBA_ERR_INVALID
        assert "injected shard fault" in str(e.value)
        assert time.perf_counter() - t0 < 30.0
        paths(abi.PATH_FAULT_SHARD, -1)
        with pytest.raises(MmbaError) as e:
            s.solve()
        assert e.value.code == abi.MMBA_ERR_COMM
    finally:
        s.close()
        ctx.close()


def test_group_stalled_shard_times_out(paths):
    """a shard that never reaches a collective costs its
    peers MMBA_ERR_COMM after the collective timeout (here 1.5 s), not a
    hang; the whole call returns once the stalled shard wakes (2 x timeout)."""
    import time
    prob = S.make_config(1, frames=24, scale=0.05)
    opt = S.config_options(prob)
    ctx, s = _group_solver(prob, opt, 2)
    try:
        assert s.num_shards == 2
        paths(abi.PATH_COMM_TIMEOUT_MS, 1500)
        paths(abi.PATH_STALL_SHARD, 2)
        t0 = time.perf_counter()
        with pytest.raises(MmbaError) as e:
            s.solve()
        dt = time.perf_counter() - t0
        assert e.value.code == abi.MMBA_ERR_COMM
        assert "timed out" in str(e.value) or "aborted" in str(e.value)
        assert 1.4 <= dt < 20.0
    finally:
        s.close()
        ctx.close()
