"""Frame-sharded solve on one MI355X: N shards in one process
(mmba_comm_create_local, one host thread and one stream per shard) run the same
code path as the one-process-per-GPU RCCL run.  Bar: every shard returns the
same x and result, and they match the CPU oracle like the unsharded solve
(1e-6 relative on x and on every ||f|| of the trace)."""
import os
import threading

import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd.solver import Comm, Context, Solver

pytestmark = pytest.mark.gpu


def run_sharded(prob, opt, n, replicated=None, band_solver=None):
    """Solve on n in-process shards.  replicated (list): receives each shard's
    shards_replicated statistic (1: the problem did not shard and every shard
    solved all of it, mmba_plan_create_sharded); band_solver (list): each
    shard's band_solver statistic (4: the separator form)."""
    comms = Comm.local_group(n)
    ctxs = [Context(0) for _ in range(n)]
    outs, errs, reps, bsol = [None] * n, [None] * n, [None] * n, [None] * n

    def work(r):
        try:
            s = Solver(prob, opt, context=ctxs[r], comm=comms[r])
            try:
                st = s.kernel_stats()
                reps[r] = st["shards_replicated"]
                bsol[r] = st["band_solver"]
                outs[r] = s.solve()
            finally:
                s.close()
        except Exception as e:  # noqa: BLE001 - reported below
            errs[r] = e

    ths = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ths), "sharded solve hung"
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
    assert errs == [None] * n, errs
    if replicated is not None:
        replicated[:] = reps
    if band_solver is not None:
        band_solver[:] = bsol
    return outs


# C4-type scenes with 4-frame tracks at depth 20-200 are too weakly determined
# at test sizes for an x comparison (the unsharded solve differs from the
# oracle by 1e-4 there too; only ||f|| is pinned): the Schur cases use 6-frame
# tracks at depth 4-10.  Changing only the band partition count moves x by up
# to 5e-7 on the first case, so the sharded run is compared at the same 1e-6.
WC = dict(window=6, depth=(4.0, 10.0))
# oracle x after the first step of the valley test's C4 scenes at 4 / 8 shards
SHARD_STEP = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "shard",
                          "c4_shard_step.npz")
CASES = [
    (3, dict(frames=40, scale=0.004, **WC), 2),   # bundle-Schur BA, 2 shards
    (1, dict(frames=24, scale=0.05), 2),          # C2 subset: pose + focal, no Schur
    (1, dict(frames=36, scale=0.05), 3),          # C2 subset, 3 shards (a middle shard)
    (4, dict(frames=32, scale=0.05), 2),          # C5 subset: lens globals (arrow rows)
]


def check_shards_agree(outs):
    for o in outs[1:]:
        np.testing.assert_array_equal(o.x, outs[0].x)
        np.testing.assert_array_equal(o.fvec, outs[0].fvec)
        assert o.result["iterations"] == outs[0].result["iterations"]


# reduced-system solve of a sharded plan: the separator form (default where
# it applies: no arrow; each shard's interior by parallel cyclic reduction,
# the separator system all-reduced), S all-reduced whole and solved by the
# log-depth solvers on every shard (MMBA_PATH_SHARD_SEP = 0), or the
# partitioned band chains with an all-reduced separator system
# (MMBA_PATH_SHARD_BCR = 0)
SOLVES = {"separator": {abi.PATH_SHARD_SEP: 1}, "whole": {},
          "partitioned": {abi.PATH_SHARD_BCR: 0}}


def pin_solve(paths, solve):
    for k, v in SOLVES[solve].items():
        paths(k, v)


# summation order of the in-process all-reduce: rank order, or the ring
# reduce-scatter order RCCL's ring all-reduce uses (mmba_comm.cpp)
ORDERS = {"rank": 0, "ring": 1}


@pytest.mark.parametrize("order", list(ORDERS))
@pytest.mark.parametrize("solve", list(SOLVES))
@pytest.mark.parametrize("idx,kw,nshards", CASES)
def test_sharded_matches_oracle(idx, kw, nshards, solve, order, oracle, paths):
    pin_solve(paths, solve)
    paths(abi.PATH_LOCAL_RING, ORDERS[order])
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    xr, fr, eur, edr, rr, trr = oracle.solve(prob, opt)
    outs = run_sharded(prob, opt, nshards)
    check_shards_agree(outs)
    g = outs[0]
    assert g.result["reason_number"] == rr.reason_number, (g.result, rr.as_dict())
    assert g.result["outer_iterations"] == rr.outer_iterations
    np.testing.assert_allclose(g.fnorm_trace, trr, rtol=1e-6, atol=1e-9 * trr[0])
    assert np.max(np.abs(g.x - xr) / np.maximum(np.abs(xr), 1e-3)) <= 1e-6
    assert abs(g.result["error_final"] - rr.error_final) <= 1e-6 * rr.error_final
    # per-residual values move with the roundoff-determined last digits of x
    # (x at 8e-7 -> residuals at 1e-5 px on the Schur case): checked loosely
    np.testing.assert_allclose(g.fvec, fr, rtol=0, atol=1e-4 * np.max(np.abs(fr)))
    np.testing.assert_allclose(g.err_dist, edr, rtol=0, atol=1e-4 * np.max(np.abs(edr)))


@pytest.mark.parametrize("solve", list(SOLVES))
def test_sharded_ba_three_shards_structure(solve, gpu_ctx, paths):
    """3 shards (one with separators on both sides) on a bundle-Schur scene,
    against the unsharded GPU solve.  This scene is not conditioned well
    enough for a 1e-6 comparison (a rejected trial point moves by 1.4e-6), so
    the check is structural: same reason and counts, trace within 1e-5, x
    within 1e-4 (decomposition errors show up at 1e-2)."""
    pin_solve(paths, solve)
    prob = S.make_config(3, frames=54, scale=0.006, **WC)
    opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
    finally:
        s.close()
    outs = run_sharded(prob, opt, 3)
    check_shards_agree(outs)
    g = outs[0]
    for k in ("reason_number", "iterations", "outer_iterations", "function_evals"):
        assert g.result[k] == ref.result[k], k
    np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-5)
    assert np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3)) <= 1e-4


@pytest.mark.parametrize("nshards", [4, 8])
def test_sharded_ba_many_shards(nshards, gpu_ctx):
    """The shard counts the 1/2/4/8-GPU bench runs (default reduced solve: the
    separator form)
    on the 2-shard oracle case's scene density (20 frames per shard), against
    the unsharded GPU solve.  Every shard agrees bit for bit; same reason;
    the first five ||f|| (where a decomposition error shows: a wrong Schur
    block or halo moves the first step by 1e-2) within 1e-6; final ||f||
    within 1e-3.  These scenes then creep for ~30 evaluations along a weakly
    determined direction, where the summation order of 4 shards moves the
    stopping point (final ||f|| 2.5e-4 apart, measured); x is therefore not
    compared (the 2- and 3-shard tests above pin x against the oracle and
    the unsharded solve)."""
    prob = S.make_config(3, frames=20 * nshards, scale=0.002 * nshards, **WC)
    opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
    finally:
        s.close()
    outs = run_sharded(prob, opt, nshards)
    check_shards_agree(outs)
    g = outs[0]
    assert g.result["reason_number"] == ref.result["reason_number"]
    np.testing.assert_allclose(g.fnorm_trace[:5], ref.fnorm_trace[:5], rtol=1e-6)
    assert abs(g.result["error_final"] - ref.result["error_final"]) <= \
        1e-3 * ref.result["error_final"]
    # x after the first full step of the same run: the
    # sharded and unsharded solves from x0 with the evaluation budget capped
    # at 2, every component within 1e-6
    opt1 = S.config_options(prob, iterations=2)
    s = Solver(prob, opt1, context=gpu_ctx)
    try:
        ref1 = s.solve()
    finally:
        s.close()
    g1 = run_sharded(prob, opt1, nshards)[0]
    np.testing.assert_allclose(g1.fnorm_trace, ref1.fnorm_trace, rtol=1e-7)
    assert np.max(np.abs(g1.x - ref1.x) / np.maximum(np.abs(ref1.x), 1e-3)) <= 1e-6


@pytest.mark.parametrize("solve", ["separator", "whole"])
@pytest.mark.parametrize("order", list(ORDERS))
@pytest.mark.parametrize("nshards", [2, 4, 8])
@pytest.mark.parametrize("scene", ["c4", "wc"])
def test_sharded_ba_x_before_the_valley(scene, nshards, order, solve, gpu_ctx, paths):
    """x itself, on the headline C4 structure (4-frame tracks at depth
    20-200) and on the 6-frame variant, sharded against unsharded, with the
    evaluation budget capped at 2 (x0 and one full LM step): past that the
    reference itself does not determine x to 1e-6 on this structure
    (profiles/r2_parity/c4_envelope.txt).  The step is a full
    Schur / reduced solve across every shard boundary, so a wrong block, a
    missing halo term or a wrong separator shows up in x at 1e-3..1e-2; the
    bar here is 1e-6 relative on every component."""
    paths(abi.PATH_LOCAL_RING, ORDERS[order])
    kw = WC if scene == "wc" else {}
    prob = S.make_config(3, frames=20 * nshards, scale=0.002 * nshards, **kw)
    opt = S.config_options(prob, iterations=2)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
    finally:
        s.close()
    pin_solve(paths, solve)
    bsol = []
    outs = run_sharded(prob, opt, nshards, band_solver=bsol)
    check_shards_agree(outs)
    # the separator form where it applies (no arrow, half bandwidth <= 23:
    # the C4 spec's 4-frame tracks; the 6-frame variant's band is wider)
    if solve == "separator" and scene == "c4":
        assert bsol == [4] * nshards, bsol
    g = outs[0]
    for k in ("reason_number", "iterations", "function_evals"):
        assert g.result[k] == ref.result[k], k
    assert ref.fnorm_trace[-1] < ref.fnorm_trace[0]  # the step was taken (and accepted)
    # the shards' S sums in another order: ||f|| after the step agrees to
    # roundoff of the step (1.8e-8 measured at 8 shards on the C4 scene)
    np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-7)
    dx = np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3))
    if solve == "separator" and scene == "c4" and nshards > 2:
        # the separator form eliminates in another order than the unsharded
        # parallel cyclic reduction (the whole-S form is the same algorithm on
        # a differently summed S), so the two steps part by the roundoff
        # the normal equations allow: cond(J^T J) eps (tests/golden/
        # make_shard_step.py: 3.3e10 at 4 shards, 2.4e11 at 8 -> 2.7e-5;
        # measured 1.6e-5 at 8).  And the step is as close to the
        # reference's (the oracle's QR step) as the unsharded solve's is.
        fx = np.load(SHARD_STEP)
        cond = float(fx["cond_%d" % nshards])
        assert dx <= max(1e-6, cond * 1.1e-16), (dx, cond)
        # the initial ||f|| is the same sum in another order
        np.testing.assert_allclose(g.fnorm_trace[0], ref.fnorm_trace[0], rtol=1e-12)
        xo = fx["x_%d" % nshards]
        xs = np.maximum(np.abs(xo), 1e-3)
        d_ref = np.max(np.abs(ref.x - xo) / xs)
        d_sep = np.max(np.abs(g.x - xo) / xs)
        assert d_sep <= max(1e-6, 2.0 * d_ref), (d_sep, d_ref)
    else:
        assert dx <= 1e-6, dx
    if scene == "c4" and nshards in (4, 8):
        # the sharded step against the ORACLE's step at the
        # north star's 1e-6, once the step's undetermined directions (scaled
        # J's sigma < 1e-4 sigma_max at x0, make_steps.RATIO, registered
        # before any GPU run; 21 of 1,671 at 4 shards, 113 of 3,351 at 8) are
        # projected out -- the bar test_gpu_steps holds every C4 step to; and
        # ||f|| after the step within 1e-6 of the oracle's
        from tests.golden.make_steps import determined_dx
        fx = np.load(SHARD_STEP)
        d = {"exp_x": fx["x_%d" % nshards], "undet_basis": fx["undet_%d" % nshards]}
        ddx = determined_dx(d, g.x)
        assert ddx <= 1e-6, ddx
        np.testing.assert_allclose(g.fnorm_trace, fx["trace_%d" % nshards], rtol=1e-6)


@pytest.mark.parametrize("nshards", [4, 8])
def test_separator_form_well_conditioned(nshards, gpu_ctx, paths):
    """The separator form at 4 and 8 shards held to the 1e-6 x bar itself
    (ADVICE r4): the C4 spec's 4-frame tracks (half bandwidth 23, so the
    separator form applies) with the bundles near the camera (depth 4-10
    instead of 20-200), first full step against the unsharded solve -- a
    missing halo term or separator-assembly error moves x by 1e-3..1e-2;
    the initial ||f|| agrees to 1e-12 and the stepped one to 1e-9."""
    prob = S.make_config(3, frames=20 * nshards, scale=0.002 * nshards, depth=(4.0, 10.0))
    opt = S.config_options(prob, iterations=2)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
    finally:
        s.close()
    bsol = []
    pin_solve(paths, "separator")
    outs = run_sharded(prob, opt, nshards, band_solver=bsol)
    check_shards_agree(outs)
    assert bsol == [4] * nshards, bsol
    g = outs[0]
    assert g.result["iterations"] == ref.result["iterations"]
    np.testing.assert_allclose(g.fnorm_trace[0], ref.fnorm_trace[0], rtol=1e-12)
    np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-9)
    dx = np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3))
    assert dx <= 1e-6, dx


@pytest.mark.parametrize("nshards", [2, 4])
def test_sharded_dense_c3_structure(nshards, gpu_ctx, paths):
    """A reduced system that is no narrow band (the C3 structure: ten cameras,
    bundles tracked across the shot) shards too (VERDICT r4 "next" 8): each
    shard assembles the rows of its own camera-frames, the dense S and its
    right-hand side are all-reduced and every shard factors it with the fp64
    MFMA dense solver.  Against the unsharded dense
    solve: the first full step's x at 1e-6 and its ||f|| at 1e-9, then the
    whole run's reason, counts and trace at 1e-6 (the committed oracle
    fixture c3_f8 pins the unsharded run, test_gpu_golden.py)."""
    prob = S.make_config(2, frames=8, scale=0.002)
    for it in (2, 1000):
        opt = S.config_options(prob, iterations=it)
        s = Solver(prob, opt, context=gpu_ctx)
        try:
            assert s.kernel_stats()["reduced_kind"] == 2
            ref = s.solve()
        finally:
            s.close()
        reps = []
        outs = run_sharded(prob, opt, nshards, replicated=reps)
        assert reps == [0] * nshards, reps  # really sharded, not replicated
        check_shards_agree(outs)
        g = outs[0]
        for k in ("reason_number", "iterations", "function_evals"):
            assert g.result[k] == ref.result[k], k
        if it == 2:
            np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-9)
            dx = np.max(np.abs(g.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3))
            assert dx <= 1e-6, dx
        else:
            np.testing.assert_allclose(g.fnorm_trace, ref.fnorm_trace, rtol=1e-6)


def test_rccl_communicator_one_rank(gpu_ctx):
    """A real RCCL communicator on the box's GPU (ncclGetUniqueId,
    ncclCommInitRank, ncclAllReduce in place on the plan's stream -- the calls
    the multi-GPU bench makes).  RCCL refuses two ranks on one device, so on a
    one-GPU box the communicator has one rank and the all-reduce is the
    identity, bit for bit, for both operations."""
    from mayamatchmovesolver_amd.solver import comm_unique_id

    c = Comm.rccl(gpu_ctx, 0, 1, comm_unique_id())
    try:
        v = np.linspace(-3.0, 7.0, 1001) ** 3
        np.testing.assert_array_equal(c.debug_allreduce(gpu_ctx, v), v)
        np.testing.assert_array_equal(c.debug_allreduce(gpu_ctx, v, "max"), v)
    finally:
        c.close()


@pytest.mark.parametrize("order", list(ORDERS))
@pytest.mark.parametrize("n", [2, 3, 8])
def test_local_group_allreduce(n, order, paths):
    """The in-process group's all-reduce (sum in rank or ring order, max) on
    n host threads, each with its own stream: every rank gets the same bits,
    equal to the numpy sum in that order."""
    paths(abi.PATH_LOCAL_RING, ORDERS[order])
    comms = Comm.local_group(n)
    ctxs = [Context(0) for _ in range(n)]
    rng = np.random.default_rng(7)
    vals = [rng.standard_normal(777) for _ in range(n)]
    outs, errs = [None] * n, [None] * n

    def work(r):
        try:
            outs[r] = (comms[r].debug_allreduce(ctxs[r], vals[r]),
                       comms[r].debug_allreduce(ctxs[r], vals[r], "max"))
        except Exception as e:  # noqa: BLE001 - reported below
            errs[r] = e

    ths = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in ths), "group all-reduce hung"
    for c in comms:
        c.close()
    for c in ctxs:
        c.close()
    assert errs == [None] * n, errs
    cnt = vals[0].size
    ref = np.empty(cnt)
    for i in range(cnt):
        r0 = (i * n // cnt + 1) % n if order == "ring" else 0
        acc = vals[r0][i]
        for k in range(1, n):
            acc = acc + vals[(r0 + k) % n][i]
        ref[i] = acc
    for s, m in outs:
        np.testing.assert_array_equal(s, ref)
        np.testing.assert_array_equal(m, np.max(np.stack(vals), axis=0))


def test_unshardable_problem_replicated(gpu_ctx):
    """A problem the frame partition cannot take (rolling shutter: the blend
    couples every camera-frame with its neighbours across a shard boundary)
    is solved whole on every shard, without collectives: the same bits as
    the unsharded plan, on every shard (mmba_plan_create_sharded)."""
    prob = S.make_config(4, frames=12, scale=0.05, rolling_shutter=0.5)
    opt = S.config_options(prob, iterations=6)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        assert s.kernel_stats()["shards_replicated"] == 0
        ref = s.solve()
    finally:
        s.close()
    reps = []
    outs = run_sharded(prob, opt, 2, replicated=reps)
    assert reps == [1, 1]
    for o in outs:
        np.testing.assert_array_equal(o.x, ref.x)
        np.testing.assert_array_equal(o.fvec, ref.fvec)
        np.testing.assert_array_equal(o.fnorm_trace, ref.fnorm_trace)
        assert o.result["iterations"] == ref.result["iterations"]
