"""The cooperative whole-solve launch (mmba_lmcoop.hip) of block-diagonal plans
against the host-driven LM loop of the same plan (MMBA_LM_COOP=0) and the
oracle.

Both paths run the MINPACK lmder / lmdif control flow of Plan::solve on the
same device arithmetic; their scalar reductions sum in different orders, so
the traces agree to roundoff, not bit for bit.  Against the oracle the bar is
the north star's (1e-6 on x and on every ||f||)."""
import os

import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd.solver import Solver

pytestmark = pytest.mark.gpu


def _solve(prob, opt, ctx, coop, **kw):
    old = os.environ.get("MMBA_LM_COOP")
    os.environ["MMBA_LM_COOP"] = "1" if coop else "0"
    try:
        s = Solver(prob, opt, context=ctx)
    finally:
        if old is None:
            del os.environ["MMBA_LM_COOP"]
        else:
            os.environ["MMBA_LM_COOP"] = old
    try:
        out = s.solve(**kw)
        used = s.kernel_stats()["solve_launch"]
    finally:
        s.close()
    return out, used


def _same(a, b, tol=1e-9):
    ga, gb = a.result, b.result
    for k in ("reason_number", "iterations", "outer_iterations", "function_evals",
              "jacobian_evals", "user_interrupted", "error_is_better"):
        assert ga[k] == gb[k], (k, ga[k], gb[k])
    assert len(a.fnorm_trace) == len(b.fnorm_trace)
    np.testing.assert_allclose(a.fnorm_trace, b.fnorm_trace, rtol=tol)
    xs = np.maximum(np.abs(b.x), 1e-3)
    assert np.max(np.abs(a.x - b.x) / xs) <= tol
    f0 = float(b.fnorm_trace[0])
    assert np.linalg.norm(a.fvec - b.fvec) <= tol * f0
    assert np.linalg.norm(a.err_user - b.err_user) <= tol * f0
    assert np.max(np.abs(a.err_dist - b.err_dist)) <= tol * max(1.0, np.max(np.abs(b.err_dist)))
    for k in ("error_final", "error_avg", "error_max", "error_rms", "error_initial_avg"):
        assert abs(ga[k] - gb[k]) <= tol * max(1.0, abs(gb[k])), (k, ga[k], gb[k])


@pytest.mark.parametrize("solver_type", [abi.SOLVER_TYPE_CMINPACK_LMDER,
                                         abi.SOLVER_TYPE_CMINPACK_LMDIF])
@pytest.mark.parametrize("mode", [abi.SCENE_GRAPH_MODE_MAYA_DAG,
                                  abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH])
def test_coop_matches_host_loop_c2(solver_type, mode, gpu_ctx):
    prob = S.make_config(1, frames=24, scale=0.2)
    opt = S.config_options(prob, scene_graph_mode=mode, solver_type=solver_type,
                           iterations=200)
    a, used_a = _solve(prob, opt, gpu_ctx, True)
    b, used_b = _solve(prob, opt, gpu_ctx, False)
    assert used_a == 1 and used_b == 0
    _same(a, b)


def test_coop_full_c2_matches_host_loop(gpu_ctx):
    prob = S.make_config(1)  # the full configs[1] scene (120 frames, 840 parameters)
    opt = S.config_options(prob)
    a, used = _solve(prob, opt, gpu_ctx, True)
    b, _ = _solve(prob, opt, gpu_ctx, False)
    assert used == 1
    _same(a, b, tol=1e-8)


@pytest.mark.parametrize("extra", ["mode2", "no_accept", "initial_given", "maxfev"])
def test_coop_options(extra, gpu_ctx):
    prob = S.make_config(1, frames=16, scale=0.1)
    kw = {}
    if extra == "mode2":
        kw["auto_param_scale"] = 0
    elif extra == "no_accept":
        kw["accept_only_better"] = 0
    elif extra == "initial_given":
        kw["initial_error_avg"] = 3.5
    elif extra == "maxfev":
        kw["iterations"] = 3
    opt = S.config_options(prob, **kw)
    if extra == "mode2":
        prob.param_weight = np.ascontiguousarray(np.linspace(0.5, 2.0, prob.num_params))
    a, used = _solve(prob, opt, gpu_ctx, True)
    b, _ = _solve(prob, opt, gpu_ctx, False)
    assert used == 1
    _same(a, b)


def test_coop_against_oracle(oracle, gpu_ctx):
    prob = S.make_config(1, frames=12, scale=0.1)
    opt = S.config_options(prob)
    xr, fr, eur, edr, rr, trr = oracle.solve(prob, opt)
    a, used = _solve(prob, opt, gpu_ctx, True)
    assert used == 1
    g = a.result
    assert g["reason_number"] == rr.reason_number
    assert g["iterations"] == rr.iterations
    assert g["function_evals"] == rr.function_evals
    assert g["jacobian_evals"] == rr.jacobian_evals
    np.testing.assert_allclose(a.fnorm_trace, trr, rtol=1e-6, atol=1e-9 * trr[0])
    xs = np.maximum(np.abs(xr), 1e-3)
    assert np.max(np.abs(a.x - xr) / xs) <= 1e-6


def test_coop_plan_reuse_is_bitwise(gpu_ctx):
    prob = S.make_config(1, frames=16, scale=0.1)
    opt = S.config_options(prob)
    old = os.environ.get("MMBA_LM_COOP")
    os.environ["MMBA_LM_COOP"] = "1"
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        a = s.solve()
        b = s.solve()
        assert s.kernel_stats()["solve_launch"] == 1
    finally:
        s.close()
        if old is None:
            del os.environ["MMBA_LM_COOP"]
        else:
            os.environ["MMBA_LM_COOP"] = old
    assert np.array_equal(a.x, b.x)
    assert np.array_equal(a.fnorm_trace, b.fnorm_trace)
    assert np.array_equal(a.fvec, b.fvec)
