"""Per-frame solve mode (mmba_solve_per_frame; FrameSolveMode::kPerFrame,
src/mmSolver/adjust/adjust_base.cpp:1430-1484) against the CPU oracle run
frame by frame on sub-problems split here, independently of the library's
own splitter: each frame's observations, that frame's animated parameters
and every static parameter; frames in order, x carried from frame to frame.
Bar: per frame the same reason code and evaluation counts, final x within
1e-6 relative (the unsharded parity bar)."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd.problem import Problem
from mayamatchmovesolver_amd.solver import solve_per_frame

pytestmark = pytest.mark.gpu


def frame_problem(prob, f, x):
    d = prob.to_npz_dict()
    oi = np.flatnonzero(np.asarray(prob.obs_frame) == f)
    pi = np.flatnonzero((np.asarray(prob.param_frame) == f) | (np.asarray(prob.param_frame) < 0))
    for k in ("obs_marker", "obs_frame", "obs_weight"):
        d[k] = np.asarray(d[k])[oi]
    d["obs_xy"] = np.asarray(d["obs_xy"]).reshape(-1, 2)[oi].reshape(-1)
    for k in ("param_attr", "param_frame", "param_min", "param_max", "param_offset",
              "param_scale", "param_weight"):
        if k in d:
            d[k] = np.asarray(d[k])[pi]
    d["x0"] = np.asarray(x)[pi]
    return Problem.from_npz_dict(d), pi


def oracle_per_frame(prob, opt, oracle, interrupt_after=-1):
    x = np.array(prob.x0, dtype=float)
    out = []
    for f in range(prob.num_frames):
        sub, pi = frame_problem(prob, f, x)
        if sub.num_params == 0 or sub.num_params > 2 * sub.num_obs:
            break
        xs, _, _, _, rr, _ = oracle.solve(sub, opt, interrupt_after=interrupt_after)
        if rr.error_is_better:  # solveFrames' write-back (adjust_base.cpp:1231-1244)
            x[pi] = xs
        out.append(rr)
    return x, out


def frame_params_only(prob):
    """The problem with its static parameters dropped (they stay at their
    scene values): every parameter is keyed at one frame."""
    d = prob.to_npz_dict()
    keep = np.flatnonzero(np.asarray(prob.param_frame) >= 0)
    for k in ("param_attr", "param_frame", "param_min", "param_max", "param_offset",
              "param_scale", "param_weight", "x0"):
        if k in d:
            d[k] = np.asarray(d[k])[keep]
    return Problem.from_npz_dict(d)


def check_frames(prob, res, rr, x, xr, rel=1e-6):
    assert len(rr) <= prob.num_frames
    for f, (g, r) in enumerate(zip(res, rr)):
        assert g["reason_number"] == r.reason_number, (f, g, r.as_dict())
        assert g["iterations"] == r.iterations, f
        assert g["function_evals"] == r.function_evals, f
        assert g["jacobian_evals"] == r.jacobian_evals, f
        assert g["outer_iterations"] == r.outer_iterations, f
        assert g["user_interrupted"] == r.user_interrupted, f
        assert g["error_is_better"] == r.error_is_better, f
        for k in ("error_final", "error_avg", "error_min", "error_max", "error_rms",
                  "error_initial_avg"):
            assert abs(g[k] - getattr(r, k)) <= rel * abs(getattr(r, k)) + 1e-9, (f, k, g[k],
                                                                                 getattr(r, k))
    for g in res[len(rr):]:
        assert g["success"] == 0
    assert np.max(np.abs(x - xr) / np.maximum(np.abs(xr), 1e-3)) <= rel


@pytest.mark.parametrize("idx,kw,conc", [
    (1, dict(frames=12, scale=0.05), 8),   # pose + focal per frame: independent frames
    (1, dict(frames=12, scale=0.05), 1),   # the same, one at a time
    (4, dict(frames=6, scale=0.05), 8),    # lens (static) + poses: frames chained
])
def test_per_frame_matches_oracle(idx, kw, conc, oracle):
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    xr, rr = oracle_per_frame(prob, opt, oracle)
    x, res = solve_per_frame(prob, opt, max_concurrency=conc)
    assert len(rr) == prob.num_frames
    for f, (g, r) in enumerate(zip(res, rr)):
        assert g["reason_number"] == r.reason_number, (f, g, r.as_dict())
        assert g["iterations"] == r.iterations, f
        assert g["function_evals"] == r.function_evals, f
        assert abs(g["error_final"] - r.error_final) <= 1e-6 * r.error_final + 1e-9, f
    assert np.max(np.abs(x - xr) / np.maximum(np.abs(xr), 1e-3)) <= 1e-6


@pytest.fixture(params=["batched", "per-frame plans"])
def path(request, paths):
    if request.param != "batched":
        paths(abi.PATH_PERFRAME_BATCH, 0)
    return request.param


@pytest.mark.parametrize("solver", ["lmder", "lmdif"])
@pytest.mark.parametrize("mode", ["mmsg", "dag"])
def test_per_frame_paths_match_oracle(path, solver, mode, oracle):
    """Both per-frame paths (one launch for every frame, and one plan per
    frame) against the oracle, for both cminpack solvers and both scene-graph
    modes: counts, error statistics and x per frame."""
    from mayamatchmovesolver_amd import abi
    prob = S.make_config(1, frames=10, scale=0.05)
    st = abi.SOLVER_TYPE_CMINPACK_LMDER if solver == "lmder" else abi.SOLVER_TYPE_CMINPACK_LMDIF
    sg = abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH if mode == "mmsg" else abi.SCENE_GRAPH_MODE_MAYA_DAG
    opt = S.config_options(prob, scene_graph_mode=sg, solver_type=st, iterations=100)
    xr, rr = oracle_per_frame(prob, opt, oracle)
    x, res = solve_per_frame(prob, opt, max_concurrency=4)
    check_frames(prob, res, rr, x, xr)


def test_per_frame_two_cameras_per_frame(path, oracle):
    """C5's two cameras with the shared lens fixed: two camera-frames (12
    parameters) per frame, solved as one frame sub-problem."""
    prob = frame_params_only(S.make_config(4, frames=6, scale=0.05))
    assert len(set(np.asarray(prob.param_frame))) == prob.num_frames
    opt = S.config_options(prob)
    xr, rr = oracle_per_frame(prob, opt, oracle)
    x, res = solve_per_frame(prob, opt)
    check_frames(prob, res, rr, x, xr)


@pytest.mark.parametrize("variant", ["no_accept_only_better", "param_weights",
                                     "initial_error_given", "maxfev"])
def test_per_frame_options(path, variant, oracle):
    prob = S.make_config(1, frames=6, scale=0.05)
    kw = {}
    if variant == "no_accept_only_better":
        kw = dict(accept_only_better=0)
    elif variant == "param_weights":
        kw = dict(auto_param_scale=0)
        prob.param_weight = np.linspace(0.5, 2.0, prob.num_params)
    elif variant == "initial_error_given":
        kw = dict(initial_error_avg=1e6)
    elif variant == "maxfev":
        kw = dict(iterations=3)
    opt = S.config_options(prob, **kw)
    xr, rr = oracle_per_frame(prob, opt, oracle)
    x, res = solve_per_frame(prob, opt)
    check_frames(prob, res, rr, x, xr)


def test_per_frame_interrupt_pending(path, oracle):
    """An interrupt already requested: every frame's solveFrames stops at
    its first poll (reason -1, one counted evaluation, nothing written back
    unless the error got better)."""
    prob = S.make_config(1, frames=5, scale=0.05)
    opt = S.config_options(prob)
    xr, rr = oracle_per_frame(prob, opt, oracle, interrupt_after=0)
    x, res = solve_per_frame(prob, opt, interrupt=lambda: True)
    check_frames(prob, res, rr, x, xr)
    assert all(g["reason_number"] == -1 for g in res)


def test_plan_per_frame_reuse(oracle):
    """mmba_plan_solve_per_frame: one plan, several per-frame solves (plan
    caching); each call equals the oracle's per-frame loop."""
    from mayamatchmovesolver_amd.solver import Solver
    prob = S.make_config(1, frames=8, scale=0.05)
    opt = S.config_options(prob)
    xr, rr = oracle_per_frame(prob, opt, oracle)
    sv = Solver(prob, opt)
    try:
        for _ in range(2):
            x, res = sv.solve_per_frame()
            check_frames(prob, res, rr, x, xr)
    finally:
        sv.close()


def test_plan_per_frame_refuses_chained():
    """A static parameter chains the frames: the plan entry point refuses
    (MMBA_ERR_UNSUPPORTED), mmba_solve_per_frame takes the chained path."""
    from mayamatchmovesolver_amd._lib import MmbaError
    from mayamatchmovesolver_amd.solver import Solver
    prob = S.make_config(4, frames=4, scale=0.05)
    sv = Solver(prob, S.config_options(prob))
    try:
        with pytest.raises(MmbaError):
            sv.solve_per_frame()
    finally:
        sv.close()
