"""Per-frame solve mode (mmba_solve_per_frame; FrameSolveMode::kPerFrame,
src/mmSolver/adjust/adjust_base.cpp:1430-1484) against the CPU oracle run
frame by frame on sub-problems split here, independently of the library's
own splitter: each frame's observations, that frame's animated parameters
and every static parameter; frames in order, x carried from frame to frame.
Bar: per frame the same reason code and evaluation counts, final x within
1e-6 relative (the unsharded parity bar)."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S
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
              "param_scale"):
        d[k] = np.asarray(d[k])[pi]
    d["x0"] = np.asarray(x)[pi]
    return Problem.from_npz_dict(d), pi


def oracle_per_frame(prob, opt, oracle):
    x = np.array(prob.x0, dtype=float)
    out = []
    for f in range(prob.num_frames):
        sub, pi = frame_problem(prob, f, x)
        if sub.num_params == 0 or sub.num_params > 2 * sub.num_obs:
            break
        xs, _, _, _, rr, _ = oracle.solve(sub, opt)
        x[pi] = xs
        out.append(rr)
    return x, out


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
