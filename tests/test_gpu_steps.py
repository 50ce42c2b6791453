"""The C4 structure and the parented rolling-shutter scene with solved
bundles, pinned step by step at the north star's 1e-6 (tests/golden/
make_steps.py; VERDICT r4 "next" 2): from waypoints of the oracle's own run
(x after K evaluations, from the first step to the stopping point) the HIP
solve's one-step call (maxfev 2: evaluation, FD Jacobian, damped solve,
trial point; adjust_cminpack_lmder.cpp:114-185) against the oracle's.

Bars: reason and every counter equal; every ||f|| of the step within 1e-6
relative; fvec within 1e-6 of the step's first ||f||; x within 1e-6 relative
once the step's undetermined directions (scaled J's singular values below
1e-4 sigma_max, fixed in make_steps.RATIO before any GPU run) are projected
out, and the whole x within the step's pre-registered 1-ulp envelope
(tests/golden/envelopes.py, 8 registered seeds) where that is wider than
1e-6."""
import numpy as np
import pytest

from mayamatchmovesolver_amd.solver import Solver
from tests.golden import make_steps as ST

pytestmark = pytest.mark.gpu
REL = 1e-6


@pytest.mark.parametrize("name", ST.fixture_names())
def test_gpu_step_from_waypoint(name, gpu_ctx):
    import os
    if not os.path.exists(os.path.join(ST.STEPS, name + ".npz")):
        pytest.skip("fixture not generated")
    prob, opt, d = ST.load(name)
    assert int(d["envelope_runs"]) == 8, "envelope not computed over the registered seeds"
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        out = s.solve(x0=d["x_start"])
    finally:
        s.close()
    g = out.result
    for k in ("reason_number", "iterations", "function_evals", "jacobian_evals",
              "outer_iterations"):
        assert g[k] == int(d["res_" + k]), k
    tr = d["exp_trace"]
    assert len(out.fnorm_trace) == len(tr)
    np.testing.assert_allclose(out.fnorm_trace, tr, rtol=REL)
    assert np.linalg.norm(out.fvec - d["exp_fvec"]) <= REL * float(tr[0])
    det = ST.determined_dx(d, out.x)
    assert det <= REL, (det, float(d["exp_x_det_envelope"]))
    xr = d["exp_x"]
    dx = float(np.max(np.abs(out.x - xr) / np.maximum(np.abs(xr), 1e-3)))
    assert dx <= max(REL, float(d["exp_x_envelope"])), (dx, float(d["exp_x_envelope"]))
