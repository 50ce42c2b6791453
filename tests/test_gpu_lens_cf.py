"""Animated lens coefficients in camera-frame blocks (VERDICT r4 "next" 7).

The reference re-measures only an animated parameter's own frame for its FD
column (adjust_solveFunc.cpp frameIndexEnable) and clones the lens per frame
(maya_lens_model_utils.cpp:654-661, read at adjust_measureErrors.cpp:244), so
an animated lens coefficient whose lens instances at its frame are read by
one camera reaches the rows of ONE camera-frame: the plan puts it in that
camera-frame's block (Plan::build, VF_LENS) instead of the global arrow,
where more than NGMAX animated frames (32 then, 48 since round 6) were refused.  Pinned here: the
residuals and the FD Jacobian against the oracle on a one-camera shot with
its distortion animated over 36 frames, the refusal that remains with the
classification pinned off, and (tests/test_gpu_golden.py,
c5_f40_lens_anim_1cam) the whole solve against the oracle's fixture."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver

pytestmark = pytest.mark.gpu


def scene(frames=36, scale=0.02):
    return S.make_config(4, frames=frames, scale=scale, lens_model="classic_animated", cameras=1)


def test_animated_lens_over_ngmax_residuals_and_jacobian(oracle, gpu_ctx):
    prob = scene()
    assert prob.num_params == 36 * 7 + 1  # pose + distortion per frame, static quartic
    opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        st = s.kernel_stats()
        assert st["reduced_dim"] == 36 * 7 + 1, st  # 36 blocks of 7, one global row
        x1 = prob.x0 + 0.01
        f1, _, _, _ = s.measure(x1)
        f1_ref, _, _, _ = oracle.measure(prob, opt, x1)
        np.testing.assert_allclose(f1, f1_ref, rtol=1e-12, atol=1e-12)
        J = s.jacobian(x1)
        _, J_ref = oracle.jacobian(prob, opt, x1)
        scale = np.max(np.abs(J_ref))
        assert np.max(np.abs(J - J_ref)) <= 1e-7 * scale
        assert np.array_equal(J != 0, J_ref != 0) or np.max(np.abs(J[J_ref == 0])) < 1e-9 * scale
    finally:
        s.close()


def test_animated_lens_as_globals_refused(gpu_ctx, paths):
    """With the classification pinned off every animated coefficient is a
    global parameter: 50 + 1 > NGMAX (48), refused as before round 5."""
    paths(abi.PATH_LENS_CF, 0)
    prob = scene(frames=50)
    with pytest.raises(MmbaError) as e:
        Solver(prob, S.config_options(prob), context=gpu_ctx).close()
    assert "48 global" in str(e.value)


def test_shared_lens_stays_global(oracle, gpu_ctx):
    """Two cameras on one animated lens: a coefficient's frame is read by both
    camera-frames, so it stays a global parameter (the C5 spec's structure),
    solved as before against the oracle."""
    from tests.test_gpu_parity import check_solve
    prob = S.make_config(4, frames=8, scale=0.05, lens_model="classic_animated")
    check_solve(prob, S.config_options(prob), oracle, gpu_ctx)
