"""Rolling shutter on the GPU (BASELINE configs[4] "rolling-shutter
per-scanline pose"; mmba.h ABI 3, csrc/mmba_rs.hip) against the CPU oracle
(oracle/refcpu.c rs_blend, pinned in tests/test_oracle_rs.py).

The reference solver has no rolling-shutter model -- its only rolling-shutter
arithmetic is the 3DE exporter's 2D correction
(share/3dequalizer/python/uvtrack_format.py:186-203, 243-330), whose blend
both sides apply to the camera pose -- so parity against the reference itself
is unpinned; these tests hold the HIP path to the oracle at the north star's
bar (reason, counts, every ||f|| and x at 1e-6; residuals 1e-12; the FD
Jacobian 1e-7 of its max entry)."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver
from tests.test_gpu_parity import check_solve

pytestmark = pytest.mark.gpu

MODES = [abi.SCENE_GRAPH_MODE_MAYA_DAG, abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH]


def rs_scene(frames=8, scale=0.05, rs=0.5, **kw):
    return S.make_config(4, frames=frames, scale=scale, rolling_shutter=rs, **kw)


@pytest.mark.parametrize("mode", MODES)
def test_rs_measure_jacobian_reproject(mode, oracle, gpu_ctx):
    prob = rs_scene()
    opt = S.config_options(prob, scene_graph_mode=mode)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        for x in (None, prob.x0 + 0.01):
            f, eu, ed, _ = s.measure(x)
            fr, eur, edr, _ = oracle.measure(prob, opt, x)
            np.testing.assert_allclose(f, fr, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(eu, eur, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(ed, edr, rtol=1e-12, atol=1e-12)
            pts, mkr = s.reproject(x)
            pr, mr = oracle.reproject_obs(prob, opt, x)
            np.testing.assert_allclose(pts, pr, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(mkr, mr, rtol=1e-15, atol=0)
        x1 = prob.x0 + 0.01
        J = s.jacobian(x1)
        _, Jr = oracle.jacobian(prob, opt, x1)
        scale = np.max(np.abs(Jr))
        assert np.max(np.abs(J - Jr)) <= 1e-7 * scale
        # the structure: neighbouring-frame columns are non-zero where the
        # oracle's are (the blend reaches frames f - 1 .. f + 1)
        assert np.max(np.abs(J[Jr == 0])) <= 1e-9 * scale
        assert np.all(J[np.abs(Jr) > 1e-6 * scale] != 0)
    finally:
        s.close()


@pytest.mark.parametrize("solver_type", [abi.SOLVER_TYPE_CMINPACK_LMDER,
                                         abi.SOLVER_TYPE_CMINPACK_LMDIF])
@pytest.mark.parametrize("mode", MODES)
def test_rs_solve_matches_oracle(solver_type, mode, oracle, gpu_ctx):
    prob = rs_scene()
    opt = S.config_options(prob, scene_graph_mode=mode, solver_type=solver_type)
    out, (xr, rr) = check_solve(prob, opt, oracle, gpu_ctx)
    assert rr.reason_number in (1, 2, 3, 5)


@pytest.mark.parametrize("kw", [
    dict(frames=24, scale=0.2, rs=0.5),              # band through every frame
    dict(frames=12, scale=0.1, rs=-0.8),             # bottom scanline first
    dict(frames=8, scale=0.05, rs=0.5, lens_model="radial"),
])
def test_rs_variants_match_oracle(kw, oracle, gpu_ctx):
    prob = rs_scene(**kw)
    opt = S.config_options(prob)
    check_solve(prob, opt, oracle, gpu_ctx)


def test_rs_refuses_mixed_animated_lens(gpu_ctx):
    """An animated lens coefficient under the reference's lens index
    arithmetic (mmba.h ABI 7): marker i at frame f reads the
    coefficient keyed at frame (i + f) % F, which the rolling-shutter
    Jacobian's per-camera-frame columns do not hold -- refused with
    MMBA_ERR_UNSUPPORTED (round 3 solved it with each marker reading its own
    frame, which is not what the reference computes)."""
    prob = rs_scene(frames=8, scale=0.05, rs=0.5, lens_model="classic_animated")
    opt = S.config_options(prob)
    with pytest.raises(MmbaError) as e:
        Solver(prob, opt, context=gpu_ctx).close()
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED


def test_rs_one_camera_only(oracle, gpu_ctx):
    """One camera with a rolling shutter, the other a global shutter."""
    prob = rs_scene(frames=10, scale=0.08)
    prob.cam_rs_value = np.array([0.7, 0.0])
    opt = S.config_options(prob)
    check_solve(prob, opt, oracle, gpu_ctx)


def test_rs_zero_equals_global_shutter(gpu_ctx):
    """cam_rs_value all 0 is the reference path, bit for bit."""
    prob = rs_scene()
    opt = S.config_options(prob)
    outs = []
    for rs in (np.zeros(prob.num_cameras), None):
        prob.cam_rs_value = rs
        s = Solver(prob, opt, context=gpu_ctx)
        try:
            outs.append(s.solve())
        finally:
            s.close()
    np.testing.assert_array_equal(outs[0].x, outs[1].x)
    np.testing.assert_array_equal(outs[0].fnorm_trace, outs[1].fnorm_trace)


def test_rs_refuses_central_differences(gpu_ctx):
    """Outside the supported scope (central differences) the plan is refused
    with MMBA_ERR_UNSUPPORTED, never silently solved without the blend."""
    prob = rs_scene()
    opt = S.config_options(prob, auto_diff_type=abi.AUTO_DIFF_TYPE_CENTRAL)
    with pytest.raises(MmbaError) as e:
        Solver(prob, opt, context=gpu_ctx)
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED


@pytest.mark.parametrize("parented", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_rs_solved_bundles(parented, mode, oracle, gpu_ctx):
    """Solved bundles under a rolling shutter: a row reaches the camera-frame
    blocks of f - 1, f, f + 1 and its bundle, so the Schur complement runs
    over virtual observations (one per block a row reaches; Plan::build,
    k_schur_obs_rs).  Measurement, the FD Jacobian (the bundle columns last
    in each row) and the solve against the oracle -- whole for the plain
    camera; for the parented one the first four evaluations: after them the
    cost crawls along a valley (16.99 -> 16.98 over 200 evaluations) where
    the oracle's own 1-ulp x envelope is 7e-2 and its evaluation count moves
    from 92 to 279."""
    prob = S.edge_scene(parented=parented, solve_bundles=True)
    prob.cam_rs_value = np.array([0.6])
    opt = S.config_options(prob, scene_graph_mode=mode, **({"iterations": 4} if parented else {}))
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        x1 = prob.x0 + 0.01
        f, _, _, _ = s.measure(x1)
        fr, _, _, _ = oracle.measure(prob, opt, x1)
        np.testing.assert_allclose(f, fr, rtol=1e-12, atol=1e-12)
        J = s.jacobian(x1)
        _, Jr = oracle.jacobian(prob, opt, x1)
        scale = np.max(np.abs(Jr))
        assert np.max(np.abs(J - Jr)) <= 1e-7 * scale
    finally:
        s.close()
    check_solve(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("solve_parent", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_rs_parented_camera(solve_parent, mode, oracle, gpu_ctx):
    """A camera under a rotated, translated group (tests/test_oracle_rs.py
    pins the model: the group's world matrix at the frame times the blended
    local pose): measurement, reprojection and the FD Jacobian at 1e-12 /
    1e-7, then the whole solve against the oracle; with the group's rotation
    solved its three static columns move every observation through the
    parent's world matrix (rs_record's attribute override)."""
    prob = S.edge_scene(parented=True, solve_bundles=False, solve_parent=solve_parent)
    prob.cam_rs_value = np.array([0.6])
    opt = S.config_options(prob, scene_graph_mode=mode)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        for x in (None, prob.x0 + 0.01):
            f, eu, ed, _ = s.measure(x)
            fr, eur, edr, _ = oracle.measure(prob, opt, x)
            np.testing.assert_allclose(f, fr, rtol=1e-12, atol=1e-12)
            pts, _ = s.reproject(x)
            pr, _ = oracle.reproject_obs(prob, opt, x)
            np.testing.assert_allclose(pts, pr, rtol=1e-12, atol=1e-14)
        x1 = prob.x0 + 0.01
        J = s.jacobian(x1)
        _, Jr = oracle.jacobian(prob, opt, x1)
        scale = np.max(np.abs(Jr))
        assert np.max(np.abs(J - Jr)) <= 1e-7 * scale
    finally:
        s.close()
    check_solve(prob, opt, oracle, gpu_ctx)
