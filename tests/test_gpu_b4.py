"""MM Scene Graph point indexing (mmba.h ABI 8) on the
device: markers listed bundle by bundle, not grouped by camera, so
observation (marker i, frame f) compares flat marker i of the camera-major
listing (flat.rs:271-356 read at adjust_measureErrors.cpp:454-459).  Each
scene: measurement, dense Jacobian, reprojection and the whole solve against
the CPU oracle (tests/test_oracle_b4.py pins the oracle), 1e-6 on x and every
||f||; a 2-shard solve; the refusal when a flat marker's x,y is unknown."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver

from test_gpu_edge import REL, check, check_measure_jacobian
from test_gpu_sharded import run_sharded

pytestmark = pytest.mark.gpu

KINDS = {"full": {}, "partial_frame_xy": {"partial": True, "frame_xy": True}}


@pytest.mark.parametrize("kind", list(KINDS))
def test_b4_solve(kind, oracle, gpu_ctx):
    prob = S.b4_scene(**KINDS[kind])
    opt = S.config_options(prob)
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx)


def test_b4_reproject(oracle, gpu_ctx):
    prob = S.b4_scene(partial=True, frame_xy=True)
    opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        for x in (None, np.asarray(prob.x0) + 0.001):
            pts, mkr = s.reproject(x)
            pr, mr = oracle.reproject_obs(prob, opt, x)
            np.testing.assert_allclose(pts, pr, rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(mkr, mr, rtol=1e-12, atol=1e-12)
    finally:
        s.close()


def test_b4_sharded(oracle):
    """Two frame shards: the remapped observations' cameras and bundles set
    the camera-frame blocks and the bundle owners.  Four iterations: after
    the second the scene's cost crawls along a valley (9.448 -> 9.4434 over
    70 iterations), where x is not comparable at 1e-6 (4.9e-5 after the
    full 2-shard solve)."""
    prob = S.b4_scene(frames=16, bundles=8)
    opt = S.config_options(prob, iterations=4)
    xr, fr, *_ = oracle.solve(prob, opt)
    outs = run_sharded(prob, opt, 2)
    assert np.array_equal(outs[0].x, outs[1].x)
    xs = np.maximum(np.abs(xr), 1e-3)
    assert np.max(np.abs(outs[0].x - xr) / xs) <= REL
    assert abs(np.linalg.norm(outs[0].fvec) - np.linalg.norm(fr)) <= REL * np.linalg.norm(fr)


def test_b4_unknown_flat_xy_refused(gpu_ctx):
    prob = S.b4_scene(partial=True)
    opt = S.config_options(prob)
    with pytest.raises(MmbaError) as e:
        Solver(prob, opt, context=gpu_ctx).close()
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED
    dag = S.config_options(prob, scene_graph_mode=abi.SCENE_GRAPH_MODE_MAYA_DAG)
    Solver(prob, dag, context=gpu_ctx).close()  # Maya-DAG mode has no B4


def test_b4_rolling_shutter_refused(gpu_ctx):
    prob = S.b4_scene()
    prob.cam_rs_value = np.full(prob.num_cameras, 0.5)
    with pytest.raises(MmbaError) as e:
        Solver(prob, S.config_options(prob), context=gpu_ctx).close()
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED
