"""Host-side checks of the raised-capacity rigs (tests/test_gpu_caps.py runs
them on the GPU): the scene generators produce the parameter structure the
GPU tests assert, and the CPU oracle solves the 40-global block-diagonal rig
(the oracle's own 1-ulp envelope there is 2.3e-8, profiles/r6_caps/)."""
import numpy as np

from mayamatchmovesolver_amd import abi, make_options, synthetic as S


def test_twelve_parameter_rig_structure():
    F = 8
    prob = S.make_config(4, frames=F, scale=0.05, lens_model="classic_wide", cameras=1)
    assert prob.num_params == 12 * F
    pf = np.asarray(prob.param_frame)
    # every solved attribute is keyed per frame: 12 per frame, one camera
    assert np.all(pf >= 0)
    assert np.all(np.bincount(pf, minlength=F) == 12)


def test_forty_global_rig_structure():
    prob = S.witness_scene(n_witness=6, n_focal=6, extra_globals=1)
    pf = np.asarray(prob.param_frame)
    # static (frame < 0) parameters: 40 camera globals + 24 bundles x 3
    assert int(np.sum(pf < 0)) == 40 + 24 * 3
    assert prob.num_params == 36 + 40 + 72
    wide = S.witness_scene(n_witness=7, n_focal=7, extra_globals=3)
    assert int(np.sum(np.asarray(wide.param_frame) < 0)) - 24 * 3 == 49


def test_forty_global_block_diagonal_rig_oracle(oracle):
    prob = S.witness_scene(n_witness=6, n_focal=6, extra_globals=1, solve_bundles=False)
    opt = make_options(scene_graph_mode=abi.SCENE_GRAPH_MODE_MAYA_DAG)
    x, f, _eu, _ed, res, trace = oracle.solve(prob, opt)
    assert res.reason_number == 1
    assert trace[-1] < 0.05 * trace[0]
    assert np.all(np.isfinite(x))
