"""Plan caching (the INTEGRATION shim keeps one plan per problem shape):
``mmba_plan_set_attr_values`` on an existing plan gives the same solve,
bit for bit, as a fresh plan built from the updated scene."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S
from mayamatchmovesolver_amd.solver import Solver

pytestmark = pytest.mark.gpu


def written_back(prob, x):
    """The scene after solveFrames' write-back of internal parameters x."""
    d = prob.to_npz_dict()
    vals = np.array(d["attr_values"], dtype=float)
    ext = prob.external_params(x)
    anim = np.asarray(prob.attr_animated)
    off = np.asarray(prob.attr_offset)
    for p, (a, f) in enumerate(zip(np.asarray(prob.param_attr), np.asarray(prob.param_frame))):
        vals[off[a] + (f if anim[a] else 0)] = ext[p]
    d["attr_values"] = vals
    d["x0"] = np.asarray(x, dtype=float)
    return type(prob).from_npz_dict(d)


@pytest.mark.parametrize("cfg,kw", [(1, dict(frames=6, scale=0.05)),
                                    (3, dict(frames=12, scale=0.05))])
def test_set_attr_values_equals_fresh_plan(cfg, kw):
    prob = S.make_config(cfg, **kw)
    opt = S.config_options(prob, iterations=8)  # stop early: the second solve still moves
    sv = Solver(prob, opt)
    try:
        first = sv.solve()
        prob2 = written_back(prob, first.x)
        sv.set_attr_values(prob2.attr_values)
        cached = sv.solve(x0=prob2.x0)
    finally:
        sv.close()
    fresh_sv = Solver(prob2, opt)
    try:
        fresh = fresh_sv.solve()
    finally:
        fresh_sv.close()
    assert cached.result["iterations"] == fresh.result["iterations"]
    np.testing.assert_array_equal(cached.x, fresh.x)
    np.testing.assert_array_equal(cached.fnorm_trace, fresh.fnorm_trace)
    np.testing.assert_array_equal(cached.err_dist, fresh.err_dist)
    assert cached.result["error_initial_avg"] == fresh.result["error_initial_avg"]


@pytest.mark.parametrize("scene", ["c3", "c2", "rows"])
@pytest.mark.parametrize("dma", [0, 1])
def test_solve_into_page_locked_buffers(scene, dma, gpu_ctx, paths):
    """Output buffers in page-locked host memory (mmba_host_alloc, as bench.py
    and a caching caller keep them) receive the same bits as ordinary numpy
    arrays, solve after solve: through the per-list DMA copies (the default,
    PATH_HANDBACK_DMA=1 pinned) and through k_handback_host's host-mapped
    stores with its speculative launch behind every decided trial
    (PATH_HANDBACK_DMA=0);
    "rows": stiffness / smoothness rows after the observations."""
    from mayamatchmovesolver_amd import abi, make_options
    from mayamatchmovesolver_amd.solver import host_array

    paths(abi.PATH_HANDBACK_DMA, dma)
    if scene == "rows":
        prob = S.edge_scene(stiffness=True)
        opt = make_options(scene_graph_mode=abi.SCENE_GRAPH_MODE_MAYA_DAG, iterations=40)
        assert prob.num_residuals > 2 * prob.num_obs
    else:
        prob = S.make_config(3 if scene == "c3" else 1, frames=12, scale=0.002)
        opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        m, M = prob.num_residuals, prob.num_obs
        ref = s.solve(out=(np.zeros(m), np.zeros(m), np.zeros(M)))
        pin = (host_array(m), host_array(m), host_array(M))
        pre0 = s.kernel_stats()["pre_handbacks"]
        for _ in range(2):
            for a in pin:
                a[:] = np.nan  # every entry rewritten by the hand-back
            got = s.solve(out=pin)
            np.testing.assert_array_equal(got.x, ref.x)
            np.testing.assert_array_equal(pin[0], ref.fvec)
            np.testing.assert_array_equal(pin[1], ref.err_user)
            np.testing.assert_array_equal(pin[2], ref.err_dist)
        pre = s.kernel_stats()["pre_handbacks"] - pre0
        if dma:
            assert pre == 0
        elif ref.result["reason_number"] in (1, 2, 3, 5, 6, 7, 8):
            # ended by the tests after a trial: the speculative hand-back
            # behind it stored the lists
            assert pre == 2
        # the on-demand fetch of a solve(fetch=False) into the same buffers
        s.solve(fetch=False)
        for a in pin:
            a[:] = np.nan
        s.outputs(out=pin)
        np.testing.assert_array_equal(pin[0], ref.fvec)
        np.testing.assert_array_equal(pin[2], ref.err_dist)
    finally:
        s.close()
