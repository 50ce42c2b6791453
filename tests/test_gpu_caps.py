"""Structural capacities raised in round 6: up to PCMAX = 12
parameters on one camera-frame block and NGMAX = 48 global parameters (the
arrow of the reduced system), csrc/mmba_internal.h.  The reference has no such
limits (adjust_relationships.cpp:223-337 groups whatever the solve list holds);
the library refuses beyond them with MMBA_ERR_UNSUPPORTED so the caller keeps
cminpack.  Each case: the library through the C ABI against the CPU oracle on
the same inputs -- identical counts, x and every ||f|| of the trace at 1e-6
(test_gpu_edge.check) -- plus the plan's reduced-system shape."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, make_options, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver

from test_gpu_edge import check, check_measure_jacobian

pytestmark = pytest.mark.gpu

DAG, MMSG = abi.SCENE_GRAPH_MODE_MAYA_DAG, abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH
BAND, BDIAG = 0, 3


def stats(prob, opt, ctx):
    s = Solver(prob, opt, context=ctx)
    try:
        return s.kernel_stats()
    finally:
        s.close()


def test_twelve_parameter_camera_frames(oracle, gpu_ctx):
    """A one-camera shot whose pose, focal length and all five 3DE classic
    coefficients are keyed per frame and solved: 12 parameters on each of its
    8 camera-frames (the coefficients join the block: one camera reads them,
    Plan::build), no solved bundle -- the block-diagonal solve with 12-wide
    blocks (k_bd_direct<PCMAX>)."""
    prob = S.make_config(4, frames=8, scale=0.05, lens_model="classic_wide", cameras=1)
    assert prob.num_params == 8 * 12
    opt = S.config_options(prob)
    st = stats(prob, opt, gpu_ctx)
    assert st["reduced_dim"] == 96 and st["reduced_kind"] == BDIAG, st
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("mode", [DAG, MMSG])
def test_forty_globals_band(mode, oracle, gpu_ctx):
    """Six static witness cameras with poses and focal lengths solved as
    static parameters plus one film back: 40 globals beside the animated
    camera's per-frame blocks and 24 solved bundles (band + a 40-wide arrow;
    block cyclic reduction, root K + nG = 24 + 40).  Four frames: the
    oracle's own x envelope under a 1-ulp change of x0 is 7.8e-8 here, where
    the six-frame rig's is 4.5e-6 to 5.8e-6 -- beyond the 1e-6 bar for any
    implementation (tools/caps_envelope.py, profiles/r6_caps/)."""
    prob = S.witness_scene(n_witness=6, n_focal=6, extra_globals=1, frames=4)
    opt = make_options(scene_graph_mode=mode)
    st = stats(prob, opt, gpu_ctx)
    assert st["reduced_dim"] == 24 + 40 and st["reduced_kind"] == BAND, st
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx)


def test_forty_globals_band_chain(oracle, gpu_ctx):
    """Six frames (half bandwidth 35 > 32): the band chain as one partition
    with the 40-wide corner factored at width 64.  The oracle's own x
    envelope on this rig is 5.8e-6 (tools/caps_envelope.py), so x is held at
    1e-5; counts, the whole trace and the outputs at 1e-6 as everywhere."""
    prob = S.witness_scene(n_witness=6, n_focal=6, extra_globals=1)
    opt = make_options(scene_graph_mode=DAG)
    st = stats(prob, opt, gpu_ctx)
    assert st["reduced_dim"] == 36 + 40 and st["reduced_kind"] == BAND, st
    check(prob, opt, oracle, gpu_ctx, x_tol=1e-5)


def test_forty_globals_block_diagonal(oracle, gpu_ctx):
    """The same 40 globals with the bundles locked: block diagonal + a 40-wide
    arrow (k_bd_root<48>, arrow lanes 12..51 of the block waves)."""
    prob = S.witness_scene(n_witness=6, n_focal=6, extra_globals=1, solve_bundles=False)
    opt = make_options(scene_graph_mode=DAG)
    st = stats(prob, opt, gpu_ctx)
    assert st["reduced_dim"] == 36 + 40 and st["reduced_kind"] == BDIAG, st
    check(prob, opt, oracle, gpu_ctx)


def test_global_capacity_refused(gpu_ctx):
    """49 globals: refused as UNSUPPORTED (the caller keeps cminpack)."""
    prob = S.witness_scene(n_witness=7, n_focal=7, extra_globals=3)
    with pytest.raises(MmbaError) as ei:
        Solver(prob, make_options(), context=gpu_ctx)
    assert ei.value.code == abi.MMBA_ERR_UNSUPPORTED
    assert "48 global" in str(ei.value)
