"""Central differences where animated FD columns skip the other frames' rows
(B15, adjust_solveFunc.cpp:331-333, 412, 468-471): errorListA keeps the
current errors and errorListB is zero-initialised, so a skipped row j of an
animated central column p holds f_j * 0.5 / (|dA| + |dB|).  The reference's
Jacobian is then J = J_s + f c^T; the library carries the rank-one term
through the column norms, J^T f, the damped solves (Woodbury), lmpar's
Newton term and ||J p|| (Plan::b15).  Each case: the dense Jacobian and the
whole solve through the C ABI against the CPU oracle (which builds the
reference's dense columns), 1e-6 on x and every ||f||, identical counts."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, make_options, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver

from test_gpu_edge import check, check_measure_jacobian

pytestmark = pytest.mark.gpu

DAG, MMSG = abi.SCENE_GRAPH_MODE_MAYA_DAG, abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH
CENTRAL = abi.AUTO_DIFF_TYPE_CENTRAL


@pytest.mark.parametrize("mode", [DAG, MMSG])
@pytest.mark.parametrize("kw", [dict(), dict(static_focal=True), dict(parented=True, frames=4),
                                dict(frames=9, bundles=12, seed=21)])
def test_central_animated_edge(kw, mode, oracle, gpu_ctx):
    """Animated camera pose + static bundles (bundle Schur path); with
    ``static_focal`` one global parameter (the arrow of the reduced system)."""
    prob = S.edge_scene(**kw)
    opt = make_options(auto_diff_type=CENTRAL, scene_graph_mode=mode)
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx, trace_atol=1e-8)


@pytest.mark.parametrize("mode", [DAG, MMSG])
def test_central_animated_c2_window(mode, oracle, gpu_ctx):
    """configs[1] structure (pose + focal per frame, no bundle solved: the
    block-diagonal reduced solve)."""
    prob = S.make_config(1, frames=8, scale=0.1)
    opt = S.config_options(prob, scene_graph_mode=mode, auto_diff_type=CENTRAL, iterations=200)
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx, trace_atol=1e-8)


def test_central_animated_c4_window(oracle, gpu_ctx):
    """configs[3] structure (pose per frame + static bundles, banded reduced
    camera system)."""
    prob = S.make_config(3, frames=8, scale=0.001)
    opt = S.config_options(prob, auto_diff_type=CENTRAL, iterations=60)
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx, trace_atol=1e-8)


def test_central_animated_refused_off_block(gpu_ctx):
    """Several cameras, each animated: an animated column's own frame holds
    rows of the other cameras it does not reach, which would take J_s out of
    its block structure -- still refused (MMBA_ERR_UNSUPPORTED)."""
    prob = S.make_config(2, frames=3, scale=0.002)
    opt = S.config_options(prob, auto_diff_type=CENTRAL)
    with pytest.raises(MmbaError) as e:
        Solver(prob, opt, context=gpu_ctx)
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED


def test_robust_loss_animated_refused(gpu_ctx):
    """The robust loss re-applies the loss to the whole errorList buffer of
    every column (adjust_measureErrors.cpp:553-558): refused where columns
    skip rows."""
    prob = S.edge_scene()
    opt = make_options(robust_loss=1, robust_loss_type=abi.ROBUST_LOSS_TYPE_CAUCHY,
                       robust_loss_scale=100.0)
    with pytest.raises(MmbaError) as e:
        Solver(prob, opt, context=gpu_ctx)
    assert e.value.code == abi.MMBA_ERR_UNSUPPORTED
