"""Global parameters beyond 16 (VERDICT r2 "missing" 5, "next" 8): the
reference has no limit on the global (static, shared) parameters
(adjust_relationships.cpp:223-337); the library's reduced system carries
them as an arrow of up to NGMAX = 48 rows (csrc/mmba_internal.h; 32 until round 6).  Scenes:
static witness cameras whose poses and focal lengths are solved as static
parameters beside an animated camera solved per frame (synthetic
witness_scene), on each reduced-system path: the band + arrow Cholesky
(every frame coupled), block cyclic reduction (bundles on 3-frame windows),
the block-diagonal + arrow solve (no solved bundle), and frame shards.  Each
case: the library through the C ABI against the CPU oracle on the same
inputs, 1e-6 on x and on every ||f|| of the trace, identical counts."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, make_options, synthetic as S
from mayamatchmovesolver_amd._lib import MmbaError
from mayamatchmovesolver_amd.solver import Solver

from test_gpu_edge import check, check_measure_jacobian
from test_gpu_sharded import check_shards_agree, run_sharded

pytestmark = pytest.mark.gpu

DAG, MMSG = abi.SCENE_GRAPH_MODE_MAYA_DAG, abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH
BAND, BDIAG = 0, 3


def reduced_kind(prob, opt, ctx):
    s = Solver(prob, opt, context=ctx)
    try:
        return s.kernel_stats()["reduced_kind"]
    finally:
        s.close()


@pytest.mark.parametrize("mode", [DAG, MMSG])
@pytest.mark.parametrize("kw,ng", [(dict(), 24), (dict(n_witness=5, n_focal=5), 32)])
def test_wide_arrow_band(kw, ng, mode, oracle, gpu_ctx):
    """Every frame coupled through the bundles: band + arrow Cholesky."""
    prob = S.witness_scene(**kw)
    opt = make_options(scene_graph_mode=mode)
    assert reduced_kind(prob, opt, gpu_ctx) == BAND
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("kw", [dict(frames=4), dict(frames=5, n_witness=5, n_focal=5)])
def test_wide_arrow_bcr(kw, oracle, gpu_ctx):
    """Four / five frames of the animated camera: half bandwidth 23 / 29, so
    the reduced system is factored by block cyclic reduction (K = 24 / 32)
    with the 24 / 32-wide arrow (roots of order 48 / 64).  The oracle's own
    1-ulp x envelope on these rigs is 4.2e-7 / 2.7e-8, inside the 1e-6 bar.
    (Windowed visibility of the animated camera over 8-12 frames leaves a rig
    without a parity bar: there the envelope is 8e1 to 3e6 and even the
    oracle's reason code and evaluation count change under a 1-ulp change of
    x0 -- tools/wide_arrow_envelope.py, profiles/r4_parity/.)"""
    prob = S.witness_scene(**kw)
    opt = make_options()
    assert reduced_kind(prob, opt, gpu_ctx) == BAND
    check(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("mode", [DAG, MMSG])
@pytest.mark.parametrize("kw", [dict(solve_bundles=False),
                                dict(solve_bundles=False, n_witness=5, n_focal=5)])
def test_wide_arrow_block_diagonal(kw, mode, oracle, gpu_ctx):
    """No solved bundle: block-diagonal camera-frame blocks + the arrow."""
    prob = S.witness_scene(**kw)
    opt = make_options(scene_graph_mode=mode)
    assert reduced_kind(prob, opt, gpu_ctx) == BDIAG
    check(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("kw,n,rep", [
    # 12 frames, no solved bundle: half bandwidth 5, four or six camera-frames
    # per shard -- the frames really shard (partitioned band + the 32-wide
    # arrow all-reduced); the oracle's 1-ulp x envelope is 3.5e-9
    (dict(frames=12, solve_bundles=False, n_witness=5, n_focal=5), 2, 0),
    (dict(frames=12, solve_bundles=False, n_witness=5, n_focal=5), 3, 0),
    # every frame coupled through the solved bundles (half bandwidth 35 / 29)
    # over 6 / 5 frames: fewer than 2 w + 8 camera-frame rows per shard, so
    # the problem does not shard and every shard solves all of it
    (dict(n_witness=5, n_focal=5), 2, 1),
    (dict(frames=5, n_witness=5, n_focal=5), 3, 1)])
def test_wide_arrow_sharded(kw, n, rep, oracle):
    """Frame shards (in-process communicators): the global rows are
    all-reduced like the narrow arrow's; a problem too small to shard is
    solved redundantly on every shard (mmba_plan_create_sharded), not refused."""
    prob = S.witness_scene(**kw)
    opt = make_options()
    reps = []
    outs = run_sharded(prob, opt, n, replicated=reps)
    assert reps == [rep] * n
    check_shards_agree(outs)
    xr, _f, _eu, _ed, rr, trr = oracle.solve(prob, opt)
    o = outs[0]
    assert o.result["reason_number"] == rr.reason_number
    assert o.result["iterations"] == rr.iterations
    np.testing.assert_allclose(o.fnorm_trace, trr, rtol=1e-6, atol=1e-9 * trr[0])
    xs = np.maximum(np.abs(xr), 1e-3)
    assert np.max(np.abs(o.x - xr) / xs) <= 1e-6


def test_arrow_beyond_32(oracle, gpu_ctx):
    """33 globals (refused up to round 5, NGMAX was 32): solved against the
    oracle (the capacity is now 48, tests/test_gpu_caps.py)."""
    prob = S.witness_scene(n_witness=5, n_focal=5, extra_globals=1)
    check(prob, make_options(), oracle, gpu_ctx)


@pytest.mark.parametrize("mode", [DAG, MMSG])
def test_more_than_20_columns_per_observation(mode, oracle, gpu_ctx):
    """A shared anamorphic lens with its ten coefficients solved beside the
    witness poses, focal lengths and film back widths: a witness observation
    reaches 21 parameters (the library's bound is LMAX = 32).  The lens
    coefficients are weakly determined by these markers (the oracle's own
    final x moves by 5e-5 under a 1-ulp change of x0), so the bar is the
    dense Jacobian and one LM step (1-ulp envelope 6e-9) at 1e-6."""
    prob = S.witness_scene(n_witness=2, n_focal=2, extra_globals=2, lens="anamorphic")
    opt = make_options(scene_graph_mode=mode, iterations=2)
    check_measure_jacobian(prob, opt, oracle, gpu_ctx)
    check(prob, opt, oracle, gpu_ctx)
