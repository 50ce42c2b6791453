"""The block-cyclic-reduction factorisation's code paths give the same solve
bit for bit: the one-launch dataflow factor (default), the per-level
launches (MMBA_BCR_DF=0) and the unblocked pivot chain (MMBA_BCR_CHOL=0) all
perform the same floating-point operations in the same order, so x, fvec and
the whole ||f|| trace must be identical (the VALU updates, MMBA_BCR_MFMA=0,
sum in another order and are checked against numpy in test_gpu_band.py).  A hand-off race in the dataflow factor (a stale block read across
workgroups) shows up here as a mismatch.  Scenes: the C4 structure (nG = 0,
K = 8 and 24) through the whole solver; band + arrow systems (nG = 2..16,
root of order K + 8 / K + 16, K = 16 / 24 / 32) through the band-solve hook."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S
from mayamatchmovesolver_amd.solver import Solver, debug_band_solve
from tests.test_gpu_band import band_arrow_spd

pytestmark = pytest.mark.gpu

SCENES = {
    "c4": (3, dict(frames=120, scale=0.02)),
    "c4_wide": (3, dict(frames=64, scale=0.01, window=6, depth=(4.0, 10.0))),
}
VARIANTS = {
    "levels": {"MMBA_BCR_DF": "0"},
    "chain": {"MMBA_BCR_CHOL": "0"},
}


def run(prob, opt, ctx, monkeypatch, env):
    for k in ("MMBA_BCR_DF", "MMBA_BCR_MFMA", "MMBA_BCR_CHOL"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    s = Solver(prob, opt, context=ctx)
    try:
        return s.solve()
    finally:
        s.close()


@pytest.mark.parametrize("scene", list(SCENES))
def test_bcr_variants_bitwise(scene, gpu_ctx, monkeypatch):
    idx, kw = SCENES[scene]
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    ref = run(prob, opt, gpu_ctx, monkeypatch, {})
    assert ref.result["success"], ref.result
    for name, env in VARIANTS.items():
        out = run(prob, opt, gpu_ctx, monkeypatch, env)
        np.testing.assert_array_equal(out.fnorm_trace, ref.fnorm_trace, err_msg=name)
        np.testing.assert_array_equal(out.x, ref.x, err_msg=name)
        np.testing.assert_array_equal(out.fvec, ref.fvec, err_msg=name)


def test_bcr_dataflow_repeatable(gpu_ctx, monkeypatch):
    """Ten solves through one plan (the dataflow factor reuses its flags with
    a new epoch per launch): identical results every time."""
    idx, kw = SCENES["c4"]
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    for k in ("MMBA_BCR_DF", "MMBA_BCR_MFMA", "MMBA_BCR_CHOL"):
        monkeypatch.delenv(k, raising=False)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
        for _ in range(9):
            out = s.solve()
            np.testing.assert_array_equal(out.x, ref.x)
            np.testing.assert_array_equal(out.fnorm_trace, ref.fnorm_trace)
    finally:
        s.close()


@pytest.mark.parametrize("nb,w,nG", [(1000, 23, 5), (1000, 32, 16), (2880, 11, 2),
                                     (1000, 16, 3), (24 * 65, 24, 1)])
def test_bcr_band_arrow_dataflow_bitwise(nb, w, nG, gpu_ctx, monkeypatch):
    S_ = band_arrow_spd(nb, w, nG, seed=nb + w + nG)
    r = np.random.default_rng(nG).standard_normal(nb + nG)
    outs = []
    for env in ({}, {"MMBA_BCR_DF": "0"}):
        monkeypatch.delenv("MMBA_BCR_DF", raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        x, yn, _used = debug_band_solve(gpu_ctx, S_, nb, w, nG, -1)(r)
        outs.append((x, yn))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    assert outs[0][1] == outs[1][1]
