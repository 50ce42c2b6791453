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
    # dataflow launches on 1 / 3 workgroups: most items are drawn (item
    # tickets) by workgroups that already ran others -- the forward-progress
    # path when few workgroups are resident
    "grid1": {"MMBA_BCR_DF_GRID": "1"},
    "grid3": {"MMBA_BCR_DF_GRID": "3"},
}
ENV_KEYS = ("MMBA_BCR_DF", "MMBA_BCR_MFMA", "MMBA_BCR_CHOL", "MMBA_BCR_DF_GRID")


def run(prob, opt, ctx, monkeypatch, env):
    for k in ENV_KEYS:
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
    for k in ENV_KEYS:
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


def _threads(n, fn):
    import threading
    outs, errs = [None] * n, [None] * n

    def work(r):
        try:
            outs[r] = fn(r)
        except Exception as e:  # noqa: BLE001 - reported below
            errs[r] = e

    ths = [threading.Thread(target=work, args=(r,), daemon=True) for r in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in ths), "concurrent solves hung"
    assert errs == [None] * n, errs
    return outs


def test_bcr_dataflow_concurrent_full_c4(gpu_ctx, monkeypatch):
    """Eight full-size C4 solves (125 band blocks: 63 workgroups of 256
    threads per dataflow factorisation, 125 per backward solve) at once, one
    host thread and one stream each: about 500 workgroups that each fill a CU
    compete for 256 CUs, so the dataflow launches cannot all be resident.
    With item tickets every wait still ends: each solve must equal the solo
    solve bit for bit (a timed-out wait would fail the solve or switch the
    plan to the per-level launches, whose bits are the same -- so the flag is
    checked too)."""
    from mayamatchmovesolver_amd.solver import Context
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    prob = S.make_config(3)
    opt = S.config_options(prob)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        ref = s.solve()
    finally:
        s.close()
    assert ref.result["success"]
    n = 8
    ctxs = [Context(0) for _ in range(n)]
    solvers = [Solver(prob, opt, context=ctxs[r]) for r in range(n)]
    try:
        for _ in range(2):
            outs = _threads(n, lambda r: solvers[r].solve())
            for o in outs:
                np.testing.assert_array_equal(o.fnorm_trace, ref.fnorm_trace)
                np.testing.assert_array_equal(o.x, ref.x)
        assert all(not sv.dataflow_fallback() for sv in solvers)
    finally:
        for sv in solvers:
            sv.close()
        for c in ctxs:
            c.close()
