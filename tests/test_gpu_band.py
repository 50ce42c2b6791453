"""Device band + arrow Cholesky (csrc/mmba_band.hip) against numpy on random
symmetric positive-definite matrices of the reduced-system shape: nb band rows
of half bandwidth w plus nG dense arrow rows, with and without the partitioned
(nested-dissection) path and with block cyclic reduction (P = -1).  Tolerance: fp64 direct solve, 1e-10 relative to
max |x| on well-conditioned matrices."""
import numpy as np
import pytest

from mayamatchmovesolver_amd.solver import debug_band_solve

pytestmark = pytest.mark.gpu


def band_arrow_spd(nb, w, nG, seed):
    rng = np.random.default_rng(seed)
    n = nb + nG
    A = np.zeros((n, n))
    for i in range(nb):
        lo = max(0, i - w)
        A[i, lo:i + 1] = rng.uniform(-1, 1, i + 1 - lo)
    A[nb:, :] = rng.uniform(-1, 1, (nG, n)) * 0.3
    S = A @ A.T
    # structure: keep band + arrow only, then make it diagonally dominant
    mask = np.zeros((n, n), bool)
    for i in range(nb):
        mask[i, max(0, i - w):min(nb, i + w + 1)] = True
    mask[nb:, :] = True
    mask[:, nb:] = True
    S = np.where(mask, S, 0.0)
    S += np.diag(np.abs(S).sum(1) + 1.0)
    return S


CASES = [
    # nb, w, nG, P
    (84, 6, 0, 1), (84, 6, 0, 3), (300, 6, 2, 8),
    (500, 23, 0, 1), (2994, 23, 0, 0), (2994, 23, 0, 11), (2994, 23, 0, 24),
    (1000, 23, 5, 6), (1000, 40, 16, 4), (640, 60, 3, 1), (777, 80, 1, 1),
    (10, 2, 16, 1), (0, 0, 4, 1), (90, 5, 0, 9),
    # P = -1: block cyclic reduction (csrc/mmba_bcr.hip), K = 8/16/24/32
    (84, 6, 0, -1), (300, 6, 2, -1), (2994, 23, 0, -1), (1000, 23, 5, -1),
    (1000, 32, 16, -1), (10, 2, 16, -1), (0, 0, 4, -1), (90, 5, 0, -1),
    (7, 3, 0, -1), (777, 31, 1, -1), (1000, 16, 3, -1), (17, 8, 2, -1),
    (2880, 11, 2, -1), (840, 6, 0, -1), (4096, 24, 0, -1), (24 * 65, 24, 1, -1),
]


@pytest.mark.parametrize("nb,w,nG,P", CASES)
def test_band_solve_matches_numpy(nb, w, nG, P, gpu_ctx):
    S = band_arrow_spd(nb, w, nG, seed=nb * 31 + w * 7 + nG + P)
    rng = np.random.default_rng(P + 5)
    r = rng.standard_normal(nb + nG)
    solve = debug_band_solve(gpu_ctx, S, nb, w, nG, P)
    x, yn, used = solve(r)
    xr = np.linalg.solve(S, r)
    assert np.max(np.abs(x - xr)) <= 1e-10 * np.max(np.abs(xr)), (used, np.max(np.abs(x - xr)))
    ynr = float(r @ xr)  # ||L^-1 r||^2 = r^T S^-1 r for any valid factor
    assert abs(yn - ynr) <= 1e-10 * abs(ynr)
    if P > 1:
        assert used > 1
