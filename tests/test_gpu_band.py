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
    # P = -1: the log-depth solvers -- parallel cyclic reduction
    # (csrc/mmba_pcr.hip) without an arrow and K <= 24, block cyclic reduction
    # (csrc/mmba_bcr.hip) otherwise, K = 8/16/24/32; P = -2: block cyclic
    # reduction only
    (2994, 23, 0, -2), (84, 6, 0, -2), (4096, 24, 0, -2), (90, 5, 0, -2), (7, 3, 0, -2),
    (840, 6, 0, -2), (24 * 257, 24, 0, -1), (24 * 256 + 5, 23, 0, -1), (24, 23, 0, -1),
    (84, 6, 0, -1), (300, 6, 2, -1), (2994, 23, 0, -1), (1000, 23, 5, -1),
    (1000, 32, 16, -1), (10, 2, 16, -1), (0, 0, 4, -1), (90, 5, 0, -1),
    (7, 3, 0, -1), (777, 31, 1, -1), (1000, 16, 3, -1), (17, 8, 2, -1),
    (2880, 11, 2, -1), (840, 6, 0, -1), (4096, 24, 0, -1), (24 * 65, 24, 1, -1),
    # arrows wider than 16 (up to NGMAX = 32): band, partitioned, BCR K = 8..32
    (1000, 23, 24, 1), (1000, 40, 32, 4), (640, 60, 32, 1), (10, 2, 32, 1), (0, 0, 32, 1),
    (1000, 23, 24, -1), (1000, 32, 32, -1), (300, 6, 32, -1), (500, 16, 17, -1),
    (24 * 65, 24, 24, -1), (0, 0, 24, -1),
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


@pytest.mark.parametrize("M,N,K", [(300, 300, 64), (129, 129, 512), (1000, 1000, 256),
                                   (257, 130, 64), (1, 1, 16)])
def test_dgemm_nt_tri_and_general(M, N, K, gpu_ctx):
    """The dense solver's hand-written fp64 MFMA GEMM / SYRK (k_dgemm_nt) on
    ragged shapes against numpy: C - A B^T (general) and the lower triangle of
    C - A A^T (SYRK, upper triangle untouched).  The MFMA sums 4 products per
    step in fp64: agreement to 1e-13 of sum |a b|."""
    from mayamatchmovesolver_amd.solver import debug_dgemm

    rng = np.random.default_rng(M * 7 + N + K)
    A = rng.standard_normal((M, K))
    B = rng.standard_normal((N, K))
    C0 = rng.standard_normal((M, N))
    scale = np.abs(A) @ np.abs(B).T + 1.0
    got = debug_dgemm(gpu_ctx, A, B, C0, alpha=-1.0, beta=1.0)
    assert np.all(np.abs(got - (C0 - A @ B.T)) <= 1e-13 * scale)
    if M == N:
        S0 = rng.standard_normal((M, M))
        got = debug_dgemm(gpu_ctx, A, None, S0, alpha=-1.0, beta=1.0, tri=True)
        ref = S0 - A @ A.T
        low = np.tril(np.ones((M, M), dtype=bool))
        sc = np.abs(A) @ np.abs(A).T + 1.0
        assert np.all(np.abs(got - ref)[low] <= 1e-13 * sc[low])
        np.testing.assert_array_equal(got[~low], S0[~low])


@pytest.mark.parametrize("M", [64, 200, 3001])
def test_dgemm_nt_in_place_panel(M, gpu_ctx):
    """The panel solve L_ip = A_ip Linv^T computed in A_ip's own array (the
    128 x 64 two-wave variant): every workgroup reads its rows in full before
    it overwrites them."""
    from mayamatchmovesolver_amd.solver import debug_dgemm

    rng = np.random.default_rng(M)
    A = rng.standard_normal((M, 64))
    Li = np.tril(rng.standard_normal((64, 64)))
    got = debug_dgemm(gpu_ctx, A, Li, np.zeros((M, 64)), alpha=1.0, beta=0.0, in_place=True)
    scale = np.abs(A) @ np.abs(Li).T + 1.0
    assert np.all(np.abs(got - A @ Li.T) <= 1e-13 * scale)


@pytest.mark.parametrize("parts", [-1, -2])
@pytest.mark.parametrize("nb,w,nG", [(2994, 23, 0), (500, 23, 3), (1000, 15, 0)])
@pytest.mark.parametrize("where", ["odd_block", "even_block", "root", "arrow", "nan"])
def test_bcr_indefinite_is_reported(nb, w, nG, where, parts, gpu_ctx):
    """A non-positive (or NaN) pivot anywhere in the block cyclic reduction --
    a block eliminated at level 0, a block eliminated at a later level, the
    root block, the arrow corner -- is reported as a failed factorisation (the
    LM then raises its damping), never returned as a solution.  The pivot
    chains test the pivots once after the chain (a bad pivot leaves 1/C_jj
    NaN, inf or 0)."""
    from mayamatchmovesolver_amd._lib import MmbaError

    if where == "arrow" and nG == 0:
        pytest.skip("no arrow rows")
    S = band_arrow_spd(nb, w, nG, seed=nb + w + nG)
    K = max(8, (w + 7) // 8 * 8)
    row = {"odd_block": K + 3, "even_block": 2 * K + 5, "root": 2, "arrow": nb + nG - 1,
           "nan": 4 * K + 1}[where]
    S[row, row] = np.nan if where == "nan" else -10.0 * abs(S[row, row])
    solve = debug_band_solve(gpu_ctx, S, nb, w, nG, parts=parts)
    with pytest.raises(MmbaError, match="non-positive pivot"):
        solve(np.ones(nb + nG))
