"""Pin the MINPACK restatement (oracle/refcpu.c) against scipy's MINPACK
(scipy.optimize._minpack, scipy 1.15.3) -- the in-container stand-in for
cminpack 1.3.8.  Same callbacks, same options; final x, info,
nfev, njev and the full sequence of evaluation points must agree."""
import numpy as np
import pytest
from scipy.optimize import _minpack

T = np.linspace(0, 4, 30)
Y = 2.5 * np.exp(-1.3 * T) + 0.5 + 0.01 * np.random.default_rng(1).standard_normal(30)


def exp_f(p):
    return p[0] * np.exp(-p[1] * T) + p[2] - Y


def exp_j(p):
    e = np.exp(-p[1] * T)
    return np.stack([e, -p[0] * T * e, np.ones_like(T)], 1)


def rosen_f(x):
    return np.array([10 * (x[1] - x[0] ** 2), 1 - x[0]])


def rosen_j(x):
    return np.array([[-20 * x[0], 10.0], [-1.0, 0.0]])


def powell_f(x):
    return np.array([x[0] + 10 * x[1], np.sqrt(5) * (x[2] - x[3]), (x[1] - 2 * x[2]) ** 2,
                     np.sqrt(10) * (x[0] - x[3]) ** 2])


def powell_j(x):
    a, b = 2 * (x[1] - 2 * x[2]), 2 * np.sqrt(10) * (x[0] - x[3])
    return np.array([[1, 10, 0, 0], [0, 0, np.sqrt(5), -np.sqrt(5)], [0, a, -2 * a, 0],
                     [b, 0, 0, -b]], dtype=float)


def box3d_f(x):
    t = 0.1 * np.arange(1, 11)
    return np.exp(-t * x[0]) - np.exp(-t * x[1]) - x[2] * (np.exp(-t) - np.exp(-10 * t))


def box3d_j(x):
    t = 0.1 * np.arange(1, 11)
    return np.stack([-t * np.exp(-t * x[0]), t * np.exp(-t * x[1]),
                     -(np.exp(-t) - np.exp(-10 * t))], 1)


CASES = [
    (exp_f, exp_j, [1.0, 0.5, 0.0], 30),
    (rosen_f, rosen_j, [-1.2, 1.0], 2),
    (powell_f, powell_j, [3.0, -1.0, 0.0, 1.0], 4),
    (box3d_f, box3d_j, [0.0, 10.0, 20.0], 10),
]


@pytest.mark.parametrize("fun,jac,x0,m", CASES)
@pytest.mark.parametrize("factor", [100.0, 1.0])
def test_lmder_matches_scipy(oracle, fun, jac, x0, m, factor):
    seq = []

    def f(x):
        seq.append((1, x.copy()))
        return fun(x)

    def J(x):
        seq.append((2, x.copy()))
        return jac(x)

    out = _minpack._lmder(f, J, np.array(x0, float), (), 1, 0, 1e-6, 1e-6, 1e-6, 1000, factor,
                          None)
    xs, info_d, info_s = out[0], out[1], out[2]
    xr, info_r, nfev, njev, calls = oracle.lmder(fun, jac, x0, m, factor=factor)
    assert info_r == info_s
    assert nfev == info_d["nfev"] and njev == info_d["njev"]
    np.testing.assert_allclose(xr, xs, rtol=1e-13, atol=1e-300)
    # scipy evaluates fun once up front for shape checking
    seq = seq[1:]
    assert [c[0] for c in seq] == [c[0] for c in calls]
    for a, b in zip(seq, calls):
        np.testing.assert_allclose(a[1], b[1], rtol=1e-13, atol=1e-300)


@pytest.mark.parametrize("fun,jac,x0,m", CASES)
def test_lmdif_matches_scipy(oracle, fun, jac, x0, m):
    out = _minpack._lmdif(fun, np.array(x0, float), (), 1, 1e-6, 1e-6, 1e-6, 2000, 1e-4, 100.0,
                          None)
    xr, info, nfev, _ = oracle.lmdif(fun, x0, m, epsfcn=1e-4, maxfev=2000)
    assert info == out[2]
    assert nfev == out[1]["nfev"]
    np.testing.assert_allclose(xr, out[0], rtol=1e-13, atol=1e-300)


def test_enorm_matches_definition(oracle):
    rng = np.random.default_rng(0)
    for scale in (1e-25, 1.0, 1e20):
        x = rng.standard_normal(100) * scale
        assert abs(oracle.enorm(x) - np.linalg.norm(x)) <= 1e-13 * np.linalg.norm(x)
    assert oracle.enorm(np.zeros(5)) == 0.0
