"""Pin the oracle's geometry to the reference's own golden values
(lib/rust/mmscenegraph/tests/reprojection.rs, math/camera.rs tests) and the
3DE-classic round trip of lib/cppbind/mmlens/tests/test_once_3de_classic.cpp."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi

EPS = 1e-5  # reprojection.rs EPSILON


def test_projection_matrix_rust_golden(oracle):
    # math/camera.rs:79-120
    P = oracle.projection_matrix(abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH, 35.0, 36 / 25.4, 24 / 25.4)
    expected = np.array([[1.94445, 0, 0, 0], [0, 2.55927, 0, 0], [0, 0, 1.00002, -1],
                         [0, 0, 0.200002, 0]]).T
    np.testing.assert_allclose(P, expected, rtol=EPS, atol=EPS)


def test_single_point_rust_golden(oracle):
    # tests/reprojection.rs:37-97
    cam = oracle.trs_matrix((-2, 2, 5), (10, -10, -10))
    P = oracle.projection_matrix(abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH, 35.0, 36 / 25.4, 24 / 25.4)
    xy = oracle.reproject(cam, P, (-0.5, 2.7, 0.0))
    np.testing.assert_allclose(xy, [0.0865145148481126, 0.0096299819122515], rtol=EPS, atol=EPS)


def test_two_bundles_under_group_rust_golden(oracle):
    # tests/reprojection.rs:100-196
    grp = oracle.trs_matrix((0, 0, -10), (0, 15, 0))
    a = grp @ oracle.trs_matrix((-5, 0, 0), (0, 0, 0))
    b = grp @ oracle.trs_matrix((5, 0, 0), (0, 0, 0))
    np.testing.assert_allclose(a[:3, 3], [-4.829629, 0.0, -8.705905], atol=EPS)
    np.testing.assert_allclose(b[:3, 3], [4.829629, 0.0, -11.294095], atol=EPS)
    cam = oracle.trs_matrix((0, 5, 10), (-10, 0, 0), roo=abi.ROO_ZXY)
    expected_cam = np.array([[1, 0, 0, 0], [0, 0.984808, -0.173648, 0], [0, 0.173648, 0.984808, 0],
                             [0, 5, 10, 1]]).T
    np.testing.assert_allclose(cam, expected_cam, atol=EPS)
    for mode in (abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH, abi.SCENE_GRAPH_MODE_MAYA_DAG):
        P = oracle.projection_matrix(mode, 35.0, 36 / 25.4, 24 / 25.4)
        np.testing.assert_allclose(oracle.reproject(cam, P, a[:3, 3]), [-0.243416, -0.111167],
                                   atol=EPS)
        np.testing.assert_allclose(oracle.reproject(cam, P, b[:3, 3]), [0.2150060, -0.071858],
                                   atol=EPS)


@pytest.mark.parametrize("roo", range(6))
def test_rotate_orders_are_rotations(oracle, roo):
    M = oracle.trs_matrix((1, 2, 3), (10, -20, 30), (1, 1, 1), roo=roo)
    R = M[:3, :3]
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-14)
    np.testing.assert_allclose(np.linalg.det(R), 1.0, atol=1e-14)


def test_film_offsets_only_move_points_in_maya_dag(oracle):
    """Appendix B6: MMSG puts film-offset terms in the z row."""
    cam = oracle.trs_matrix((0, 0, 0), (0, 0, 0))
    pt = (1.0, 0.5, -10.0)
    for mode, moves in ((abi.SCENE_GRAPH_MODE_MAYA_DAG, True),
                        (abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH, False)):
        P0 = oracle.projection_matrix(mode, 35.0, 36 / 25.4, 24 / 25.4)
        P1 = oracle.projection_matrix(mode, 35.0, 36 / 25.4, 24 / 25.4, offx=0.1)
        d = np.abs(oracle.reproject(cam, P1, pt) - oracle.reproject(cam, P0, pt))
        assert (d[0] > 1e-6) == moves


def test_lens_3de_classic_round_trip(oracle):
    """mmlens test_once_3de_classic.cpp:32-81: undistort(redistort(p)) == p."""
    coeff = [0.1, 1.0, 0.0, 0.0, 0.1]
    for x in np.linspace(-0.5, 0.5, 7):
        for y in np.linspace(-0.5, 0.5, 7):
            dx, dy = oracle.lens_distort(coeff, x, y)
            ux, uy = oracle.lens_undistort(coeff, dx, dy)
            assert abs(ux - x) < 1e-5 and abs(uy - y) < 1e-5
    assert oracle.lens_distort([0, 1, 0, 0, 0], 0.3, -0.2) == pytest.approx((0.3, -0.2), abs=1e-15)


RADIAL_TEST_COEFF = [0.1, 0.01, -0.01, 0.05, -0.02, 0.02, 45.0, 0.5]


def test_lens_3de_radial_round_trip(oracle):
    """mmlens test_once_3de_radial_std_deg4.cpp:40-67 (the coefficients of that
    test, its order: undistort, then redistort).  The reference test prints and
    asserts nothing; the fixed-point inverse (20 + 2 iterations,
    ldpk_generic_distortion_base.h) is not converged at the far corner
    (-0.5, 0.5) with this strong bending (1.2e-3 there), so the bound is 1e-5
    inside |x|, |y| <= 0.45 and 2e-3 on the whole frame."""
    for x in np.linspace(-0.5, 0.5, 9):
        for y in np.linspace(-0.5, 0.5, 9):
            ux, uy = oracle.lens_radial_undistort(RADIAL_TEST_COEFF, x, y)
            dx, dy = oracle.lens_radial_distort(RADIAL_TEST_COEFF, ux, uy)
            tol = 1e-5 if max(abs(x), abs(y)) <= 0.45 else 2e-3
            assert abs(dx - x) < tol and abs(dy - y) < tol
    zero = [0.0] * 8
    assert oracle.lens_radial_distort(zero, 0.3, -0.2) == pytest.approx((0.3, -0.2), abs=1e-15)
    assert oracle.lens_radial_undistort(zero, 0.3, -0.2) == pytest.approx((0.3, -0.2), abs=1e-15)


def test_lens_3de_radial_undistort_model(oracle):
    """The undistort map restated independently in numpy from the LDPK text:
    cylindric M (ldpk_cylindric_extender.h calc_m) applied to the radial
    decentered polynomial (ldpk_radial_decentered_distortion.h operator()),
    in diagonal-normalised coordinates (mmlens lib.h:45-58, back 3.6 x 2.4)."""
    c2, u2, v2, c4, u4, v4, phi, b = RADIAL_TEST_COEFF
    w, h = 3.6, 2.4
    r = np.hypot(w, h) / 2
    q = np.sqrt(1 + b)
    cs, sn = np.cos(np.radians(phi)), np.sin(np.radians(phi))
    M = np.array([[cs * cs * q + sn * sn / q, (q - 1 / q) * cs * sn],
                  [(q - 1 / q) * cs * sn, cs * cs / q + sn * sn * q]])
    for x, y in [(0.3, -0.2), (-0.45, 0.4), (0.01, 0.02), (0.5, 0.5)]:
        px, py = x * w / r, y * h / r
        r2 = px * px + py * py
        rad = 1 + c2 * r2 + c4 * r2 * r2
        qx = px * rad + (r2 + 2 * px * px) * (u2 + u4 * r2) + 2 * px * py * (v2 + v4 * r2)
        qy = py * rad + (r2 + 2 * py * py) * (v2 + v4 * r2) + 2 * px * py * (u2 + u4 * r2)
        ox, oy = M @ [qx, qy]
        got = oracle.lens_radial_undistort(RADIAL_TEST_COEFF, x, y)
        assert got == pytest.approx((ox * r / w, oy * r / h), abs=1e-13)


ANAM_TEST_COEFF = [0.05, 0.05, -0.05, -0.05, 0.05, 0.05, -0.05, -0.05, 0.15, 0.15,
                   45.0, 1.1, 1.0]


@pytest.mark.parametrize("rescale", [1.0, 2.0])
def test_lens_3de_anamorphic_round_trip(oracle, rescale):
    """mmlens test_once_3de_anamorphic_std_deg4[_rescaled].cpp:58-74 (its
    coefficients; rescale 1.0 is the non-rescaled model): undistort, then
    redistort, returns the input (the reference test prints, asserts nothing)."""
    c = ANAM_TEST_COEFF + [rescale]
    worst = 0.0
    for x in np.linspace(-0.4, 0.4, 9):
        for y in np.linspace(-0.4, 0.4, 9):
            ux, uy = oracle.lens_anamorphic_undistort(c, x, y)
            dx, dy = oracle.lens_anamorphic_distort(c, ux, uy)
            worst = max(worst, abs(dx - x), abs(dy - y))
    assert worst < 1e-5, worst
    ident = [0.0] * 10 + [0.0, 1.0, 1.0, 1.0]
    assert oracle.lens_anamorphic_distort(ident, 0.3, -0.2) == pytest.approx((0.3, -0.2), abs=1e-15)


@pytest.mark.parametrize("rescale", [1.0, 2.0])
def test_lens_3de_anamorphic_undistort_generic_form(oracle, rescale):
    """The oracle's undistort uses the degree-4 specialisation (prepare()'s
    combined coefficients); restate it here from the GENERIC r / phi form of
    ldpk_generic_anamorphic_distortion.h operator() (sum of
    c(i_phi, i_r) cos(i_phi phi) r^i_r), with the extender matrices built
    independently (rotation, squeeze x / y, rescale; pixel aspect 1)."""
    c = ANAM_TEST_COEFF + [rescale]
    cx = {(0, 0): 1.0, (0, 2): c[0], (2, 2): c[2], (0, 4): c[4], (2, 4): c[6], (4, 4): c[8]}
    cy = {(0, 0): 1.0, (0, 2): c[1], (2, 2): c[3], (0, 4): c[5], (2, 4): c[7], (4, 4): c[9]}
    ph = np.radians(c[10])
    R = np.array([[np.cos(ph), -np.sin(ph)], [np.sin(ph), np.cos(ph)]])
    Sx, Sy, Rs = np.diag([c[11], 1.0]), np.diag([1.0, c[12]]), np.diag([c[13], 1.0])
    rsp = R @ Sx @ Sy @ Rs
    par = Rs @ R
    w, h = 3.6, 2.4
    rr = np.hypot(w, h) / 2
    for x, y in [(0.3, -0.2), (-0.35, 0.25), (0.01, 0.02), (0.4, 0.4)]:
        p = np.linalg.solve(par, [x * w / rr, y * h / rr])
        r, phi = np.hypot(*p), np.arctan2(p[1], p[0])
        qx = sum(v * np.cos(k[0] * phi) * r ** k[1] for k, v in cx.items())
        qy = sum(v * np.cos(k[0] * phi) * r ** k[1] for k, v in cy.items())
        o = rsp @ [p[0] * qx, p[1] * qy]
        got = oracle.lens_anamorphic_undistort(c, x, y)
        assert got == pytest.approx((o[0] * rr / w, o[1] * rr / h), abs=1e-12)


def test_bound_transforms(oracle):
    from mayamatchmovesolver_amd.problem import (FLOAT_MAX, param_external_to_internal,
                                                 param_internal_to_external)
    cases = [(-FLOAT_MAX, FLOAT_MAX, 0.0, 1.0), (-5.0, 5.0, 0.0, 1.0), (-5.0, FLOAT_MAX, 0.0, 1.0),
             (-FLOAT_MAX, 5.0, 0.0, 1.0), (-2.0, 8.0, 0.5, 2.0)]
    for lo, hi, off, sc in cases:
        for v in (-4.0, -1.0, 0.0, 2.5, 4.9):
            a = oracle.param_external_to_internal(v, lo, hi, off, sc)
            b = param_external_to_internal(v, lo, hi, off, sc)
            assert a == pytest.approx(b, rel=1e-15, abs=1e-15)
            assert oracle.param_internal_to_external(a, lo, hi, off, sc) == pytest.approx(
                param_internal_to_external(a, lo, hi, off, sc), rel=1e-15, abs=1e-15)
    # B2: lower-bound-only attributes are clamped to xmin by int->ext
    assert oracle.param_internal_to_external(3.0, -5.0, FLOAT_MAX, 0.0, 1.0) == -5.0


def test_vectorised_external_params_match_scalar(oracle):
    """Problem.external_params (vectorised) == adjust_base.cpp:194-220 per element."""
    from mayamatchmovesolver_amd import synthetic as S
    from mayamatchmovesolver_amd.problem import FLOAT_MAX
    prob = S.known_scene("test1")
    n = 40
    rng = np.random.default_rng(3)
    lo = np.where(rng.random(n) < 0.5, -FLOAT_MAX, rng.uniform(-5, 0, n))
    hi = np.where(rng.random(n) < 0.5, FLOAT_MAX, rng.uniform(1, 5, n))
    prob.param_min, prob.param_max = lo, hi
    prob.param_offset = np.where(rng.random(n) < 0.3, 0.5, 0.0)
    prob.param_scale = np.where(rng.random(n) < 0.3, 2.0, 1.0)
    x = rng.uniform(-3, 3, n)
    got = prob.external_params(x)
    for i in range(n):
        ref = oracle.param_internal_to_external(x[i], lo[i], hi[i], prob.param_offset[i],
                                                prob.param_scale[i])
        assert got[i] == pytest.approx(ref, rel=1e-15, abs=1e-15)
