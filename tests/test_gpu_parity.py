"""GPU parity: libmmba.so (HIP, gfx950) against the CPU oracle on the same inputs.

Bar (BASELINE.json north_star): final parameter vector and per-iteration
residual norm within 1e-6 relative (fp64).
"""
import numpy as np
import pytest

from mayamatchmovesolver_amd import abi, make_options, synthetic as S
from mayamatchmovesolver_amd.problem import FLOAT_MAX
from mayamatchmovesolver_amd.solver import Solver

pytestmark = pytest.mark.gpu

REL = 1e-6


def rel_err(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-300))) if a.size else 0.0


def check_solve(prob, opt, oracle, gpu_ctx, x_tol=REL, trace_tol=REL):
    xr, fr, eur, edr, rr, trr = oracle.solve(prob, opt)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        out = s.solve()
    finally:
        s.close()
    g = out.result
    assert g["reason_number"] == rr.reason_number, (g, rr.as_dict())
    assert g["iterations"] == rr.iterations
    assert g["outer_iterations"] == rr.outer_iterations
    assert g["function_evals"] == rr.function_evals
    assert g["jacobian_evals"] == rr.jacobian_evals
    assert len(out.fnorm_trace) == len(trr)
    # Relative 1e-6 per evaluation; exact-fit scenes converge to ||f|| ~ 1e-10
    # where only roundoff is left, so an absolute floor of 1e-9 * ||f0|| applies.
    np.testing.assert_allclose(out.fnorm_trace, trr, rtol=trace_tol, atol=1e-9 * trr[0])
    xs = np.maximum(np.abs(xr), 1e-3)
    assert np.max(np.abs(out.x - xr) / xs) <= x_tol, (out.x, xr)
    assert abs(g["error_final"] - rr.error_final) <= REL * rr.error_final + 1e-9 * trr[0]
    return out, (xr, rr)


@pytest.mark.parametrize("name", sorted(S.KNOWN_ANSWERS))
@pytest.mark.parametrize("solver_type", [abi.SOLVER_TYPE_CMINPACK_LMDER,
                                         abi.SOLVER_TYPE_CMINPACK_LMDIF])
@pytest.mark.parametrize("mode", [abi.SCENE_GRAPH_MODE_MAYA_DAG,
                                  abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH])
def test_known_scenes(name, solver_type, mode, oracle, gpu_ctx):
    prob = S.known_scene(name)
    opt = S.known_options(name, solver_type, mode)
    out, _ = check_solve(prob, opt, oracle, gpu_ctx)
    expected, tol = S.KNOWN_ANSWERS[name]
    ext = prob.external_params(out.x)
    if S.known_answer_applies(name, solver_type):
        assert np.all(np.abs(ext - np.array(expected)) <= tol), (ext, expected)


@pytest.mark.parametrize("mode", [abi.SCENE_GRAPH_MODE_MAYA_DAG,
                                  abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH])
def test_measure_and_jacobian_small(mode, oracle, gpu_ctx):
    prob = S.make_config(3, frames=8, scale=0.001)
    opt = S.config_options(prob, scene_graph_mode=mode)
    f_ref, eu_ref, ed_ref, st_ref = oracle.measure(prob, opt)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        f, eu, ed, st = s.measure()
        np.testing.assert_allclose(f, f_ref, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(ed, ed_ref, rtol=1e-12, atol=1e-12)
        f2, _, _, _ = s.measure(prob.x0)
        f2_ref, _, _, _ = oracle.measure(prob, opt, prob.x0)
        np.testing.assert_allclose(f2, f2_ref, rtol=1e-12, atol=1e-12)
        J = s.jacobian(prob.x0)
        _, J_ref = oracle.jacobian(prob, opt, prob.x0)
        scale = np.max(np.abs(J_ref))
        assert np.max(np.abs(J - J_ref)) <= 1e-7 * scale
        assert np.array_equal(J != 0, J_ref != 0) or np.max(np.abs(J[J_ref == 0])) < 1e-9 * scale
    finally:
        s.close()


@pytest.mark.parametrize("lens_model", ["classic", "classic_animated", "radial",
                                        "anamorphic", "anamorphic_rescaled"])
def test_measure_and_jacobian_lens(lens_model, oracle, gpu_ctx):
    """Residuals (1e-12) and FD Jacobian (1e-7 of its max entry) through each
    lens model, lens coefficients solved (SURVEY 8(f) row 2 for "radial")."""
    prob = S.make_config(4, frames=8, scale=0.05, lens_model=lens_model)
    opt = S.config_options(prob)
    f_ref, eu_ref, ed_ref, _ = oracle.measure(prob, opt)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        f, eu, ed, _ = s.measure()
        np.testing.assert_allclose(f, f_ref, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(ed, ed_ref, rtol=1e-12, atol=1e-12)
        x1 = prob.x0 + 0.01
        f1, _, _, _ = s.measure(x1)
        f1_ref, _, _, _ = oracle.measure(prob, opt, x1)
        np.testing.assert_allclose(f1, f1_ref, rtol=1e-12, atol=1e-12)
        J = s.jacobian(x1)
        _, J_ref = oracle.jacobian(prob, opt, x1)
        scale = np.max(np.abs(J_ref))
        assert np.max(np.abs(J - J_ref)) <= 1e-7 * scale
    finally:
        s.close()


SMALL_CONFIGS = [
    (0, dict()),                              # C1 full (lmdif, 90 params)
    (1, dict(frames=12, scale=0.05)),         # C2 subset (pose + focal per frame)
    (2, dict(frames=8, scale=0.002)),         # C3 subset (10 cams, Schur)
    (3, dict(frames=8, scale=0.001)),         # C4 subset (Schur BA)
    (4, dict(frames=8, scale=0.05)),          # C5 subset (3DE classic lens)
    (4, dict(frames=8, scale=0.05, lens_model="radial")),  # C5 subset, 3DE radial std deg 4
    (4, dict(frames=24, scale=0.2, lens_model="radial")),
    (4, dict(frames=8, scale=0.05, lens_model="anamorphic")),  # 3DE anamorphic std deg 4
    (4, dict(frames=24, scale=0.2, lens_model="anamorphic_rescaled")),
    (4, dict(frames=8, scale=0.05, lens_model="classic_animated")),  # animated lens attr
    (4, dict(frames=8, scale=0.05, lens_model="layered")),  # classic over a radial input (ABI 5)
    (4, dict(frames=24, scale=0.2, lens_model="layered")),
]


@pytest.mark.parametrize("idx,kw", SMALL_CONFIGS)
def test_config_parity(idx, kw, oracle, gpu_ctx):
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    check_solve(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("dense", [0, 1])
def test_reduced_system_dense_and_tiled(dense, oracle, gpu_ctx, paths):
    """The C3 structure (bundles tracked by several cameras across the whole
    shot: an almost dense reduced system) through both reduced-system solvers:
    the tiled Cholesky and the dense blocked Cholesky (fp64 MFMA GEMM / SYRK
    trailing updates, two-wave panel kernel), each against the oracle."""
    paths(abi.PATH_DENSE, dense)
    prob = S.make_config(2, frames=8, scale=0.002)
    opt = S.config_options(prob)
    check_solve(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("idx,kw,dense", [(2, dict(frames=8, scale=0.002), 1),
                                         (2, dict(frames=8, scale=0.002), 0),
                                         (3, dict(frames=8, scale=0.001), -1)])
def test_schur_dest_lane_bit_identical(idx, kw, dense, oracle, gpu_ctx, paths):
    """The lane-per-destination Schur pass (k_schur_dest_lane: off-diagonal
    destinations of at most 32 pairs, C3's common case) forms every entry of
    S with the sums of the wave-per-destination pass in the same order: the
    solve is bit-identical with the pass pinned on and off, and matches the
    oracle.  (Full-size C3 takes it by default: 9.3M destinations.)"""
    paths(abi.PATH_DENSE, dense)
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    runs = []
    for lane in (0, 1):
        paths(abi.PATH_DEST_LANE, lane)
        s = Solver(prob, opt, context=gpu_ctx)
        try:
            runs.append(s.solve())
        finally:
            s.close()
    np.testing.assert_array_equal(runs[1].x, runs[0].x)
    np.testing.assert_array_equal(runs[1].fnorm_trace, runs[0].fnorm_trace)
    check_solve(prob, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("mode", [abi.SCENE_GRAPH_MODE_MAYA_DAG,
                                  abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH])
@pytest.mark.parametrize("idx,kw", [(3, dict(frames=8, scale=0.001)),
                                    (4, dict(frames=8, scale=0.05)),
                                    (4, dict(frames=8, scale=0.05, lens_model="radial")),
                                    (4, dict(frames=8, scale=0.05,
                                             lens_model="anamorphic_rescaled"))])
def test_reproject_matches_oracle(idx, kw, mode, oracle, gpu_ctx):
    """mmba_plan_reproject (the FlatScene::evaluate point /
    marker lists): reprojected point and corrected marker per observation,
    1e-12, at x0 and at a moved x."""
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob, scene_graph_mode=mode)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        for x in (None, prob.x0 + 0.002):
            pts, mkr = s.reproject(x)
            pr, mr = oracle.reproject_obs(prob, opt, x)
            np.testing.assert_allclose(pts, pr, rtol=1e-12, atol=1e-14)
            np.testing.assert_allclose(mkr, mr, rtol=1e-15, atol=0)
    finally:
        s.close()


def test_layered_lens_measure_jacobian_and_input_attr(oracle, gpu_ctx):
    """Layered lens nodes (mmba.h ABI 5): the measurement and Jacobian of the
    C5 subset with its classic lens over a static radial input layer, then the
    same scene with an input layer's attribute solved -- the reference's
    column is zero there (the input chain is never re-pointed at the solved
    clones, maya_lens_model_utils.cpp:715) -- through the whole solve."""
    prob = S.make_config(4, frames=8, scale=0.05, lens_model="layered")
    opt = S.config_options(prob)
    x1 = prob.x0.copy()
    x1[0], x1[1] = 0.04, 0.008
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        fv, *_ = s.measure(x1)
        fr, *_ = oracle.measure(prob, opt, x1)
        assert np.max(np.abs(fv - fr)) <= 1e-9 * max(1.0, np.max(np.abs(fr)))
        J = s.jacobian(x1)
        _, J_ref = oracle.jacobian(prob, opt, x1)
        assert np.max(np.abs(J - J_ref)) <= 1e-7 * np.max(np.abs(J_ref))
    finally:
        s.close()
    # solve the input layer's degree-2 distortion too (a static attribute)
    a = int(prob.lens_attrs[14 + 0])
    d = prob.to_npz_dict()
    v = float(prob.attr_values[prob.attr_offset[a]])
    for name, val in (("param_attr", a), ("param_frame", -1), ("param_min", -FLOAT_MAX),
                      ("param_max", FLOAT_MAX), ("param_offset", 0.0),
                      ("param_scale", 1.0), ("x0", v)):
        d[name] = np.append(d[name], val)
    p2 = type(prob).from_npz_dict(d)
    p2.meta = dict(prob.meta)
    # attrList (ABI 7): the solved attributes in flag order, then
    # unsolved entries, the input layer's attribute at index 16 -- its static
    # writes (attrIndex + j, j < 8) land on entry 2, a camera attribute, whose
    # lens list entries are null.  (Appended right after the others, index 14,
    # they would land on the classic lens's entry 1 and write a radial slot
    # into a classic model: undefined in the reference, refused.)
    order = []
    for q in range(p2.num_params - 1):
        if int(p2.param_attr[q]) not in order:
            order.append(int(p2.param_attr[q]))
    la = np.asarray(p2.lens_attrs).reshape(-1, 14)
    lens_of = {int(la[l, k]): l for l in range(la.shape[0]) for k in range(14) if la[l, k] >= 0}
    p2.param_ref_attr = np.array([order.index(int(p2.param_attr[q]))
                                  for q in range(p2.num_params - 1)] + [16], np.int32)
    ref_lens = [lens_of.get(a, -1) for a in order] + [-1] * (24 - len(order))
    ref_lens[16] = lens_of[a]
    p2.ref_attr_lens = np.array(ref_lens, np.int32)
    _, J2 = oracle.jacobian(p2, opt, p2.x0)
    assert not np.any(J2[:, -1])
    check_solve(p2, opt, oracle, gpu_ctx)


@pytest.mark.parametrize("solver_type", [abi.SOLVER_TYPE_CMINPACK_LMDER, abi.SOLVER_TYPE_CMINPACK_LMDIF])
def test_k2_records_and_backsub_forms_bit_identical(solver_type, gpu_ctx, paths):
    """Round 6 forms of the C4 iteration, pinned on and off: the bundle pass
    re-evaluating each observation's bundle columns instead of reading the
    records the fused Jacobian pass stores (MMBA_PATH_JB_RECOMPUTE, jac_obs_u's
    arithmetic) and the trial back substitution forming W_i^T x itself
    (MMBA_PATH_BACKSUB_ONEPASS, k_obs_wtx's sums) give the same bits, and so
    does k_schur_obs enqueued ahead of the host's decision or after it
    (MMBA_PATH_PRE_SCHUR): x, the ||f|| trace and fvec identical.  300 frames: the
    fused Jacobian + camera-frame pass (>= 256 camera-frames) is taken."""
    prob = S.make_config(3, frames=300, scale=0.06)
    # lmdif's maxfev counts the n FD evaluations of a Jacobian too
    its = 12 if solver_type == abi.SOLVER_TYPE_CMINPACK_LMDER else 2 * prob.num_params + 6
    opt = S.config_options(prob, solver_type=solver_type, iterations=its)
    runs = {}
    for jb, one, pre in ((0, 0, 1), (0, 1, 1), (1, 0, 1), (1, 1, 1), (0, 0, 0)):
        # pre: the next damped solve's k_schur_obs enqueued with the gated
        # Jacobian (MMBA_PATH_PRE_SCHUR = 1) or after the decision (default)
        paths(abi.PATH_JB_RECOMPUTE, jb)
        paths(abi.PATH_BACKSUB_ONEPASS, one)
        paths(abi.PATH_PRE_SCHUR, pre)
        s = Solver(prob, opt, context=gpu_ctx)
        try:
            runs[(jb, one, pre)] = s.solve()
        finally:
            s.close()
    ref = runs[(0, 0, 1)]
    assert ref.result["iterations"] > 2
    for k, r in runs.items():
        np.testing.assert_array_equal(r.x, ref.x, err_msg=str(k))
        np.testing.assert_array_equal(r.fnorm_trace, ref.fnorm_trace, err_msg=str(k))
        np.testing.assert_array_equal(r.fvec, ref.fvec, err_msg=str(k))
