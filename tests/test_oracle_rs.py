"""Rolling shutter in the CPU oracle (mmba.h ABI 3; BASELINE configs[4]).

The reference solver has no rolling-shutter model; its only rolling-shutter
arithmetic is the 3DE exporter's 2D correction
(share/3dequalizer/python/uvtrack_format.py:186-203, 243-330), whose blend the
oracle applies to the camera pose.  These tests pin the oracle's arithmetic
against an independent numpy restatement of that blend and check the
structural consequences (parity against the reference itself is unpinned:
there is no reference counterpart)."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S


def scene(rs=0.5, frames=6):
    return S.make_config(4, frames=frames, scale=0.02, rolling_shutter=rs)


def test_rs_zero_is_the_global_shutter(oracle):
    p = scene()
    o = S.config_options(p)
    f_rs = oracle.measure(p, o)[0]
    p.cam_rs_value = np.zeros(p.num_cameras)
    f0 = oracle.measure(p, o)[0]
    p.cam_rs_value = None
    f1 = oracle.measure(p, o)[0]
    np.testing.assert_array_equal(f0, f1)
    assert np.max(np.abs(f_rs - f0)) > 0.0


def test_rs_blend_matches_exporter_formula():
    """synthetic.rs_blend (numpy) against a literal restatement of
    _apply_rs_correction with the exporter's end extrapolation."""
    rng = np.random.default_rng(3)
    v = rng.standard_normal(7)
    tau = rng.uniform(-0.5, 0.5, 7)
    got = S.rs_blend(v, tau)
    for f in range(7):
        cur = v[f]
        prev = v[f - 1] if f > 0 else None
        nxt = v[f + 1] if f < 6 else None
        if f == 0:
            prev = cur + (cur - nxt)
        if f == 6:
            nxt = cur + (cur - prev)
        b = (nxt - prev) / 2.0
        c = -cur + (nxt + prev) / 2.0
        assert got[f] == (cur + tau[f] * b) + (tau[f] * tau[f]) * c


def test_rs_reprojection_matches_numpy(oracle):
    """The oracle's reprojected point of every observation against the numpy
    model the synthetic markers come from (pinhole + the same pose blend,
    before the lens): 1e-10 in film units."""
    p = scene()
    p.lens_type[:] = 0  # no lens: compare the pinhole point directly
    o = S.config_options(p)
    pts, mkr = oracle.reproject_obs(p, o)
    F = p.num_frames
    ta = p.tfm_attrs.reshape(-1, 9)
    for c in range(p.num_cameras):
        t = p.cam_tfm[c]
        vals = []
        for k in range(6):
            a = ta[t, k]
            off = p.attr_offset[a]
            vals.append(p.attr_values[off:off + F] if p.attr_animated[a]
                        else np.full(F, p.attr_values[off]))
        tr = np.stack(vals[:3], 1)
        rr = np.stack(vals[3:], 1)
        sel = np.nonzero(p.mkr_cam[p.obs_marker] == c)[0]
        fs = p.obs_frame[sel]
        bpos = []
        for i in sel:
            bt = p.bnd_tfm[p.mkr_bnd[p.obs_marker[i]]]
            bpos.append([p.attr_values[p.attr_offset[ta[bt, k]]] for k in range(3)])
        tau = p.cam_rs_value[c] * (0.5 - p.obs_xy[2 * sel + 1])
        tb = np.stack([S._blend_at(tr[:, k], fs, tau) for k in range(3)], 1)
        rb = np.stack([S._blend_at(rr[:, k], fs, tau) for k in range(3)], 1)
        R = S._euler_xyz(rb[:, 0], rb[:, 1], rb[:, 2])
        pc = np.einsum("nij,ni->nj", R, np.array(bpos) - tb)
        mx = S.FOCAL_MM * pc[:, 0] / (S.FILM_W_MM * -pc[:, 2])
        my = S.FOCAL_MM * pc[:, 1] / (S.FILM_H_MM * -pc[:, 2])
        ra = S.RENDER[0] / S.RENDER[1]
        fa = S.FILM_W_MM / S.FILM_H_MM
        np.testing.assert_allclose(pts[2 * sel], mx, rtol=0, atol=1e-10)
        np.testing.assert_allclose(pts[2 * sel + 1], my * (ra / fa), rtol=0, atol=1e-10)


def test_rs_fd_column_reaches_neighbour_frames(oracle):
    """With a rolling shutter the FD column of a camera parameter at frame f
    re-measures frames f-1..f+1 (the blend's support): its non-zero rows are
    exactly the observations of that camera in those frames."""
    p = scene(frames=6)
    o = S.config_options(p)
    fvec, J = oracle.jacobian(p, o, p.x0)
    obs_frame = np.repeat(p.obs_frame, 2)
    obs_cam = np.repeat(p.mkr_cam[p.obs_marker], 2)
    for q in range(p.num_params):
        f = int(p.param_frame[q])
        if f < 0:
            continue
        c = int(np.argmax([p.param_attr[q] in p.tfm_attrs.reshape(-1, 9)[t, :6]
                           for t in p.cam_tfm]))
        rows = np.nonzero(J[:2 * p.num_obs, q])[0]
        assert rows.size > 0
        assert np.all(np.abs(obs_frame[rows] - f) <= 1)
        assert np.all(obs_cam[rows] == c)
        # and it does reach a neighbouring frame (where that camera has rows)
        nb = (np.abs(obs_frame - f) == 1) & (obs_cam == c)
        if nb.any():
            assert np.any(np.abs(obs_frame[rows] - f) == 1)


@pytest.mark.parametrize("rs", [0.5, -0.8])
def test_rs_scene_solves(rs, oracle):
    """The oracle's lmder on a rolling-shutter C5 window converges (reason 1-3)
    to a fit at the synthetic noise level."""
    p = S.make_config(4, frames=8, scale=0.05, rolling_shutter=rs)
    o = S.config_options(p)
    x, f, eu, ed, res, tr = oracle.solve(p, o)
    assert res.reason_number in (1, 2, 3), res.as_dict()
    assert res.error_rms < 1.0


# ---------------------------------------------------------------------------
# The forward model against the exporter's removal (VERDICT r3 "next" 2).
# ---------------------------------------------------------------------------
def exporter_remove_rs(xy, f, F, rs, cam_t, cam_R, focal, fbw, fbh, depth, sign=-1.0):
    """numpy restatement of the 3DE exporter's _remove_rs_from_2d_point
    (share/3dequalizer/python/uvtrack_format.py:243-333, with
    _convert_2d_to_3d_point_undistort :206-240 and _apply_rs_correction
    :186-203).  The tde4 calls are replaced by the synthetic camera: frame
    f (0-based here, 1-based in 3DE) has world position cam_t[f] and
    camera-to-world rotation cam_R[f] (getPGroupPosition3D / Rotation3D),
    the FOV is the whole image (0, 1, 0, 1), the lens centre offset is 0 and
    there is no lens (removeDistortion2D / applyDistortion2D are the
    identity).  xy: the 2D point in 3DE units (0..1, +y up); depth: the
    content distance; sign = -1 is the exporter's (+1: the negative control
    of the test below).  Returns the corrected 2D point (3DE units)."""
    xy = np.asarray(xy, dtype=np.float64)

    def to_3d(fr):  # :229-240
        p2d_cm = np.array([(xy[0] - 0.5) * fbw, (xy[1] - 0.5) * fbh])
        v = np.array([p2d_cm[0], p2d_cm[1], -focal])
        return cam_R[fr] @ (v / np.linalg.norm(v)) * depth + cam_t[fr]

    if F == 1:
        return xy
    prev_pos = to_3d(f - 1) if f > 0 else np.zeros(3)        # frame > 1
    next_pos = to_3d(f + 1) if f < F - 1 else np.zeros(3)    # frame < num_frames
    curr_pos = to_3d(f)
    if f == 0:
        prev_pos = curr_pos + (curr_pos - next_pos)
    if f == F - 1:
        next_pos = curr_pos + (curr_pos - prev_pos)
    t = rs * (1.0 - xy[1])
    dt = sign * t  # _apply_rs_correction(-t, prev, curr, next)
    b = (next_pos - prev_pos) / 2.0
    c = -curr_pos + (next_pos + prev_pos) / 2.0
    curr_pos = curr_pos + dt * b + dt * dt * c
    d = cam_R[f].T @ (curr_pos - cam_t[f])  # back-projection, :320-325
    p = np.array([d[0] * focal / (-d[2] * fbw) + 0.5, d[1] * focal / (-d[2] * fbh) + 0.5])
    return xy + (xy - p)


def _rs_rig(rs, F=7, seed=5):
    """One animated camera (smooth translate + rotate), no lens, render
    aspect = film aspect (film fit is the identity), bundles 8-40 units in
    front of it; markers are made RS-consistent below."""
    from mayamatchmovesolver_amd.problem import SceneBuilder
    rng = np.random.default_rng(seed)
    fr = np.arange(F, dtype=np.float64)
    t = np.stack([0.4 * fr + 0.03 * fr ** 2, 0.1 - 0.05 * fr, 0.2 * fr], 1)
    r = np.stack([1.0 + 1.5 * fr, -3.0 + 2.0 * fr - 0.1 * fr ** 2, 0.5 * fr], 1)
    b = SceneBuilder(F)
    tfm, _ = b.transform(t=tuple(t[:, k] for k in range(3)), r=tuple(r[:, k] for k in range(3)))
    cam, _ = b.camera(tfm, focal=S.FOCAL_MM, film_back=(S.FILM_W_IN, S.FILM_H_IN),
                      render_size=(1800, 1200))
    pts = []
    for j in range(12):
        z = -rng.uniform(8.0, 40.0)
        X = np.array([rng.uniform(-0.3, 0.3) * -z + 1.0, rng.uniform(-0.2, 0.2) * -z, z])
        bt, ids = b.transform(t=tuple(X))
        b.bundle(bt)
        b.marker(cam, j, np.zeros((F, 2)))
        pts.append(X)
    b.solve(ids[0])  # any parameter (the reprojection entry needs a problem)
    p = b.build()
    p.cam_rs_value = np.array([rs])
    return p, np.array(pts), t, S._euler_xyz(r[:, 0], r[:, 1], r[:, 2])


def _rs_consistent_markers(p, oracle):
    """Markers that the forward model reproduces exactly: y enters the
    scanline time, so iterate marker <- reprojection(marker) to the fixed
    point (rs |dy/dtau| << 1: a contraction)."""
    o = S.config_options(p)
    for _ in range(60):
        pts, _m = oracle.reproject_obs(p, o)
        if np.max(np.abs(pts - p.obs_xy)) < 1e-15:
            break
        p.obs_xy = pts.copy()
    pts, _m = oracle.reproject_obs(p, o)
    assert np.max(np.abs(pts - p.obs_xy)) < 1e-14
    return p.obs_xy.copy()


@pytest.mark.parametrize("rs", [0.3, -0.4])
def test_rs_forward_model_inverts_the_exporter(rs, oracle):
    """The library's rolling-shutter forward model is the inverse of the 3DE
    exporter's removal: markers the oracle's model reproduces exactly, run
    through the exporter's _remove_rs_from_2d_point (content distance = the
    bundle's distance from the camera at the frame), return the
    global-shutter projection to second order in the scanline time.  Both
    sides: an observation at scanline y (film units, +y up; 3DE y' = y + 0.5)
    was captured at time f + tau, tau = rs (1 - y') = rs (0.5 - y); the
    exporter blends back by -tau.  With the opposite sign the first-order
    terms would add instead of cancel."""
    errs, shifts, wrong = [], [], []
    for scale in (1.0, 0.5):
        p, X, cam_t, cam_R = _rs_rig(rs * scale)
        m = _rs_consistent_markers(p, oracle)
        o = S.config_options(p)
        p_gs = _rs_rig(0.0)[0]
        p_gs.obs_xy = m.copy()
        gs, _ = oracle.reproject_obs(p_gs, o)  # rs = 0: the global shutter
        F = p.num_frames
        fb_w, fb_h = S.FILM_W_MM, S.FILM_H_MM
        e = s = w = 0.0
        for i in range(p.num_obs):
            f = int(p.obs_frame[i])
            j = int(p.mkr_bnd[p.obs_marker[i]])
            depth = float(np.linalg.norm(X[j] - cam_t[f]))
            xy3de = m[2 * i:2 * i + 2] + 0.5
            cor = exporter_remove_rs(xy3de, f, F, rs * scale, cam_t, cam_R, S.FOCAL_MM,
                                     fb_w, fb_h, depth) - 0.5
            e = max(e, float(np.max(np.abs(cor - gs[2 * i:2 * i + 2]))))
            bad = exporter_remove_rs(xy3de, f, F, rs * scale, cam_t, cam_R, S.FOCAL_MM,
                                     fb_w, fb_h, depth, sign=1.0) - 0.5
            w = max(w, float(np.max(np.abs(bad - gs[2 * i:2 * i + 2]))))
            s = max(s, float(np.max(np.abs(m[2 * i:2 * i + 2] - gs[2 * i:2 * i + 2]))))
        errs.append(e)
        shifts.append(s)
        wrong.append(w)
    # the rolling shutter moves the markers by O(tau) ...
    assert shifts[0] > 5e-3 and 1.7 < shifts[0] / shifts[1] < 2.3
    # ... and the exporter removes that to O(tau^2): the residual error is a
    # small fraction of the shift and quarters when tau halves
    assert errs[0] < 0.1 * shifts[0], (errs, shifts)
    assert 3.0 < errs[0] / errs[1] < 5.0, errs
    # negative control: blending forward (the opposite sign convention)
    # doubles the shift instead of removing it
    assert wrong[0] > 1.5 * shifts[0], (wrong, shifts)


def test_rs_parented_reprojection_matches_numpy(oracle):
    """A camera under a (static, rotated and translated) group: the blend
    moves the camera's own translate / rotate values and the world pose is the
    group's world matrix times the blended local one (oracle
    rs_camera_world) -- the oracle's reprojected points against that numpy
    model, 1e-10 in film units."""
    p = S.edge_scene(parented=True, solve_bundles=False)
    p.cam_rs_value = np.array([0.6])
    o = S.config_options(p)
    pts, _ = oracle.reproject_obs(p, o)
    F = p.num_frames
    ta = p.tfm_attrs.reshape(-1, 9)
    t = p.cam_tfm[0]
    par = p.tfm_parent[t]
    assert par >= 0

    def vals(tf, k):
        a = ta[tf, k]
        off = p.attr_offset[a]
        return p.attr_values[off:off + F] if p.attr_animated[a] else np.full(F, p.attr_values[off])

    tr = np.stack([vals(t, k) for k in range(3)], 1)
    rr = np.stack([vals(t, k) for k in range(3, 6)], 1)
    tp = np.array([vals(par, k)[0] for k in range(3)])
    Rp = S._euler_xyz(*[vals(par, k)[0] for k in range(3, 6)])
    fs = p.obs_frame
    tau = p.cam_rs_value[0] * (0.5 - p.obs_xy[1::2])
    tb = np.stack([S._blend_at(tr[:, k], fs, tau) for k in range(3)], 1)
    rb = np.stack([S._blend_at(rr[:, k], fs, tau) for k in range(3)], 1)
    Rw = Rp[None] @ S._euler_xyz(rb[:, 0], rb[:, 1], rb[:, 2])
    tw = tb @ Rp.T + tp
    bpos = np.array([[p.attr_values[p.attr_offset[ta[p.bnd_tfm[p.mkr_bnd[k]], j]]] for j in range(3)]
                     for k in p.obs_marker])
    pc = np.einsum("nji,nj->ni", Rw, bpos - tw)
    mx = S.FOCAL_MM * pc[:, 0] / (S.FILM_W_MM * -pc[:, 2])
    my = S.FOCAL_MM * pc[:, 1] / (S.FILM_H_MM * -pc[:, 2])
    ra = S.EDGE_RENDERS["narrow"][0] / S.EDGE_RENDERS["narrow"][1]
    fa = S.FILM_W_MM / S.FILM_H_MM
    np.testing.assert_allclose(pts[0::2], mx, rtol=0, atol=1e-10)
    np.testing.assert_allclose(pts[1::2], my * (ra / fa), rtol=0, atol=1e-10)
    # and the blend matters
    p.cam_rs_value = np.array([0.0])
    pts0, _ = oracle.reproject_obs(p, o)
    assert np.max(np.abs(pts0 - pts)) > 1e-6
