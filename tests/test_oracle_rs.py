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
