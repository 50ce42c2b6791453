"""Synthetic scenes.

Two families:

1. ``known_scene(name)`` -- the reference's Maya solver tests rebuilt without
   Maya (tests/test/test_solver/*.py).  They carry the published known answers
   (SURVEY.md section 4).
2. ``make_config(i)`` -- the five BASELINE.json configurations as concrete
   synthetic inputs: numpy PCG64 seeded with
   ``20241008 + i``, 35 mm lens on a 36 x 24 mm back, Horizontal film fit,
   2048 x 1556 render, zero film offsets, markers = true projection +
   N(0, 0.5 px) noise, initial guesses = truth + perturbation, gauge locked
   (camera-0 pose at frame 0 and bundle 0) when cameras and bundles are both
   solved.

Everything here is host-side input generation (the role Maya + the Python
caller play for the reference); it contains no solver arithmetic.
"""
from __future__ import annotations

import math

import numpy as np

from . import abi
from .problem import AttrRef, FLOAT_MAX, Problem, SceneBuilder, param_external_to_internal

FOCAL_MM = 35.0
FILM_W_MM = 36.0
FILM_H_MM = 24.0
FILM_W_IN = FILM_W_MM / 25.4
FILM_H_IN = FILM_H_MM / 25.4
RENDER = (2048, 1556)
IMAGE_WIDTH = 2048.0

# ---------------------------------------------------------------------------
# Reference known-answer scenes (tests/test/test_solver).
# ---------------------------------------------------------------------------
KNOWN_ANSWERS = {
    # name: (expected external values of the solved attrs, tolerance)
    "test1": ([-6.0, 3.6], 1e-4),                       # test1.py:116-121
    "test3": ([7.44014, -32.3891], 1e-3),               # test3.py:117-118
    "minmax_both": ([-5.0, 2.3], 1e-4),                 # test_min_max_values.py:43-99
    "minmax_lower": ([-5.0, 2.3], 1e-4),                # :101-160
    "minmax_upper": ([-6.0, 2.3], 1e-4),                # :163-220
    "weight_high": ([-2.2252424, 1.65], 1e-4),          # test_marker_weight.py:86-146
    "weight_low": ([-2.2252424, 1.65], 1e-4),           # :148-206
    "weight_ratio": ([-0.333333333333, 1.3], 1e-4),     # :208-274
    "weight_same": ([-1.00000134, 1.65000055], 1e-4),   # :276-336
    "weight_zero": ([-2.25, 1.65], 1e-3),               # :338-398
    "test12_single": ([-6.0, 3.6], 1e-4),               # test12.py (driven bundle)
    # test_marker_enabled.py:43-111 (marker_02 disabled)
    "enabled_single": ([-2.24999755, 1.65000644], 1e-4),
    # test_marker_enabled.py:113-237, solved frame by frame (frames 1, 5, 10 of
    # the keyed scene; marker_02 disabled on frames 5-9 by a stepped key)
    "enabled_multi_f1": ([-0.51855463, 1.30993172], 1e-3),
    "enabled_multi_f5": ([-2.266493967, 1.631927621], 1e-3),
    "enabled_multi_f10": ([-1.48144697, 2.10503952], 1e-3),
    # test_issue54.py:113-235: nodal camera, rotate x/y solved with a +360
    # attribute offset, 10 iterations
    "issue54_zero": ([-2.85, -2.86], 1e-1),
    "issue54_twenty": ([0.0, 0.0], 1e-2),
    "issue54_threesixty": ([360.0, 360.0], 1e-2),
}


def known_options(name, solver_type=abi.SOLVER_TYPE_CMINPACK_LMDER,
                  scene_graph_mode=abi.SCENE_GRAPH_MODE_MAYA_DAG, **overrides):
    """The mmSolver flags each known-answer test runs with (iterations 1000 for
    test1, 10 for issue54, else the default 100; delta 1e-5 for test3)."""
    from .options import make_options
    iters = {"test1": 1000}.get(name, 10 if name.startswith("issue54_") else 100)
    kw = dict(solver_type=solver_type, scene_graph_mode=scene_graph_mode, iterations=iters,
              delta=1e-5 if name == "test3" else 1e-4)
    kw.update(overrides)
    return make_options(**kw)


def known_answer_applies(name, solver_type):
    """The per-frame marker-enabled test runs the default solver (lmder,
    SOLVER_TYPE_DEFAULT_VALUE); its answers pin lmder only."""
    return not (name.startswith("enabled_multi") and
                solver_type != abi.SOLVER_TYPE_CMINPACK_LMDER)


def _hermite_flat(a, b, s):
    """A two-key Maya animation curve with flat (auto-clamped) end tangents
    at parameter s in [0, 1]."""
    return a + (b - a) * (3.0 * s * s - 2.0 * s * s * s)


def _camera(b: SceneBuilder, t, r=(0.0, 0.0, 0.0)):
    tfm, tids = b.transform(t=t, r=r)
    cam, cids = b.camera(tfm, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN),
                         film_fit=abi.FILM_FIT_HORIZONTAL, render_size=RENDER)
    return cam, tids, cids


def known_scene(name: str) -> Problem:
    """Rebuild one of the reference's Maya test scenes as a flat problem."""
    b = SceneBuilder(1)
    if name in ("test1", "test3", "test12_single"):
        cam, ctids, _ = _camera(b, (-1.0, 1.0, -5.0))
        if name == "test12_single":
            # tfm_a drives tfm_b drives the bundle: one shared attribute block.
            ta, aids = b.transform(t=(-5.5, 6.4, -25.0))
            btfm, _ = b.transform(t=tuple(AttrRef(a) for a in aids[:3]))
            solve_ids = aids[:2]
        else:
            btfm, bids = b.transform(t=(5.5, 6.4, -25.0))
            solve_ids = bids[:2] if name == "test1" else ctids[3:5]
        bnd = b.bundle(btfm)
        b.marker(cam, bnd, [[-0.243056042, 0.189583713]])
        for a in solve_ids:
            b.solve(a)
        return b.build(meta={"name": name})
    if name.startswith("minmax"):
        cam, _, _ = _camera(b, (-1.0, 1.0, 10.0))
        btfm, bids = b.transform()
        bnd = b.bundle(btfm)
        b.marker(cam, bnd, [[-0.486112083, 0.189583713]])
        lo, hi = {"minmax_both": (-5.0, 5.0), "minmax_lower": (-5.0, None),
                  "minmax_upper": (None, 5.0)}[name]
        b.solve(bids[0], xmin=lo, xmax=hi)
        b.solve(bids[1])
        return b.build(meta={"name": name})
    if name.startswith("weight"):
        w1, w2 = {"weight_high": (100.0, 1.0), "weight_low": (1.0, 0.01),
                  "weight_ratio": (100.0, 50.0), "weight_same": (0.5, 0.5),
                  "weight_zero": (1.0, 0.0)}[name]
        ratio = name == "weight_ratio"  # test_marker_weight.py:227-232
        cam, _, _ = _camera(b, (0.0, 0.0, 0.0) if ratio else (-1.0, 1.0, -5.0))
        mx = 0.097222417 if ratio else 0.243056042
        grp, gids = b.transform(t=(0.0, 0.0, -10.0))
        b1t, _ = b.transform(parent=grp)
        b2t, _ = b.transform(parent=grp)
        bnd1, bnd2 = b.bundle(b1t), b.bundle(b2t)
        b.marker(cam, bnd1, [[-mx, 0.189583713]], weight=w1)
        b.marker(cam, bnd2, [[mx, 0.189583713]], weight=w2)
        b.solve(gids[0])
        b.solve(gids[1])
        return b.build(meta={"name": name})
    if name == "enabled_single":
        cam, _, _ = _camera(b, (-1.0, 1.0, -5.0))
        grp, gids = b.transform(t=(0.0, 0.0, -10.0))
        b1t, _ = b.transform(parent=grp)
        b2t, _ = b.transform(parent=grp)
        bnd1, bnd2 = b.bundle(b1t), b.bundle(b2t)
        b.marker(cam, bnd1, [[-0.243056042, 0.189583713]])
        b.marker(cam, bnd2, [[0.243056042, 0.189583713]], enable=[False])
        b.solve(gids[0])
        b.solve(gids[1])
        return b.build(meta={"name": name})
    if name.startswith("enabled_multi_f"):
        # keys at frames 1 and 10; frame f of the curve (flat tangents)
        f = int(name[len("enabled_multi_f"):])
        sfr = (f - 1) / 9.0
        rx = _hermite_flat(-5.0, 5.0, sfr)
        ry = _hermite_flat(-5.5, 5.5, sfr)
        m1 = (_hermite_flat(-0.243056042, -0.29166725, sfr),
              _hermite_flat(0.218750438, 0.189583713, sfr))
        m2 = (_hermite_flat(0.243056042, 0.29166725, sfr),
              _hermite_flat(0.218750438, 0.189583713, sfr))
        en2 = not (5 <= f < 10)  # enable keys 1 / 0 / 1 at 1 / 5 / 10, stepped
        cam, _, _ = _camera(b, (-1.0, 1.0, -5.0), r=(rx, ry, 0.0))
        grp, gids = b.transform(t=(np.zeros(1), np.zeros(1), -10.0))
        b1t, _ = b.transform(parent=grp)
        b2t, _ = b.transform(parent=grp)
        bnd1, bnd2 = b.bundle(b1t), b.bundle(b2t)
        b.marker(cam, bnd1, [list(m1)])
        b.marker(cam, bnd2, [list(m2)], enable=[en2])
        b.solve(gids[0])
        b.solve(gids[1])
        return b.build(meta={"name": name})
    if name.startswith("issue54_"):
        kind = name[len("issue54_"):]
        cam_t, cam_r = {"zero": ((-2.0, 2.0, -5.0), (0.0, 0.0, 0.0)),
                        "twenty": ((-1.0, 1.0, -5.0), (20.0, 20.0, 20.0)),
                        "threesixty": ((-1.0, 1.0, -5.0), (360.0, 360.0, 360.0))}[kind]
        cam, ctids, _ = _camera(b, cam_t, r=cam_r)
        btfm, _ = b.transform(t=(-1.0, 1.0, -25.0))
        bnd = b.bundle(btfm)
        b.marker(cam, bnd, [[0.0, 0.0]])
        b.solve(ctids[3], offset=360.0)  # (attr, min, max, offset '360', scale)
        b.solve(ctids[4], offset=360.0)
        return b.build(meta={"name": name, "iterations": 10})
    raise KeyError(name)


# ---------------------------------------------------------------------------
# BASELINE.json configurations.
# ---------------------------------------------------------------------------
def _euler_xyz(rx, ry, rz):
    """Column-vector rotation Rz @ Ry @ Rx (degrees), vectorised over frames."""
    rx, ry, rz = (np.radians(np.asarray(v, dtype=np.float64)) for v in (rx, ry, rz))
    cx, sx, cy, sy, cz, sz = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry), np.cos(rz), np.sin(rz)
    R = np.empty(rx.shape + (3, 3))
    R[..., 0, 0] = cz * cy
    R[..., 0, 1] = cz * sy * sx - sz * cx
    R[..., 0, 2] = cz * sy * cx + sz * sx
    R[..., 1, 0] = sz * cy
    R[..., 1, 1] = sz * sy * sx + cz * cx
    R[..., 1, 2] = sz * sy * cx - cz * sx
    R[..., 2, 0] = -sy
    R[..., 2, 1] = cy * sx
    R[..., 2, 2] = cy * cx
    return R


def _project(cam_t, cam_r, focal, pts):
    """True marker coordinates of world points for one camera pose
    (pinhole, Horizontal film fit: x in film-width units, y in film-height units)."""
    R = _euler_xyz(*cam_r)
    pc = (pts - cam_t) @ R  # R^T (p - t)
    depth = -pc[..., 2]
    mx = focal * pc[..., 0] / (FILM_W_MM * depth)
    my = focal * pc[..., 1] / (FILM_H_MM * depth)
    return mx, my, depth


def _lens_distort_truth(c, x, y):
    """Forward model used only to synthesise lens-distorted markers
    (LDPK classic map_inverse of the undistort polynomial, fixed-point)."""
    ld, sq, cx, cy, qu = c
    w, h = 3.6, 2.4
    r = math.sqrt(w * w + h * h) / 2.0
    qx, qy = x * w / r, y * h / r

    def ev(px, py):
        p02, p12 = px * px, py * py
        fx = px * (1 + ld / sq * p02 + (ld + cx) / sq * p12 + qu / sq * p02 * p02
                   + 2 * qu / sq * p02 * p12 + qu / sq * p12 * p12)
        fy = py * (1 + (ld + cy) * p02 + ld * p12 + qu * p02 * p02 + 2 * qu * p02 * p12
                   + qu * p12 * p12)
        return fx, fy

    fx, fy = ev(qx, qy)
    px, py = qx - (fx - qx), qy - (fy - qy)
    for _ in range(40):
        ix, iy = ev(px, py)
        px, py = px + qx - ix, py + qy - iy
    return px * r / w, py * r / h


def _radial_distort_truth(c, x, y):
    """Forward model used only to synthesise markers through a 3DE radial
    decentered deg 4 cylindric lens: cylindric^-1 then the fixed-point inverse
    of the radial decentered polynomial (LDPK radial_decentered_distortion,
    cylindric_extender_2)."""
    c2, u2, v2, c4, u4, v4, phi, bend = c
    w, h = 3.6, 2.4
    r = math.sqrt(w * w + h * h) / 2.0
    q = math.sqrt(1.0 + bend)
    cs, sn = math.cos(math.radians(phi)), math.sin(math.radians(phi))
    m = np.array([[cs * cs * q + sn * sn / q, (q - 1 / q) * cs * sn],
                  [(q - 1 / q) * cs * sn, cs * cs / q + sn * sn * q]])
    mi = np.linalg.inv(m)
    dx, dy = x * w / r, y * h / r
    qx, qy = mi[0, 0] * dx + mi[0, 1] * dy, mi[1, 0] * dx + mi[1, 1] * dy

    def ev(px, py):
        x2, y2, xy = px * px, py * py, px * py
        r2 = x2 + y2
        rad = 1.0 + c2 * r2 + c4 * r2 * r2
        return (px * rad + (r2 + 2 * x2) * (u2 + u4 * r2) + 2 * xy * (v2 + v4 * r2),
                py * rad + (r2 + 2 * y2) * (v2 + v4 * r2) + 2 * xy * (u2 + u4 * r2))

    fx, fy = ev(qx, qy)
    px, py = qx - (fx - qx), qy - (fy - qy)
    for _ in range(40):
        ix, iy = ev(px, py)
        px, py = px + qx - ix, py + qy - iy
    return px * r / w, py * r / h


def _anamorphic_distort_truth(c, x, y):
    """Forward model used only to synthesise markers through a 3DE anamorphic
    deg 4 rotate squeeze xy (rescaled) lens: PAR * fixed-point inverse of the
    anamorphic polynomial at RSP^-1 q (LDPK generic_anamorphic_distortion<4>,
    rotation / squeeze extenders)."""
    cx02, cy02, cx22, cy22, cx04, cy04, cx24, cy24, cx44, cy44, rot, sqx, sqy, rs = c
    w, h = 3.6, 2.4
    r = math.sqrt(w * w + h * h) / 2.0
    ph = math.radians(rot)
    R = np.array([[math.cos(ph), -math.sin(ph)], [math.sin(ph), math.cos(ph)]])
    rsp = R @ np.diag([sqx, 1.0]) @ np.diag([1.0, sqy]) @ np.diag([rs, 1.0])
    par = np.diag([rs, 1.0]) @ R
    ri = np.linalg.inv(rsp)
    dx, dy = x * w / r, y * h / r
    qx, qy = ri[0, 0] * dx + ri[0, 1] * dy, ri[1, 0] * dx + ri[1, 1] * dy
    kx = (cx02 + cx22, cx02 - cx22, cx04 + cx24 + cx44, 2 * cx04 - 6 * cx44, cx04 - cx24 + cx44)
    ky = (cy02 + cy22, cy02 - cy22, cy04 + cy24 + cy44, 2 * cy04 - 6 * cy44, cy04 - cy24 + cy44)

    def ev(px, py):
        x2, y2 = px * px, py * py
        return (px * (1 + x2 * kx[0] + y2 * kx[1] + x2 * x2 * kx[2] + x2 * y2 * kx[3]
                      + y2 * y2 * kx[4]),
                py * (1 + x2 * ky[0] + y2 * ky[1] + x2 * x2 * ky[2] + x2 * y2 * ky[3]
                      + y2 * y2 * ky[4]))

    fx, fy = ev(qx, qy)
    px, py = qx - (fx - qx), qy - (fy - qy)
    for _ in range(40):
        ix, iy = ev(px, py)
        px, py = px + qx - ix, py + qy - iy
    ox, oy = par[0, 0] * px + par[0, 1] * py, par[1, 0] * px + par[1, 1] * py
    return ox * r / w, oy * r / h


CONFIG_NAMES = {
    0: "c1_1cam_20bnd_50mkr_10f_lmdif",
    1: "c2_1cam_1kbnd_5kmkr_120f_pose_focal",
    2: "c3_10cam_10kbnd_50kmkr_500f_schur",
    3: "c4_500pose_50kbnd_200kobs",
    4: "c5_lens3de_2cam_2kmkr_240f",
}


def make_config(index: int, frames: int | None = None, scale: float = 1.0,
                scene_graph_mode=abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH, window: int = 4,
                depth=(20.0, 200.0), lens_model: str = "classic",
                init_noise: float = 1.0, obs_noise: float = 1.0,
                rolling_shutter: float = 0.0, cameras: int = 2) -> Problem:
    """Concrete synthetic input for BASELINE.json ``configs[index]``.

    ``frames`` / ``scale`` shrink a configuration (frame-window subsets and
    fewer markers) for parity tests and the bounded CPU-baseline sample;
    the defaults give the full configuration.  ``window`` (track length in
    frames) and ``depth`` (bundle depth range) apply to configs[3] only: the
    defaults are the C4 spec; longer tracks / nearer bundles give the
    well-conditioned variants the sharded-solve tests compare x on.
    ``init_noise`` (configs[2] / configs[3]) scales the initial-guess
    perturbation of poses and bundles (1.0 = the spec).  ``obs_noise`` (configs[2] / configs[3]) scales
    the 0.5 px marker noise: 0 gives a zero-residual minimum, where x is
    determined to roundoff; with the spec noise the minimum of the C4
    structure lies in a flat valley (far bundles on a 1.5-unit baseline) and
    the lmder stopping point moves along it by ~1e-3 under a 1-ulp change of
    x0 -- in the reference as in any fp64 implementation.
    ``lens_model`` (configs[4] only): "classic" (the C5 spec), "radial" (the
    same scene through a 3DE radial decentered deg 4 cylindric lens, degree-2
    and degree-4 distortion solved), "anamorphic" / "anamorphic_rescaled"
    (3DE anamorphic deg 4 rotate squeeze xy [rescaled], cx02 / cy02 solved),
    "classic_animated" (the classic lens with its distortion animated, one
    parameter per frame):
    SURVEY 8(f) row 2.
    ``rolling_shutter`` (configs[4] only): rs in frames (time shift x fps),
    the configs[4] "rolling-shutter per-scanline pose" (mmba.h ABI 3; 0 = off).
    ``cameras`` (configs[4] only): cameras sharing the lens (the spec's 2; 1
    gives the one-camera shot whose animated lens coefficients each reach one
    camera-frame).
    """
    rng = np.random.Generator(np.random.PCG64(20241008 + index))
    if index == 0:
        return _config_c1(rng, frames or 10)
    if index == 1:
        return _config_c2(rng, frames or 120, scale)
    if index == 2:
        return _config_ba(rng, index, n_cams=10, F=frames or 500, B=int(10000 * scale),
                          K=int(50000 * scale), window=20, per_cam_markers=True,
                          init_noise=init_noise, obs_noise=obs_noise)
    if index == 3:
        return _config_ba(rng, index, n_cams=1, F=frames or 500, B=int(50000 * scale),
                          K=int(50000 * scale), window=window, per_cam_markers=False,
                          depth=depth, init_noise=init_noise, obs_noise=obs_noise)
    if index == 4:
        return _config_c5(rng, frames or 240, scale, lens_model, rolling_shutter, cameras)
    raise KeyError(index)


def _camera_path(rng, F, c):
    f = np.arange(F, dtype=np.float64)
    phase = rng.uniform(0, 2 * math.pi, size=6)
    t = np.stack([2.0 * c + 0.04 * f + 0.3 * np.sin(0.05 * f + phase[0]),
                  1.5 + 0.2 * np.sin(0.03 * f + phase[1]),
                  0.02 * f + 0.2 * np.sin(0.04 * f + phase[2])], axis=1)
    r = np.stack([2.0 * np.sin(0.02 * f + phase[3]),
                  -3.0 * c + 4.0 * np.sin(0.015 * f + phase[4]),
                  1.0 * np.sin(0.025 * f + phase[5])], axis=1)
    return t, r


def _bundles_in_front(rng, B, depth_lo=20.0, depth_hi=200.0):
    depth = rng.uniform(depth_lo, depth_hi, size=B)
    x = rng.uniform(-0.35, 0.35, size=B) * depth
    y = rng.uniform(-0.22, 0.22, size=B) * depth
    return np.stack([x, y + 1.5, -depth], axis=1)


def _noisy(rng, v, a=1.0):
    return v + a * rng.normal(0.0, 0.5, size=v.shape) / IMAGE_WIDTH


def _config_c1(rng, F):
    """1 cam, F frames, 20 bundles, 50 markers (k -> bundle k mod 20);
    solve bundle translate (static) + camera rotate (animated); lmdif."""
    B, K = 20, 50
    b = SceneBuilder(F)
    t_true, r_true = _camera_path(rng, F, 0)
    r_init = r_true + rng.uniform(-2.0, 2.0, size=r_true.shape)
    tfm, tids = b.transform(t=[t_true[:, 0], t_true[:, 1], t_true[:, 2]],
                            r=[r_init[:, 0], r_init[:, 1], r_init[:, 2]])
    cam, _ = b.camera(tfm, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN), render_size=RENDER)
    P = _bundles_in_front(rng, B, 20.0, 60.0)
    P_init = P * (1.0 + rng.uniform(-0.05, 0.05, size=(B, 1)))
    bnd_attr = []
    for j in range(B):
        bt, bids = b.transform(t=tuple(P_init[j]))
        b.bundle(bt)
        bnd_attr.append(bids[:3])
    for k in range(K):
        j = k % B
        fs = np.arange(F)
        mx, my = _pose_project(t_true, r_true, FOCAL_MM, np.repeat(P[j][None], F, 0), fs)
        b.marker(cam, j, np.stack([_noisy(rng, mx), _noisy(rng, my)], axis=1))
    for ids in bnd_attr:
        for a in ids:
            b.solve(a)
    for a in tids[3:6]:
        b.solve(a)
    return b.build(meta={"name": CONFIG_NAMES[0], "solver_type": abi.SOLVER_TYPE_CMINPACK_LMDIF,
                         "iterations": 1000})


def _bulk_problem(F, cams_t, cams_r, cams_focal, cam_solve, bnd_init, bnd_solved, mkr_cam,
                  mkr_bnd, obs_m, obs_f, obs_xy, lens=None, gauge_cam0=False,
                  lens_first=False, meta=None, cams_offset=None):
    """Vectorised problem assembly (same semantics as SceneBuilder.build)."""
    b = SceneBuilder(F)
    lens_ids = []
    lens_idx = -1
    if lens is not None:
        if lens.get("model") == "radial":
            lens_idx, lens_ids = b.lens_3de_radial_std_deg4(*lens["init"])
        elif lens.get("model") == "anamorphic":
            lens_idx, lens_ids = b.lens_3de_anamorphic_std_deg4(*lens["init"])
        else:
            lens_idx, lens_ids = b.lens_3de_classic(*lens["init"])
        if "input" in lens:
            kind, vals = lens["input"]
            assert kind == "radial"
            in_idx, _ = b.lens_3de_radial_std_deg4(*vals)
            b.lens_input(lens_idx, in_idx)
    cam_attr_ids = []
    for c in range(len(cams_t)):
        tfm, tids = b.transform(t=[cams_t[c][:, 0], cams_t[c][:, 1], cams_t[c][:, 2]],
                                r=[cams_r[c][:, 0], cams_r[c][:, 1], cams_r[c][:, 2]])
        _, cids = b.camera(tfm, focal=cams_focal[c], film_back=(FILM_W_IN, FILM_H_IN),
                           film_offset=(0.0, 0.0) if cams_offset is None else cams_offset[c],
                           render_size=RENDER, lens=lens_idx)
        cam_attr_ids.append((tids, cids))
    bnd_attr_ids = []
    for j in range(len(bnd_init)):
        bt, bids = b.transform(t=tuple(bnd_init[j]))
        b.bundle(bt)
        bnd_attr_ids.append(bids[:3])
    b.markers_bulk(mkr_cam, mkr_bnd, obs_m, obs_f, obs_xy)
    # solve list (attribute-major)
    if lens is not None and lens_first:
        for slot in lens["solve_slots"]:
            b.solve(lens_ids[slot])
    params_excluded = set()
    for c, (tids, cids) in enumerate(cam_attr_ids):
        for a in cam_solve(tids, cids):
            b.solve(a)
            if gauge_cam0 and c == 0:
                params_excluded.add(a)
    for j, ids in enumerate(bnd_attr_ids):
        if bnd_solved[j]:
            for a in ids:
                b.solve(a)
    prob = b.build(meta=meta)
    if gauge_cam0:
        keep = ~(np.isin(prob.param_attr, list(params_excluded)) & (prob.param_frame == 0))
        for name in ("param_attr", "param_frame", "param_min", "param_max", "param_offset",
                     "param_scale", "x0"):
            setattr(prob, name, np.ascontiguousarray(getattr(prob, name)[keep]))
    return prob


def _windows(rng, K, F, mean_len, lo=None, hi=None):
    if lo is None:
        length = np.clip(rng.poisson(mean_len, size=K), 2, F)
    else:
        length = rng.integers(lo, hi + 1, size=K)
        length = np.minimum(length, F)
    start = rng.integers(0, F - length + 1)
    return start, length


def _obs_from_windows(rng, start, length, project_fn, noise=1.0):
    ks = np.repeat(np.arange(start.size), length)
    offs = np.arange(length.sum()) - np.repeat(np.cumsum(length) - length, length)
    fs = np.repeat(start, length) + offs
    mx, my = project_fn(ks, fs)
    xy = np.stack([_noisy(rng, mx, noise), _noisy(rng, my, noise)], axis=1)
    return ks, fs, xy


_ROO_FACTORS = {abi.ROO_XYZ: "zyx", abi.ROO_YZX: "xzy", abi.ROO_ZXY: "yxz",
                abi.ROO_XZY: "yzx", abi.ROO_YXZ: "zxy", abi.ROO_ZYX: "xyz"}


def _euler(rx, ry, rz, roo=abi.ROO_XYZ):
    """Column-vector rotation of any rotate order (degrees): the product of the
    three axis rotations in the order mmba_geom.h trs_matrix chains them."""
    rx, ry, rz = (np.radians(np.asarray(v, dtype=np.float64)) for v in (rx, ry, rz))

    def axis(a, ang):
        c, s_ = np.cos(ang), np.sin(ang)
        R = np.zeros(np.shape(ang) + (3, 3))
        i, j = {"x": (1, 2), "y": (2, 0), "z": (0, 1)}[a]
        k = "xyz".index(a)
        R[..., k, k] = 1.0
        R[..., i, i] = c
        R[..., j, j] = c
        R[..., i, j] = -s_
        R[..., j, i] = s_
        return R

    ang = {"x": rx, "y": ry, "z": rz}
    a, b_, c = _ROO_FACTORS[roo]
    return axis(a, ang[a]) @ axis(b_, ang[b_]) @ axis(c, ang[c])


def _pose_project(t, r, focal, pts, fs):
    R = _euler_xyz(r[fs, 0], r[fs, 1], r[fs, 2])
    pc = np.einsum("nij,ni->nj", R, pts - t[fs])
    depth = -pc[:, 2]
    fcl = focal[fs] if np.ndim(focal) else focal
    return fcl * pc[:, 0] / (FILM_W_MM * depth), fcl * pc[:, 1] / (FILM_H_MM * depth)


def rs_blend(v, tau):
    """Rolling-shutter pose blend (mmba.h ABI 3; the 3DE exporter's
    _apply_rs_correction, uvtrack_format.py:186-203, with its end-frame
    extrapolation :311-314): per-frame values v[F, ...] at time f + tau[f].
    Used here only to synthesise markers through the same model."""
    v = np.asarray(v, dtype=np.float64)
    pv = np.concatenate([v[:1] + (v[:1] - v[1:2]), v[:-1]])
    nv = np.concatenate([v[1:], v[-1:] + (v[-1:] - v[-2:-1])])
    b = (nv - pv) / 2.0
    c = -v + ((nv + pv) / 2.0)
    tau = np.asarray(tau, dtype=np.float64).reshape((-1,) + (1,) * (v.ndim - 1))
    return (v + tau * b) + (tau * tau) * c


def _pose_project_rs(t, r, focal, pts, fs, rs, y_guess, iters=4):
    """_pose_project with the camera pose of each observation taken at its
    scanline time tau = rs * (0.5 - y) (a fixed point in the marker's own y)."""
    y = np.asarray(y_guess, dtype=np.float64)
    mx = my = None
    for _ in range(iters):
        tau = rs * (0.5 - y)
        tb = np.empty((fs.size, 3))
        rb = np.empty((fs.size, 3))
        for k in range(3):
            tb[:, k] = _blend_at(t[:, k], fs, tau)
            rb[:, k] = _blend_at(r[:, k], fs, tau)
        R = _euler_xyz(rb[:, 0], rb[:, 1], rb[:, 2])
        pc = np.einsum("nij,ni->nj", R, pts - tb)
        depth = -pc[:, 2]
        fcl = focal[fs] if np.ndim(focal) else focal
        mx, my = fcl * pc[:, 0] / (FILM_W_MM * depth), fcl * pc[:, 1] / (FILM_H_MM * depth)
        y = my
    return mx, my


def _blend_at(v, fs, tau):
    """rs_blend of the per-frame series v evaluated per observation (frame fs,
    time offset tau)."""
    F = v.size
    cv = v[fs]
    pv = np.where(fs > 0, v[np.maximum(fs - 1, 0)], 0.0)
    nv = np.where(fs < F - 1, v[np.minimum(fs + 1, F - 1)], 0.0)
    pv = np.where(fs == 0, cv + (cv - nv), pv)
    nv = np.where(fs == F - 1, cv + (cv - pv), nv)
    b = (nv - pv) / 2.0
    c = -cv + ((nv + pv) / 2.0)
    return (cv + tau * b) + (tau * tau) * c


def _config_c2(rng, F, scale):
    """1 camera, 1k locked bundles, 5k markers (k -> k mod 1000), windows U[20,60];
    solve camera translate/rotate + focal per frame."""
    B, K = max(1, int(1000 * scale)), max(1, int(5000 * scale))
    t, r = _camera_path(rng, F, 0)
    focal = FOCAL_MM * (1.0 + 0.05 * np.sin(0.02 * np.arange(F)))
    P = _bundles_in_front(rng, B)
    start, length = _windows(rng, K, F, None, 20, 60)
    mkr_bnd = np.arange(K) % B
    ks, fs, xy = _obs_from_windows(rng, start, length,
                                   lambda ks, fs: _pose_project(t, r, focal, P[mkr_bnd[ks]], fs))
    t0 = t + rng.uniform(-0.05, 0.05, size=t.shape)
    r0 = r + rng.uniform(-2.0, 2.0, size=r.shape)
    f0 = focal * (1.0 + rng.uniform(-0.05, 0.05, size=F))
    return _bulk_problem(F, [t0], [r0], [f0],
                         lambda tids, cids: list(tids[:6]) + [cids[abi.CAM_FOCAL_MM]],
                         P, np.zeros(B, bool), np.zeros(K, np.int32), mkr_bnd, ks, fs, xy,
                         meta={"name": CONFIG_NAMES[1]})


def _config_ba(rng, index, n_cams, F, B, K, window, per_cam_markers, depth=(20.0, 200.0),
               init_noise=1.0, obs_noise=1.0):
    """Full BA: animated cameras (t, r per frame) + static bundles, gauge-locked.

    C3 (``per_cam_markers``): a 10-camera rig (2 units apart) moving slowly,
    bundles in a box in front, 5 markers per bundle spread over the cameras.
    C4: one camera dollying 0.5 units/frame; every bundle is placed in front of
    the camera at the middle of its 4-frame window so the window's baseline
    (1.5 units) gives usable parallax at depth 20-200."""
    if per_cam_markers:
        ts, rs = zip(*[_camera_path(rng, F, c) for c in range(n_cams)])
        P = _bundles_in_front(rng, B)
        L = K // n_cams
        mkr_cam = np.repeat(np.arange(n_cams), L)
        K = mkr_cam.size
        # camera c sees bundles [c*B/n_cams, c*B/n_cams + L) mod B: every bundle
        # is seen by K/B consecutive cameras and the camera/bundle graph is
        # connected (a plain k mod B splits odd/even cameras into two
        # disconnected, gauge-free components).
        k = np.arange(K)
        mkr_bnd = ((k % L) + (k // L) * max(1, B // n_cams)) % B
        start, length = _windows(rng, K, F, window)
    else:
        f = np.arange(F, dtype=np.float64)
        phase = rng.uniform(0, 2 * math.pi, size=4)
        t = np.stack([0.5 * f, 1.5 + 0.3 * np.sin(0.05 * f + phase[0]),
                      -0.1 * f + 0.3 * np.sin(0.03 * f + phase[1])], axis=1)
        r = np.stack([1.5 * np.sin(0.02 * f + phase[2]), -10.0 + 3.0 * np.sin(0.01 * f + phase[3]),
                      0.5 * np.sin(0.04 * f)], axis=1)
        ts, rs = (t,), (r,)
        mkr_cam = np.zeros(K, np.int64)
        mkr_bnd = np.arange(K) % B
        length = np.full(K, min(window, F))
        start = rng.integers(0, F - length[0] + 1, size=K)
        # bundle j placed relative to the camera at the middle of its window
        mid = np.minimum(start + length // 2, F - 1)
        P = np.empty((B, 3))
        depth = rng.uniform(depth[0], depth[1], size=B)
        u = rng.uniform(-0.35, 0.35, size=B)
        v = rng.uniform(-0.22, 0.22, size=B)
        owner = np.full(B, -1)
        owner[mkr_bnd[::-1]] = np.arange(K)[::-1]  # first marker of each bundle
        fm = mid[np.maximum(owner, 0)]
        Rm = _euler_xyz(r[fm, 0], r[fm, 1], r[fm, 2])
        pc = np.stack([u * depth, v * depth, -depth], axis=1)
        P = t[fm] + np.einsum("nij,nj->ni", Rm, pc)

    def proj(ks, fs):
        mx = np.empty(ks.size)
        my = np.empty(ks.size)
        for c in range(n_cams):
            sel = mkr_cam[ks] == c
            mx[sel], my[sel] = _pose_project(ts[c], rs[c], FOCAL_MM, P[mkr_bnd[ks[sel]]], fs[sel])
        return mx, my

    ks, fs, xy = _obs_from_windows(rng, start, length, proj, obs_noise)
    a = init_noise
    t0 = [tc + a * rng.uniform(-0.05, 0.05, size=tc.shape) for tc in ts]
    r0 = [rc + a * rng.uniform(-2.0, 2.0, size=rc.shape) for rc in rs]
    for c in (0,):  # gauge: camera-0 pose at frame 0 exact
        t0[c][0] = ts[c][0]
        r0[c][0] = rs[c][0]
    # bundles perturbed +-5% along the ray from the camera that first sees them
    first_f = np.zeros(B, np.int64)
    first_c = np.zeros(B, np.int64)
    seen = np.zeros(B, bool)
    for q in range(ks.size):
        j = mkr_bnd[ks[q]]
        if not seen[j]:
            seen[j] = True
            first_f[j] = fs[q]
            first_c[j] = mkr_cam[ks[q]]
    origin = np.stack([ts[first_c[j]][first_f[j]] for j in range(B)]) if B else np.zeros((0, 3))
    P0 = origin + (P - origin) * (1.0 + a * rng.uniform(-0.05, 0.05, size=(B, 1)))
    P0[0] = P[0]  # gauge: bundle 0 locked at truth
    solved = np.ones(B, bool)
    solved[0] = False
    return _bulk_problem(F, t0, r0, [FOCAL_MM] * n_cams, lambda tids, cids: list(tids[:6]),
                         P0, solved, mkr_cam, mkr_bnd, ks, fs, xy, gauge_cam0=True,
                         meta={"name": CONFIG_NAMES[index]})


def _config_c5(rng, F, scale, lens_model="classic", rolling_shutter=0.0, n_cams=2):
    """2 cams, 1k locked bundles, 2k markers (1k per cam), windows mean 60,
    one shared 3DE-classic lens with distortion + quartic solved (lens attrs first).
    ``rolling_shutter`` = rs (frames, time shift x fps) != 0: both cameras
    have that rolling shutter (mmba.h ABI 3) and the markers are synthesised
    through the same per-scanline pose blend."""
    B, K = max(1, int(1000 * scale)), max(2, int(2000 * scale))
    ts, rs = zip(*[_camera_path(rng, F, c) for c in range(n_cams)])
    P = _bundles_in_front(rng, B)
    mkr_cam = np.repeat(np.arange(n_cams), K // n_cams)
    K = mkr_cam.size
    mkr_bnd = np.arange(K) % B
    start, length = _windows(rng, K, F, 60)
    if lens_model in ("anamorphic", "anamorphic_rescaled"):
        resc = lens_model == "anamorphic_rescaled"
        lens_true = (0.03, 0.02, -0.01, 0.01, 0.005, 0.005, 0.0, 0.0, 0.0, 0.0, 5.0, 1.05, 1.0,
                     1.2 if resc else 1.0)
        distort = _anamorphic_distort_truth
        init = (0.0, 0.0) + lens_true[2:13]
        lens = {"model": "anamorphic", "init": init + ((lens_true[13],) if resc else ()),
                "solve_slots": (0, 1)}
    elif lens_model == "radial":
        lens_true = (0.05, 0.002, -0.002, 0.01, 0.0, 0.0, 20.0, 0.05)
        distort = _radial_distort_truth
        lens = {"model": "radial", "init": (0.0,) + lens_true[1:3] + (0.0,) + lens_true[4:],
                "solve_slots": (0, 3)}
    elif lens_model == "layered":
        # the classic lens (distortion + quartic solved) layered over a
        # static radial deg 4 input lens (mmba.h ABI 5): the input is applied
        # first, with its values as read (constants of the solve)
        lens_true = (0.05, 1.0, 0.0, 0.0, 0.01)
        in_true = (0.03, 0.002, -0.001, 0.008, 0.0, 0.0, 15.0, 0.02)

        def distort(c, x, y):
            ix, iy = _radial_distort_truth(in_true, x, y)
            return _lens_distort_truth(c, ix, iy)
        lens = {"init": (0.0, 1.0, 0.0, 0.0, 0.0), "solve_slots": (0, 4),
                "input": ("radial", in_true)}
    else:
        lens_true = (0.05, 1.0, 0.0, 0.0, 0.01)
        distort = _lens_distort_truth
        lens = {"init": (0.0, 1.0, 0.0, 0.0, 0.0), "solve_slots": (0, 4)}
        if lens_model == "classic_animated":  # distortion keyed per frame (F params)
            lens["init"] = (np.zeros(F),) + lens["init"][1:]
        elif lens_model == "classic_wide":
            # all five classic coefficients keyed per frame and solved, with the
            # camera's focal length: 6 + 1 + 5 = 12 parameters on each
            # camera-frame of a one-camera shot
            lens["init"] = (np.zeros(F), np.ones(F), np.zeros(F), np.zeros(F), np.zeros(F))
            lens["solve_slots"] = (0, 1, 2, 3, 4)

    def proj(ks, fs):
        mx = np.empty(ks.size)
        my = np.empty(ks.size)
        for c in range(n_cams):
            sel = mkr_cam[ks] == c
            mx[sel], my[sel] = _pose_project(ts[c], rs[c], FOCAL_MM, P[mkr_bnd[ks[sel]]], fs[sel])
            if rolling_shutter:
                # the scanline pose: a fixed point in the distorted marker y
                for _ in range(4):
                    _dx, _dy = _c5_lens(mx[sel], my[sel])
                    mx[sel], my[sel] = _pose_project_rs(
                        ts[c], rs[c], FOCAL_MM, P[mkr_bnd[ks[sel]]], fs[sel], rolling_shutter,
                        _dy, iters=1)
        # Horizontal fit marker y is in film-height units; the lens works on the
        # projected (film-fit scaled) point, see adjust_measureErrors.cpp:458-472.
        return _c5_lens(mx, my)

    def _c5_lens(mx, my):
        ra = RENDER[0] / RENDER[1]
        fa = FILM_W_MM / FILM_H_MM
        py = my * (ra / fa)
        dx, dy = distort(lens_true, mx, py)
        return dx, dy / (ra / fa)

    ks, fs, xy = _obs_from_windows(rng, start, length, proj)
    t0 = [tc + rng.uniform(-0.05, 0.05, size=tc.shape) for tc in ts]
    r0 = [rc + rng.uniform(-2.0, 2.0, size=rc.shape) for rc in rs]
    wide = lens_model == "classic_wide"
    focal0 = [FOCAL_MM * (1.0 + rng.uniform(-0.01, 0.01, F)) if wide else FOCAL_MM
              for _ in range(n_cams)]
    offset0 = None

    def cam_solve(tids, cids):
        return list(tids[:6]) + ([cids[abi.CAM_FOCAL_MM]] if wide else [])
    prob = _bulk_problem(F, t0, r0, focal0, cam_solve,
                         P, np.zeros(B, bool), mkr_cam, mkr_bnd, ks, fs, xy, lens=lens,
                         lens_first=True, cams_offset=offset0,
                         meta={"name": CONFIG_NAMES[4] + ("" if lens_model == "classic"
                                                          else "_" + lens_model) +
                               ("" if n_cams == 2 else "_%dcam" % n_cams) +
                               ("_rs" if rolling_shutter else "")})
    if rolling_shutter:
        prob.cam_rs_value = np.full(prob.num_cameras, float(rolling_shutter))
    return prob


EDGE_RENDERS = {"wide": (2048, 858), "narrow": (2048, 1556)}  # aspect above / below 36x24 mm


def edge_scene(film_fit=abi.FILM_FIT_HORIZONTAL, render="narrow", film_offset=(0.0, 0.0),
               camera_scale=1.0, rotate_order=abi.ROO_XYZ, parented=False, frames=6,
               bundles=24, seed=9, stiffness=False, static_focal=False,
               offset_shifts=True, gauge=True, solve_bundles=True,
               solve_parent=False, duplicate_markers=0) -> Problem:
    """Small bundle-adjustment scene over the camera settings the synthetic
    configs keep benign: any film fit, a render aspect above or
    below the film aspect, film offsets (inches, Appendix B5/B6), a camera
    scale, any rotate order (camera and its parent), and a parented camera
    (camera transform under a static, rotated group).  One camera animated
    over ``frames`` frames (pose solved, frame 0 locked), ``bundles`` bundles
    seen on every frame (translate solved, bundle 0 locked).  Markers are a
    plain pinhole projection of the truth plus noise: the reference geometry
    (film fit, offsets, scale) then has something to fit, which is all a
    parity scene needs.  ``stiffness``: stiffness rows on two bundle
    translates and a smoothness row on one camera rotate
    (adjust_measureErrors.cpp:311-387).  ``static_focal``: the camera focal
    is solved too, as one static (global) parameter.  ``gauge=False``: nothing
    locked (with one frame: a bundle-only solve against a fixed camera).
    ``solve_bundles=False``: the bundles stay at their true positions, unsolved
    (the rolling-shutter plans' restriction).  ``solve_parent`` (with
    ``parented``): the parent group's rotation is solved too -- three static
    (global) parameters starting 0.5-1 degree off.  ``duplicate_markers`` = k:
    bundles 1..k get a second marker of the same camera (a bundle seen twice
    in one camera-frame), its positions offset by 0.002."""
    rng = np.random.Generator(np.random.PCG64(seed))
    F, B = frames, bundles
    b = SceneBuilder(F)
    f = np.arange(F, dtype=np.float64)
    t_true = np.stack([0.4 * f, 1.5 + 0.1 * f, -0.2 * f], axis=1)
    r_true = np.stack([2.0 + 0.5 * f, -8.0 + 0.7 * f, 1.0 + 0.3 * f], axis=1)
    depth = rng.uniform(15.0, 40.0, size=B)
    P = np.stack([rng.uniform(-0.3, 0.3, B) * depth, 1.5 + rng.uniform(-0.2, 0.2, B) * depth,
                  -depth], axis=1)
    t0 = t_true + rng.uniform(-0.05, 0.05, size=t_true.shape)
    r0 = r_true + rng.uniform(-1.0, 1.0, size=r_true.shape)
    t0[0], r0[0] = t_true[0], r_true[0]
    parent = None
    pids = None
    if parented:
        pr0 = (2.0, -2.8, 3.6) if solve_parent else (1.5, -2.0, 3.0)
        parent, pids = b.transform(t=(0.3, -0.2, 0.5), r=pr0, s=(1.0, 1.0, 1.0),
                                   rotate_order=rotate_order)
    ctfm, tids = b.transform(t=[t0[:, 0], t0[:, 1], t0[:, 2]], r=[r0[:, 0], r0[:, 1], r0[:, 2]],
                             parent=parent, rotate_order=rotate_order)
    cam, cids = b.camera(ctfm, focal=FOCAL_MM * (1.03 if static_focal else 1.0),
                         film_back=(FILM_W_IN, FILM_H_IN), film_offset=film_offset,
                         film_fit=film_fit, render_size=EDGE_RENDERS[render],
                         camera_scale=camera_scale)
    P0 = P * (1.0 + rng.uniform(-0.03, 0.03, size=(B, 1)))
    if gauge or not solve_bundles:
        P0[0] = P[0]
    if not solve_bundles:
        P0 = P.copy()
    bids = []
    for j in range(B):
        bt, ids = b.transform(t=tuple(P0[j]))
        b.bundle(bt)
        bids.append(ids)
    # truth camera world pose (parent o local, any rotate order)
    Rl = _euler(r_true[:, 0], r_true[:, 1], r_true[:, 2], rotate_order)
    if parented:
        Rp = _euler(1.5, -2.0, 3.0, rotate_order)
        Rw = Rp[None] @ Rl
        tw = t_true @ Rp.T + np.array([0.3, -0.2, 0.5])
    else:
        Rw, tw = Rl, t_true
    fs = np.tile(np.arange(F), B)
    pc = np.einsum("nji,nj->ni", Rw[fs], np.repeat(P, F, 0) - tw[fs])
    mx = FOCAL_MM * pc[:, 0] / (FILM_W_MM * -pc[:, 2]) / camera_scale
    my = FOCAL_MM * pc[:, 1] / (FILM_H_MM * -pc[:, 2]) / camera_scale
    if offset_shifts:  # Maya DAG: the offset moves the image; MM Scene Graph: not (B6)
        mx = mx - film_offset[0] / FILM_W_IN
        my = my - film_offset[1] / FILM_H_IN
    mx, my = _noisy(rng, mx).reshape(B, F), _noisy(rng, my).reshape(B, F)
    for j in range(B):
        b.marker(cam, j, np.stack([mx[j], my[j]], axis=1))
    for j in range(1, 1 + duplicate_markers):
        b.marker(cam, j, np.stack([mx[j] + 0.002, my[j] - 0.002], axis=1))
    if static_focal:
        b.solve(cids[abi.CAM_FOCAL_MM])
    for a in tids[:6]:
        b.solve(a)
    if solve_parent and pids is not None:
        for a in pids[3:6]:
            b.solve(a)
    for j in range(1 if gauge else 0, B if solve_bundles else 0):
        for a in bids[j][:3]:
            b.solve(a)
    if stiffness:
        b.stiffness(bids[1][0], weight=2.0, variance=0.5, value=float(P0[1][0]) + 0.1)
        b.stiffness(bids[2][2], weight=1.0, variance=2.0, value=float(P0[2][2]) - 0.2)
        b.smoothness(tids[4], weight=0.5, variance=1.5, value=float(r0[3][1]) + 0.3, frame=3)
    prob = b.build(meta={"name": "edge"})
    if gauge:  # camera pose at frame 0 locked (parameters of frame 0 dropped)
        keep = ~(np.isin(prob.param_attr, tids[:6]) & (prob.param_frame == 0))
        for name in ("param_attr", "param_frame", "param_min", "param_max", "param_offset",
                     "param_scale", "x0"):
            setattr(prob, name, np.ascontiguousarray(getattr(prob, name)[keep]))
    return prob


def rig_scene(n_cams=2, bundles=10, solve_cam1=True, stiffness=False, seed=11) -> Problem:
    """Static rig: ``n_cams`` cameras with static (non-animated) poses 1.5
    units apart on one frame, bundles in front solved (translate), camera 1's
    rotation solved as three static (global) parameters (its translation
    stays: it sets the scale).  Every parameter is static,
    so every FD column re-measures every row: the scene on which the
    reference's central differences and robust loss are well defined (see
    Plan::build).  Markers camera-major (B4).  ``stiffness``: a stiffness row
    on a bundle translate and a smoothness row on camera 1's rotate y."""
    rng = np.random.Generator(np.random.PCG64(seed))
    b = SceneBuilder(1)
    B = bundles
    depth = rng.uniform(12.0, 30.0, size=B)
    P = np.stack([rng.uniform(-0.3, 0.3, B) * depth, rng.uniform(-0.2, 0.2, B) * depth,
                  -depth], axis=1)
    cams, cam_ids = [], []
    for c in range(n_cams):
        t = np.array([1.5 * c, 0.2 * c, 0.0])
        r = np.array([0.5 * c, -2.0 * c, 0.3 * c])
        t0 = t + (rng.uniform(-0.05, 0.05, 3) if c == 1 and solve_cam1 else 0.0)
        r0 = r + (rng.uniform(-1.0, 1.0, 3) if c == 1 and solve_cam1 else 0.0)
        tfm, tids = b.transform(t=tuple(t0), r=tuple(r0))
        cam, _ = b.camera(tfm, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN),
                          render_size=RENDER)
        cams.append((cam, t, r))
        cam_ids.append(tids)
    P0 = P * (1.0 + rng.uniform(-0.04, 0.04, size=(B, 1)))
    bids = []
    for j in range(B):
        bt, ids = b.transform(t=tuple(P0[j]))
        b.bundle(bt)
        bids.append(ids)
    for cam, t, r in cams:
        R = _euler_xyz(*r)
        pc = (P - t) @ R
        mx = FOCAL_MM * pc[:, 0] / (FILM_W_MM * -pc[:, 2])
        my = FOCAL_MM * pc[:, 1] / (FILM_H_MM * -pc[:, 2])
        for j in range(B):
            b.marker(cam, j, [[_noisy(rng, mx[j]), _noisy(rng, my[j])]])
    if solve_cam1 and n_cams > 1:  # rotate only: translating camera 1 is the free scale
        for a in cam_ids[1][3:6]:
            b.solve(a)
    for j in range(B):
        for a in bids[j][:3]:
            b.solve(a)
    if stiffness:
        b.stiffness(bids[0][1], weight=1.5, variance=0.3, value=float(P0[0][1]) + 0.05)
        if solve_cam1 and n_cams > 1:
            b.smoothness(cam_ids[1][4], weight=0.7, variance=0.8, value=-1.5)
    return b.build(meta={"name": "rig"})


B3_VARIANTS = ("lens_first", "cam_first", "animated", "animated_late", "one_lens")


def b3_scene(variant="lens_first", frames=5, markers_per_cam=4, seed=23) -> Problem:
    """Two cameras, each with its own 3DE classic lens (distortion 0.04 and
    -0.03): the scene on which the reference's lens index arithmetic (SURVEY
    Appendix B3, mmba.h ABI 7) distorts marker i at frame f with the lens of
    marker (i + f) / F and writes a lens attribute solved at frame g into the
    lens of attrList entry (a + g) / F.  Camera 0 moves along x with its
    rotation solved per frame; camera 1 is static with its rotation solved
    (three globals); the bundles are fixed.  Markers: the plain projection
    of each marker's own camera and lens, plus noise.  Variants:
      "lens_first": both lenses' distortion solved, listed before the cameras
      "cam_first":  the same, the lens attributes listed after the rotations
      "animated":   lens 0's distortion animated and solved (one parameter
                    per frame, values differing per frame), lens attributes
                    first: lens 1's static distortion then overwrites lens 0's
                    clones at frames 1.. (attrList entry 1 + j lands in entry
                    0's range), and marker i at frame f reads frame (i+f) % F
      "animated_late": the same, the lens attributes after the rotations
                    (their writes land on attrList entries of no lens)
      "one_lens":   camera 0 without a lens, camera 1's lens solved."""
    assert variant in B3_VARIANTS, variant
    rng = np.random.Generator(np.random.PCG64(seed))
    F = frames
    b = SceneBuilder(F)
    fr = np.arange(F, dtype=np.float64)
    render = (1500, 1000)  # the film aspect: film fit is the identity
    K = markers_per_cam
    depth = rng.uniform(10.0, 25.0, size=2 * K)
    P = np.stack([rng.uniform(-0.25, 0.25, 2 * K) * depth, rng.uniform(-0.2, 0.2, 2 * K) * depth,
                  -depth], axis=1)
    truth = [(0.04, 1.0, 0.0, 0.0, 0.0), (-0.03, 1.0, 0.0, 0.0, 0.0)]
    if variant in ("animated", "animated_late"):
        d0 = 0.04 + 0.005 * fr
        lens0, lids0 = b.lens_3de_classic(distortion=np.zeros(F) + 0.01 * fr)
    else:
        d0 = np.full(F, 0.04)
        lens0, lids0 = b.lens_3de_classic(distortion=0.0)
    lens1, lids1 = b.lens_3de_classic(distortion=0.0)
    t0 = np.stack([0.3 * fr, 0.1 + 0.0 * fr, 0.0 * fr], 1)
    r0 = np.stack([1.0 + 0.2 * fr, -1.5 + 0.1 * fr, 0.5 + 0.0 * fr], 1)
    tfm0, tids0 = b.transform(t=[t0[:, 0], t0[:, 1], t0[:, 2]],
                              r=[r0[:, 0] + rng.uniform(-0.5, 0.5, F),
                                 r0[:, 1] + rng.uniform(-0.5, 0.5, F),
                                 r0[:, 2] + rng.uniform(-0.5, 0.5, F)])
    t1, r1 = np.array([1.0, 0.2, 0.5]), np.array([0.5, 2.0, -0.3])
    tfm1, tids1 = b.transform(t=tuple(t1), r=tuple(r1 + rng.uniform(-0.8, 0.8, 3)))
    cam0, _ = b.camera(tfm0, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN),
                       render_size=render, lens=-1 if variant == "one_lens" else lens0)
    cam1, _ = b.camera(tfm1, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN),
                       render_size=render, lens=lens1)
    for j in range(2 * K):
        bt, _ = b.transform(t=tuple(P[j]))
        b.bundle(bt)
    for c, cam in enumerate((cam0, cam1)):
        for k in range(K):
            j = c * K + k
            xy = np.empty((F, 2))
            for f in range(F):
                t, r = (t0[f], r0[f]) if c == 0 else (t1, r1)
                mx, my, _ = _project(t, r, FOCAL_MM, P[j])
                if c == 1 or variant != "one_lens":
                    lt = truth[c] if c == 1 else (d0[f],) + truth[0][1:]
                    mx, my = _lens_distort_truth(lt, float(mx), float(my))
                xy[f] = (float(_noisy(rng, np.asarray(mx))), float(_noisy(rng, np.asarray(my))))
            b.marker(cam, j, xy)
    lens_solve = [lids1[0]] if variant == "one_lens" else [lids0[0], lids1[0]]
    first = variant in ("lens_first", "animated")
    if first:
        for a in lens_solve:
            b.solve(a)
    for a in tids0[3:6] + tids1[3:6]:
        b.solve(a)
    if not first:
        for a in lens_solve:
            b.solve(a)
    return b.build(meta={"name": "b3_" + variant})


def b4_scene(frames=4, bundles=6, partial=False, frame_xy=False, seed=29) -> Problem:
    """Two cameras seeing every bundle, the markers listed bundle by bundle
    (camera 1's, then camera 0's): not grouped by camera, so in MM Scene
    Graph mode observation (marker i, frame f) reads the flat point and marker
    lists at i * F + f, which hold the i-th marker in camera order (SURVEY
    Appendix B4, mmba.h ABI 8).  Camera 0 moves along x with its rotation
    solved per frame, camera 1 is static with its rotation solved (three
    globals), the bundles' translates are solved.  Marker weights differ per
    marker.  ``partial``: some markers disabled on some frames, so a remapped
    observation can read a flat marker with no observation there;
    ``frame_xy``: mkr_frame_xy filled with every marker's x,y at every frame."""
    rng = np.random.Generator(np.random.PCG64(seed))
    F, B = frames, bundles
    b = SceneBuilder(F)
    fr = np.arange(F, dtype=np.float64)
    render = (1500, 1000)
    depth = rng.uniform(10.0, 25.0, size=B)
    P = np.stack([rng.uniform(-0.25, 0.25, B) * depth, rng.uniform(-0.2, 0.2, B) * depth,
                  -depth], axis=1)
    t0 = np.stack([0.3 * fr, 0.1 + 0.0 * fr, 0.0 * fr], 1)
    r0 = np.stack([1.0 + 0.2 * fr, -1.5 + 0.1 * fr, 0.5 + 0.0 * fr], 1)
    tfm0, tids0 = b.transform(t=[t0[:, 0], t0[:, 1], t0[:, 2]],
                              r=[r0[:, 0] + rng.uniform(-0.5, 0.5, F),
                                 r0[:, 1] + rng.uniform(-0.5, 0.5, F),
                                 r0[:, 2] + rng.uniform(-0.5, 0.5, F)])
    t1, r1 = np.array([1.0, 0.2, 0.5]), np.array([0.5, 2.0, -0.3])
    tfm1, tids1 = b.transform(t=tuple(t1), r=tuple(r1 + rng.uniform(-0.8, 0.8, 3)))
    cam0, _ = b.camera(tfm0, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN), render_size=render)
    cam1, _ = b.camera(tfm1, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN), render_size=render)
    P0 = P * (1.0 + rng.uniform(-0.03, 0.03, size=(B, 1)))
    bids = []
    for j in range(B):
        bt, ids = b.transform(t=tuple(P0[j]))
        b.bundle(bt)
        bids.append(ids)
    all_xy = []
    for j in range(B):
        for c, cam in ((1, cam1), (0, cam0)):
            xy = np.empty((F, 2))
            for f in range(F):
                t, r = (t0[f], r0[f]) if c == 0 else (t1, r1)
                mx, my, _ = _project(t, r, FOCAL_MM, P[j])
                xy[f] = (float(_noisy(rng, np.asarray(mx))), float(_noisy(rng, np.asarray(my))))
            en = None
            if partial and (j + c) % 3 == 1:  # a gap of one frame
                en = np.ones(F, bool)
                en[(j + 2 * c) % F] = False
            b.marker(cam, j, xy, enable=en, weight=1.0 + 0.25 * ((2 * j + c) % 3))
            all_xy.append(xy)
    for a in tids0[3:6] + tids1[3:6]:
        b.solve(a)
    for j in range(B):
        for a in bids[j][:3]:
            b.solve(a)
    prob = b.build(meta={"name": "b4" + ("_partial" if partial else "")})
    if frame_xy:
        prob.mkr_frame_xy = np.ascontiguousarray(np.stack(all_xy), dtype=np.float64).reshape(-1)
    return prob


def b4_grouped_twin(prob: Problem) -> Problem:
    """The grouped scene a B4 problem is equivalent to in MM Scene Graph mode
    (tests): the markers renumbered into the flat (camera-major) order and
    each observation's x,y replaced by that of the flat marker it reads --
    its own weight, frame and marker number kept."""
    K, F = prob.num_markers, int(prob.num_frames)
    flat = np.concatenate([np.flatnonzero(prob.mkr_cam == c) for c in range(prob.num_cameras)])
    g = flat[prob.obs_marker]
    if prob.mkr_frame_xy is not None:
        fxy = prob.mkr_frame_xy.reshape(K, F, 2)
    else:
        fxy = np.full((K, F, 2), np.nan)
        fxy[prob.obs_marker, prob.obs_frame] = prob.obs_xy.reshape(-1, 2)
    xy = prob.obs_xy.reshape(-1, 2).copy()
    moved = g != prob.obs_marker
    xy[moved] = fxy[g[moved], prob.obs_frame[moved]]
    d = prob.to_npz_dict()
    d["mkr_cam"] = prob.mkr_cam[flat]
    d["mkr_bnd"] = prob.mkr_bnd[flat]
    d["obs_xy"] = xy.reshape(-1)
    d.pop("mkr_frame_xy", None)
    twin = Problem.from_npz_dict(d)
    twin.meta = dict(prob.meta)
    return twin


def witness_scene(n_witness=4, frames=6, bundles=24, solve_bundles=True, n_focal=3,
                  extra_globals=0, window=None, lens=None, wide_block=False,
                  seed=17) -> Problem:
    """Witness-camera rig with a wide arrow of global parameters: a fixed
    static reference camera 0, ``n_witness`` static witness cameras whose
    poses are solved as static (global) parameters (witness 1: rotation
    only -- its fixed translation sets the scale; the others: translate and
    rotate), static focal lengths solved on the first ``n_focal`` witnesses,
    one animated camera whose pose is solved per frame (camera-frame blocks),
    and ``bundles`` bundles (translate solved with ``solve_bundles``).
    n_witness = 4, n_focal = 3 gives 24 globals; 5 / 5 gives 32, the
    library's arrow capacity.  ``extra_globals`` adds solved static film back
    widths on the witnesses (to step past it).  ``window``: the animated
    camera sees bundle j only on ``window`` consecutive frames (a banded
    reduced system instead of a dense one).  ``lens="anamorphic"``: every
    camera shares one 3DE anamorphic deg 4 lens whose ten polynomial
    coefficients are solved (created and solved first: B3), so a witness
    observation reaches more than 20 parameters.  ``wide_block``: the animated
    camera also solves its focal length and film offsets per frame and has
    its own 3DE classic lens whose distortion and x / y curvature are keyed
    per frame -- 6 + 3 + 3 = 12 parameters on each of its camera-frames (the
    lens coefficients join the block: one camera reads them, Plan::build).
    Markers camera-major (B4)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    F = int(frames)
    b = SceneBuilder(F)
    lens_idx, lens_solve = -1, []
    if lens == "anamorphic":
        lens_idx, lids = b.lens_3de_anamorphic_std_deg4()
        lens_solve = list(lids[:10])
    elif lens is not None:
        raise ValueError(lens)
    B = bundles
    depth = rng.uniform(12.0, 30.0, size=B)
    P = np.stack([rng.uniform(-0.3, 0.3, B) * depth, rng.uniform(-0.2, 0.2, B) * depth,
                  -depth], axis=1)
    views = []  # (cam index, per-frame t (F,3), per-frame r (F,3), focal)
    solve_ids = []
    gl_cams = []
    for c in range(n_witness + 1):
        # on an arc around the bundle cloud, each aimed at its centre
        X = 5.0 * (c - n_witness / 2.0)
        t = np.array([X, 0.4 * c, 0.5 * (c % 2)])
        r = np.array([0.5 * c, np.degrees(np.arctan2(X, 20.0)), 0.3 * c])
        foc = FOCAL_MM * (1.0 + 0.05 * c)
        solved = c >= 1
        t0 = t + (rng.uniform(-0.05, 0.05, 3) if c >= 2 else 0.0)
        r0 = r + (rng.uniform(-1.0, 1.0, 3) if solved else 0.0)
        f0 = foc * (1.0 + (rng.uniform(-0.03, 0.03) if 1 <= c <= n_focal else 0.0))
        tfm, tids = b.transform(t=tuple(t0), r=tuple(r0))
        cam, cids = b.camera(tfm, focal=f0, film_back=(FILM_W_IN, FILM_H_IN),
                             render_size=RENDER, lens=lens_idx)
        views.append((cam, np.tile(t, (F, 1)), np.tile(r, (F, 1)), foc))
        if c == 1:
            solve_ids += tids[3:6]
        elif c >= 2:
            solve_ids += tids[0:6]
        if 1 <= c <= n_focal:
            solve_ids.append(cids[abi.CAM_FOCAL_MM])
        if c >= 1:
            gl_cams.append(cids)
    for k in range(int(extra_globals)):
        solve_ids.append(gl_cams[k % len(gl_cams)][abi.CAM_FILM_BACK_W_INCH])
    # the animated camera: pose solved per frame
    fr = np.arange(F, dtype=np.float64)
    ta = np.stack([0.7 + 0.25 * fr, 0.1 + 0.02 * fr, 0.5 - 0.05 * fr], axis=1)
    ra = np.stack([0.4 + 0.3 * np.sin(fr), -1.0 + 0.5 * fr, 0.2 * np.cos(fr)], axis=1)
    ta0 = ta + rng.uniform(-0.05, 0.05, size=ta.shape)
    ra0 = ra + rng.uniform(-1.0, 1.0, size=ra.shape)
    tfm, aids = b.transform(t=tuple(ta0[:, k] for k in range(3)),
                            r=tuple(ra0[:, k] for k in range(3)))
    block_ids = []
    if wide_block:
        wl, wlids = b.lens_3de_classic(distortion=np.full(F, 0.01), curvature_x=np.full(F, -0.01),
                                       curvature_y=np.full(F, 0.01))
        cam, acids = b.camera(tfm, focal=FOCAL_MM * (1.0 + rng.uniform(-0.02, 0.02, F)),
                              film_back=(FILM_W_IN, FILM_H_IN),
                              film_offset=(rng.uniform(-0.01, 0.01, F), rng.uniform(-0.01, 0.01, F)),
                              render_size=RENDER, lens=wl)
        block_ids = [acids[abi.CAM_FOCAL_MM], acids[abi.CAM_FILM_OFFSET_X_INCH],
                     acids[abi.CAM_FILM_OFFSET_Y_INCH]]
        lens_solve = [wlids[0], wlids[2], wlids[3]] + lens_solve  # lens first (B3)
    else:
        cam, _ = b.camera(tfm, focal=FOCAL_MM, film_back=(FILM_W_IN, FILM_H_IN),
                          render_size=RENDER, lens=lens_idx)
    views.append((cam, ta, ra, FOCAL_MM))
    P0 = P * (1.0 + rng.uniform(-0.04, 0.04, size=(B, 1))) if solve_bundles else P
    bids = []
    for j in range(B):
        bt, ids = b.transform(t=tuple(P0[j]))
        b.bundle(bt)
        bids.append(ids)
    for cam, tt, rr, foc in views:
        xy = np.zeros((B, F, 2))
        for f in range(F):
            R = _euler_xyz(*rr[f])
            pc = (P - tt[f]) @ R
            xy[:, f, 0] = foc * pc[:, 0] / (FILM_W_MM * -pc[:, 2])
            xy[:, f, 1] = foc * pc[:, 1] / (FILM_H_MM * -pc[:, 2])
        animated = cam == views[-1][0]
        for j in range(B):
            en = None
            if animated and window is not None:
                s0 = (j * max(F - window, 0)) // max(B - 1, 1)
                en = (fr >= s0) & (fr < s0 + window)
            b.marker(cam, j, _noisy(rng, xy[j]), enable=en)
    for a in lens_solve + solve_ids:
        b.solve(a)
    for a in list(aids[0:6]) + block_ids:
        b.solve(a)
    if solve_bundles:
        for j in range(B):
            for a in bids[j][:3]:
                b.solve(a)
    return b.build(meta={"name": "witness"})


def config_options(prob: Problem, scene_graph_mode=abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH,
                   **overrides):
    """Solver options for a synthetic config (lmder, forward FD,
    delta 1e-4, tau 1, mode 1, tolerances 1e-6; C1 uses lmdif with iterMax 1000)."""
    from .options import make_options
    kw = dict(solver_type=prob.meta.get("solver_type", abi.SOLVER_TYPE_CMINPACK_LMDER),
              iterations=prob.meta.get("iterations", 1000), scene_graph_mode=scene_graph_mode,
              image_width=IMAGE_WIDTH)
    kw.update(overrides)
    return make_options(**kw)
