"""Markers of shim scenes 2 / 3 (tests/shim/shim_core_test.cpp,
tests/test_shim_core.py::python_scene): the oracle's forward model (layered
lens, rolling shutter 0.5, the scanline time taken from the marker's own y)
evaluated at a "true" pose and lens -- rotations offset from the scene's
starting values by up to ~1.5 degrees, classic distortion 0.025 instead of
0.02 -- so the solve has an exact answer to find.  The printed 17-digit
literals are pasted into both files (the C++ and Python scenes must hold the
same bits).  Run from the repo root: python tests/shim/gen_scene2_markers.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from mayamatchmovesolver_amd import make_options  # noqa: E402
from oracle import refcpu as R  # noqa: E402
from test_shim_core import python_scene  # noqa: E402  (its markers are what this prints)


def main():
    q = python_scene(2)
    F = q.num_frames
    f = np.arange(F, dtype=np.float64)
    x = q.x0.copy()
    # parameters: rx, ry, rz per frame (frame-minor), then the distortion
    x[0:F] += 1.2 * np.sin(f + 1.0)
    x[F:2 * F] += -0.8 + 0.4 * f
    x[2 * F:3 * F] += 0.6 * np.cos(2.0 * f)
    x[3 * F] = 0.025
    opt = make_options(iterations=100)
    # the film-fit corrected marker must equal the reprojected point, and the
    # scanline time reads the marker's own y: iterate to the fixed point
    # (the film-fit correction scales each axis: marker = k * obs_xy)
    pts, mkr = R.reproject_obs(q, opt, x)
    k = np.ones(2)
    for a in range(2):
        nz = np.nonzero(q.obs_xy[a::2])[0][0]
        k[a] = mkr[2 * nz + a] / q.obs_xy[2 * nz + a]
    kk = np.tile(k, q.num_obs)
    for _ in range(200):
        pts, mkr = R.reproject_obs(q, opt, x)
        if np.max(np.abs(pts - mkr)) < 1e-16:
            break
        q.obs_xy = q.obs_xy + (pts - mkr) / kk
    f, _eu, _ed, _st = R.measure(q, opt, x)
    assert np.max(np.abs(f)) < 1e-9, np.max(np.abs(f))
    # ~0.2 px of marker noise: the solution is a well-defined least-squares
    # minimum, not an exact fit at the finite differences' noise floor
    q.obs_xy = q.obs_xy + 1e-4 * np.random.default_rng(7).standard_normal(q.obs_xy.size)
    print("MARKERS = [")
    for i in range(q.num_obs):
        print("    (%.17g, %.17g)," % (q.obs_xy[2 * i], q.obs_xy[2 * i + 1]))
    print("]")


if __name__ == "__main__":
    main()
