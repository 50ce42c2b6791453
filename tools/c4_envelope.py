#!/usr/bin/env python3
"""How closely the reference's lmder determines x on the C4 structure.

For each row: the CPU oracle (oracle/refcpu.c) solves the scene, then solves
it again from x0 perturbed by ~1 ulp (relative 1e-15, 3 seeds); the
"envelope" is the largest relative change of any x component.  A GPU result
cannot be pinned to the reference closer than that, whatever its arithmetic.
Rows vary the scene size, the stopping tolerances and the evaluation budget;
the last block gives the singular values of J at the solution and the final
||f|| of the perturbed runs (the objective is flat along the direction x
moves: far bundles on a 1.5-unit baseline, 0.5 px marker noise, forward
differences with delta 1e-4).

Run from the repo root (CPU only, ~3 minutes):
    python tools/c4_envelope.py > profiles/r2_parity/c4_envelope.txt
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mayamatchmovesolver_amd import synthetic as S  # noqa: E402
from oracle import refcpu as R  # noqa: E402


def envelope(prob, opt, seeds=3):
    t = time.time()
    x, fv, _eu, _ed, res, _tr = R.solve(prob, opt)
    dt = time.time() - t
    env, fns = 0.0, []
    for seed in range(seeds):
        rng = np.random.default_rng(seed)
        x0p = prob.x0 * (1.0 + 1e-15 * rng.standard_normal(prob.x0.size))
        xp, fp = R.solve(prob, opt, x0=x0p)[:2]
        env = max(env, float(np.max(np.abs(xp - x) / np.maximum(np.abs(x), 1e-3))))
        fns.append(float(np.linalg.norm(fp)))
    return x, fv, res, env, fns, dt


def row(tag, prob, opt):
    x, fv, res, env, fns, dt = envelope(prob, opt)
    print("%-34s n=%4d m=%5d reason=%d evals=%3d  ||f||=%.9e  envelope=%.1e  (%.1f s)" % (
        tag, prob.num_params, prob.num_residuals, res.reason_number, res.function_evals,
        float(np.linalg.norm(fv)), env, dt), flush=True)
    return x, fv, fns


def main():
    print("# oracle x envelope on the C4 structure (1 camera, 4-frame tracks, depth 20-200)")
    print("# default options: lmder, forward FD delta 1e-4, tolerances 1e-6, iterMax 1000")
    for frames, scale in ((8, 0.001), (8, 0.002), (12, 0.002), (16, 0.002)):
        prob = S.make_config(3, frames=frames, scale=scale)
        row("f%d scale %.3f" % (frames, scale), prob, S.config_options(prob))
    print("# tighter stopping tolerances do not determine x (the valley is flat)")
    prob = S.make_config(3, frames=16, scale=0.002)
    for eps in (1e-10, 1e-14):
        row("f16 scale 0.002 tol %.0e" % eps, prob,
            S.config_options(prob, epsilon1=eps, epsilon2=eps, epsilon3=eps))
    print("# evaluation budget capped: x determined before the valley")
    for frames, scale in ((16, 0.002), (32, 0.004)):
        p = S.make_config(3, frames=frames, scale=scale)
        for it in (2, 3, 4, 6, 10):
            row("f%d scale %.3f iterations %d" % (frames, scale, it), p,
                S.config_options(p, iterations=it))
    print("# c4_f16 at the solution: singular values of J and ||f|| of the perturbed runs")
    opt = S.config_options(prob)
    x, fv, fns = row("f16 scale 0.002", prob, opt)
    _f, J = R.jacobian(prob, opt, x)
    s = np.linalg.svd(J, compute_uv=False)
    print("sigma_max %.3e  sigma_min %.3e  cond %.1e" % (s[0], s[-1], s[0] / s[-1]))
    print("perturbed-run ||f||:", " ".join("%.9e" % v for v in fns),
          " (relative spread %.1e)" % ((max(fns) - min(fns)) / float(np.linalg.norm(fv))))


if __name__ == "__main__":
    main()
