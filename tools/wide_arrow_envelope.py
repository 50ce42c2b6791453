#!/usr/bin/env python3
"""How closely the reference's lmder determines x on the wide-arrow witness
rigs (tests/test_gpu_wide_arrow.py): the CPU oracle solves each rig, then
solves it again from x0 perturbed by ~1 ulp (relative 1e-15, 3 seeds); the
envelope is the largest relative change of any x component (as
tools/c4_envelope.py).  The windowed rigs (the animated camera seen through
3-frame bundle windows over 8-12 frames) are the ones the BCR test no longer
uses; the 4 / 5-frame rigs are the ones it does.

Run from the repo root (CPU only, ~2 minutes):
    python tools/wide_arrow_envelope.py > profiles/r4_parity/wide_arrow_envelope.txt
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mayamatchmovesolver_amd import make_options, synthetic as S  # noqa: E402
from oracle import refcpu as R  # noqa: E402


def row(tag, prob, opt, seeds=3):
    t = time.time()
    x, fv, _eu, _ed, res, _tr = R.solve(prob, opt)
    env = 0.0
    fns = []
    for seed in range(seeds):
        rng = np.random.default_rng(seed)
        x0p = prob.x0 * (1.0 + 1e-15 * rng.standard_normal(prob.x0.size))
        xp, fp, _e, _d, rp, _t = R.solve(prob, opt, x0=x0p)
        env = max(env, float(np.max(np.abs(xp - x) / np.maximum(np.abs(x), 1e-3))))
        fns.append("%d/%d" % (rp.reason_number, rp.function_evals))
    print("%-40s n=%4d m=%5d reason=%d evals=%4d ||f||=%.9e envelope=%.1e perturbed=%s (%.1f s)" % (
        tag, prob.num_params, prob.num_residuals, res.reason_number, res.function_evals,
        float(np.linalg.norm(fv)), env, ",".join(fns), time.time() - t), flush=True)


def main():
    print("# oracle x envelope on the witness rigs (lmder, forward FD delta 1e-4, tol 1e-6)")
    print("# the rigs the BCR test uses")
    for kw in (dict(frames=4), dict(frames=5, n_witness=5, n_focal=5)):
        row("witness %s" % kw, S.witness_scene(**kw), make_options())
    print("# windowed visibility (3-frame bundle windows), the rigs it stopped using")
    for kw in (dict(frames=8, window=3), dict(frames=12, window=3),
               dict(frames=12, window=3, n_witness=5, n_focal=5)):
        row("witness %s" % kw, S.witness_scene(**kw), make_options())


if __name__ == "__main__":
    main()
