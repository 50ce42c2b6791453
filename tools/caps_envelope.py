#!/usr/bin/env python3
"""The oracle's own x envelope on the raised-capacity rigs of
tests/test_gpu_caps.py (the method of tools/wide_arrow_envelope.py: solve, then
solve again from x0 perturbed by ~1 ulp, relative 1e-15, 3 seeds; the
envelope is the largest relative change of any x component, floor 1e-3).  A
rig whose envelope approaches the tests' 1e-6 bar cannot hold it.

Run from the repo root (CPU only):
    python tools/caps_envelope.py > profiles/r6_caps/caps_envelope.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from mayamatchmovesolver_amd import abi, make_options, synthetic as S  # noqa: E402
from wide_arrow_envelope import row  # noqa: E402

DAG, MMSG = abi.SCENE_GRAPH_MODE_MAYA_DAG, abi.SCENE_GRAPH_MODE_MM_SCENE_GRAPH


def main():
    print("# oracle x envelope on the capacity rigs (lmder, forward FD delta 1e-4, tol 1e-6)")
    p = S.make_config(4, frames=8, scale=0.05, lens_model="classic_wide", cameras=1)
    row("12-parameter camera-frames", p, S.config_options(p))
    for kw in (dict(n_witness=6, n_focal=6, extra_globals=1, frames=4),
               dict(n_witness=6, n_focal=6, extra_globals=1),
               dict(n_witness=6, n_focal=6, extra_globals=1, frames=8),
               dict(n_witness=6, n_focal=6, extra_globals=1, bundles=40),
               dict(n_witness=6, n_focal=6, extra_globals=1, solve_bundles=False)):
        for mode in (DAG, MMSG):
            row("40 globals %s mode %d" % (kw, mode), S.witness_scene(**kw),
                make_options(scene_graph_mode=mode))


if __name__ == "__main__":
    main()
