"""Diagnostics for the rolling shutter with solved bundles (GPU): the solve
under each reduced-system path pin, and the first iterations against the
oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mayamatchmovesolver_amd import abi, synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Context, Solver, set_path
from oracle import refcpu as R

prob = S.edge_scene(parented=False, solve_bundles=True)
prob.cam_rs_value = np.array([0.6])
ctx = Context(0)
for pins in ({}, {abi.PATH_PCR: 0}, {abi.PATH_PCR: 0, abi.PATH_BCR_DATAFLOW: 0}):
    for k, v in pins.items():
        set_path(k, v)
    for it in (1, 2, 3, 100):
        opt = S.config_options(prob, scene_graph_mode=1, iterations=it)
        xr, fr, _, _, rr, trr = R.solve(prob, opt)
        s = Solver(prob, opt, context=ctx)
        try:
            st = s.kernel_stats()
            try:
                out = s.solve()
                dx = np.max(np.abs(out.x - xr) / np.maximum(np.abs(xr), 1e-3))
                print(pins, it, "band_solver", st["band_solver"], "reason", out.result["reason_number"],
                      rr.reason_number, "trace", out.fnorm_trace[:4], trr[:4], "dx %.2e" % dx, flush=True)
            except Exception as e:  # noqa: BLE001
                print(pins, it, "band_solver", st["band_solver"], "FAILED", e, "oracle", trr[:4], flush=True)
        finally:
            s.close()
    for k in pins:
        set_path(k, -1)
