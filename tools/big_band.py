"""The reduced band system every rank solves in the whole-S sharded form, on
one device: the C4 structure over N x 500 frames solved unsharded (the
same nb = N x 2,994 band system), with the builder's reduced solver and
with block cyclic reduction pinned (MMBA_PATH_PCR = 0).  Prints per run the
band solver, LM reason / iterations, seconds per solve (median of 3 after a
warm-up) and, from one more solve with the plan's timers on, the reduced
solve's event time per damped solve.
usage: python tools/big_band.py N [N ...]"""
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mayamatchmovesolver_amd import abi, synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Context, Solver, set_path  # noqa: E402

ctx = Context(0)
for n in [int(a) for a in sys.argv[1:]] or [8]:
    frames = 500 * n
    prob = S.make_config(3, frames=frames, scale=frames / 500.0)
    opt = S.config_options(prob, iterations=40)
    for name, pins in (("default", {}), ("bcr", {abi.PATH_PCR: 0})):
        for k, v in pins.items():
            set_path(k, v)
        s = Solver(prob, opt, context=ctx)
        try:
            s.solve()  # warm-up
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                o = s.solve()
                ts.append(time.perf_counter() - t0)
            s.set_timing(True)  # the reduced solve's event time, in a separate solve
            s.solve()
            st = s.kernel_stats()
            s.set_timing(False)
        finally:
            s.close()
            for k in pins:
                set_path(k, -1)
        r = o.result
        print(json.dumps({"N": n, "run": name, "band_solver": st.get("band_solver"),
                          "reduced_dim": st.get("reduced_dim"), "reason": r["reason_number"],
                          "iterations": r["iterations"], "rms": r["error_rms"],
                          "reduced_solve_us": 1e3 * st["chol_ms_avg"],
                          "reduced_solves": st["chol_launches"],
                          "s_per_solve": statistics.median(ts),
                          "ms_per_iteration": 1e3 * statistics.median(ts) / max(1, r["iterations"])}),
              flush=True)
ctx.close()
