"""Diagnostic: x error vs the oracle for unsharded and sharded GPU solves."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from mayamatchmovesolver_amd import synthetic as S
from mayamatchmovesolver_amd.solver import Context, Solver
from oracle import refcpu as R
from tests.test_gpu_sharded import run_sharded

def xerr(a, b):
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-3)))

for idx, kw, ns in [(3, dict(frames=40, scale=0.004, window=6, depth=(4.0, 10.0)), 2),
                    (3, dict(frames=60, scale=0.004, window=6, depth=(4.0, 10.0)), 3),
                    (1, dict(frames=24, scale=0.05), 2), (4, dict(frames=32, scale=0.05), 2)]:
    prob = S.make_config(idx, **kw)
    opt = S.config_options(prob)
    xr, fr, eur, edr, rr, trr = R.solve(prob, opt)
    ctx = Context(0)
    s = Solver(prob, opt, context=ctx)
    o1 = s.solve()
    s.close()
    line = "%d %s n=%d M=%d | oracle it=%d info=%d | gpu1 it=%d xerr=%.2e trerr=%.2e" % (
        idx, kw, prob.num_params, prob.num_obs, rr.outer_iterations, rr.reason_number,
        o1.result["outer_iterations"], xerr(o1.x, xr),
        float(np.max(np.abs(o1.fnorm_trace[:len(trr)] - trr[:len(o1.fnorm_trace)]) / trr[0])))
    if ns > 1:
        o2 = run_sharded(prob, opt, ns)[0]
        line += " | shard%d it=%d xerr=%.2e vs1=%.2e" % (ns, o2.result["outer_iterations"],
                                                        xerr(o2.x, xr), xerr(o2.x, o1.x))
    print(line, flush=True)
