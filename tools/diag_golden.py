"""Diagnostic: GPU solve of one golden fixture, per-parameter deviation from the oracle."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.golden import make_golden as G
from mayamatchmovesolver_amd.solver import Solver, Context
name = sys.argv[1]
prob, opt, d = G.load(name)
ctx = Context(0)
s = Solver(prob, opt, context=ctx)
out = s.solve()
s.close()
xr = d["exp_x"]
rel = np.abs(out.x - xr) / np.maximum(np.abs(xr), 1e-3)
k = int(np.argmax(rel))
print(name, "iters", out.result["outer_iterations"], "max rel %.3e at p=%d (attr %d frame %d) x=%.12g ref=%.12g" % (
    rel[k], k, prob.param_attr[k], prob.param_frame[k], out.x[k], xr[k]))
print("norm rel %.3e" % (np.linalg.norm(out.x - xr) / np.linalg.norm(xr)))
print("trace rel max %.3e" % np.max(np.abs(out.fnorm_trace - d["exp_trace"]) / d["exp_trace"]))
print("top5 rel", np.sort(rel)[-5:])
