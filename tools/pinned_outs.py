"""A/B: the caller's output buffers (fvec, errorList, errorDistanceList) in
pageable vs page-locked host memory (mmba_host_alloc) for repeated solves."""
import sys
import time

import numpy as np

from mayamatchmovesolver_amd import synthetic as S
from mayamatchmovesolver_amd.solver import Context, Solver

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 1
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
prob = S.make_config(cfg)
opt = S.config_options(prob)
ctx = Context(0)
sv = Solver(prob, opt, context=ctx)
m, M = prob.num_residuals, prob.num_obs


def run(outs, label):
    for _ in range(2):
        sv.solve(out=outs)
    ctx.synchronize()
    t0 = time.perf_counter()
    it = 0
    for _ in range(steps):
        r = sv.solve(out=outs)
        it += r.result["outer_iterations"]
    ctx.synchronize()
    dt = time.perf_counter() - t0
    print("%-10s %.3f ms/solve  %.1f it/s" % (label, 1e3 * dt / steps, it / dt), flush=True)


run((np.zeros(m), np.zeros(m), np.zeros(M)), "pageable")
from mayamatchmovesolver_amd.solver import host_array  # noqa: E402

run((host_array(m), host_array(m), host_array(M)), "pinned")
run((np.zeros(m), np.zeros(m), np.zeros(M)), "pageable")
sv.close()
ctx.close()
