"""Round-6 diagnostic: the one-step x of the C4-spec sharded-test scenes
(tests/golden/shard/c4_shard_step.npz, the oracle's step) through the
unsharded solver with each parallel-cyclic-reduction pivot chain
(MMBA_PATH_PCR_CHAIN 0 = one-pivot Cholesky, the default; 1 = 2 x 2 pivots) and the
block cyclic reduction (MMBA_PATH_PCR = 0): ||f|| after the step and the
largest relative deviation of x from the oracle's."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mayamatchmovesolver_amd import abi, synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Context, Solver, set_path  # noqa: E402

fx = np.load(os.path.join(ROOT, "tests/golden/shard/c4_shard_step.npz"))
ctx = Context(0)
for n in (4, 8):
    prob = S.make_config(3, frames=20 * n, scale=0.002 * n)
    opt = S.config_options(prob, iterations=2)
    xo, tro = fx["x_%d" % n], fx["trace_%d" % n]
    for name, paths in (("chol", {abi.PATH_PCR_CHAIN: 0}), ("ldl2", {abi.PATH_PCR_CHAIN: 1}),
                        ("ldl1", {abi.PATH_PCR_CHAIN: 2}),
                        ("bcr", {abi.PATH_PCR: 0})):
        for k in range(1, abi.PATH_NUM):
            set_path(k, -1)
        for k, v in paths.items():
            set_path(k, v)
        s = Solver(prob, opt, context=ctx)
        try:
            out = s.solve()
        finally:
            s.close()
        dx = np.max(np.abs(out.x - xo) / np.maximum(np.abs(xo), 1e-3))
        print("n=%d %-5s trace %s oracle %s  df %.2e  max rel dx %.2e" % (
            n, name, np.array2string(out.fnorm_trace, precision=9),
            np.array2string(tro, precision=9), abs(out.fnorm_trace[-1] - tro[-1]) / tro[-1], dx),
            flush=True)
for k in range(1, abi.PATH_NUM):
    set_path(k, -1)
ctx.close()
