"""Oracle x after the first full LM step (iterations = 2: x0 and one step) of
the C4-spec scenes the sharded valley test runs at 4 and 8 shards
(tests/test_gpu_sharded.py::test_sharded_ba_x_before_the_valley), so the
sharded forms can be held against the reference instead of only against the
unsharded GPU solve.  Run from the repo root:

    python tests/golden/make_shard_step.py

Writes tests/golden/shard/c4_shard_step.npz: for n in (4, 8), x_n (the
oracle's x), trace_n, and cond_n (the condition number of J^T J at x0, which
bounds how closely any fp64 solve pins the step: about cond * 1e-16)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mayamatchmovesolver_amd import synthetic as S  # noqa: E402
from oracle import refcpu as R  # noqa: E402


def main():
    out = {}
    for n in (4, 8):
        prob = S.make_config(3, frames=20 * n, scale=0.002 * n)
        opt = S.config_options(prob, iterations=2)
        x, _, _, _, rr, tr = R.solve(prob, opt)
        _, J = R.jacobian(prob, opt, np.asarray(prob.x0))
        w = np.linalg.eigvalsh(J.T @ J)
        out["x_%d" % n] = x
        out["trace_%d" % n] = tr
        out["cond_%d" % n] = np.float64(w[-1] / w[0])
        print(n, rr.reason_number, rr.iterations, "cond %.3e" % out["cond_%d" % n], flush=True)
    path = os.path.join(ROOT, "tests", "golden", "shard", "c4_shard_step.npz")
    np.savez_compressed(path, **out)
    print("wrote", path)


if __name__ == "__main__":
    main()
