"""Oracle x after the first full LM step (iterations = 2: x0 and one step) of
the C4-spec scenes the sharded valley test runs at 4 and 8 shards
(tests/test_gpu_sharded.py::test_sharded_ba_x_before_the_valley), so the
sharded forms can be held against the reference instead of only against the
unsharded GPU solve.  Run from the repo root:

    python tests/golden/make_shard_step.py

Writes tests/golden/shard/c4_shard_step.npz: for n in (4, 8), x_n (the
oracle's x), trace_n, and cond_n (the condition number of J^T J at x0, which
bounds how closely any fp64 solve pins the step: about cond * 1e-16).

Round 6: also undet_n / sigma_n, the step's
undetermined directions exactly as tests/golden/make_steps.py defines them
(right singular vectors of the oracle's J at the step's start x0, columns
scaled by max(|x_n|, 1e-3), with sigma < make_steps.RATIO sigma_max; RATIO
fixed there before any GPU run), so the sharded step is held at 1e-6 against
the ORACLE's step once those directions are projected out
(make_steps.determined_dx).  ``--basis`` adds them to an existing fixture
without touching x_n / trace_n / cond_n."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from mayamatchmovesolver_amd import synthetic as S  # noqa: E402
from oracle import refcpu as R  # noqa: E402
from tests.golden.make_steps import undetermined_basis  # noqa: E402

PATH = os.path.join(ROOT, "tests", "golden", "shard", "c4_shard_step.npz")


def add_basis():
    out = dict(np.load(PATH, allow_pickle=False))
    for n in (4, 8):
        prob = S.make_config(3, frames=20 * n, scale=0.002 * n)
        opt = S.config_options(prob, iterations=2)
        scale = np.maximum(np.abs(out["x_%d" % n]), 1e-3)
        Vu, sv = undetermined_basis(prob, opt, np.asarray(prob.x0, dtype=np.float64), scale)
        out["undet_%d" % n] = Vu
        out["sigma_%d" % n] = sv
        print(n, "undetermined %d of %d (scaled cond %.2e)" % (Vu.shape[1], sv.size, sv[0] / sv[-1]),
              flush=True)
    np.savez_compressed(PATH, **out)
    print("wrote", PATH)


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
    np.savez_compressed(PATH, **out)
    print("wrote", PATH)
    add_basis()


if __name__ == "__main__":
    if "--basis" in sys.argv[1:]:
        add_basis()
    else:
        main()
