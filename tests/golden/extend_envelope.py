#!/usr/bin/env python3
"""Widen the sample behind a full-size fixture's ``exp_x_envelope`` (see
make_full_golden.py): more oracle runs from x0 perturbed by ~1 ulp
(relative 1e-15), each seed one process, then --combine folds every seed's x
into the envelope (the largest relative move of any component against the
fixture's exp_x) and ``envelope_runs``; every other field stays.

    python tests/golden/extend_envelope.py --case c4_w10_full --seed 1   # per seed
    python tests/golden/extend_envelope.py --case c4_w10_full --combine
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.golden import make_full_golden as FG  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--combine", action="store_true")
    a = ap.parse_args()
    if a.seed is not None:
        from oracle import refcpu as R
        prob, opt, _d = FG.load(a.case)
        rng = np.random.default_rng(a.seed)
        x0 = prob.x0 * (1.0 + 1e-15 * rng.standard_normal(prob.x0.size))
        x = R.solve(prob, opt, x0=x0)[0]
        os.makedirs(FG.PARTS, exist_ok=True)
        np.save(os.path.join(FG.PARTS, "%s_env_s%d.npy" % (a.case, a.seed)), x)
    if a.combine:
        path = os.path.join(FG.FULL, a.case + ".npz")
        d = dict(np.load(path, allow_pickle=False))
        x = d["exp_x"]
        env, runs = float(d["exp_x_envelope"]), int(d["envelope_runs"])
        for f in sorted(os.listdir(FG.PARTS)):
            if f.startswith(a.case + "_env_s"):
                xp = np.load(os.path.join(FG.PARTS, f), allow_pickle=False)
                env = max(env, float(np.max(np.abs(xp - x) / np.maximum(np.abs(x), 1e-3))))
                runs += 1
        d["exp_x_envelope"] = np.array(env)
        d["envelope_runs"] = np.array(runs)
        np.savez_compressed(path, **d)
        print("%s: x-envelope %.3e over %d runs" % (a.case, env, runs))


if __name__ == "__main__":
    main()
