"""Diagnostic: repeatability of the C4-structure solve with the dataflow BCR
factor (default) and the per-level launches (MMBA_BCR_DF=0)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mayamatchmovesolver_amd import synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Context, Solver  # noqa: E402

prob = S.make_config(3, frames=120, scale=0.02)
opt = S.config_options(prob)
ctx = Context(0)
s = Solver(prob, opt, context=ctx)
outs = [s.solve() for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6)]
ref = outs[0]
for i, o in enumerate(outs):
    tr, rt = o.fnorm_trace, ref.fnorm_trace
    n = min(len(tr), len(rt))
    d = np.flatnonzero(tr[:n] != rt[:n])
    print(os.environ.get("MMBA_BCR_DF", "df"), i, o.result["reason_number"], o.result["iterations"],
          o.result["function_evals"], "len", len(tr), "first diff", d[:1],
          "rel %.1e" % (np.max(np.abs(tr[:n] - rt[:n]) / rt[:n]) if n else 0),
          "x %.1e" % np.max(np.abs(o.x - ref.x) / np.maximum(np.abs(ref.x), 1e-3)), flush=True)
s.close()
ctx.close()
