"""Diagnostic: the weak-scaling bench scene (N x 500 frames) solved unsharded
and through the group entry with N in-process shards on device 0 in each
reduced-solve form; prints reason, iterations, RMS and the first ||f|| of
each trace.  usage: python tools/shard_diag.py N [max_evals]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from mayamatchmovesolver_amd import abi, synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Context, Solver, set_path  # noqa: E402

n = int(sys.argv[1])
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 200
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 500 * n
prob = S.make_config(3, frames=frames, scale=frames / 500.0)
opt = S.config_options(prob, iterations=cap)
runs = [("unsharded", None, {}), ("default", n, {}), ("whole", n, {abi.PATH_SHARD_SEP: 0}),
        ("separator", n, {abi.PATH_SHARD_SEP: 1}), ("partitioned", n, {abi.PATH_SHARD_BCR: 0})]
ref = None
for name, shards, pins in runs:
    for k, v in pins.items():
        set_path(k, v)
    ctx = Context(0) if shards is None else Context.multi([0] * shards)
    s = Solver(prob, opt, context=ctx)
    st = s.kernel_stats()
    t0 = time.perf_counter()
    o = s.solve()
    dt = time.perf_counter() - t0
    s.close()
    ctx.close()
    for k in pins:
        set_path(k, -1)
    r = o.result
    line = {"run": name, "band_solver": st["band_solver"], "reason": r["reason_number"],
            "evals": r["iterations"], "outer": r["outer_iterations"], "rms": r["error_rms"],
            "s": round(dt, 3), "trace": [float("%.10g" % v) for v in o.fnorm_trace[:8]]}
    if ref is None:
        ref = o
    else:
        k = min(len(o.fnorm_trace), len(ref.fnorm_trace))
        line["trace_rel_dev"] = float(np.max(np.abs(o.fnorm_trace[:k] - ref.fnorm_trace[:k]) /
                                             ref.fnorm_trace[:k]))
        line["first_dev_eval"] = int(np.argmax(np.abs(o.fnorm_trace[:k] - ref.fnorm_trace[:k]) >
                                               1e-6 * ref.fnorm_trace[:k]))
    print(json.dumps(line), flush=True)
