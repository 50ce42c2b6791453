"""Sharded-path timing on ONE GPU: N shards in one process over the in-process
communicator (one thread + stream per shard, all on device 0), weak scaling as
bench.py does it (N x 500 frames).  The shards share the GPU, so this is not
an N-GPU number; it shows the per-iteration latency of the sharded algorithm
(partitioned band solve, all-reduces) against the unsharded one.
usage: python tools/shard_bench.py N [steps]"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mayamatchmovesolver_amd import synthetic as S  # noqa: E402
from mayamatchmovesolver_amd.solver import Comm, Context, Solver  # noqa: E402

n = int(sys.argv[1])
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
prob = S.make_config(3, frames=500 * n, scale=float(n))
opt = S.config_options(prob)
comms = Comm.local_group(n) if n > 1 else [None]
ctxs = [Context(0) for _ in range(n)]
solvers = [None] * n
res = [None] * n
bar = threading.Barrier(n)
times = [0.0] * n


def work(r):
    s = Solver(prob, opt, context=ctxs[r], comm=comms[r])
    solvers[r] = s
    s.solve()  # warm-up
    bar.wait()
    t0 = time.perf_counter()
    for _ in range(steps):
        res[r] = s.solve()
    ctxs[r].synchronize()
    times[r] = time.perf_counter() - t0
    s.close()


ths = [threading.Thread(target=work, args=(r,)) for r in range(n)]
for t in ths:
    t.start()
for t in ths:
    t.join()
dt = max(times)
r = res[0].result
print(json.dumps({"shards": n, "frames": prob.num_frames, "obs": prob.num_obs,
                  "ms_per_solve": 1e3 * dt / steps, "iterations": r["outer_iterations"],
                  "ms_per_iteration": 1e3 * dt / steps / r["outer_iterations"],
                  "rms": r["error_rms"], "reason": r["reason_number"]}))
