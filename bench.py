#!/usr/bin/env python3
"""Benchmark: mmSolver LM bundle adjustment on MI355X (libmmba.so).

Metric (BASELINE.json): LM iterations/sec + residuals/sec (markers x frames)
at 1/2/4/8 MI355X; final RMS reprojection error.  Workload: configs[3],
"500 cameras, 50k bundles, 200k observations" (one animated
camera x 500 frames, 50k bundles, 4-frame tracks, 152,991 parameters).  One
step = one full LM solve of the scene from its initial guess, with the problem
already resident in HBM (the plan is uploaded before the timed region); every
solve hands errorList / ud->errorList / errorDistanceList back to the caller's
page-locked host buffers, as the seam's caller needs them.  The same solves
leaving those outputs in HBM (mmba_plan_outputs) are timed beside it
(`device_resident`).

`value` is whole-job residuals/s: observations x (residual evaluations +
Jacobian evaluations) per second (SURVEY 8(d) metric definitions); LM
iterations/s is reported beside it.

Multi-GPU: weak scaling, the per-GPU shard is the C4 scene -- N GPUs solve
ONE N x 500-frame scene (N x 50k bundles, N x 200k observations)
frame-sharded over the GPUs, the library exchanging over RCCL (xGMI).
  - under torch.distributed.run (WORLD_SIZE = N): one process per GPU, each
    rank a shard (mmba_comm_create_rccl); torch.distributed (gloo) only
    broadcasts the RCCL id and brackets the timed region;
  - run plainly with --gpus N: one process, the seam's single caller, over
    mmba_context_create_multi(devices 0..N-1) (mmba.h ABI 9) -- the library
    drives the N devices from its own threads (ncclCommInitAll).  With fewer
    than N visible devices the N shards run on device 0 (the in-process
    transport), labelled in `config.devices` and `parallelism`: a rehearsal
    of the sharded path, not a multi-GPU measurement.

The CPU baseline (rank 0, N = 1) is the oracle (oracle/refcpu.c, a
cost-faithful restatement of the reference MM-Scene-Graph + cminpack path)
timed single-threaded on full-density frame windows of the same scene (one LM
iteration each), with the GPU timed on the same windows in the same run; the
full scene needs a 490 GB dense Jacobian on the CPU, so its rate is only
reported as a labelled extrapolation.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
FP64_MFMA_PEAK_TF = 78.6  # MI355X dense FP64 matrix rate (spec)
FP64_VALU_PEAK_TF = 78.6  # MI355X FP64 vector rate (spec)
BASE_FRAMES = {1: 120, 2: 500, 3: 500, 4: 240}


_last_note = [time.perf_counter()]


def progress(msg, every=20.0):
    """A line on stderr at most every `every` seconds (long configurations,
    e.g. C3 at ~11 s per solve, would otherwise run silent for minutes)."""
    now = time.perf_counter()
    if now - _last_note[0] >= every:
        _last_note[0] = now
        print("[bench] %s" % msg, file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=3, help="BASELINE.json configs index")
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--lens-model", default="classic",
                    choices=["classic", "classic_animated", "radial", "anamorphic",
                             "anamorphic_rescaled"],
                    help="configs[4] lens model (classic = the C5 spec)")
    ap.add_argument("--rolling-shutter", type=float, default=0.0, metavar="RS",
                    help="configs[4]: rolling-shutter value in frames (time shift x fps; "
                         "the configs[4] per-scanline pose, mmba.h ABI 3)")
    ap.add_argument("--per-frame", type=int, default=0, metavar="CONC",
                    help="per-frame solve mode (mmba_solve_per_frame) with CONC frames at "
                         "once; prints its own JSON line (not the headline metric)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget-s", type=float, default=30.0,
                    help="skip the larger CPU window once this much CPU time is spent")
    ap.add_argument("--no-traffic", action="store_true",
                    help="skip the rocprofv3 PMC passes that fill roofline.traffic")
    ap.add_argument("--path", action="append", default=[], metavar="NAME=VALUE",
                    help="A/B diagnostics: pin a plan-builder choice through the "
                         "mmba_debug_set_path test hook (e.g. pcr=0); the line records it")
    return ap.parse_args()


def apply_paths(args):
    """--path NAME=VALUE -> mmba_debug_set_path(abi.PATH_NAME, VALUE)."""
    from mayamatchmovesolver_amd import abi
    from mayamatchmovesolver_amd.solver import set_path
    pinned = {}
    for item in args.path:
        name, val = item.split("=")
        set_path(getattr(abi, "PATH_" + name.upper()), int(val))
        pinned[name.lower()] = int(val)
    return pinned


def dist_setup():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local, dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def allreduce(dist, v, op="max"):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM)
    return float(t.item())


def allgather_float(dist, v):
    """Every rank's v, in rank order (one value per rank)."""
    if dist is None:
        return [v]
    import torch
    out = [torch.zeros(1, dtype=torch.float64) for _ in range(dist.get_world_size())]
    dist.all_gather(out, torch.tensor([v], dtype=torch.float64))
    return [float(t.item()) for t in out]


def broadcast_bytes(dist, data: bytes | None, n: int) -> bytes:
    import torch
    t = torch.zeros(n, dtype=torch.uint8)
    if data is not None:
        t[:] = torch.frombuffer(bytearray(data), dtype=torch.uint8)
    dist.broadcast(t, src=0)
    return bytes(t.numpy().tobytes())


# Kernels inside the K2 span (Plan::jac: span_begin .. span_end), i.e. the
# launches whose HIP-event time is roofline.avg_ms.
K2_REGEX = "k_jacobian|k_jac_ne|k_ne_|k_colnorms|k_jac_epilogue"
VALU_F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
            "SQ_INSTS_VALU_TRANS_F64")
# the reduced solve's kernels (Plan::solve_damped_enqueue's factorisations) and
# their matrix-core counters: SQ_VALU_MFMA_BUSY_CYCLES counts cycles (summed
# over the SIMDs), SQ_WAVE_CYCLES quad-cycles (MI355X_MICROARCH.md, PMC units)
RED_REGEX = "k_pcr_solve|k_bcr_|k_band_factor|k_dense_|k_dgemm|k_bd_"
MFMA_PASS = ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES")


def pmc_traffic(args):
    """HBM bytes per K2 pass from PMC counters (MI355X_MICROARCH.md, HBM /
    rocprofv3 section): one rocprofv3 --pmc pass per counter (FETCH_SIZE and
    WRITE_SIZE do not fit one pass), each a child process running one solve
    of the same workload, started before this process touches the GPU.
    FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts half the bytes of
    streaming reads, so it is doubled.  Returns (bytes, detail) or (None, why)."""
    import csv
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if prof is None:
        return None, "rocprofv3 not found"
    base = [sys.executable, os.path.abspath(__file__), "--steps", "1", "--warmup", "0",
            "--no-cpu-baseline", "--no-traffic", "--config", str(args.config),
            "--scale", str(args.scale)]
    if args.frames:
        base += ["--frames", str(args.frames)]
    if args.config == 4:
        base += ["--lens-model", args.lens_model, "--rolling-shutter", str(args.rolling_shutter)]
    for item in args.path:
        base += ["--path", item]
    env = dict(os.environ, TMPDIR="/tmp")
    per = {}
    tmp = tempfile.mkdtemp(prefix="mmba_pmc_", dir="/tmp")
    # one pass per counter group: FETCH_SIZE and WRITE_SIZE do not fit one
    # pass; the four fp64 VALU instruction counters (SQ) fit one
    passes = (("FETCH_SIZE",), ("WRITE_SIZE",), VALU_F64, MFMA_PASS)
    try:
        for group in passes:
            out = os.path.join(tmp, group[0])
            rx = RED_REGEX if group is MFMA_PASS else K2_REGEX
            cmd = ["timeout", "-s", "KILL", "150", prof, "--pmc", *group,
                   "--kernel-include-regex", rx, "-d", out, "-o", "k2",
                   "--output-format", "csv", "--"] + base
            r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL,
                               stderr=subprocess.DEVNULL)
            files = [os.path.join(dp, f) for dp, _, fs in os.walk(out) for f in fs
                     if f.endswith("counter_collection.csv")]
            if r.returncode != 0 or not files:
                if group is VALU_F64:  # optional: the traffic stands without it
                    per["valu_error"] = "rocprofv3 --pmc pass failed (rc=%d)" % r.returncode
                    continue
                if group is MFMA_PASS:
                    per["mfma_error"] = "rocprofv3 --pmc pass failed (rc=%d)" % r.returncode
                    continue
                return None, "rocprofv3 --pmc %s pass failed (rc=%d)" % (group[0], r.returncode)
            acc = {}
            for row in csv.DictReader(open(files[0])):
                k = row["Kernel_Name"].split("(")[0]
                c = row.get("Counter_Name", group[0])
                acc.setdefault(c, {}).setdefault(k, []).append(float(row["Counter_Value"]))
            for c, kv in acc.items():
                per[("red:" if group is MFMA_PASS else "") + c] = {
                    k: sum(v) / len(v) for k, v in kv.items()}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = sum(per["FETCH_SIZE"].values()) * 1024.0
    write = sum(per["WRITE_SIZE"].values()) * 1024.0
    valu = None
    if all(c in per for c in VALU_F64):
        # fp64 flops per K2 pass from the instruction counts (per wave, 64
        # lanes): 2 per FMA, 1 per add / mul / transcendental
        n = {c: sum(per[c].values()) for c in VALU_F64}
        flops = 64.0 * (2.0 * n["SQ_INSTS_VALU_FMA_F64"] + n["SQ_INSTS_VALU_ADD_F64"] +
                        n["SQ_INSTS_VALU_MUL_F64"] + n["SQ_INSTS_VALU_TRANS_F64"])
        valu = {"flops_per_launch": flops, "instructions_per_launch": n,
                "per_kernel": {c: per[c] for c in VALU_F64},
                "note": "64 x (2 FMA + ADD + MUL + TRANS) fp64 VALU instructions, rocprofv3 "
                        "--pmc, averaged per launch, summed over the K2 kernels"}
    mfma = None
    if all("red:" + c in per for c in MFMA_PASS):
        # per launch of each reduced-solve kernel: matrix-core busy cycles and
        # the waves' lifetime (quad-cycles x 4)
        mfma = {k: {"mfma_busy_cycles": per["red:SQ_VALU_MFMA_BUSY_CYCLES"][k],
                    "valu_instructions": per["red:SQ_INSTS_VALU"].get(k),
                    "waves": per["red:SQ_WAVES"].get(k),
                    "wave_cycles": 4.0 * per["red:SQ_WAVE_CYCLES"].get(k, 0.0)}
                for k in per["red:SQ_VALU_MFMA_BUSY_CYCLES"]}
    detail = {"fetch_size_bytes_raw": fetch, "write_size_bytes": write,
              "valu_f64": valu, "valu_error": per.get("valu_error"),
              "reduced_solve_mfma": mfma, "mfma_error": per.get("mfma_error"),
              "per_kernel_kib": {"FETCH_SIZE": per["FETCH_SIZE"],
                                 "WRITE_SIZE": per["WRITE_SIZE"]},
              "correction": "traffic = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE "
                            "halving, MI355X_MICROARCH.md HBM section), averaged per launch "
                            "over one solve, summed over the K2 kernels (%s)" % K2_REGEX}
    return 2.0 * fetch + write, detail


# Full-density frame windows of the workload timed on the CPU: the same
# scene generator with the window's share of bundles (C4: 100 new bundles per
# frame, each tracked over 4 frames), i.e. the full C4 density on F' frames.
# Sized so the largest window's oracle iteration takes ~10-30 s (cost ~ F'^3:
# the full C2 iteration is ~980 s on 120 frames, the full C5 ~3,860 s on 240).
CPU_WINDOWS = {3: (5, 10), 2: (2, 3), 1: (12, 32), 4: (16, 40), 0: (10,)}


def _pinned_core():
    """One core of this process's CPU set (the reference solve is single
    threaded: `taskset -c <core>` for the oracle's timed calls)."""
    try:
        return min(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return None


def _window(cfg_index, frames):
    from mayamatchmovesolver_amd import synthetic as S
    base = BASE_FRAMES.get(cfg_index, 10)
    if cfg_index == 0:
        return S.make_config(0)
    return S.make_config(cfg_index, frames=frames, scale=frames / base)


def cpu_baseline(cfg_index, budget_s, ctx):
    """The oracle (oracle/refcpu.c: cost-faithful restatement of the reference
    MM-Scene-Graph + cminpack lmder path, single thread) TIMED on full-density
    frame windows of the benchmarked scene, one LM iteration each (lmder
    iterMax 2: initial evaluation, one FD Jacobian + QR + lmpar, one trial
    point); the GPU runs the identical call on the identical window in the
    same process, so the ratio is measured, not modelled.  The full C4 scene
    needs a 490 GB dense Jacobian on the CPU; its per-iteration time is only
    given as a separately labelled extrapolation (t ~ m n^2, the QR term)."""
    from mayamatchmovesolver_amd import synthetic as S
    from mayamatchmovesolver_amd.solver import Solver
    from oracle import refcpu as R

    full = S.make_config(cfg_index)
    n_full, m_full = full.num_params, full.num_residuals
    del full
    samples = []
    spent = 0.0
    core = _pinned_core()
    for frames in CPU_WINDOWS.get(cfg_index, (2,)):
        if samples and spent > budget_s:
            break
        p = _window(cfg_index, frames)
        o = S.config_options(p, iterations=2)
        R.lib()  # loaded outside the timing
        # the oracle call runs pinned to one core (taskset -c <core>): the
        # reference solve is single threaded on Maya's main thread
        prev = os.sched_getaffinity(0) if core is not None else None
        if core is not None:
            os.sched_setaffinity(0, {core})
        try:
            t0 = time.perf_counter()
            _x, _f, _eu, _ed, res, _tr = R.solve(p, o)
            dt = time.perf_counter() - t0
        finally:
            if prev is not None:
                os.sched_setaffinity(0, prev)
        spent += dt
        it = max(1, res.outer_iterations)
        # the GPU on the same window and call (plan built outside the timing)
        sv = Solver(p, o, context=ctx)
        try:
            sv.solve()
            gts = []
            for _ in range(5):
                ctx.synchronize()
                g0 = time.perf_counter()
                gr = sv.solve().result
                ctx.synchronize()
                gts.append(time.perf_counter() - g0)
            gt = float(np.median(gts))
            git = max(1, gr["outer_iterations"])
        finally:
            sv.close()
        samples.append({"frames": frames, "params": p.num_params, "residuals": p.num_residuals,
                        "observations": p.num_obs, "cpu_s": dt, "cpu_lm_iterations": it,
                        "cpu_lm_iterations_per_s": it / dt, "gpu_s": gt,
                        "gpu_lm_iterations_per_s": git / gt,
                        "speedup_measured": (git / gt) / (it / dt)})
    big = samples[-1]
    # separately labelled: the full scene's per-iteration time from the
    # largest window by the dense-QR cost ratio m n^2 (not a measurement)
    t_full = (big["cpu_s"] / big["cpu_lm_iterations"]) * (
        (m_full * float(n_full) ** 2) / (big["residuals"] * float(big["params"]) ** 2))
    desc = ("oracle/refcpu.c single thread pinned to core %s (taskset), one LM iteration "
            "(lmder iterMax 2) on full-density "
            "frame windows of the same scene: %s; the GPU timed on the same windows and calls "
            "(median of 5) in this process" % (core, "; ".join(
                "F'=%d n=%d m=%d: CPU %.2f s, GPU %.2f ms" % (
                    q["frames"], q["params"], q["residuals"], q["cpu_s"], 1e3 * q["gpu_s"])
                for q in samples)))
    full_run = None
    fx = {1: "c2_full_it1", 4: "c5_full_it1"}.get(cfg_index)
    if fx:
        # the oracle on the WHOLE configuration, one LM iteration (lmder
        # iterMax 2): measured once when the full-size parity fixture was
        # made (tests/golden/make_full_golden.py, one thread, this repo's
        # build container) -- a measurement on another host, labelled so
        path = os.path.join(ROOT, "tests", "golden", "full", fx + ".npz")
        if os.path.exists(path):
            d = np.load(path, allow_pickle=False)
            it = max(1, int(d["res_outer_iterations"]))
            full_run = {"fixture": os.path.relpath(path, ROOT),
                        "seconds": float(d["oracle_seconds"]), "lm_iterations": it,
                        "lm_iterations_per_s": it / float(d["oracle_seconds"]),
                        "host": "build container (one thread), not the GPU box",
                        "params": int(d["exp_x"].size)}
    return {"value": big["cpu_lm_iterations_per_s"], "unit": "LM iterations/s", "cores": 1,
            "kind": "port", "sample": desc, "windows": samples, "full_config_run": full_run,
            "speedup_measured_same_window": big["speedup_measured"],
            "extrapolated_full_scene": {
                "label": "EXTRAPOLATION, not a measurement: largest window's per-iteration time "
                         "scaled by the dense-QR cost ratio m*n^2",
                "t_iter_s": t_full, "lm_iterations_per_s": 1.0 / t_full}}


def per_frame_line(args):
    """Per-frame solve mode (FrameSolveMode::kPerFrame) over the config's
    frames: residuals/s over all frame solves.  When the frames are
    independent the plan is built once (setup_s) and every step solves every
    frame in one launch (mmba_plan_solve_per_frame); otherwise each step is
    one mmba_solve_per_frame call with CONC frame solves in flight."""
    from mayamatchmovesolver_amd import synthetic as S
    from mayamatchmovesolver_amd._lib import MmbaError
    from mayamatchmovesolver_amd.solver import Solver, solve_per_frame
    kw = ({"lens_model": args.lens_model, "rolling_shutter": args.rolling_shutter}
          if args.config == 4 else {})
    prob = S.make_config(args.config, frames=args.frames, scale=args.scale, **kw)
    opt = S.config_options(prob)
    obs_per_frame = np.bincount(np.asarray(prob.obs_frame), minlength=prob.num_frames)
    t0 = time.perf_counter()
    sv = Solver(prob, opt)
    setup = time.perf_counter() - t0
    try:
        sv.solve_per_frame()
        step = sv.solve_per_frame
        path = "batched (one launch per call, plan cached)"
    except MmbaError:
        sv.close()
        sv, setup = None, None

        def step():
            return solve_per_frame(prob, opt, max_concurrency=args.per_frame)
        path = "per-frame plans, %d in flight" % args.per_frame
    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    resid = iters = 0
    for _ in range(args.steps):
        _, res = step()
        for f, r in enumerate(res):
            resid += int(obs_per_frame[f]) * (r["function_evals"] + r["outer_iterations"])
            iters += r["outer_iterations"]
    dt = time.perf_counter() - t0
    rms = float(np.sqrt(np.mean([r["error_rms"] ** 2 for r in res if r["success"]])))
    print(json.dumps({
        "metric": "per-frame solve mode residuals/s", "value": resid / dt,
        "unit": "residuals/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "dtype": "f64",
        "data": "synthetic", "config": {"workload": prob.meta.get("name"),
                                        "frames": prob.num_frames, "path": path,
                                        "concurrent_frames": args.per_frame},
        "lm_iterations_per_s": iters / dt, "frames_per_s": prob.num_frames * args.steps / dt,
        "final_rms_px_frames": rms, "setup_s": setup}),
        flush=True)
    if sv is not None:
        sv.close()


def parallelism(world, group, devices):
    if world > 1:
        return "frame-sharded x%d, one process per GPU (RCCL)" % world
    if group and len(set(devices)) == len(devices):
        return "frame-sharded x%d, one caller over %d GPUs (mmba_context_create_multi, " \
               "RCCL)" % (len(devices), len(devices))
    if group:
        return ("frame-sharded x%d in-process on device %d (one-GPU rehearsal of the sharded "
                "path through mmba_context_create_multi; not a multi-GPU measurement)"
                % (len(devices), devices[0]))
    return "single"


def main():
    args = parse()
    if args.per_frame:
        return per_frame_line(args)
    world, rank, local, dist = dist_setup()
    # one process over --gpus N devices (mmba_context_create_multi)
    group = world == 1 and args.gpus > 1
    nshards = args.gpus if group else world
    # PMC passes first, as child processes, before this process initialises
    # the GPU (rank 0 of a 1-GPU run only)
    traffic, traffic_detail = None, None
    if nshards == 1 and not args.no_traffic:
        traffic, traffic_detail = pmc_traffic(args)
    from mayamatchmovesolver_amd import synthetic as S
    from mayamatchmovesolver_amd.solver import Comm, Context, Solver, comm_unique_id
    pinned = apply_paths(args)

    frames = args.frames
    scale = args.scale
    if nshards > 1:  # weak scaling: the per-GPU shard is the single-GPU scene
        frames = (frames or BASE_FRAMES.get(args.config, 500)) * nshards
        scale = scale * nshards
    t0 = time.perf_counter()
    kw = ({"lens_model": args.lens_model, "rolling_shutter": args.rolling_shutter}
          if args.config == 4 else {})
    prob = S.make_config(args.config, frames=frames, scale=scale, **kw)
    opt = S.config_options(prob)
    gen_s = time.perf_counter() - t0
    progress("scene built (%.1f s)" % gen_s, every=0.0)
    # MMBA_BENCH_DEVICE: every rank on one device (RCCL path rehearsal on a
    # one-GPU box; the driver's multi-GPU runs leave it unset)
    devices = [int(os.environ.get("MMBA_BENCH_DEVICE", local))]
    if group:
        from mayamatchmovesolver_amd.solver import device_count
        visible = device_count()
        devices = list(range(nshards)) if visible >= nshards else [0] * nshards
        ctx = Context.multi(devices)
        progress("%d shards on devices %s" % (nshards, devices), every=0.0)
    else:
        ctx = Context(devices[0])
    comm = None
    rccl_ranks = None
    if world > 1:
        uid = broadcast_bytes(dist, comm_unique_id() if rank == 0 else None, 128)
        comm = Comm.rccl(ctx, rank, world, uid)
        rccl_ranks = comm.count()  # ncclCommCount: the ranks RCCL itself reports
        progress("rank %d: RCCL communicator up, ncclCommCount = %d" % (rank, rccl_ranks),
                 every=0.0)
    t0 = time.perf_counter()
    solver = Solver(prob, opt, context=ctx, comm=comm)
    upload_s = time.perf_counter() - t0
    if group and solver.num_shards != nshards:
        raise SystemExit("bench: the scene did not shard over %d devices" % nshards)
    progress("plan built (%.1f s)" % upload_s, every=0.0)

    # the caller's output buffers (errorList, ud->errorList,
    # errorDistanceList) are allocated once, in page-locked host memory
    # (mmba_host_alloc), and refilled by every solve
    from mayamatchmovesolver_amd.solver import host_array
    outs = (host_array(prob.num_residuals), host_array(prob.num_residuals),
            host_array(prob.num_obs))
    for w in range(args.warmup):
        solver.solve(out=outs)
        progress("warmup %d/%d" % (w + 1, args.warmup))

    # value: inputs resident in HBM before the timed region; every solve hands
    # errorList / ud->errorList / errorDistanceList (plus x, the result
    # record and the ||f|| trace) back to the caller's page-locked buffers,
    # as the seam's caller reads them (compute_error_stats and
    # accept-only-better, adjust_base.cpp:1201-1250; the shim's call)
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    iters = nfev = njev = 0
    last = None
    for st in range(args.steps):
        last = solver.solve(out=outs)
        progress("step %d/%d" % (st + 1, args.steps))
        iters += last.result["outer_iterations"]
        nfev += last.result["function_evals"]
        njev += last.result["outer_iterations"]
    ctx.synchronize()
    barrier(dist)
    dt = time.perf_counter() - t0
    dt_max = allreduce(dist, dt, "max")
    dt_ranks = allgather_float(dist, dt)  # per-shard times (the max is the value's clock)
    # device-resident rate (reported beside value, never as value): the same
    # solves leaving the per-residual outputs in HBM (mmba_plan_solve with
    # NULL output pointers; mmba_plan_outputs fetches them on demand)
    barrier(dist)
    ctx.synchronize()
    t0 = time.perf_counter()
    for st in range(args.steps):
        solver.solve(fetch=False)
        progress("device-resident step %d/%d" % (st + 1, args.steps))
    ctx.synchronize()
    barrier(dist)
    dt_dev = allreduce(dist, time.perf_counter() - t0, "max")
    # kernel timing (HIP events around the spans) on separate, untimed
    # solves, so the events do not weigh on the timed steps
    solver.set_timing(True)
    for _ in range(max(1, min(args.steps, 5))):
        solver.solve(out=outs)
    stats = solver.kernel_stats()
    solver.set_timing(False)

    if rank == 0:
        # one solve of the whole scene per step: count observations once
        resid = float(prob.num_obs) * (nfev + njev)
        value = resid / dt_max
        lm_rate = iters / dt_max
        # Roofline: the FD-Jacobian + normal-equation pass (HBM class) on this
        # rank's shard, bytes = B_J x observations per launch
        jac_ms = stats["jac_ms_avg"]
        jac_bytes = stats["jac_bytes"]
        achieved = (jac_bytes / (jac_ms * 1e-3)) / 1e9 if jac_ms > 0 else 0.0
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "kernel": "k_jacobian+k_ne_* (FD Jacobian blocks + normal equations)",
                    "avg_ms": jac_ms, "bytes_per_launch": jac_bytes,
                    "launches": stats["jac_launches"], "traffic_pmc": traffic_detail}
        valu = (traffic_detail or {}).get("valu_f64")
        if valu and jac_ms > 0:
            # the same K2 pass against the fp64 VALU peak: the FD Jacobian's
            # re-projections are arithmetic (C5: the LDPK fixed-point inverse)
            vt = valu["flops_per_launch"] / (jac_ms * 1e-3) / 1e12
            roofline["valu_fp64"] = {"achieved_tflops": vt, "peak_tflops": FP64_VALU_PEAK_TF,
                                     "frac": vt / FP64_VALU_PEAK_TF,
                                     "flops_per_launch": valu["flops_per_launch"]}
        kind = stats.get("reduced_kind", 0)
        band_names = {1: "band: partitioned Cholesky chains", 2: "band: block cyclic reduction",
                      3: "band: parallel cyclic reduction (k_pcr_solve, one launch, x out)",
                      4: "band: separator form (shard interiors by parallel cyclic reduction)",
                      5: "block diagonal + arrow (per camera-frame Cholesky)"}
        chol = {"avg_ms": stats["chol_ms_avg"], "launches": stats["chol_launches"],
                "reduced_dim": stats["reduced_dim"],
                "solver": band_names.get(stats.get("band_solver", 0), "band") if kind in (0, 3)
                else ["", "tiled sparse Cholesky",
                      "dense blocked Cholesky (MFMA GEMM trailing updates)"][kind],
                "note": "time per damped solve's factorisation (+ fused solve), HIP events"}
        if kind in (0, 3) and stats["chol_ms_avg"] > 0:
            # latency-bound (a dependent pivot chain per elimination level):
            # the fp64 fraction is reported on the ALGORITHMIC flops of the
            # band system (n_b w^2 + 4 n_b w, + the arrow), as measured, not
            # as a target; what the solver executes is beside it
            t_s = stats["chol_ms_avg"] * 1e-3
            tf = stats["chol_flops_alg"] / t_s / 1e12
            chol.update({"bound": "latency (a dependent 24-step pivot chain and a neighbour "
                                  "hand-off per level)"
                         if kind == 0 else "latency (one wave per camera-frame block)",
                         "dominant": stats["chol_ms_avg"] > jac_ms,
                         "achieved_tflops": tf, "peak_tflops": FP64_MFMA_PEAK_TF,
                         "frac": tf / FP64_MFMA_PEAK_TF, "flops": stats["chol_flops_alg"],
                         "flops_note": "algorithmic: n_b w^2 + 4 n_b w (+ arrow) for the band "
                                       "system, per damped solve",
                         "executed_flops": stats["chol_flops"],
                         "executed_tflops": stats["chol_flops"] / t_s / 1e12})
            if stats.get("band_levels", 0) > 0:
                lv = stats["band_levels"]
                # latency model: one launch whose levels run back to back --
                # per level one K-step pivot chain, the products and one
                # neighbour hand-off; the time per level is what a faster
                # chain or hand-off would cut
                chol["latency_model"] = {
                    "levels": lv, "block": stats["band_block"],
                    "us_per_level": 1e3 * stats["chol_ms_avg"] / (lv + 1),
                    "model": "t = (levels + 1) x (K-step pivot chain + products + neighbour "
                             "hand-off); the last term is the uncoupled block's solve"}
        mf = (traffic_detail or {}).get("reduced_solve_mfma")
        if mf:
            # matrix-core occupancy of the reduced solve (rocprofv3 --pmc):
            # busy cycles over launch time x 2.4 GHz x 1,024 SIMDs
            chol["mfma_pmc"] = {k: dict(v, busy_frac_of_chip=(
                v["mfma_busy_cycles"] / (stats["chol_ms_avg"] * 1e-3 * 2.4e9 * 1024.0)
                if stats["chol_ms_avg"] > 0 else None)) for k, v in mf.items()}
            chol["mfma_pmc_note"] = ("SQ_VALU_MFMA_BUSY_CYCLES per launch (cycles, summed over "
                                     "SIMDs), SQ_WAVE_CYCLES x 4; busy_frac_of_chip against the "
                                     "damped solve's HIP-event time")
        elif traffic_detail and traffic_detail.get("mfma_error"):
            chol["mfma_pmc"] = traffic_detail["mfma_error"]
        if kind == 2 and stats["chol_ms_avg"] > 0:
            tf = stats["chol_flops"] / (stats["chol_ms_avg"] * 1e-3) / 1e12
            chol.update({"achieved_tflops": tf, "peak_tflops": FP64_MFMA_PEAK_TF,
                         "frac": tf / FP64_MFMA_PEAK_TF, "flops": stats["chol_flops"]})
            # the dense reduced solve dominates such a workload: it is the
            # roofline kernel (fp64 MFMA bound), the K2 figure stays beside it
            if stats["chol_ms_avg"] > jac_ms:
                roofline = {"bound": "mfma", "achieved": tf, "peak": FP64_MFMA_PEAK_TF,
                            "unit": "TFLOP/s", "frac": tf / FP64_MFMA_PEAK_TF, "traffic": None,
                            "kernel": "dense reduced-system Cholesky (n_r^3/3 flop per "
                                      "factorisation; k_dense_potf64 + the hand-written "
                                      "fp64 MFMA GEMM/SYRK k_dgemm_nt)",
                            "avg_ms": stats["chol_ms_avg"], "flops_per_launch":
                            stats["chol_flops"], "launches": stats["chol_launches"],
                            "k2_hbm": roofline}
        cpu = None
        if not args.no_cpu_baseline and nshards == 1:
            cpu = cpu_baseline(args.config, args.cpu_budget_s, ctx)
        r = last.result
        line = {
            "metric": "LM iterations/sec + residuals/sec (markers x frames) at 1/2/4/8 MI355X; "
                      "final RMS reproj error",
            "value": value,
            "unit": "residuals/s",
            "n_gpus": nshards,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * dt_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY 8(d) generator, seed 20241008+i)",
            "config": {"workload": prob.meta.get("name", S.CONFIG_NAMES[args.config]),
                       "frames": prob.num_frames,
                       "cameras": prob.num_cameras, "bundles": prob.num_bundles,
                       "markers": prob.num_markers, "observations": prob.num_obs,
                       "parameters": prob.num_params, "residuals": prob.num_residuals,
                       "parallelism": parallelism(world, group, devices),
                       **({"devices": devices} if group else {}),
                       "solver": "lmder fwd-FD delta=1e-4 tau=1 tol=1e-6",
                       **({"pinned_paths": pinned} if pinned else {})},
            "lm_iterations_per_s": lm_rate,
            **({"shards": {"rccl_ranks": rccl_ranks, "num_shards": solver.num_shards,
                           "per_rank_ms_per_step": [1e3 * t / args.steps for t in dt_ranks]}}
               if nshards > 1 else {}),
            "final_rms_px": r["error_rms"],
            "d2h_bytes_per_step": 8.0 * (2 * prob.num_residuals + prob.num_obs),
            "device_resident": {
                "note": "the same solves leaving errorList / ud->errorList / "
                        "errorDistanceList in HBM (mmba_plan_outputs); not the value",
                "ms_per_step": 1e3 * dt_dev / args.steps,
                "value": resid / dt_dev,
                "lm_iterations_per_s": iters / dt_dev},
            "lm_iterations_per_solve": r["outer_iterations"],
            "nfev_per_solve": r["iterations"],
            "reason_number": r["reason_number"],
            "roofline": roofline,
            "reduced_cholesky": chol,
            "cpu_baseline": cpu,
            "setup_s": {"generate": gen_s, "upload": upload_s},
            "time_split_s": {"func": r["time_func_s"], "jac": r["time_jac_s"],
                             "linear": r["time_linear_s"], "solve": r["time_solve_s"]},
        }
        print(json.dumps(line), flush=True)
    solver.close()
    if comm is not None:
        comm.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
