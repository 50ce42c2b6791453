"""Solve entry point: the host-side mirror of ``solveFrames`` -> LM -> results.

``Solver`` keeps the problem resident in HBM (an ``mmba_plan``) so repeated
solves on the same structure (the Python standard solver issues many,
``_api/solverstandardutils.py``) do not re-upload.  Results are returned both
as raw doubles and as the reference's ``key=value`` result strings
(``SolverResult::appendToMStringArray``, adjust_results.h:117-160) parsed by
``mmSolver.api.SolveResult`` (python/mmSolver/_api/solveresult.py:127-149).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from . import abi
from ._lib import check, lib
from .problem import Problem


def _dp(a):
    return None if a is None else a.ctypes.data_as(C.POINTER(C.c_double))


def _addr(a):
    """Data address of a C-contiguous array (for c_void_p arguments)."""
    return None if a is None else a.__array_interface__["data"][0]


def _num(v):
    # mmstring::numberToString uses default 6 significant digits (B10)
    return "%g" % v


@dataclass
class SolveResult:
    x: np.ndarray
    fvec: np.ndarray
    err_user: np.ndarray
    err_dist: np.ndarray
    result: Dict
    fnorm_trace: np.ndarray
    kernel_stats: Optional[Dict] = None

    problem: Optional[Problem] = None
    x0: Optional[np.ndarray] = None

    @property
    def accepted_x(self):
        """What solveFrames writes back: the solved x when the error got
        better (adjust_base.cpp:1231-1244), else the starting x."""
        if self.result.get("error_is_better", 1) or self.x0 is None:
            return self.x
        return self.x0

    @property
    def external(self):
        """Attribute values at the solution (what setParameters writes back)."""
        return self.problem.external_params(self.x)

    def result_strings(self) -> List[str]:
        r = self.result
        return [
            "success=%d" % int(r["success"]),
            "reason_num=%d" % int(r["reason_number"]),
            "error_final=" + _num(r["error_final"]),
            "error_final_average=" + _num(r["error_avg"]),
            "error_final_maximum=" + _num(r["error_max"]),
            "error_final_minimum=" + _num(r["error_min"]),
            "iteration_num=%d" % int(r["iterations"]),
            "iteration_function_num=%d" % int(r["function_evals"]),
            "iteration_jacobian_num=%d" % int(r["jacobian_evals"]),
            "user_interrupted=%d" % int(r["user_interrupted"]),
        ]


class Context:
    """A device context (``mmba_context``).  ``Context.multi(devices)``: one
    context over several devices (ABI 9) -- a ``Solver`` on it is frame-sharded
    over every device and driven from this thread (the library runs the other
    devices' shards on its own threads); naming one device N times runs the N
    shards there (the in-process transport)."""

    def __init__(self, device: int = 0, _handle=None):
        self._h = C.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            check(lib().mmba_context_create(int(device), C.byref(self._h)))

    @classmethod
    def multi(cls, devices) -> "Context":
        devs = [int(d) for d in devices]
        arr = (C.c_int * len(devs))(*devs)
        h = C.c_void_p()
        check(lib().mmba_context_create_multi(arr, len(devs), C.byref(h)))
        return cls(_handle=h)

    @property
    def num_devices(self) -> int:
        return int(lib().mmba_context_num_devices(self._h))

    @property
    def handle(self):
        return self._h

    def synchronize(self):
        check(lib().mmba_context_synchronize(self._h))

    def close(self):
        if self._h:
            lib().mmba_context_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """One shard's communicator for the frame-sharded solve (``mmba_comm``).

    ``Comm.rccl(ctx, rank, nranks, uid)``: RCCL, one process per GPU; ``uid`` is
    ``comm_unique_id()`` from one rank, broadcast by the caller.
    ``Comm.local_group(n)``: n in-process shards (one host thread each)."""

    def __init__(self, handle, rank, nranks):
        self._h = handle
        self.rank, self.nranks = rank, nranks

    @classmethod
    def rccl(cls, ctx: "Context", rank: int, nranks: int, unique_id: bytes) -> "Comm":
        h = C.c_void_p()
        check(lib().mmba_comm_create_rccl(ctx.handle, int(rank), int(nranks),
                                          bytes(unique_id), C.byref(h)))
        return cls(h, rank, nranks)

    @classmethod
    def local_group(cls, nranks: int) -> List["Comm"]:
        hs = (C.c_void_p * nranks)()
        check(lib().mmba_comm_create_local(int(nranks), hs))
        return [cls(C.c_void_p(hs[r]), r, nranks) for r in range(nranks)]

    @property
    def handle(self):
        return self._h

    def count(self) -> int:
        """Ranks as the transport reports them (``ncclCommCount`` for RCCL)."""
        n = lib().mmba_comm_count(self._h)
        check(min(n, 0))
        return n

    def debug_allreduce(self, ctx: "Context", values, op: str = "sum") -> np.ndarray:
        """The plan's in-place all-reduce on a copy of ``values`` (test hook,
        ``mmba_debug_comm_allreduce``); collective over the communicator."""
        buf = np.ascontiguousarray(values, dtype=np.float64).copy()
        check(lib().mmba_debug_comm_allreduce(ctx.handle, self._h, _dp(buf), int(buf.size),
                                              1 if op == "max" else 0))
        return buf

    def close(self):
        if self._h:
            lib().mmba_comm_destroy(self._h)
            self._h = C.c_void_p()


def debug_dgemm(ctx: "Context", A, B, Cm, alpha=1.0, beta=0.0, tri=False, in_place=False):
    """The dense solver's fp64 MFMA GEMM / SYRK (test hook, ``mmba_debug_dgemm``):
    returns beta Cm + alpha A B^T (``tri``: lower triangle of a SYRK with B = A,
    entries above the diagonal keep Cm's; ``in_place``: the panel-solve form,
    computed in A's array, beta 0)."""
    A = np.asfortranarray(A, dtype=np.float64)
    out = np.array(Cm, dtype=np.float64, order="F", copy=True)
    M, K = A.shape
    N = out.shape[1]
    bp, ldb = None, 0
    if B is not None:
        B = np.asfortranarray(B, dtype=np.float64)
        bp, ldb = B.ctypes.data_as(C.c_void_p), B.shape[0]
    flat = out.ravel(order="K")  # a view: the hook writes the result into `out`
    af = A.ravel(order="F")
    check(lib().mmba_debug_dgemm(ctx.handle, int(bool(tri)), int(bool(in_place)), M, N, K,
                                 _dp(af), M, bp, ldb, _dp(flat), M, float(alpha),
                                 float(beta)))
    return out


class _HostBlock:
    """Owner of one mmba_host_alloc block (freed with the last array view)."""

    def __init__(self, nbytes: int):
        self.ptr = C.c_void_p()
        check(lib().mmba_host_alloc(int(nbytes), C.byref(self.ptr)))

    def __del__(self):
        if self.ptr:
            lib().mmba_host_free(self.ptr)
            self.ptr = C.c_void_p()


class _Pinned(np.ndarray):
    """ndarray over page-locked host memory; holds the block (views keep it
    alive through their base)."""


def host_array(n: int) -> np.ndarray:
    """A float64 array of n entries in page-locked host memory
    (``mmba_host_alloc``) for buffers kept across solves (``Solver.solve(out=...)``):
    the end-of-solve device-to-host copies run at full link rate."""
    n = max(int(n), 1)
    blk = _HostBlock(8 * n)
    arr = np.ctypeslib.as_array((C.c_double * n).from_address(blk.ptr.value)).view(_Pinned)
    arr._blk = blk
    arr[:] = 0.0
    return arr


def comm_unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check(lib().mmba_comm_unique_id(buf))
    return buf.raw


class Solver:
    """A problem uploaded to one MI355X (``mmba_plan``); with ``comm``, this
    shard of a frame-sharded plan (every shard passes the same problem)."""

    def __init__(self, problem: Problem, options, context: Optional[Context] = None,
                 device: int = 0, comm: Optional[Comm] = None):
        self.problem = problem
        self.options = options
        self.ctx = context or Context(device)
        self.comm = comm
        self._prob_c, self._keep = problem.to_ctypes()
        self._h = C.c_void_p()
        check(lib().mmba_plan_create_sharded(self.ctx.handle, C.byref(self._prob_c),
                                             C.byref(self.options),
                                             comm.handle if comm is not None else None,
                                             C.byref(self._h)))

    def close(self):
        if self._h:
            lib().mmba_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def num_shards(self) -> int:
        """Shards this plan solves on (``mmba_plan_num_shards``)."""
        return int(lib().mmba_plan_num_shards(self._h))

    def reduced_residual(self, x=None, lam: float = 0.0) -> float:
        """||S x - r|| / ||r|| of the damped reduced system the plan forms at x
        (test hook ``mmba_debug_reduced_residual``; dense reduced plans)."""
        xx = np.ascontiguousarray(self.problem.x0 if x is None else x, dtype=np.float64)
        out = np.zeros(1)
        check(lib().mmba_debug_reduced_residual(self._h, _dp(xx), float(lam), _dp(out)))
        return float(out[0])

    def set_timing(self, enable=True):
        st = abi.MmbaKernelStats()
        self._timing = bool(enable)
        check(lib().mmba_plan_kernel_stats(self._h, 1 if enable else 0, C.byref(st)))

    def kernel_stats(self):
        """The plan's kernel statistics (the timing switch is left as set)."""
        st = abi.MmbaKernelStats()
        check(lib().mmba_plan_kernel_stats(self._h, 1 if getattr(self, "_timing", False) else 0,
                                           C.byref(st)))
        return st.as_dict()

    def dataflow_fallback(self) -> bool:
        """True once a timed-out dataflow wait switched this plan's block
        cyclic reduction to the per-level launches."""
        return bool(self.kernel_stats()["dataflow_fallback"])

    def measure(self, x=None):
        p = self.problem
        m, M = p.num_residuals, p.num_obs
        fvec, eu, ed, st = np.zeros(m), np.zeros(m), np.zeros(M), np.zeros(3)
        xx = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
        check(lib().mmba_plan_measure(self._h, _dp(xx), _dp(fvec), _dp(eu), _dp(ed), _dp(st)))
        return fvec, eu, ed, st

    def reproject(self, x=None):
        """Per-observation reprojected (lens-distorted) point and film-fit
        corrected marker at internal parameters x (``mmba_plan_reproject``):
        two [2M] arrays in observation order."""
        M = self.problem.num_obs
        pts, mkr = np.zeros(2 * M), np.zeros(2 * M)
        xx = None if x is None else np.ascontiguousarray(x, dtype=np.float64)
        check(lib().mmba_plan_reproject(self._h, _dp(xx), _dp(pts), _dp(mkr)))
        return pts, mkr

    def jacobian(self, x):
        """Dense reference-layout Jacobian (m x n) at internal parameters x."""
        p = self.problem
        m, n = p.num_residuals, p.num_params
        xx = np.ascontiguousarray(x, dtype=np.float64)
        fjac = np.zeros(m * n)
        check(lib().mmba_plan_jacobian(self._h, _dp(xx), _dp(fjac)))
        return fjac.reshape(n, m).T

    def solve(self, x0=None, trace_capacity=4096, interrupt=None, out=None,
              fetch=True) -> SolveResult:
        """LM solve from x0 (internal parameters).  ``SolveResult.x`` is the
        solved x as lmder leaves paramList; ``result["error_is_better"]`` says
        whether solveFrames would write it back (``accepted_x``).
        ``interrupt``: a callable polled where the reference polls
        MComputation::isInterruptRequested (non-zero / True stops).
        ``out``: (fvec, err_user, err_dist) float64 arrays to fill instead of
        fresh ones (a caller solving repeatedly keeps its buffers).
        ``fetch=False``: the per-residual outputs stay in HBM (NULL output
        pointers; ``fvec`` / ``err_user`` / ``err_dist`` are None) until
        ``outputs()`` fetches them."""
        p = self.problem
        m, M = p.num_residuals, p.num_obs
        x = np.array(p.x0 if x0 is None else x0, dtype=np.float64)
        if not fetch:
            fvec = eu = ed = None
        elif out is None:
            fvec, eu, ed = np.zeros(m), np.zeros(m), np.zeros(M)
        else:
            fvec, eu, ed = out
            assert fvec.dtype == eu.dtype == ed.dtype == np.float64
            assert fvec.size >= m and eu.size >= m and ed.size >= M
            assert fvec.flags.c_contiguous and eu.flags.c_contiguous and ed.flags.c_contiguous
        res = abi.MmbaResult()
        # the ||f|| trace buffer and its descriptor are kept across solves of
        # the same capacity (the library resets count; the used part is copied)
        if getattr(self, "_trace_cap", None) != trace_capacity:
            self._tbuf = np.zeros(max(1, trace_capacity))
            self._tr = abi.MmbaTrace(_dp(self._tbuf), trace_capacity, 0)
            self._trace_cap = trace_capacity
        tbuf, tr = self._tbuf, self._tr
        cbs = _callbacks(interrupt)
        rc = lib().mmba_plan_solve(self._h, _addr(x), _addr(fvec), _addr(eu), _addr(ed),
                                   C.byref(res), C.byref(cbs) if cbs is not None else None,
                                   C.byref(tr))
        if rc not in (abi.MMBA_OK, abi.MMBA_ERR_INTERRUPTED):
            check(rc)
        return SolveResult(x=x, fvec=fvec, err_user=eu, err_dist=ed, result=res.as_dict(),
                           fnorm_trace=tbuf[:min(tr.count, trace_capacity)].copy(), problem=p,
                           x0=np.array(p.x0 if x0 is None else x0, dtype=np.float64))


    def outputs(self, out=None):
        """(fvec, err_user, err_dist) of the last ``solve`` / ``measure``
        (``mmba_plan_outputs``): the fetch a ``solve(fetch=False)`` left in
        HBM.  ``out``: arrays to fill (e.g. ``host_array`` page-locked ones)."""
        p = self.problem
        m, M = p.num_residuals, p.num_obs
        fvec, eu, ed = out if out is not None else (np.zeros(m), np.zeros(m), np.zeros(M))
        check(lib().mmba_plan_outputs(self._h, _dp(fvec), _dp(eu), _dp(ed)))
        return fvec, eu, ed

    def set_attr_values(self, attr_values):
        """Replace the scene's attribute values of this plan
        (``mmba_plan_set_attr_values``; plan caching across solves)."""
        v = np.ascontiguousarray(attr_values, dtype=np.float64)
        assert v.size >= np.asarray(self.problem.attr_values).size
        check(lib().mmba_plan_set_attr_values(self._h, _dp(v)))

    def solve_per_frame(self, x0=None, interrupt=None):
        """Per-frame solve mode on this plan (``mmba_plan_solve_per_frame``):
        every frame in one launch.  Returns (x, [per-frame result dicts]);
        raises MmbaError (MMBA_ERR_UNSUPPORTED) when the parameters do not
        split into independent frames."""
        p = self.problem
        x = np.array(p.x0 if x0 is None else x0, dtype=np.float64)
        res = (abi.MmbaResult * p.num_frames)()
        cbs = _callbacks(interrupt)
        check(lib().mmba_plan_solve_per_frame(self._h, _dp(x), res,
                                              C.byref(cbs) if cbs is not None else None))
        return x, [r.as_dict() for r in res]


def solve(problem: Problem, options, x0=None, device: int = 0) -> SolveResult:
    """One-shot solve (``mmba_solve``)."""
    s = Solver(problem, options, device=device)
    try:
        return s.solve(x0)
    finally:
        s.close()


def _callbacks(interrupt):
    if interrupt is None:
        return None
    return abi.MmbaCallbacks(abi.INTERRUPT_FN(lambda _u: 1 if interrupt() else 0),
                             abi.PROGRESS_FN(lambda _u, _i: None), None)


def solve_per_frame(problem: Problem, options, x0=None, device: int = 0,
                    max_concurrency: int = 0, interrupt=None, context=None):
    """Per-frame solve mode (``mmba_solve_per_frame``; FrameSolveMode::kPerFrame,
    adjust_base.cpp:1430-1484).  Returns (x, [per-frame result dicts]); x holds
    what each frame's solveFrames wrote back."""
    p, keep = problem.to_ctypes()
    x = np.array(problem.x0 if x0 is None else x0, dtype=np.float64)
    F = problem.num_frames
    res = (abi.MmbaResult * F)()
    ctx = context or Context(device)
    cbs = _callbacks(interrupt)
    try:
        rc = lib().mmba_solve_per_frame(ctx.handle, C.byref(p), C.byref(options), _dp(x),
                                        res, int(max_concurrency),
                                        C.byref(cbs) if cbs is not None else None)
        if rc not in (abi.MMBA_OK, abi.MMBA_ERR_INTERRUPTED):
            check(rc)
    finally:
        if context is None:
            ctx.close()
    return x, [r.as_dict() for r in res]


def shard_layout(problem: Problem, nranks: int):
    """Frame partition a sharded plan of `problem` uses (host only): returns
    (bounds[nranks + 1], bundle_owner[num_bundles]); shard k owns frames
    [bounds[k], bounds[k + 1]) and the bundles whose first observation is there."""
    p = problem
    frames = np.ascontiguousarray(p.obs_frame, dtype=np.int32)
    bnd = np.ascontiguousarray(np.asarray(p.mkr_bnd)[np.asarray(p.obs_marker)], dtype=np.int32)
    bounds = np.zeros(nranks + 1, dtype=np.int32)
    owner = np.zeros(max(p.num_bundles, 1), dtype=np.int32)
    check(lib().mmba_shard_layout(p.num_frames, p.num_obs, frames, bnd, p.num_bundles, nranks,
                                  bounds, owner))
    return bounds, owner[:p.num_bundles]


def device_count() -> int:
    return int(lib().mmba_device_count())


def set_path(key: int, value: int = -1) -> None:
    """Test hook (``mmba_debug_set_path``): pin a plan-builder choice
    (``abi.PATH_*``) for the plans and in-process communicators created
    afterwards; -1 restores the builder's own choice."""
    check(lib().mmba_debug_set_path(int(key), int(value)))


def debug_band_solve(ctx: "Context", S: np.ndarray, nb: int, w: int, nG: int, parts: int = 0):
    """Test hook: solve S x = r-style systems with the device band + arrow
    Cholesky (``mmba_debug_band_solve``).  Returns a function r -> (x, ||L^-1 r||^2, P)."""
    S = np.ascontiguousarray(S, dtype=np.float64)

    def solve(r):
        r = np.ascontiguousarray(r, dtype=np.float64)
        x = np.empty_like(r)
        yn = C.c_double(0.0)
        pu = C.c_int(0)
        check(lib().mmba_debug_band_solve(ctx.handle, int(nb), int(w), int(nG), int(parts),
                                          _dp(S), _dp(r), _dp(x), C.byref(yn), C.byref(pu)))
        return x, yn.value, pu.value
    return solve
