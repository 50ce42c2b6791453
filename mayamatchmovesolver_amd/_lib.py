"""Loader for ``csrc/libmmba.so`` (the HIP/gfx950 product library).

There is deliberately no fallback: if the library is missing or no gfx950
device is visible, every compute entry point raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import os
import subprocess

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(_HERE, "csrc")
LIB_PATH = os.environ.get("MMBA_LIB", os.path.join(CSRC, "libmmba.so"))  # override: diagnostics only
_lib = None


class MmbaError(RuntimeError):
    def __init__(self, code, message):
        super().__init__("mmba error %d: %s" % (code, message))
        self.code = code


def build(jobs=8):
    """Compile libmmba.so for gfx950 in-tree (hipcc cross-compiles without a GPU)."""
    subprocess.check_call(["make", "-s", "-j%d" % jobs, "-C", CSRC])
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MmbaError(abi.MMBA_ERR_NO_DEVICE,
                            "libmmba.so not built (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        if L.mmba_abi_version() != abi.ABI_VERSION:
            raise MmbaError(abi.MMBA_ERR_INVALID, "libmmba.so ABI %d, bindings expect %d "
                            "(rebuild)" % (L.mmba_abi_version(), abi.ABI_VERSION))
        dp = C.POINTER(C.c_double)
        L.mmba_abi_version.restype = C.c_int
        L.mmba_device_count.restype = C.c_int
        L.mmba_last_error.restype = C.c_char_p
        L.mmba_options_default.restype = None
        L.mmba_options_default.argtypes = [C.POINTER(abi.MmbaOptions), C.c_int32]
        for name in ("mmba_param_external_to_internal", "mmba_param_internal_to_external"):
            f = getattr(L, name)
            f.restype = C.c_double
            f.argtypes = [C.c_double] * 5
        L.mmba_context_create.restype = C.c_int
        L.mmba_context_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.mmba_context_create_multi.restype = C.c_int
        L.mmba_context_create_multi.argtypes = [C.POINTER(C.c_int), C.c_int,
                                                C.POINTER(C.c_void_p)]
        L.mmba_debug_reduced_residual.restype = C.c_int
        L.mmba_debug_reduced_residual.argtypes = [C.c_void_p, dp, C.c_double, dp]
        L.mmba_context_num_devices.restype = C.c_int
        L.mmba_context_num_devices.argtypes = [C.c_void_p]
        L.mmba_plan_num_shards.restype = C.c_int
        L.mmba_plan_num_shards.argtypes = [C.c_void_p]
        L.mmba_context_synchronize.restype = C.c_int
        L.mmba_context_synchronize.argtypes = [C.c_void_p]
        L.mmba_host_alloc.restype = C.c_int
        L.mmba_host_alloc.argtypes = [C.c_size_t, C.POINTER(C.c_void_p)]
        L.mmba_host_free.restype = None
        L.mmba_host_free.argtypes = [C.c_void_p]
        L.mmba_context_destroy.restype = None
        L.mmba_context_destroy.argtypes = [C.c_void_p]
        L.mmba_plan_create.restype = C.c_int
        L.mmba_plan_create.argtypes = [C.c_void_p, C.POINTER(abi.MmbaProblem),
                                       C.POINTER(abi.MmbaOptions), C.POINTER(C.c_void_p)]
        L.mmba_plan_destroy.restype = None
        L.mmba_plan_destroy.argtypes = [C.c_void_p]
        L.mmba_plan_measure.restype = C.c_int
        L.mmba_plan_measure.argtypes = [C.c_void_p, dp, dp, dp, dp, dp]
        L.mmba_plan_reproject.restype = C.c_int
        L.mmba_solve_per_frame.restype = C.c_int
        L.mmba_solve_per_frame.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, dp, C.c_void_p,
                                           C.c_int32, C.POINTER(abi.MmbaCallbacks)]
        L.mmba_plan_reproject.argtypes = [C.c_void_p, dp, dp, dp]
        L.mmba_plan_set_attr_values.restype = C.c_int
        L.mmba_plan_set_attr_values.argtypes = [C.c_void_p, dp]
        L.mmba_plan_solve_per_frame.restype = C.c_int
        L.mmba_plan_solve_per_frame.argtypes = [C.c_void_p, dp, C.c_void_p,
                                                C.POINTER(abi.MmbaCallbacks)]
        L.mmba_plan_jacobian.restype = C.c_int
        L.mmba_plan_jacobian.argtypes = [C.c_void_p, dp, dp]
        L.mmba_plan_solve.restype = C.c_int
        # (x and the three output lists as plain addresses: Solver.solve passes
        # the arrays' data pointers, ~2 us each instead of ~5 for data_as)
        L.mmba_plan_solve.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.POINTER(abi.MmbaResult),
                                      C.POINTER(abi.MmbaCallbacks), C.POINTER(abi.MmbaTrace)]
        L.mmba_plan_outputs.restype = C.c_int
        L.mmba_plan_outputs.argtypes = [C.c_void_p, dp, dp, dp]
        L.mmba_solve.restype = C.c_int
        L.mmba_solve.argtypes = [C.c_void_p, C.POINTER(abi.MmbaProblem),
                                 C.POINTER(abi.MmbaOptions), dp, dp, dp, dp,
                                 C.POINTER(abi.MmbaResult), C.POINTER(abi.MmbaCallbacks),
                                 C.POINTER(abi.MmbaTrace)]
        L.mmba_debug_set_path.restype = C.c_int
        L.mmba_debug_set_path.argtypes = [C.c_int, C.c_int]
        L.mmba_debug_band_solve.restype = C.c_int
        L.mmba_debug_band_solve.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, dp, dp,
                                            dp, dp, C.POINTER(C.c_int)]
        L.mmba_plan_kernel_stats.restype = C.c_int
        L.mmba_plan_kernel_stats.argtypes = [C.c_void_p, C.c_int, C.POINTER(abi.MmbaKernelStats)]
        L.mmba_comm_unique_id.restype = C.c_int
        L.mmba_comm_unique_id.argtypes = [C.c_char_p]
        L.mmba_comm_create_rccl.restype = C.c_int
        L.mmba_comm_create_rccl.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_char_p,
                                            C.POINTER(C.c_void_p)]
        L.mmba_comm_create_local.restype = C.c_int
        L.mmba_comm_create_local.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.mmba_comm_destroy.restype = None
        L.mmba_comm_destroy.argtypes = [C.c_void_p]
        L.mmba_comm_count.restype = C.c_int
        L.mmba_comm_count.argtypes = [C.c_void_p]
        L.mmba_debug_dgemm.restype = C.c_int
        L.mmba_debug_dgemm.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                       dp, C.c_int, C.c_void_p, C.c_int, dp, C.c_int,
                                       C.c_double, C.c_double]
        L.mmba_debug_comm_allreduce.restype = C.c_int
        L.mmba_debug_comm_allreduce.argtypes = [C.c_void_p, C.c_void_p, dp, C.c_int, C.c_int]
        L.mmba_plan_create_sharded.restype = C.c_int
        L.mmba_plan_create_sharded.argtypes = [C.c_void_p, C.POINTER(abi.MmbaProblem),
                                               C.POINTER(abi.MmbaOptions), C.c_void_p,
                                               C.POINTER(C.c_void_p)]
        ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
        L.mmba_shard_layout.restype = C.c_int
        L.mmba_shard_layout.argtypes = [C.c_int32, C.c_int32, ip, ip, C.c_int32, C.c_int32, ip,
                                        ip]
        _lib = L
    return _lib


def check(rc):
    if rc != abi.MMBA_OK:
        msg = lib().mmba_last_error()
        raise MmbaError(rc, msg.decode() if msg else "")
    return rc
