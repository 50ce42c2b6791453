"""The drop-in boundary: libmmba.so builds for gfx950, loads, exports every
function include/mmba.h declares, and its host-only helpers agree with the
oracle.  No device compute here (runs on CPU-only machines)."""
import ctypes as C
import os
import re
import subprocess

import pytest

from mayamatchmovesolver_amd import _lib, abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mmba.h")


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mmba_[a-z_]+)\s*\(", text)) -
                  {"mmba_problem", "mmba_options", "mmba_result"})


def test_header_declares_abi():
    fns = declared_functions()
    assert set(fns) == set(abi.EXPORTED_SYMBOLS), set(fns) ^ set(abi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(L):
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [f for f in declared_functions() if f not in exported]
    assert not missing, missing
    for f in declared_functions():
        assert hasattr(L, f)


def test_library_is_gfx950_code_object(L):
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for other in (b"--gfx942", b"--gfx90a", b"--gfx1100"):
        assert other not in blob


def test_struct_layouts_match_header():
    # sizes of the C structs as ctypes sees them (x86_64 LP64 rules)
    import shutil
    import tempfile
    src = ('#include <stdio.h>\n#include "%s"\nint main(){printf("%%zu %%zu %%zu %%zu %%zu",'
           'sizeof(mmba_problem),sizeof(mmba_options),sizeof(mmba_result),sizeof(mmba_trace),'
           'sizeof(mmba_kernel_stats));}' % HEADER)
    d = tempfile.mkdtemp()
    try:
        open(os.path.join(d, "s.c"), "w").write(src)
        subprocess.check_call(["gcc", os.path.join(d, "s.c"), "-o", os.path.join(d, "s")])
        sizes = [int(v) for v in subprocess.check_output([os.path.join(d, "s")]).split()]
    finally:
        shutil.rmtree(d)
    assert sizes == [C.sizeof(abi.MmbaProblem), C.sizeof(abi.MmbaOptions),
                     C.sizeof(abi.MmbaResult), C.sizeof(abi.MmbaTrace),
                     C.sizeof(abi.MmbaKernelStats)]


def test_host_helpers(L, oracle):
    assert L.mmba_abi_version() == abi.ABI_VERSION == 10
    o = abi.MmbaOptions()
    L.mmba_options_default(C.byref(o), abi.SOLVER_TYPE_CMINPACK_LMDER)
    assert (o.iter_max, o.tau, o.eps1, o.delta, o.auto_param_scale, o.image_width) == \
        (100, 1.0, 1e-6, 1e-4, 1, 2048.0)
    assert o.scene_graph_mode == abi.SCENE_GRAPH_MODE_MAYA_DAG
    from mayamatchmovesolver_amd.problem import FLOAT_MAX
    for lo, hi in ((-FLOAT_MAX, FLOAT_MAX), (-5.0, 5.0), (-FLOAT_MAX, 5.0), (-5.0, FLOAT_MAX)):
        for v in (-3.0, 0.0, 1.5):
            a = L.mmba_param_external_to_internal(v, lo, hi, 0.0, 1.0)
            assert a == oracle.param_external_to_internal(v, lo, hi, 0.0, 1.0)
            assert L.mmba_param_internal_to_external(a, lo, hi, 0.0, 1.0) == \
                oracle.param_internal_to_external(a, lo, hi, 0.0, 1.0)


def test_no_device_fails_loudly(L):
    if L.mmba_device_count() > 0:
        pytest.skip("a gfx950 device is visible")
    h = C.c_void_p()
    rc = L.mmba_context_create(0, C.byref(h))
    assert rc == abi.MMBA_ERR_NO_DEVICE
    assert b"gfx950" in L.mmba_last_error()
    devs = (C.c_int * 2)(0, 0)
    assert L.mmba_context_create_multi(devs, 2, C.byref(h)) == abi.MMBA_ERR_NO_DEVICE


def test_bound_transforms_keep_nan(L, oracle):
    """std::max<double>(v, xmin) / std::min<double>(v, xmax) (adjust_base.cpp:
    202-203,217-218,232-233) return v when v is NaN: a NaN parameter stays NaN
    instead of snapping to a bound, in the library and in the oracle alike."""
    import math
    from mayamatchmovesolver_amd.problem import FLOAT_MAX
    nan = float("nan")
    for lo, hi in ((-FLOAT_MAX, FLOAT_MAX), (-5.0, 5.0), (-FLOAT_MAX, 5.0), (-5.0, FLOAT_MAX)):
        assert math.isnan(L.mmba_param_internal_to_external(nan, lo, hi, 0.0, 1.0))
        assert math.isnan(oracle.param_internal_to_external(nan, lo, hi, 0.0, 1.0))
        assert math.isnan(L.mmba_param_external_to_internal(nan, lo, hi, 0.0, 1.0))
        assert math.isnan(oracle.param_external_to_internal(nan, lo, hi, 0.0, 1.0))
