"""GPU (libmmba.so through the C ABI) against the committed golden fixtures:
same reason code and evaluation counts, every ||f|| of the trace and the final
parameter vector within 1e-6 relative (BASELINE.json north_star), final
residual vector within 1e-6 of the initial ||f||."""
import numpy as np
import pytest

from mayamatchmovesolver_amd.solver import Solver
from tests.golden import make_golden as G

pytestmark = pytest.mark.gpu
REL = 1e-6


@pytest.mark.parametrize("name", G.fixture_names())
def test_gpu_matches_fixture(name, gpu_ctx):
    prob, opt, d = G.load(name)
    s = Solver(prob, opt, context=gpu_ctx)
    try:
        out = s.solve()
    finally:
        s.close()
    g = out.result
    assert g["reason_number"] == int(d["res_reason_number"])
    assert g["iterations"] == int(d["res_iterations"])
    assert g["function_evals"] == int(d["res_function_evals"])
    assert g["jacobian_evals"] == int(d["res_jacobian_evals"])
    tr = d["exp_trace"]
    assert len(out.fnorm_trace) == len(tr)
    np.testing.assert_allclose(out.fnorm_trace, tr, rtol=REL, atol=1e-9 * tr[0])
    # final x: 1e-6 relative, or -- on ill-conditioned scenes -- the oracle's
    # own roundoff envelope (how far its x moves under a 1-ulp change of x0,
    # stored in the fixture by make_golden.py)
    xr = d["exp_x"]
    tol = max(REL, float(d["exp_x_envelope"]))
    assert np.max(np.abs(out.x - xr) / np.maximum(np.abs(xr), 1e-3)) <= tol
    # final residual vector: norm of the difference against the initial ||f||
    assert np.linalg.norm(out.fvec - d["exp_fvec"]) <= REL * float(tr[0])
