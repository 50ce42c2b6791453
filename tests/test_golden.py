"""The committed golden fixtures (tests/golden/*.npz, made by
tests/golden/make_golden.py) against the CPU oracle and the reference's own
known answers.  CPU only: the oracle must reproduce every fixture exactly, so a
change to oracle/refcpu.c or to the synthetic generator cannot go unnoticed."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S
from tests.golden import make_golden as G

NAMES = G.fixture_names()


def test_fixtures_present():
    assert len(NAMES) >= 14, NAMES


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(name, oracle):
    prob, opt, d = G.load(name)
    x, fvec, eu, ed, res, tr = oracle.solve(prob, opt)
    np.testing.assert_array_equal(x, d["exp_x"])
    np.testing.assert_array_equal(fvec, d["exp_fvec"])
    np.testing.assert_array_equal(ed, d["exp_err_dist"])
    np.testing.assert_array_equal(tr, d["exp_trace"])
    assert res.reason_number == int(d["res_reason_number"])
    assert res.iterations == int(d["res_iterations"])
    assert res.jacobian_evals == int(d["res_jacobian_evals"])


@pytest.mark.parametrize("name", [n for n in NAMES if n.startswith("known_")])
def test_fixture_known_answer(name):
    """mmSolver's Maya solver tests: converged external values."""
    prob, _opt, d = G.load(name)
    scene = name[len("known_"):].rsplit("_", 1)[0]
    expected, tol = S.KNOWN_ANSWERS[scene]
    ext = prob.external_params(d["exp_x"])
    assert np.all(np.abs(ext - np.array(expected)) <= tol), (ext, expected)


@pytest.mark.parametrize("name", NAMES)
def test_fixture_consistency(name):
    _prob, _opt, d = G.load(name)
    # only the deliberately ill-conditioned C4 16-frame window needs the envelope
    assert float(d["exp_x_envelope"]) <= (1e-2 if name == "c4_f16" else 1e-4)
    assert d["exp_trace"].size == int(d["res_function_evals"])
    assert abs(np.linalg.norm(d["exp_fvec"]) - float(d["res_error_final"])) <= \
        1e-12 * max(1.0, float(d["res_error_final"]))


# ---- full-size fixtures (tests/golden/make_full_golden.py): the oracle's
# outputs on the full BASELINE configurations / full-density C4 windows; the
# scenes are regenerated from their seed, so the generator must reproduce the
# exact problem the oracle ran on (SHA-256 digest).
from tests.golden import make_full_golden as FG  # noqa: E402

FULL = FG.fixture_names()


@pytest.mark.parametrize("name", FULL)
def test_full_fixture_scene_digest(name):
    prob, opt, d = FG.load(name)  # raises on a digest mismatch
    assert d["exp_x"].size == prob.num_params
    if "exp_fvec" in d:
        assert d["exp_fvec"].size == prob.num_residuals
        assert abs(np.linalg.norm(d["exp_fvec"]) - float(d["res_error_final"])) <= \
            1e-12 * float(d["res_error_final"])
    assert d["exp_trace"].size == int(d["res_function_evals"])
    assert int(d["envelope_runs"]) >= 1
