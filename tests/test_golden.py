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
    # every envelope comes from tests/golden/envelopes.py over exactly its
    # registered seeds, never from a GPU run
    from tests.golden.envelopes import SEEDS
    assert tuple(d["envelope_seeds"]) == SEEDS and int(d["envelope_runs"]) == len(SEEDS)
    # only the deliberately ill-conditioned C4 16-frame window needs a wide
    # one (registered: 1.31e-2; round 4's 3-seed sample gave 8.1e-3)
    assert float(d["exp_x_envelope"]) <= (2e-2 if name == "c4_f16" else 1e-4)
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
    # an envelope, where the fixture has one, is the registered one; a fixture
    # without one (envelope_runs 0) is held at the flat 1e-6 bar on the GPU
    if int(d["envelope_runs"]) > 0 and "envelope_seeds" in d:
        from tests.golden.envelopes import SEEDS
        assert tuple(d["envelope_seeds"]) == SEEDS and int(d["envelope_runs"]) == len(SEEDS)


# ---- waypoint one-step fixtures (tests/golden/make_steps.py): the scene
# regenerates to the digest the oracle ran on, the envelope is the registered
# one, and the stored undetermined directions are orthonormal right singular
# vectors of the step's scaled Jacobian below the pre-stated ratio
from tests.golden import make_steps as ST  # noqa: E402


@pytest.mark.parametrize("name", ST.fixture_names())
def test_step_fixture_consistency(name):
    from tests.golden.envelopes import SEEDS
    prob, opt, d = ST.load(name)  # raises on a digest mismatch
    assert d["x_start"].size == prob.num_params == d["exp_x"].size
    assert tuple(d["envelope_seeds"]) == SEEDS and int(d["envelope_runs"]) == len(SEEDS)
    assert float(d["ratio"]) == ST.RATIO
    V = d["undet_basis"].astype(np.float64)
    if V.size:
        np.testing.assert_allclose(V.T @ V, np.eye(V.shape[1]), atol=1e-5)
        sv = d["sigma"]
        assert V.shape[1] == int(np.sum(sv < ST.RATIO * sv[0]))
    # the oracle's own 1-ulp runs stay inside the bar in the determined subspace
    assert float(d["exp_x_det_envelope"]) <= 1e-6
    assert d["exp_trace"].size == int(d["res_function_evals"])
