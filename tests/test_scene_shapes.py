"""Shapes of the synthetic scenes the wide-arrow and layered-lens GPU tests
rely on (CPU only): the number of global parameters (static, not a bundle's
translate) each witness rig carries, the parameters reaching one
observation, and the layered C5 lens chain."""
import numpy as np
import pytest

from mayamatchmovesolver_amd import synthetic as S


def globals_and_reach(prob):
    bnd_attrs = set()
    for b in range(prob.num_bundles):
        t = prob.bnd_tfm[b]
        bnd_attrs.update(int(a) for a in prob.tfm_attrs[9 * t:9 * t + 3])
    static = [p for p in range(prob.num_params) if prob.param_frame[p] < 0]
    ng = sum(1 for p in static if int(prob.param_attr[p]) not in bnd_attrs)
    return ng


@pytest.mark.parametrize("kw,ng", [(dict(), 24), (dict(n_witness=5, n_focal=5), 32),
                                   (dict(n_witness=5, n_focal=5, extra_globals=1), 33),
                                   (dict(frames=4), 24), (dict(frames=5, n_witness=5, n_focal=5), 32),
                                   (dict(n_witness=2, n_focal=2, extra_globals=2,
                                         lens="anamorphic"), 23)])
def test_witness_scene_globals(kw, ng):
    assert globals_and_reach(S.witness_scene(**kw)) == ng


def test_layered_c5_chain():
    prob = S.make_config(4, frames=6, scale=0.02, lens_model="layered")
    assert prob.lens_type.size == 2 and list(prob.lens_input) == [1, -1]
    assert np.all(prob.cam_lens == 0)
    d = prob.to_npz_dict()
    assert list(type(prob).from_npz_dict(d).lens_input) == [1, -1]
