"""Layered lens nodes in the oracle (mmba.h ABI 5): the camera's lens is
applied last, over its input layers, which run first with their values as
read (lens_model_3de_classic.cpp:82-88: applyModelDistort runs the input
model's before its own; maya_lens_model_utils.cpp:715: the solver never
re-points the input chain, so its values are constants of the solve).  Pinned
against the single-model distortion functions composed by hand."""
import numpy as np

from mayamatchmovesolver_amd import synthetic as S


def _layered():
    prob = S.make_config(4, frames=6, scale=0.02, lens_model="layered")
    assert prob.lens_input is not None and list(prob.lens_input) == [1, -1]
    return prob


def test_layered_lens_applies_input_first(oracle):
    prob = _layered()
    opt = S.config_options(prob)
    x = prob.x0.copy()
    x[0], x[1] = 0.05, 0.01  # the top lens's distortion and quartic (solved first)
    pts, _ = oracle.reproject_obs(prob, opt, x)
    bare = prob.with_x0(x)
    bare.cam_lens = np.full(bare.num_cameras, -1, np.int32)
    raw, _ = oracle.reproject_obs(bare, opt)
    c_in = np.array([0.03, 0.002, -0.001, 0.008, 0.0, 0.0, 15.0, 0.02])
    c_top = np.array([0.05, 1.0, 0.0, 0.0, 0.01])
    want = np.empty_like(raw)
    other = np.empty_like(raw)
    for i in range(prob.num_obs):
        ix, iy = oracle.lens_radial_distort(c_in, raw[2 * i], raw[2 * i + 1])
        want[2 * i], want[2 * i + 1] = oracle.lens_distort(c_top, ix, iy)
        tx, ty = oracle.lens_distort(c_top, raw[2 * i], raw[2 * i + 1])
        other[2 * i], other[2 * i + 1] = oracle.lens_radial_distort(c_in, tx, ty)
    np.testing.assert_allclose(pts, want, rtol=0, atol=1e-13)
    assert np.max(np.abs(pts - other)) > 1e-6  # the order matters on this scene


def test_input_layer_values_override_attributes(oracle):
    """lens_input_values (the plug-read values) replace the input layer's
    attribute values; solving an input layer's attribute changes nothing."""
    prob = _layered()
    opt = S.config_options(prob)
    f0, *_ = oracle.measure(prob, opt)
    vals = np.zeros(2 * 14)
    # the top lens's own plug values (ABI 7: a slot no parameter writes, and
    # every slot before setParameters runs): its attributes at frame 0
    la = np.asarray(prob.lens_attrs).reshape(-1, 14)[0]
    for k, a in enumerate(la):
        vals[k] = prob.attr_values[prob.attr_offset[a]] if a >= 0 else (1.0 if k == 1 else 0.0)
    vals[14:22] = [0.03, 0.002, -0.001, 0.008, 0.0, 0.0, 15.0, 0.02]
    p2 = prob.with_x0(prob.x0)
    p2.lens_input_values = vals
    f1, *_ = oracle.measure(p2, opt)
    np.testing.assert_array_equal(f0, f1)
    vals[14] = 0.0
    p2.lens_input_values = vals
    f2, *_ = oracle.measure(p2, opt)
    assert np.max(np.abs(f2 - f0)) > 1e-3
