"""Host-side problem assembly: the Maya-free counterpart of what ``solveFrames``
builds before it calls the LM (src/mmSolver/adjust/adjust_base.cpp:713-1047).

``SceneBuilder`` plays the role of the Maya scene + ``construct_scene_graph``
(src/mmSolver/mayahelper/maya_scene_graph.cpp:1114) and of the relationship
pre-pass:

* observations follow ``countUpNumberOfErrors``
  (src/mmSolver/adjust/adjust_relationships.cpp:75-221): marker-major,
  frame-minor, only frames with ``enable`` and ``weight > 0``, marker position
  divided by the MarkerGroup overscan, weights normalised by the per-frame
  maximum weight;
* parameters follow ``countUpNumberOfUnknownParameters`` (:223-337):
  attribute-major, an animated attribute expands to one parameter per frame,
  a static one to a single parameter with frame ``-1``;
* initial parameters follow ``get_initial_parameters``
  (adjust_base.cpp:260-295): external value -> internal via the box-constraint
  transform.

``Problem`` holds the flat SoA arrays of ``include/mmba.h::mmba_problem``.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Union

import numpy as np

from . import abi

FLOAT_MAX = float(np.finfo(np.float32).max)  # std::numeric_limits<float>::max()

Value = Union[float, Sequence[float], np.ndarray]


def param_external_to_internal(value, xmin, xmax, offset, scale):
    """``parameterBoundFromExternalToInternal`` (adjust_base.cpp:225-258),
    bug-compatible (lower-bound-only is treated as unbounded, Appendix B2)."""
    value = max(value, xmin)
    value = min(value, xmax)
    value = value * scale + offset
    xmin = xmin * scale + offset
    xmax = xmax * scale + offset
    if xmin <= FLOAT_MAX and xmax >= FLOAT_MAX:
        return value
    if xmax >= FLOAT_MAX:
        return math.sqrt(((value - xmin) + 1.0) ** 2 - 1.0)
    if xmin <= -FLOAT_MAX:
        return math.sqrt(((xmax - value) + 1.0) ** 2 - 1.0)
    return math.asin((2.0 * (value - xmin) / (xmax - xmin)) - 1.0)


def param_internal_to_external(value, xmin, xmax, offset, scale):
    """``parameterBoundFromInternalToExternal`` (adjust_base.cpp:194-220)."""
    if xmin <= -FLOAT_MAX and xmax >= FLOAT_MAX:
        value = value / scale - offset
        return min(max(value, xmin), xmax)
    if xmax >= FLOAT_MAX:
        value = xmin - (1.0 + math.sqrt(value * value + 1.0))
    elif xmin <= -FLOAT_MAX:
        value = xmax + (1.0 - math.sqrt(value * value + 1.0))
    else:
        value = xmin + ((xmax - xmin) / 2.0) * (math.sin(value) + 1.0)
    value = value / scale - offset
    return min(max(value, xmin), xmax)


_FIELDS_I32 = [
    "attr_animated", "tfm_parent", "tfm_rotate_order", "tfm_attrs", "cam_tfm",
    "cam_attrs", "cam_film_fit", "cam_render_size", "cam_lens", "lens_type",
    "lens_attrs", "bnd_tfm", "mkr_cam", "mkr_bnd", "obs_marker", "obs_frame",
    "param_attr", "param_frame",
]
_FIELDS_I64 = ["attr_offset"]
_FIELDS_F64 = [
    "attr_values", "obs_xy", "obs_weight", "param_min", "param_max",
    "param_offset", "param_scale", "x0",
]
# ABI 2 (optional: absent in fixtures written before it)
_FIELDS_OPT_I32 = ["stiff_attr", "stiff_frame", "smooth_attr", "smooth_frame"]
_FIELDS_OPT_F64 = ["stiff_weight", "stiff_variance", "stiff_value", "smooth_weight",
                   "smooth_variance", "smooth_value"]


@dataclass
class Problem:
    """Flat problem, field-for-field ``mmba_problem`` plus ``x0``."""

    num_frames: int
    attr_animated: np.ndarray
    attr_offset: np.ndarray
    attr_values: np.ndarray
    tfm_parent: np.ndarray
    tfm_rotate_order: np.ndarray
    tfm_attrs: np.ndarray
    cam_tfm: np.ndarray
    cam_attrs: np.ndarray
    cam_film_fit: np.ndarray
    cam_render_size: np.ndarray
    cam_lens: np.ndarray
    lens_type: np.ndarray
    lens_attrs: np.ndarray
    bnd_tfm: np.ndarray
    mkr_cam: np.ndarray
    mkr_bnd: np.ndarray
    obs_marker: np.ndarray
    obs_frame: np.ndarray
    obs_xy: np.ndarray
    obs_weight: np.ndarray
    param_attr: np.ndarray
    param_frame: np.ndarray
    param_min: np.ndarray
    param_max: np.ndarray
    param_offset: np.ndarray
    param_scale: np.ndarray
    x0: np.ndarray
    meta: Dict = field(default_factory=dict)
    # ABI 2: paramWeightList (None = 1.0) and attribute stiffness / smoothness
    # rows (adjust_measureErrors.cpp:311-387)
    param_weight: Optional[np.ndarray] = None
    stiff_attr: Optional[np.ndarray] = None
    stiff_frame: Optional[np.ndarray] = None
    stiff_weight: Optional[np.ndarray] = None
    stiff_variance: Optional[np.ndarray] = None
    stiff_value: Optional[np.ndarray] = None
    smooth_attr: Optional[np.ndarray] = None
    smooth_frame: Optional[np.ndarray] = None
    smooth_weight: Optional[np.ndarray] = None
    smooth_variance: Optional[np.ndarray] = None
    smooth_value: Optional[np.ndarray] = None
    # ABI 3: per-camera rolling-shutter value in frames (time shift x fps;
    # None = every camera a global shutter, the reference behaviour)
    cam_rs_value: Optional[np.ndarray] = None
    # ABI 5: layered lens nodes -- the input lens of each lens (-1 none) and
    # the input layers' plug-read values (None = the attributes at frame 0)
    lens_input: Optional[np.ndarray] = None
    lens_input_values: Optional[np.ndarray] = None
    # ABI 7: the reference's lens index arithmetic (Appendix B3, mmba.h) --
    # each parameter's attrList index (paramToAttrList[p].first) and the lens
    # of each attrList entry (-1 not a lens attribute); None = derived
    param_ref_attr: Optional[np.ndarray] = None
    ref_attr_lens: Optional[np.ndarray] = None
    # ABI 8: every marker's x,y at every frame, [num_markers, num_frames, 2]
    # flattened (the MMSG flat marker list, Appendix B4; None = taken from the
    # observations)
    mkr_frame_xy: Optional[np.ndarray] = None

    def __post_init__(self):
        for name in _FIELDS_I32:
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dtype=np.int32).reshape(-1))
        for name in _FIELDS_I64:
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dtype=np.int64).reshape(-1))
        for name in _FIELDS_F64:
            setattr(self, name, np.ascontiguousarray(getattr(self, name), dtype=np.float64).reshape(-1))
        for name in _FIELDS_OPT_I32:
            v = getattr(self, name)
            setattr(self, name, np.zeros(0, np.int32) if v is None else
                    np.ascontiguousarray(v, dtype=np.int32).reshape(-1))
        for name in _FIELDS_OPT_F64:
            v = getattr(self, name)
            setattr(self, name, np.zeros(0, np.float64) if v is None else
                    np.ascontiguousarray(v, dtype=np.float64).reshape(-1))
        if self.param_weight is not None:
            self.param_weight = np.ascontiguousarray(self.param_weight,
                                                     dtype=np.float64).reshape(-1)
        if self.cam_rs_value is not None:
            self.cam_rs_value = np.ascontiguousarray(self.cam_rs_value,
                                                     dtype=np.float64).reshape(-1)
        if self.lens_input is not None:
            self.lens_input = np.ascontiguousarray(self.lens_input, dtype=np.int32).reshape(-1)
        if self.lens_input_values is not None:
            self.lens_input_values = np.ascontiguousarray(self.lens_input_values,
                                                          dtype=np.float64).reshape(-1)
        for name in ("param_ref_attr", "ref_attr_lens"):
            if getattr(self, name) is not None:
                setattr(self, name, np.ascontiguousarray(getattr(self, name),
                                                         dtype=np.int32).reshape(-1))
        if self.mkr_frame_xy is not None:
            self.mkr_frame_xy = np.ascontiguousarray(self.mkr_frame_xy,
                                                     dtype=np.float64).reshape(-1)

    # sizes -------------------------------------------------------------
    @property
    def num_obs(self):
        return int(self.obs_marker.size)

    @property
    def num_params(self):
        return int(self.param_attr.size)

    @property
    def num_stiff(self):
        return int(self.stiff_attr.size)

    @property
    def num_smooth(self):
        return int(self.smooth_attr.size)

    @property
    def num_residuals(self):
        """2 per observation, then the stiffness and smoothness rows."""
        return 2 * self.num_obs + self.num_stiff + self.num_smooth

    @property
    def num_cameras(self):
        return int(self.cam_tfm.size)

    @property
    def num_bundles(self):
        return int(self.bnd_tfm.size)

    @property
    def num_markers(self):
        return int(self.mkr_cam.size)

    # ctypes -------------------------------------------------------------
    def to_ctypes(self):
        """Return (MmbaProblem, keepalive).  The arrays are referenced, not copied."""
        def ptr(arr, ctype):
            if arr.size == 0:
                return C.cast(None, C.POINTER(ctype))
            return arr.ctypes.data_as(C.POINTER(ctype))

        p = abi.MmbaProblem()
        p.num_frames = int(self.num_frames)
        p.num_attrs = int(self.attr_animated.size)
        p.attr_animated = ptr(self.attr_animated, C.c_int32)
        p.attr_offset = ptr(self.attr_offset, C.c_int64)
        p.attr_values = ptr(self.attr_values, C.c_double)
        p.num_transforms = int(self.tfm_parent.size)
        p.tfm_parent = ptr(self.tfm_parent, C.c_int32)
        p.tfm_rotate_order = ptr(self.tfm_rotate_order, C.c_int32)
        p.tfm_attrs = ptr(self.tfm_attrs, C.c_int32)
        p.num_cameras = self.num_cameras
        p.cam_tfm = ptr(self.cam_tfm, C.c_int32)
        p.cam_attrs = ptr(self.cam_attrs, C.c_int32)
        p.cam_film_fit = ptr(self.cam_film_fit, C.c_int32)
        p.cam_render_size = ptr(self.cam_render_size, C.c_int32)
        p.cam_lens = ptr(self.cam_lens, C.c_int32)
        p.num_lenses = int(self.lens_type.size)
        p.lens_type = ptr(self.lens_type, C.c_int32)
        p.lens_attrs = ptr(self.lens_attrs, C.c_int32)
        p.num_bundles = self.num_bundles
        p.bnd_tfm = ptr(self.bnd_tfm, C.c_int32)
        p.num_markers = self.num_markers
        p.mkr_cam = ptr(self.mkr_cam, C.c_int32)
        p.mkr_bnd = ptr(self.mkr_bnd, C.c_int32)
        p.num_obs = self.num_obs
        p.obs_marker = ptr(self.obs_marker, C.c_int32)
        p.obs_frame = ptr(self.obs_frame, C.c_int32)
        p.obs_xy = ptr(self.obs_xy, C.c_double)
        p.obs_weight = ptr(self.obs_weight, C.c_double)
        p.num_params = self.num_params
        p.param_attr = ptr(self.param_attr, C.c_int32)
        p.param_frame = ptr(self.param_frame, C.c_int32)
        p.param_min = ptr(self.param_min, C.c_double)
        p.param_max = ptr(self.param_max, C.c_double)
        p.param_offset = ptr(self.param_offset, C.c_double)
        p.param_scale = ptr(self.param_scale, C.c_double)
        p.param_weight = (ptr(self.param_weight, C.c_double) if self.param_weight is not None
                          else C.cast(None, C.POINTER(C.c_double)))
        p.num_stiff = self.num_stiff
        p.stiff_attr = ptr(self.stiff_attr, C.c_int32)
        p.stiff_frame = ptr(self.stiff_frame, C.c_int32)
        p.stiff_weight = ptr(self.stiff_weight, C.c_double)
        p.stiff_variance = ptr(self.stiff_variance, C.c_double)
        p.stiff_value = ptr(self.stiff_value, C.c_double)
        p.num_smooth = self.num_smooth
        p.smooth_attr = ptr(self.smooth_attr, C.c_int32)
        p.smooth_frame = ptr(self.smooth_frame, C.c_int32)
        p.smooth_weight = ptr(self.smooth_weight, C.c_double)
        p.smooth_variance = ptr(self.smooth_variance, C.c_double)
        p.smooth_value = ptr(self.smooth_value, C.c_double)
        p.cam_rs_value = (ptr(self.cam_rs_value, C.c_double) if self.cam_rs_value is not None
                          else C.cast(None, C.POINTER(C.c_double)))
        p.lens_input = (ptr(self.lens_input, C.c_int32) if self.lens_input is not None
                        else C.cast(None, C.POINTER(C.c_int32)))
        p.lens_input_values = (ptr(self.lens_input_values, C.c_double)
                               if self.lens_input_values is not None
                               else C.cast(None, C.POINTER(C.c_double)))
        p.param_ref_attr = (ptr(self.param_ref_attr, C.c_int32)
                            if self.param_ref_attr is not None
                            else C.cast(None, C.POINTER(C.c_int32)))
        p.num_ref_attrs = int(self.ref_attr_lens.size) if self.ref_attr_lens is not None else 0
        p.ref_attr_lens = (ptr(self.ref_attr_lens, C.c_int32) if self.ref_attr_lens is not None
                           else C.cast(None, C.POINTER(C.c_int32)))
        p.mkr_frame_xy = (ptr(self.mkr_frame_xy, C.c_double) if self.mkr_frame_xy is not None
                          else C.cast(None, C.POINTER(C.c_double)))
        return p, [self]

    # (de)serialisation ---------------------------------------------------
    def to_npz_dict(self):
        d = {name: getattr(self, name) for name in _FIELDS_I32 + _FIELDS_I64 + _FIELDS_F64}
        d["num_frames"] = np.array(self.num_frames, dtype=np.int64)
        if self.num_stiff or self.num_smooth:
            for name in _FIELDS_OPT_I32 + _FIELDS_OPT_F64:
                d[name] = getattr(self, name)
        if self.param_weight is not None:
            d["param_weight"] = self.param_weight
        if self.cam_rs_value is not None:
            d["cam_rs_value"] = self.cam_rs_value
        for name in ("lens_input", "lens_input_values", "param_ref_attr", "ref_attr_lens",
                     "mkr_frame_xy"):
            if getattr(self, name) is not None:
                d[name] = getattr(self, name)
        return d

    @classmethod
    def from_npz_dict(cls, d):
        kw = {name: np.asarray(d[name]) for name in _FIELDS_I32 + _FIELDS_I64 + _FIELDS_F64}
        nl = int(np.asarray(kw["lens_type"]).size)
        la = np.asarray(kw["lens_attrs"], dtype=np.int32).reshape(-1)
        if nl and la.size == 5 * nl:  # fixtures written with the 5-slot (classic-only) stride
            la = np.concatenate([la.reshape(nl, 5), -np.ones((nl, abi.LENS_NUM_ATTRS - 5),
                                                             np.int32)], axis=1).reshape(-1)
            kw["lens_attrs"] = la
        for name in _FIELDS_OPT_I32 + _FIELDS_OPT_F64 + ["param_weight", "cam_rs_value",
                                                          "lens_input", "lens_input_values",
                                                          "param_ref_attr", "ref_attr_lens",
                                                          "mkr_frame_xy"]:
            if name in d:
                kw[name] = np.asarray(d[name])
        return cls(num_frames=int(d["num_frames"]), **kw)

    def with_x0(self, x0):
        d = self.to_npz_dict()
        d["x0"] = np.asarray(x0, dtype=np.float64)
        p = Problem.from_npz_dict(d)
        p.meta = dict(self.meta)
        return p

    def external_params(self, x):
        """Internal parameter vector -> attribute (external) values
        (``parameterBoundFromInternalToExternal`` vectorised over parameters)."""
        v = np.asarray(x, dtype=np.float64)
        lo, hi = self.param_min, self.param_max
        off, sc = self.param_offset, self.param_scale
        unb = (lo <= -FLOAT_MAX) & (hi >= FLOAT_MAX)
        up_inf = ~unb & (hi >= FLOAT_MAX)
        lo_inf = ~unb & ~up_inf & (lo <= -FLOAT_MAX)
        both = ~unb & ~up_inf & ~lo_inf
        out = np.where(unb, v, 0.0)
        r = np.sqrt(v * v + 1.0)
        out = np.where(up_inf, lo - (1.0 + r), out)
        out = np.where(lo_inf, hi + (1.0 - r), out)
        out = np.where(both, lo + ((hi - lo) / 2.0) * (np.sin(v) + 1.0), out)
        out = out / sc - off
        return np.minimum(np.maximum(out, lo), hi)


class SceneBuilder:
    """Build an mmSolver-like scene (cameras, bundles, markers, frames).

    Attribute values use Maya UI units (degrees, mm focal, inch film back).
    """

    def __init__(self, num_frames: int):
        assert num_frames > 0
        self.F = int(num_frames)
        self._attr_animated: List[int] = []
        self._attr_offset: List[int] = []
        self._values: List[float] = []
        self._tfm_parent: List[int] = []
        self._tfm_roo: List[int] = []
        self._tfm_attrs: List[List[int]] = []
        self._cam_tfm: List[int] = []
        self._cam_attrs: List[List[int]] = []
        self._cam_fit: List[int] = []
        self._cam_size: List[List[int]] = []
        self._cam_lens: List[int] = []
        self._lens_type: List[int] = []
        self._lens_attrs: List[List[int]] = []
        self._lens_input: Dict[int, int] = {}
        self._bnd_tfm: List[int] = []
        self._mkr_cam: List[int] = []
        self._mkr_bnd: List[int] = []
        self._mkr_xy: List[np.ndarray] = []
        self._mkr_enable: List[np.ndarray] = []
        self._mkr_weight: List[np.ndarray] = []
        self._mkr_overscan: List[tuple] = []
        self._solve: List[tuple] = []
        self._bulk = None
        self._stiff: List[tuple] = []
        self._smooth: List[tuple] = []

    # attributes -----------------------------------------------------------
    def attr(self, value: Value) -> int:
        """Create an attribute; a scalar is static, an F-length array animated."""
        arr = np.asarray(value, dtype=np.float64)
        aid = len(self._attr_animated)
        self._attr_offset.append(len(self._values))
        if arr.ndim == 0:
            self._attr_animated.append(0)
            self._values.append(float(arr))
        else:
            assert arr.shape == (self.F,), arr.shape
            self._attr_animated.append(1)
            self._values.extend(float(v) for v in arr)
        return aid

    def attr_value(self, aid: int, frame: int) -> float:
        off = self._attr_offset[aid]
        return self._values[off + (frame if self._attr_animated[aid] else 0)]

    def _as_attr(self, v, default):
        if v is None:
            v = default
        if isinstance(v, AttrRef):
            return v.aid
        return self.attr(v)

    # nodes ----------------------------------------------------------------
    def transform(self, t=(0.0, 0.0, 0.0), r=(0.0, 0.0, 0.0), s=(1.0, 1.0, 1.0),
                  parent: Optional[int] = None, rotate_order: int = abi.ROO_XYZ):
        """Returns (transform index, [9 attr ids])."""
        ids = [self._as_attr(v, 0.0) for v in t] + [self._as_attr(v, 0.0) for v in r] + \
              [self._as_attr(v, 1.0) for v in s]
        idx = len(self._tfm_parent)
        if parent is not None:
            assert 0 <= parent < idx, "transforms must be created parent-first"
        self._tfm_parent.append(-1 if parent is None else int(parent))
        self._tfm_roo.append(int(rotate_order))
        self._tfm_attrs.append(ids)
        return idx, ids

    def camera(self, tfm: int, focal=35.0, film_back=(36.0 / 25.4, 24.0 / 25.4),
               film_offset=(0.0, 0.0), film_fit=abi.FILM_FIT_HORIZONTAL,
               render_size=(2048, 1556), far_clip=10000.0, camera_scale=1.0,
               lens: int = -1):
        """Returns (camera index, [8 attr ids])."""
        ids = [None] * abi.CAM_NUM_ATTRS
        ids[abi.CAM_FILM_BACK_W_INCH] = self._as_attr(film_back[0], 36.0 / 25.4)
        ids[abi.CAM_FILM_BACK_H_INCH] = self._as_attr(film_back[1], 24.0 / 25.4)
        ids[abi.CAM_FOCAL_MM] = self._as_attr(focal, 35.0)
        ids[abi.CAM_FILM_OFFSET_X_INCH] = self._as_attr(film_offset[0], 0.0)
        ids[abi.CAM_FILM_OFFSET_Y_INCH] = self._as_attr(film_offset[1], 0.0)
        ids[abi.CAM_NEAR_CLIP] = self._as_attr(0.1, 0.1)
        ids[abi.CAM_FAR_CLIP] = self._as_attr(far_clip, 10000.0)
        ids[abi.CAM_SCALE] = self._as_attr(camera_scale, 1.0)
        idx = len(self._cam_tfm)
        self._cam_tfm.append(int(tfm))
        self._cam_attrs.append(ids)
        self._cam_fit.append(int(film_fit))
        self._cam_size.append([int(render_size[0]), int(render_size[1])])
        self._cam_lens.append(int(lens))
        return idx, ids

    def lens_3de_classic(self, distortion=0.0, anamorphic_squeeze=1.0, curvature_x=0.0,
                         curvature_y=0.0, quartic_distortion=0.0):
        """Returns (lens index, [5 attr ids])."""
        ids = [self._as_attr(distortion, 0.0), self._as_attr(anamorphic_squeeze, 1.0),
               self._as_attr(curvature_x, 0.0), self._as_attr(curvature_y, 0.0),
               self._as_attr(quartic_distortion, 0.0)]
        idx = len(self._lens_type)
        self._lens_type.append(abi.LENS_3DE_CLASSIC)
        self._lens_attrs.append(ids + [-1] * (abi.LENS_NUM_ATTRS - len(ids)))
        return idx, ids

    def lens_3de_radial_std_deg4(self, degree2_distortion=0.0, degree2_u=0.0, degree2_v=0.0,
                                 degree4_distortion=0.0, degree4_u=0.0, degree4_v=0.0,
                                 cylindric_direction=0.0, cylindric_bending=0.0):
        """3DE radial decentered deg 4 cylindric lens (mmlens
        LensModel3deRadialDecenteredDeg4Cylindric).  Returns (lens index, [8 attr ids])."""
        vals = (degree2_distortion, degree2_u, degree2_v, degree4_distortion, degree4_u,
                degree4_v, cylindric_direction, cylindric_bending)
        ids = [self._as_attr(v, 0.0) for v in vals]
        idx = len(self._lens_type)
        self._lens_type.append(abi.LENS_3DE_RADIAL_STD_DEG4)
        self._lens_attrs.append(ids + [-1] * (abi.LENS_NUM_ATTRS - len(ids)))
        return idx, ids

    def lens_3de_anamorphic_std_deg4(self, cx02=0.0, cy02=0.0, cx22=0.0, cy22=0.0, cx04=0.0,
                                     cy04=0.0, cx24=0.0, cy24=0.0, cx44=0.0, cy44=0.0,
                                     lens_rotation=0.0, squeeze_x=1.0, squeeze_y=1.0,
                                     rescale=None):
        """3DE anamorphic deg 4 rotate squeeze xy lens (mmlens
        LensModel3deAnamorphicDeg4RotateSqueezeXY); with ``rescale`` the
        "Rescaled" variant.  Returns (lens index, [13 or 14 attr ids])."""
        vals = (cx02, cy02, cx22, cy22, cx04, cy04, cx24, cy24, cx44, cy44, lens_rotation)
        ids = [self._as_attr(v, 0.0) for v in vals]
        ids += [self._as_attr(squeeze_x, 1.0), self._as_attr(squeeze_y, 1.0)]
        kind = abi.LENS_3DE_ANAMORPHIC_STD_DEG4
        if rescale is not None:
            ids.append(self._as_attr(rescale, 1.0))
            kind = abi.LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED
        idx = len(self._lens_type)
        self._lens_type.append(kind)
        self._lens_attrs.append(ids + [-1] * (abi.LENS_NUM_ATTRS - len(ids)))
        return idx, ids

    def lens_input(self, lens: int, input_lens: int):
        """Layer ``input_lens`` under ``lens`` (a lens node's inLens connection,
        mmba.h ABI 5): the input layer's values are constants of the solve."""
        assert 0 <= lens < len(self._lens_type) and 0 <= input_lens < len(self._lens_type)
        self._lens_input[int(lens)] = int(input_lens)

    def bundle(self, tfm: int) -> int:
        self._bnd_tfm.append(int(tfm))
        return len(self._bnd_tfm) - 1

    def marker(self, cam: int, bnd: int, xy, enable=None, weight=None,
               overscan=(1.0, 1.0)) -> int:
        """``xy``: (F, 2) marker translate X/Y (film-back units, -0.5..0.5)."""
        xy = np.asarray(xy, dtype=np.float64).reshape(self.F, 2)
        en = np.ones(self.F, dtype=bool) if enable is None else np.asarray(enable, dtype=bool)
        if weight is None:
            w = np.ones(self.F)
        else:
            w = np.broadcast_to(np.asarray(weight, dtype=np.float64), (self.F,)).copy()
        self._mkr_cam.append(int(cam))
        self._mkr_bnd.append(int(bnd))
        self._mkr_xy.append(xy)
        self._mkr_enable.append(en)
        self._mkr_weight.append(w)
        self._mkr_overscan.append((float(overscan[0]), float(overscan[1])))
        return len(self._mkr_cam) - 1

    def markers_bulk(self, mkr_cam, mkr_bnd, obs_marker, obs_frame, obs_xy, obs_weight=None):
        """Bulk markers for large scenes: observations given directly (already
        overscan-corrected, any order; sorted marker-major/frame-minor here)."""
        assert not self._mkr_cam, "bulk markers cannot be mixed with marker()"
        m = np.asarray(obs_marker, dtype=np.int64)
        f = np.asarray(obs_frame, dtype=np.int64)
        order = np.lexsort((f, m))
        xy = np.asarray(obs_xy, dtype=np.float64).reshape(-1, 2)[order]
        w = np.ones(m.size) if obs_weight is None else np.asarray(obs_weight, np.float64)[order]
        self._bulk = (np.asarray(mkr_cam, np.int32), np.asarray(mkr_bnd, np.int32),
                      m[order].astype(np.int32), f[order].astype(np.int32), xy, w)

    def solve(self, aid: int, xmin=None, xmax=None, offset=None, scale=None):
        """Mark an attribute as solved (the ``-attr`` flag order = param order)."""
        self._solve.append((int(aid),
                            -FLOAT_MAX if xmin is None else float(xmin),
                            FLOAT_MAX if xmax is None else float(xmax),
                            0.0 if offset is None else float(offset),
                            1.0 if scale is None else float(scale)))

    def stiffness(self, aid: int, weight: float, variance: float, value: float, frame: int = 0):
        """Attribute stiffness row (StiffAttrs: weight / variance / value
        attributes, adjust_measureErrors.cpp:318-348); rows with weight <= 0
        are not counted (adjust_relationships.cpp:186-199)."""
        self._stiff.append((int(aid), int(frame), float(weight), float(variance), float(value)))

    def smoothness(self, aid: int, weight: float, variance: float, value: float, frame: int = 0):
        """Attribute smoothness row (adjust_measureErrors.cpp:353-387)."""
        self._smooth.append((int(aid), int(frame), float(weight), float(variance), float(value)))

    # assembly ---------------------------------------------------------------
    def build(self, meta=None) -> Problem:
        F = self.F
        # countUpNumberOfErrors
        obs_m, obs_f, obs_xy, obs_w = [], [], [], []
        mkr_cam, mkr_bnd = self._mkr_cam, self._mkr_bnd
        if self._bulk is not None:
            mkr_cam, mkr_bnd, obs_m, obs_f, obs_xy, obs_w = self._bulk
            keep = obs_w > 0.0
            obs_m, obs_f, obs_xy, obs_w = obs_m[keep], obs_f[keep], obs_xy[keep], obs_w[keep]
        for k in range(len(self._mkr_cam)):
            ox, oy = self._mkr_overscan[k]
            sx, sy = 1.0 / ox, 1.0 / oy
            for f in range(F):
                w = self._mkr_weight[k][f]
                if self._mkr_enable[k][f] and w > 0.0:
                    obs_m.append(k)
                    obs_f.append(f)
                    obs_xy.append((self._mkr_xy[k][f, 0] * sx, self._mkr_xy[k][f, 1] * sy))
                    obs_w.append(w)
        obs_m = np.asarray(obs_m, dtype=np.int32)
        obs_f = np.asarray(obs_f, dtype=np.int32)
        obs_w = np.asarray(obs_w, dtype=np.float64)
        if obs_w.size:
            wmax = np.zeros(F)
            np.maximum.at(wmax, obs_f, obs_w)
            obs_w = obs_w / wmax[obs_f]
        # countUpNumberOfUnknownParameters
        pa, pf, pmin, pmax, poff, pscl, x0 = [], [], [], [], [], [], []
        for aid, xmin, xmax, off, scl in self._solve:
            frames = range(F) if self._attr_animated[aid] else [-1]
            for f in frames:
                pa.append(aid)
                pf.append(f)
                pmin.append(xmin)
                pmax.append(xmax)
                poff.append(off)
                pscl.append(scl)
                v = self.attr_value(aid, max(f, 0))
                x0.append(param_external_to_internal(v, xmin, xmax, off, scl))
        prob = Problem(
            num_frames=F,
            attr_animated=self._attr_animated,
            attr_offset=self._attr_offset,
            attr_values=self._values,
            tfm_parent=self._tfm_parent,
            tfm_rotate_order=self._tfm_roo,
            tfm_attrs=np.asarray(self._tfm_attrs, dtype=np.int32).reshape(-1),
            cam_tfm=self._cam_tfm,
            cam_attrs=np.asarray(self._cam_attrs, dtype=np.int32).reshape(-1),
            cam_film_fit=self._cam_fit,
            cam_render_size=np.asarray(self._cam_size, dtype=np.int32).reshape(-1),
            cam_lens=self._cam_lens,
            lens_type=self._lens_type,
            lens_attrs=np.asarray(self._lens_attrs, dtype=np.int32).reshape(-1),
            bnd_tfm=self._bnd_tfm,
            mkr_cam=mkr_cam,
            mkr_bnd=mkr_bnd,
            obs_marker=obs_m,
            obs_frame=obs_f,
            obs_xy=np.asarray(obs_xy, dtype=np.float64).reshape(-1),
            obs_weight=obs_w,
            param_attr=pa,
            param_frame=pf,
            param_min=pmin,
            param_max=pmax,
            param_offset=poff,
            param_scale=pscl,
            x0=x0,
        )
        # countUpNumberOfErrors counts rows with weight > 0; measureErrors then
        # reads the first `count` entries of the list (reference indexing)
        for kind, rows in (("stiff", self._stiff), ("smooth", self._smooth)):
            count = sum(1 for r in rows if r[2] > 0.0)
            use = rows[:count]
            setattr(prob, kind + "_attr", np.array([r[0] for r in use], np.int32))
            setattr(prob, kind + "_frame", np.array([r[1] for r in use], np.int32))
            setattr(prob, kind + "_weight", np.array([r[2] for r in use], np.float64))
            setattr(prob, kind + "_variance", np.array([r[3] for r in use], np.float64))
            setattr(prob, kind + "_value", np.array([r[4] for r in use], np.float64))
        if self._lens_input:
            li = np.full(len(self._lens_type), -1, np.int32)
            for k, v in self._lens_input.items():
                li[k] = v
            prob.lens_input = li
        prob.meta = dict(meta or {})
        return prob


class AttrRef:
    """Reference an existing attribute id when creating nodes."""

    def __init__(self, aid: int):
        self.aid = int(aid)
