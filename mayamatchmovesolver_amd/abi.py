"""ctypes mirror of include/mmba.h (the drop-in C ABI).

Only plain data layouts live here; loading the HIP library is in ``_lib.py``.
Field order and types must match ``include/mmba.h`` exactly.
"""
import ctypes as C

MMBA_OK = 0
MMBA_ERR_INVALID = -1
MMBA_ERR_DEVICE = -2
MMBA_ERR_UNSUPPORTED = -3
MMBA_ERR_INTERRUPTED = -4
MMBA_ERR_NO_DEVICE = -5
MMBA_ERR_COMM = -6

SOLVER_TYPE_CMINPACK_LMDIF = 1
SOLVER_TYPE_CMINPACK_LMDER = 2
SCENE_GRAPH_MODE_MAYA_DAG = 1
SCENE_GRAPH_MODE_MM_SCENE_GRAPH = 2
AUTO_DIFF_TYPE_FORWARD = 0
AUTO_DIFF_TYPE_CENTRAL = 1
ROBUST_LOSS_TYPE_TRIVIAL = 0
ROBUST_LOSS_TYPE_SOFT_L_ONE = 1
ROBUST_LOSS_TYPE_CAUCHY = 2
ABI_VERSION = 10

# mmba_debug_set_path keys (test hook: pin a plan-builder choice)
PATH_PCR = 1
PATH_SHARD_BCR = 2
PATH_BCR_DATAFLOW = 3
PATH_BCR_GRID = 4
PATH_DENSE = 5
PATH_PERFRAME_BATCH = 6
PATH_LOCAL_RING = 7
PATH_PROBE = 8
PATH_SHARD_SEP = 9
PATH_TRIAL_RECORDS = 10
PATH_LENS_CF = 11
PATH_DEST_LANE = 12
PATH_FAULT_SHARD = 13
PATH_COMM_TIMEOUT_MS = 14
PATH_STALL_SHARD = 15
PATH_PCR_CHAIN = 16
PATH_BACKSUB_ONEPASS = 17
PATH_JB_RECOMPUTE = 18
PATH_NE_CF_SPLIT = 19
PATH_RED_BD = 20
PATH_HANDBACK_DMA = 21
PATH_PRE_HANDBACK = 22
PATH_PRE_SCHUR = 23
PATH_NUM = 24

FILM_FIT_FILL = 0
FILM_FIT_HORIZONTAL = 1
FILM_FIT_VERTICAL = 2
FILM_FIT_OVERSCAN = 3

ROO_XYZ, ROO_YZX, ROO_ZXY, ROO_XZY, ROO_YXZ, ROO_ZYX = range(6)

LENS_NONE = 0
LENS_3DE_CLASSIC = 1
LENS_3DE_RADIAL_STD_DEG4 = 2
LENS_3DE_ANAMORPHIC_STD_DEG4 = 3
LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED = 4

CAM_FILM_BACK_W_INCH = 0
CAM_FILM_BACK_H_INCH = 1
CAM_FOCAL_MM = 2
CAM_FILM_OFFSET_X_INCH = 3
CAM_FILM_OFFSET_Y_INCH = 4
CAM_NEAR_CLIP = 5
CAM_FAR_CLIP = 6
CAM_SCALE = 7
CAM_NUM_ATTRS = 8
LENS_NUM_ATTRS = 14

_i32p = C.POINTER(C.c_int32)
_i64p = C.POINTER(C.c_int64)
_f64p = C.POINTER(C.c_double)


class MmbaProblem(C.Structure):
    _fields_ = [
        ("num_frames", C.c_int32),
        ("num_attrs", C.c_int32),
        ("attr_animated", _i32p),
        ("attr_offset", _i64p),
        ("attr_values", _f64p),
        ("num_transforms", C.c_int32),
        ("tfm_parent", _i32p),
        ("tfm_rotate_order", _i32p),
        ("tfm_attrs", _i32p),
        ("num_cameras", C.c_int32),
        ("cam_tfm", _i32p),
        ("cam_attrs", _i32p),
        ("cam_film_fit", _i32p),
        ("cam_render_size", _i32p),
        ("cam_lens", _i32p),
        ("num_lenses", C.c_int32),
        ("lens_type", _i32p),
        ("lens_attrs", _i32p),
        ("num_bundles", C.c_int32),
        ("bnd_tfm", _i32p),
        ("num_markers", C.c_int32),
        ("mkr_cam", _i32p),
        ("mkr_bnd", _i32p),
        ("num_obs", C.c_int32),
        ("obs_marker", _i32p),
        ("obs_frame", _i32p),
        ("obs_xy", _f64p),
        ("obs_weight", _f64p),
        ("num_params", C.c_int32),
        ("param_attr", _i32p),
        ("param_frame", _i32p),
        ("param_min", _f64p),
        ("param_max", _f64p),
        ("param_offset", _f64p),
        ("param_scale", _f64p),
        # ABI 2
        ("param_weight", _f64p),
        ("num_stiff", C.c_int32),
        ("stiff_attr", _i32p),
        ("stiff_frame", _i32p),
        ("stiff_weight", _f64p),
        ("stiff_variance", _f64p),
        ("stiff_value", _f64p),
        ("num_smooth", C.c_int32),
        ("smooth_attr", _i32p),
        ("smooth_frame", _i32p),
        ("smooth_weight", _f64p),
        ("smooth_variance", _f64p),
        ("smooth_value", _f64p),
        # ---- ABI 3 ----
        ("cam_rs_value", _f64p),
        # ---- ABI 5 ----
        ("lens_input", _i32p),
        ("lens_input_values", _f64p),
        # ABI 7: the reference's lens index arithmetic (Appendix B3)
        ("param_ref_attr", _i32p),
        ("num_ref_attrs", C.c_int32),
        ("ref_attr_lens", _i32p),
        # ABI 8: MMSG flat marker positions (Appendix B4)
        ("mkr_frame_xy", _f64p),
    ]


class MmbaOptions(C.Structure):
    _fields_ = [
        ("solver_type", C.c_int32),
        ("iter_max", C.c_int32),
        ("tau", C.c_double),
        ("eps1", C.c_double),
        ("eps2", C.c_double),
        ("eps3", C.c_double),
        ("delta", C.c_double),
        ("auto_diff_type", C.c_int32),
        ("auto_param_scale", C.c_int32),
        ("scene_graph_mode", C.c_int32),
        ("image_width", C.c_double),
        ("accept_only_better", C.c_int32),
        ("log_level", C.c_int32),
        # ABI 2
        ("robust_loss", C.c_int32),
        ("robust_loss_type", C.c_int32),
        ("robust_loss_scale", C.c_double),
        ("initial_error_given", C.c_int32),
        ("pad_opt0", C.c_int32),
        ("initial_error_avg", C.c_double),
    ]


class MmbaResult(C.Structure):
    _fields_ = [
        ("success", C.c_int32),
        ("reason_number", C.c_int32),
        ("iterations", C.c_int32),
        ("function_evals", C.c_int32),
        ("jacobian_evals", C.c_int32),
        ("outer_iterations", C.c_int32),
        ("user_interrupted", C.c_int32),
        ("error_is_better", C.c_int32),
        ("error_final", C.c_double),
        ("error_avg", C.c_double),
        ("error_min", C.c_double),
        ("error_max", C.c_double),
        ("error_initial_avg", C.c_double),
        ("error_rms", C.c_double),
        ("num_trace", C.c_int32),
        ("pad0", C.c_int32),
        ("time_solve_s", C.c_double),
        ("time_func_s", C.c_double),
        ("time_jac_s", C.c_double),
        ("time_linear_s", C.c_double),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_ if name != "pad0"}


INTERRUPT_FN = C.CFUNCTYPE(C.c_int, C.c_void_p)
PROGRESS_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int)


class MmbaCallbacks(C.Structure):
    _fields_ = [
        ("interrupt", INTERRUPT_FN),
        ("progress", PROGRESS_FN),
        ("user", C.c_void_p),
    ]


class MmbaTrace(C.Structure):
    _fields_ = [
        ("fnorm", _f64p),
        ("capacity", C.c_int32),
        ("count", C.c_int32),
    ]


class MmbaKernelStats(C.Structure):
    _fields_ = [
        ("jac_ms_avg", C.c_double),
        ("jac_bytes", C.c_double),
        ("jac_launches", C.c_int32),
        ("resid_ms_avg", C.c_double),
        ("resid_bytes", C.c_double),
        ("resid_launches", C.c_int32),
        ("chol_ms_avg", C.c_double),
        ("chol_flops", C.c_double),
        ("chol_launches", C.c_int32),
        ("reduced_dim", C.c_int32),
        ("reduced_kind", C.c_int32),
        ("dataflow_fallback", C.c_int32),
        ("shards_replicated", C.c_int32),
        ("spec_replays", C.c_int32),
        ("band_solver", C.c_int32),
        ("band_levels", C.c_int32),
        ("band_block", C.c_int32),
        ("chol_flops_alg", C.c_double),
        ("pre_handbacks", C.c_int32),
        ("reserved10", C.c_int32),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# Functions exported by libmmba.so (checked by tests/test_abi.py against
# include/mmba.h).
EXPORTED_SYMBOLS = [
    "mmba_abi_version",
    "mmba_device_count",
    "mmba_last_error",
    "mmba_options_default",
    "mmba_param_external_to_internal",
    "mmba_param_internal_to_external",
    "mmba_context_create",
    "mmba_context_create_multi",
    "mmba_context_num_devices",
    "mmba_plan_num_shards",
    "mmba_debug_reduced_residual",
    "mmba_context_destroy",
    "mmba_context_synchronize",
    "mmba_host_alloc",
    "mmba_host_free",
    "mmba_plan_create",
    "mmba_plan_destroy",
    "mmba_comm_unique_id",
    "mmba_shard_layout",
    "mmba_comm_create_rccl",
    "mmba_comm_create_local",
    "mmba_comm_destroy",
    "mmba_comm_count",
    "mmba_plan_create_sharded",
    "mmba_plan_measure",
    "mmba_plan_reproject",
    "mmba_solve_per_frame",
    "mmba_plan_solve_per_frame",
    "mmba_plan_set_attr_values",
    "mmba_plan_jacobian",
    "mmba_plan_solve",
    "mmba_plan_outputs",
    "mmba_solve",
    "mmba_plan_kernel_stats",
    "mmba_debug_set_path",
    "mmba_debug_band_solve",
    "mmba_debug_comm_allreduce",
    "mmba_debug_dgemm",
]
