/*
 * mmba.h -- C ABI of the MI355X bundle-adjustment core ("mmba").
 *
 * This is the drop-in seam for mmSolver's Levenberg-Marquardt hot path.
 * In the reference, `solveFrames` (src/mmSolver/adjust/adjust_base.cpp:1167-1190)
 * dispatches to
 *
 *   bool solve_3d_cminpack_lmder(SolverOptions&, int numberOfParameters,
 *                                int numberOfErrors,
 *                                std::vector<double>& paramList,   // in: x0 (internal), out: x
 *                                std::vector<double>& errorList,   // out: fvec
 *                                std::vector<double>& paramWeightList,
 *                                SolverData& userData, SolverResult& out);
 *   (src/mmSolver/adjust/adjust_cminpack_lmder.cpp:64-69; lmdif twin at
 *    src/mmSolver/adjust/adjust_cminpack_lmdif.cpp:61-66)
 *
 * `mmba_solve` / `mmba_plan_solve` replace that call.  `mmba_problem` is the
 * Maya-free flattening of `SolverData` after `construct_scene_graph`
 * (src/mmSolver/mayahelper/maya_scene_graph.cpp:1114) and
 * `countUpNumberOfErrors` / `countUpNumberOfUnknownParameters`
 * (src/mmSolver/adjust/adjust_relationships.cpp:75,223): plain SoA arrays,
 * host pointers, no ownership transfer.  Nothing is retained after return
 * except inside an explicitly created plan.
 *
 * All arithmetic is IEEE fp64; all indices are int32.
 */
#ifndef MMBA_H
#define MMBA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MMBA_ABI_VERSION 10

/* Return codes. */
#define MMBA_OK 0
#define MMBA_ERR_INVALID (-1)     /* malformed problem / options          */
#define MMBA_ERR_DEVICE (-2)      /* HIP runtime error                    */
#define MMBA_ERR_UNSUPPORTED (-3) /* valid mmSolver input this core does not (yet) map */
#define MMBA_ERR_INTERRUPTED (-4) /* interrupt callback returned non-zero */
#define MMBA_ERR_NO_DEVICE (-5)   /* no gfx950 device visible             */
#define MMBA_ERR_COMM (-6)        /* RCCL communicator error              */

/* Solver types: same numbers as SOLVER_TYPE_CMINPACK_* (adjust_defines.h:44-52). */
#define MMBA_SOLVER_CMINPACK_LMDIF 1
#define MMBA_SOLVER_CMINPACK_LMDER 2

/* Scene graph modes: same numbers as SCENE_GRAPH_MODE_* (adjust_defines.h:76-77). */
#define MMBA_SCENE_GRAPH_MAYA_DAG 1
#define MMBA_SCENE_GRAPH_MM_SCENE_GRAPH 2

/* Auto-diff types (adjust_defines.h:96-97). */
#define MMBA_AUTO_DIFF_FORWARD 0
#define MMBA_AUTO_DIFF_CENTRAL 1

/* Film fit (lib/rust/mmscenegraph/src/math/camera.rs FilmFit; Maya enum). */
#define MMBA_FILM_FIT_FILL 0
#define MMBA_FILM_FIT_HORIZONTAL 1
#define MMBA_FILM_FIT_VERTICAL 2
#define MMBA_FILM_FIT_OVERSCAN 3

/* Rotate orders (maya_camera.cpp:921-941 / euler.rs). */
#define MMBA_ROO_XYZ 0
#define MMBA_ROO_YZX 1
#define MMBA_ROO_ZXY 2
#define MMBA_ROO_XZY 3
#define MMBA_ROO_YXZ 4
#define MMBA_ROO_ZYX 5

/* Lens model types (mmlens LensModelType, lib/cppbind/mmlens/include/mmlens/
 * _cxxbridge.h:414-421: k3deClassic, k3deRadialStdDeg4). */
#define MMBA_LENS_NONE 0
#define MMBA_LENS_3DE_CLASSIC 1
#define MMBA_LENS_3DE_RADIAL_STD_DEG4 2
#define MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4 3
#define MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED 4

/* Camera attribute slots in `cam_attrs` (8 per camera). */
#define MMBA_CAM_FILM_BACK_W_INCH 0
#define MMBA_CAM_FILM_BACK_H_INCH 1
#define MMBA_CAM_FOCAL_MM 2
#define MMBA_CAM_FILM_OFFSET_X_INCH 3
#define MMBA_CAM_FILM_OFFSET_Y_INCH 4
#define MMBA_CAM_NEAR_CLIP 5
#define MMBA_CAM_FAR_CLIP 6
#define MMBA_CAM_SCALE 7
#define MMBA_CAM_NUM_ATTRS 8

/* Lens attribute slots in `lens_attrs` (14 per lens; -1 = attribute absent,
 * the model's default is used).
 *   3DE classic (LDPK classic order, lens_model_3de_classic.cpp:75-113):
 *     0 distortion, 1 anamorphic squeeze (default 1), 2 curvature x,
 *     3 curvature y, 4 quartic distortion; 5-7 unused.
 *   3DE radial decentered deg 4 cylindric
 *   (lens_model_3de_radial_decentered_deg_4_cylindric.cpp:70-80):
 *     0 degree-2 distortion, 1 degree-2 u, 2 degree-2 v, 3 degree-4 distortion,
 *     4 degree-4 u, 5 degree-4 v, 6 cylindric direction (degrees),
 *     7 cylindric bending.  All default 0.
 *   3DE anamorphic deg 4 rotate squeeze xy (+ rescaled)
 *   (lens_model_3de_anamorphic_deg_4_rotate_squeeze_xy[_rescaled].cpp:53-66):
 *     0 cx02, 1 cy02, 2 cx22, 3 cy22, 4 cx04, 5 cy04, 6 cx24, 7 cy24, 8 cx44,
 *     9 cy44 (default 0), 10 lens rotation (degrees, default 0), 11 squeeze x,
 *     12 squeeze y, 13 rescale (rescaled model only; defaults 1). */
#define MMBA_LENS_NUM_ATTRS 14

/*
 * Flattened problem.  Units are Maya UI units, exactly as the reference
 * solver sees attribute values: translations in scene units, rotations in
 * degrees, focal length in mm, film back / film offset in inches.
 *
 * Attribute values (the mmscenegraph AttrDataBlock, attr/datablock.rs):
 * attribute `a` is static (one value at attr_values[attr_offset[a]]) or
 * animated (num_frames values starting at attr_offset[a]).  An attribute id
 * of -1 in any attribute slot means "constant" with the slot's default
 * (0 for translate/rotate/offset, 1 for scale/camera scale/squeeze,
 * 10000 for far clip, 0.1 for near clip).
 */
typedef struct mmba_problem {
    int32_t num_frames;

    int32_t num_attrs;
    const int32_t *attr_animated; /* [num_attrs] */
    const int64_t *attr_offset;   /* [num_attrs] */
    const double *attr_values;    /* initial (external) values */

    /* Transforms, topologically sorted (parent index < child index). */
    int32_t num_transforms;
    const int32_t *tfm_parent;       /* [num_transforms], -1 = world   */
    const int32_t *tfm_rotate_order; /* [num_transforms]               */
    const int32_t *tfm_attrs;        /* [9*num_transforms] tx ty tz rx ry rz sx sy sz */

    int32_t num_cameras;
    const int32_t *cam_tfm;         /* [num_cameras] transform index  */
    const int32_t *cam_attrs;       /* [8*num_cameras] see MMBA_CAM_* */
    const int32_t *cam_film_fit;    /* [num_cameras]                  */
    const int32_t *cam_render_size; /* [2*num_cameras] width, height  */
    const int32_t *cam_lens;        /* [num_cameras] lens index or -1 (NULL = none) */

    int32_t num_lenses;
    const int32_t *lens_type;  /* [num_lenses] MMBA_LENS_*     */
    const int32_t *lens_attrs; /* [14*num_lenses] attribute ids */

    int32_t num_bundles;
    const int32_t *bnd_tfm; /* [num_bundles] transform index */

    int32_t num_markers;
    const int32_t *mkr_cam; /* [num_markers] camera index */
    const int32_t *mkr_bnd; /* [num_markers] bundle index */

    /* Observations = errorToMarkerList (adjust_relationships.cpp:124-160):
     * marker-major, frame-minor, only enabled frames with weight > 0. */
    int32_t num_obs;
    const int32_t *obs_marker; /* [num_obs] */
    const int32_t *obs_frame;  /* [num_obs] frame index        */
    const double *obs_xy;      /* [2*num_obs] marker x,y with MarkerGroup overscan applied
                                  (markerPosList), before film-fit correction */
    const double *obs_weight;  /* [num_obs] markerWeightList, already normalised per frame
                                  (adjust_relationships.cpp:166-182); sqrt is taken inside */

    /* Parameters = paramToAttrList (adjust_relationships.cpp:223-337). */
    int32_t num_params;
    const int32_t *param_attr;    /* [num_params] attribute id         */
    const int32_t *param_frame;   /* [num_params] frame index, -1 static */
    const double *param_min;      /* [num_params] Attr::getMinimumValue (-FLT_MAX = none) */
    const double *param_max;      /* [num_params] Attr::getMaximumValue (+FLT_MAX = none) */
    const double *param_offset;   /* [num_params] Attr::getOffsetValue */
    const double *param_scale;    /* [num_params] Attr::getScaleValue  */

    /* ---- ABI 2 ---- */
    /* paramWeightList (adjust_base.cpp countUpNumberOfUnknownParameters), the
     * `diag` lmder/lmdif read in mode 2 (auto_param_scale off,
     * adjust_cminpack_lmder.cpp:103-106,151).  NULL = 1.0 for every parameter. */
    const double *param_weight;   /* [num_params] */

    /* Attribute stiffness and smoothness error rows
     * (adjust_measureErrors.cpp:311-387; counted by countUpNumberOfErrors,
     * adjust_relationships.cpp:184-215).  Row i of each list is
     *   ((1 / gaussian(v, value, variance)) - 1) * weight,
     *   gaussian(x, mean, sigma) = exp(-((x - mean)^2 / (2 sigma^2))),
     * with v the attribute's current value (at `frame` for an animated
     * attribute).  The rows follow the 2*num_obs marker rows: stiffness rows,
     * then smoothness rows, exactly as the reference indexes errorList.  Pass
     * the first num_stiff entries of stiffAttrsList (the reference indexes
     * that list by row).  Only the Maya DAG path computes them: in MM Scene
     * Graph mode they stay 0 (adjust_measureErrors.cpp:518). */
    int32_t num_stiff;
    const int32_t *stiff_attr;     /* [num_stiff] attribute id            */
    const int32_t *stiff_frame;    /* [num_stiff] frame index (animated attrs; ignored for static) */
    const double *stiff_weight;    /* [num_stiff] stiffness weight  (> 0)  */
    const double *stiff_variance;  /* [num_stiff] stiffness variance       */
    const double *stiff_value;     /* [num_stiff] stiffness value (mean)   */
    int32_t num_smooth;
    const int32_t *smooth_attr;
    const int32_t *smooth_frame;
    const double *smooth_weight;
    const double *smooth_variance;
    const double *smooth_value;

    /* ---- ABI 3 ---- */
    /* Rolling shutter (BASELINE configs[4]; an extension: the reference
     * solver has no rolling-shutter model, its only rolling-shutter
     * arithmetic is the 3DE exporter's 2D correction,
     * share/3dequalizer/python/uvtrack_format.py:243-330).  Per camera the
     * rolling-shutter value in frames, rs = time shift x fps (:269-270);
     * 0 = a global shutter.  NULL = off for every camera (the reference
     * behaviour).  With rs != 0 and num_frames > 1, the camera transform's
     * translate / rotate attributes seen by observation (marker, frame f) are
     * the exporter's three-frame blend (_apply_rs_correction, :186-203) at the
     * scanline time tau = rs * (0.5 - y) (y = obs_xy's y, film-height units,
     * +y up: the top scanline is read first, :318):
     *   b = (v(f+1) - v(f-1)) / 2,  c = -v(f) + (v(f+1) + v(f-1)) / 2,
     *   v(f + tau) = v(f) + tau b + tau^2 c,
     * with the exporter's end extrapolation v(-1) = v(0) + (v(0) - v(1)),
     * v(F) = v(F-1) + (v(F-1) - v(F-2)) (:311-314).  The FD column of an
     * animated parameter then re-measures frames f-1..f+1.  A camera under a
     * parent blends its own translate / rotate values; its world pose is the
     * parent's world matrix at frame f times the blended local matrix.
     * Supported with forward differences, unsharded, without bundle-side
     * global parameters (MMBA_ERR_UNSUPPORTED otherwise). */
    const double *cam_rs_value;   /* [num_cameras] */

    /* ---- ABI 5 ---- */
    /* Layered lens nodes.  lens_input[l] = the lens chained as the input of
     * lens l (-1 = none).  What the reference solver evaluates for a camera
     * whose lens node has upstream nodes: the per-frame models are clones of
     * the camera-connected node's plug model (maya_lens_model_utils.cpp:
     * 655-662), whose input chain the node's compute set from the upstream
     * nodes' values at the time the plug was read (MMLensModel3deNode.cpp:
     * 164); connectLensModels never re-points it (its loop, :715, does not
     * run), so the input layers are constants of the solve and their
     * attributes, if solved, have zero Jacobian columns.  Distortion applies
     * the deepest input first, the camera's own lens last
     * (lens_model_3de_classic.cpp:82-88).  lens_input_values[14*l + k] =
     * slot k of layer l as read with the plug (absent slots: the model's
     * default); NULL = each slot's attribute value at frame 0.  At most 4
     * input layers per lens; lens_input NULL = no layers (ABI <= 4). */
    const int32_t *lens_input;        /* [num_lenses] */
    const double *lens_input_values;  /* [14*num_lenses] */

    /* ---- ABI 7 ---- */
    /* The reference's lens index arithmetic, reproduced
     * for any lens layout.  The solver keeps num_frames clones of every lens
     * model, instance (l, f) at lensModelList[l*F + f], and two lookup lists
     * built as markerFrame[i*F + f] = instance (cam_lens[mkr_cam[i]], f) and
     * attrFrame[a*F + f] = instance (lens of attrList entry a, f)
     * (maya_lens_model_utils.cpp:655-662, 782-799, 836-851), but reads them at
     * markerIndex + frameIndex (adjust_measureErrors.cpp:244, 463) and at
     * attrIndex + frameIndex / attrIndex + j (adjust_setParameters.cpp:
     * 113-121, 206-214).  So observation (marker i, frame f) is distorted by
     * instance (cam_lens[mkr_cam[(i+f) / F]], (i+f) % F), and solving
     * attribute a at frame g writes its value into the slot of its type of
     * instance (lens of attrList entry (a+g) / F, (a+g) % F) -- a static
     * attribute for every g < F, entries without a lens skipped
     * (setLensModelAttributeValue ignores a null model); the last parameter
     * written wins.  A slot no parameter writes keeps the value the plug
     * model was cloned with (lens_input_values, or each slot's attribute at
     * frame 0; lens attributes are never read per frame, Appendix B11).  With
     * one lens shared by every camera and its attributes first in attrList,
     * every instance holds the same values and this is the plain model.
     *   param_ref_attr[p] = paramToAttrList[p].first, the attribute's index
     *                       in the solver's attrList (NULL: the attributes
     *                       numbered in order of first appearance in the
     *                       parameter list, which is attrList's order when
     *                       every entry has a parameter);
     *   ref_attr_lens[a]  = the lens whose attribute attrList entry a is, -1
     *                       if it is not a lens attribute (NULL: from
     *                       lens_attrs). */
    const int32_t *param_ref_attr;  /* [num_params] */
    int32_t num_ref_attrs;
    const int32_t *ref_attr_lens;   /* [num_ref_attrs] */

    /* ---- ABI 8 ---- */
    /* MM Scene Graph point indexing.  FlatScene emits its
     * point and marker lists camera -> marker -> frame (flat.rs:271-356: the
     * markers of camera 0 in marker order, then camera 1's ...), but
     * measureErrors_mmSceneGraph reads both at markerIndex * F + frameIndex
     * (adjust_measureErrors.cpp:454-459).  So with markers not grouped by
     * ascending camera, observation (marker i, frame f) compares the point
     * and marker position of flat marker k = (i-th marker in camera order) --
     * its camera, bundle, film fit and x,y at frame f -- while its weight,
     * frame enable and lens (B3) stay those of marker i.  mkr_frame_xy gives
     * every marker's x,y at every frame, as obs_xy (the flat marker list
     * before film fit); NULL: a remapped observation takes the x,y of the
     * observation (k, f), and MMBA_ERR_UNSUPPORTED when marker k has none at
     * frame f.  Unused in Maya-DAG mode and when markers are grouped. */
    const double *mkr_frame_xy; /* [2*num_markers*num_frames] */
} mmba_problem;

/* SolverOptions subset that the LM path reads (adjust_data.h:133-185). */
typedef struct mmba_options {
    int32_t solver_type;      /* MMBA_SOLVER_CMINPACK_LMDIF / _LMDER     */
    int32_t iter_max;         /* maxfev                                  */
    double tau;               /* factor = tau * 100                      */
    double eps1;              /* ftol */
    double eps2;              /* xtol */
    double eps3;              /* gtol */
    double delta;             /* FD step (lmder) / epsfcn = |delta| (lmdif) */
    int32_t auto_diff_type;   /* MMBA_AUTO_DIFF_*                        */
    int32_t auto_param_scale; /* 1 -> MINPACK mode 1, else mode 2        */
    int32_t scene_graph_mode; /* MMBA_SCENE_GRAPH_*                      */
    double image_width;       /* pixels (default 2048)                   */
    int32_t accept_only_better; /* report error_is_better against the initial error */
    int32_t log_level;        /* 0 error .. 4 debug                      */

    /* ---- ABI 2 ---- */
    /* Robust loss (applyLossFunctionToErrors, adjust_base.cpp:132-187), applied
     * to every residual row only when robust_loss != 0, i.e. when the solver
     * type supports it (SolverOptions::solverSupportsRobustLoss; false for
     * both cminpack types, adjust_defines.h:122,141 -- so off by default). */
    int32_t robust_loss;        /* solverSupportsRobustLoss                 */
    int32_t robust_loss_type;   /* MMBA_ROBUST_LOSS_*                       */
    double robust_loss_scale;
    /* Initial measurement of solveFrames (adjust_base.cpp:1080-1103).
     * 0 (default): the library measures the errors at the scene's current
     * values before solving.  1: the caller already did; its average error
     * distance is `initial_error_avg` (used for accept-only-better).  Every
     * ABI-2 field is 0 in the reference behaviour, so a zeroed struct plus
     * the ABI-1 fields keeps it. */
    int32_t initial_error_given;
    int32_t pad_opt0;
    double initial_error_avg;
} mmba_options;

/* Robust loss types (adjust_defines.h:96-98). */
#define MMBA_ROBUST_LOSS_TRIVIAL 0
#define MMBA_ROBUST_LOSS_SOFT_L_ONE 1
#define MMBA_ROBUST_LOSS_CAUCHY 2

/* SolverResult mirror (adjust_results.h:59-72) plus run statistics. */
typedef struct mmba_result {
    int32_t success;          /* functionEvals > 0 (adjust_cminpack_lmder.cpp:191) */
    int32_t reason_number;    /* MINPACK info 0..8, negative on interrupt */
    int32_t iterations;       /* nfev */
    int32_t function_evals;   /* iflag=1 calls (userData.iterNum)         */
    int32_t jacobian_evals;   /* FD columns / iflag=2 calls (jacIterNum)  */
    int32_t outer_iterations; /* njev: LM iterations                      */
    int32_t user_interrupted;
    int32_t error_is_better;  /* acceptOnlyBetter outcome (1 = kept solution) */
    double error_final;       /* enorm(fvec) at returned x                */
    double error_avg;         /* pixels; errorDistanceList stats (adjust_base.cpp:346) */
    double error_min;
    double error_max;
    double error_initial_avg; /* before solving (adjust_base.cpp:1080-1103) */
    double error_rms;         /* sqrt(sum dist^2 / M) at returned x, pixels */
    int32_t num_trace;        /* entries written to the fnorm trace        */
    int32_t pad0;
    double time_solve_s;      /* wall time inside the solve                */
    double time_func_s;       /* residual kernels                          */
    double time_jac_s;        /* Jacobian + normal-equation kernels        */
    double time_linear_s;     /* Schur + Cholesky + solves                 */
} mmba_result;

/* Interrupt / progress callbacks.  `interrupt` is polled where the
 * reference polls MComputation::isInterruptRequested: at every solveFunc call
 * (each residual evaluation and each Jacobian request,
 * adjust_solveFunc.cpp:567-571) and before every finite-difference column
 * (:321-325); a non-zero return stops the solve with reason_number -1 and the
 * counts the reference would report.  `progress` is called once per LM outer
 * iteration with the Jacobian count.  Either pointer may be NULL. */
typedef struct mmba_callbacks {
    int (*interrupt)(void *user);           /* non-zero -> stop */
    void (*progress)(void *user, int iter);
    void *user;
} mmba_callbacks;

/* Optional per-evaluation trace: fnorm of every iflag=1 residual
 * evaluation, in call order (first entry = initial point). */
typedef struct mmba_trace {
    double *fnorm;     /* [capacity] */
    int32_t capacity;
    int32_t count;     /* out */
} mmba_trace;

typedef struct mmba_context mmba_context;
typedef struct mmba_plan mmba_plan;

int mmba_abi_version(void);
/* Number of visible gfx950 devices (0 when none). */
int mmba_device_count(void);
/* Last error message of the calling thread. */
const char *mmba_last_error(void);

/* Defaults identical to the cminpack_lmder defaults (adjust_defines.h:129-141). */
void mmba_options_default(mmba_options *opt, int32_t solver_type);

/* Box-constraint reparametrisation (adjust_base.cpp:194-258), bug-compatible. */
double mmba_param_external_to_internal(double value, double xmin, double xmax,
                                       double offset, double scale);
double mmba_param_internal_to_external(double value, double xmin, double xmax,
                                       double offset, double scale);

int mmba_context_create(int device, mmba_context **out);
/* ABI 9: one caller, several devices.  The reference calls solveFrames once,
 * on Maya's main thread (adjust_base.cpp:1174-1183), so the multi-GPU
 * fan-out stays inside the library (SURVEY 8(b) "Threading"): a context over
 * `ndevices` devices (<= 8) -- one stream per device and the group's
 * communicators, RCCL (ncclCommInitAll, in this process) when the devices are
 * distinct, the in-process transport when one device is named ndevices times
 * (a one-GPU box runs the sharded path this way; mixing is MMBA_ERR_INVALID).
 * mmba_plan_create on it builds the frame-sharded plan of
 * mmba_plan_create_sharded over every device, and the plan's entry points
 * (solve, measure, reproject, outputs, set_attr_values, kernel_stats) run all
 * shards from the calling thread: the library's own threads drive devices
 * 1..N-1, the interrupt callback is polled on the calling thread only (its
 * answer reaches every shard), and every shard writes its own parameters and
 * observations straight into the caller's buffers.  A problem that does not
 * shard is solved by the first device alone.  Destroy every plan before the
 * context. */
int mmba_context_create_multi(const int *devices, int ndevices, mmba_context **out);
/* Devices of a context (1 for mmba_context_create). */
int mmba_context_num_devices(const mmba_context *ctx);
void mmba_context_destroy(mmba_context *ctx);
/* Wait for all work on the context's device (bench timing brackets). */
int mmba_context_synchronize(mmba_context *ctx);
/* Page-locked host memory (hipHostMalloc) for buffers a caller keeps across
 * solves -- x, fvec, errorList, errorDistanceList: the end-of-solve
 * device-to-host copies then run at full link rate instead of through the
 * driver's staging copies of pageable memory.  Optional; any host pointer
 * works. */
int mmba_host_alloc(size_t bytes, void **out);
void mmba_host_free(void *p);

/* Upload a problem into HBM once; the plan can then be solved many times
 * (cached device context for the many small calls the Python standard solver
 * issues, _api/solverstandardutils.py). */
int mmba_plan_create(mmba_context *ctx, const mmba_problem *prob,
                     const mmba_options *opt, mmba_plan **out);
void mmba_plan_destroy(mmba_plan *plan);

/*
 * Frame-sharded solve: one plan per shard (one process per GPU
 * over RCCL, or one thread per shard in one process for tests).  Every shard
 * passes the SAME full problem; the library partitions the frames by
 * observation count and each shard evaluates the observations of its frames
 * (plus the other observations of the bundles tracked in them), owns the
 * reduced-system rows of its camera-frames and factors them; the shards
 * all-reduce scalars, the global-parameter block, the small separator system
 * of the partitioned band factorisation and the reduced step.  Every shard
 * returns the same x, fvec and result.  No reference counterpart (the
 * reference solver is single-threaded).
 */
typedef struct mmba_comm mmba_comm;
/* 128-byte RCCL unique id, made on one rank and broadcast by the caller. */
int mmba_comm_unique_id(unsigned char out_id[128]);
/* RCCL communicator on ctx's device (ncclCommInitRankConfig, non-blocking:
 * the initialisation and every collective wait at most the collective timeout
 * -- MMBA_PATH_COMM_TIMEOUT_MS / MMBA_COMM_TIMEOUT_MS, 120 s by default --
 * before the communicator is aborted and the call returns MMBA_ERR_COMM). */
int mmba_comm_create_rccl(mmba_context *ctx, int rank, int nranks,
                          const unsigned char unique_id[128], mmba_comm **out);
/* nranks in-process communicators (out[0..nranks-1], nranks <= 8), each used
 * by one host thread with its own context. */
int mmba_comm_create_local(int nranks, mmba_comm **out);
void mmba_comm_destroy(mmba_comm *comm);
/* Ranks of the communicator as the transport reports them (ncclCommCount for
 * RCCL, the group size in-process); negative on error. */
int mmba_comm_count(const mmba_comm *comm);
/* Like mmba_plan_create, for the shard `comm` stands for.  Collective: every
 * shard calls it (and then every solve / measure / outputs call) together,
 * with the same pattern of NULL / non-NULL output pointers.  Each shard's
 * results reach the others by one all-gather of its own rows (parameters,
 * observations), not by an all-reduce of full vectors. */
int mmba_plan_create_sharded(mmba_context *ctx, const mmba_problem *prob,
                             const mmba_options *opt, mmba_comm *comm, mmba_plan **out);
/* The frame partition a sharded plan uses (host only, no device needed):
 * shard k owns frames [bounds[k], bounds[k+1]) (balanced by observation
 * count) and the bundles whose earliest observation lies in them
 * (bundle_owner, nullable).  obs_bundle[i] = bundle of observation i. */
/* Shards a plan solves on: 1 unsharded (or replicated), N for a sharded
 * plan or a plan over an N-device context (ABI 9). */
int mmba_plan_num_shards(const mmba_plan *plan);
int mmba_shard_layout(int32_t num_frames, int32_t num_obs, const int32_t *obs_frame,
                      const int32_t *obs_bundle, int32_t num_bundles, int32_t nranks,
                      int32_t *bounds_out /* nranks + 1 */, int32_t *bundle_owner_out);

/* Plan caching (the Maya-side shim keeps one plan per problem shape):
 * replace the scene's attribute values (the problem's attr_values, same
 * attr_offset layout) of an existing plan, e.g. after a previous solve's
 * results were written back.  Structure, observations, parameters and
 * options are kept; the next solve / measure starts from these values. */
int mmba_plan_set_attr_values(mmba_plan *plan, const double *attr_values);

/* One residual evaluation (measureErrors, adjust_measureErrors.cpp:523) at
 * internal parameters x.  Any output pointer may be NULL. */
int mmba_plan_measure(mmba_plan *plan, const double *x, double *fvec_out,
                      double *err_user_out, double *err_dist_out,
                      double *avg_min_max_out /* [3] */);

/* Per-observation reprojection at internal parameters x (NULL: the problem's
 * x0): the lens-distorted reprojected point and the film-fit corrected
 * marker, [2*num_obs] each in observation order -- the out_point_list /
 * out_marker_list pair FlatScene::evaluate produces
 * (lib/rust/mmscenegraph/src/scene/flat.rs:271-356) and measureErrors
 * compares (adjust_measureErrors.cpp:444-472); |marker - point| * imageWidth
 * is err_user of mmba_plan_measure.  Either output may be NULL. */
int mmba_plan_reproject(mmba_plan *plan, const double *x, double *point_xy_out,
                        double *marker_xy_out);

/* Reference-layout Jacobian at internal parameters x (the fjac the reference
 * builds in solveFunc_calculateJacobianMatrix, adjust_solveFunc.cpp:482-525):
 * column-major num_residuals x num_params, ldfjac = num_residuals.  Dense
 * output -- meant for tests and small problems. */
int mmba_plan_jacobian(mmba_plan *plan, const double *x, double *fjac);

/* Run the LM solve from internal parameters x_inout: the
 * solve_3d_cminpack_lmder / _lmdif call inside solveFrames, bracketed by the
 * initial error measurement (adjust_base.cpp:1080-1103; it runs unless
 * opt->initial_error_given != 0 or opt->accept_only_better == 0) and the
 * accept-only-better test (:1208-1229).
 *   x_inout      [num_params]      in: x0; out: the solved x, as lmder leaves
 *                                  paramList.  res->error_is_better says
 *                                  whether the caller should write it back
 *                                  (:1231-1244) or keep x0.
 *   fvec_out     [num_residuals]   errorList (weighted, |dx|*imageWidth*sqrt(w),
 *                                  then the stiffness / smoothness rows)
 *   err_user_out [num_residuals]   ud->errorList (no weight, no loss)
 *   err_dist_out [num_obs]         ud->errorDistanceList
 * num_residuals = 2*num_obs + num_stiff + num_smooth.  Any output may be NULL. */
int mmba_plan_solve(mmba_plan *plan, double *x_inout, double *fvec_out,
                    double *err_user_out, double *err_dist_out,
                    mmba_result *res, const mmba_callbacks *cb,
                    mmba_trace *trace);

/* Outputs of the plan's last mmba_plan_solve / mmba_plan_measure, kept in
 * HBM: a caller that solves with NULL output pointers (device-resident
 * results) fetches errorList / ud->errorList / errorDistanceList here, in
 * the same layouts as mmba_plan_solve's.  MMBA_ERR_INVALID when the last
 * call on the plan was neither (reproject, jacobian and per-frame solves
 * overwrite the buffers).  Sharded plans: a collective, like the solve.  Any
 * output may be NULL. */
int mmba_plan_outputs(mmba_plan *plan, double *fvec_out, double *err_user_out,
                      double *err_dist_out);

/* Per-frame solve mode (FrameSolveMode::kPerFrame, adjust_base.cpp:1430-1484):
 * one solveFrames per frame over that frame's observations and the
 * parameters keyed at it plus every static parameter; results[num_frames]
 * gets each frame's SolverResult and x_inout the parameters each frame's
 * solveFrames writes back (the solved values when error_is_better, else the
 * frame's starting values).  The first frame with no parameters or fewer
 * residuals than parameters stops the sequence (later frames: success = 0).
 *   - No static parameter, every parameter on one camera-frame, forward
 *     differences, no robust loss / attribute rows, <= 8 cameras and <= 32
 *     parameters per frame: every frame is solved in ONE launch (one
 *     workgroup runs one frame's whole lmder / lmdif, mmba_batch.hip).
 *     cb->interrupt is polled on the calling thread while the launch runs;
 *     once it returns non-zero every frame stops at its next evaluation or
 *     Jacobian poll (reason_number -1).  max_concurrency is not used.
 *     mmba_debug_set_path(MMBA_PATH_PERFRAME_BATCH, 0) selects the path
 *     below (a test hook).
 *   - Otherwise one plan per frame: frames without a static parameter run
 *     max_concurrency at a time (0 = all) on host worker threads, each with
 *     its own stream; with a static parameter they are chained in order, as
 *     in the reference, and cb->interrupt is polled at every reference poll
 *     point. */
int mmba_solve_per_frame(mmba_context *ctx, const mmba_problem *prob,
                         const mmba_options *opt, double *x_inout,
                         mmba_result *results /* [num_frames] */, int32_t max_concurrency,
                         const mmba_callbacks *cb);

/* Per-frame solve mode on a plan of the whole problem (plan caching: the
 * caller builds the plan once and solves every frame per call in one
 * launch).  Same semantics as the batched path of mmba_solve_per_frame;
 * results[num_frames].  MMBA_ERR_UNSUPPORTED (mmba_last_error says why)
 * when the plan's parameters do not split into independent frames -- use
 * mmba_solve_per_frame then. */
int mmba_plan_solve_per_frame(mmba_plan *plan, double *x_inout, mmba_result *results,
                              const mmba_callbacks *cb);

/* One-shot convenience: plan_create + plan_solve + plan_destroy. */
int mmba_solve(mmba_context *ctx, const mmba_problem *prob,
               const mmba_options *opt, double *x_inout, double *fvec_out,
               double *err_user_out, double *err_dist_out, mmba_result *res,
               const mmba_callbacks *cb, mmba_trace *trace);

/* Kernel-level timing of the last solve for roofline accounting: average
 * device time (ms) of the dominant kernels measured with HIP events on the
 * plan's stream, and the algorithmic bytes / flops they moved per launch. */
typedef struct mmba_kernel_stats {
    double jac_ms_avg;      /* FD-Jacobian + normal-equation kernel       */
    double jac_bytes;       /* algorithmic HBM bytes per launch           */
    int32_t jac_launches;
    double resid_ms_avg;    /* residual kernel                            */
    double resid_bytes;
    int32_t resid_launches;
    double chol_ms_avg;     /* reduced camera system Cholesky             */
    double chol_flops;      /* flops per factorisation as performed: n_r^3/3
                               (dense / tiled), block cyclic reduction's
                               per-block count, band or block-diagonal
                               Cholesky counts                             */
    int32_t chol_launches;
    int32_t reduced_dim;    /* n_r = camera-frame + global parameters     */
    int32_t reduced_kind;   /* 0 band (block cyclic reduction / partitioned),
                               1 tiled sparse Cholesky, 2 dense blocked
                               Cholesky,
                               3 block diagonal + arrow (no solved bundle) */
    int32_t dataflow_fallback; /* 1 once a timed-out dataflow wait in the block
                               cyclic reduction switched this plan to the
                               per-level launches (ABI 3)                  */
    int32_t shards_replicated; /* ABI 6 (the slot of ABI 4's solve_launch,
                               whose cooperative solve was removed): 1 when
                               mmba_plan_create_sharded found that the
                               problem does not shard (too few camera-frame
                               rows per shard, a band wider than the
                               partitioned solver takes, rolling shutter,
                               B15 ...) and every shard solves the whole
                               problem redundantly, without collectives    */
    int32_t spec_replays;   /* ABI 6: solves of this plan replayed from x0
                               because a Jacobian enqueued ahead of the
                               host's lmder decision was not the one the
                               host took (expected 0; the replay enqueues
                               every Jacobian after the decision)          */
    int32_t band_solver;    /* ABI 7: the band reduced system's solver --
                               0 none (not a band plan), 1 partitioned band
                               Cholesky chains, 2 block cyclic reduction,
                               3 parallel cyclic reduction, 4 separator form
                               (sharded: interiors by parallel cyclic
                               reduction, separator system all-reduced),
                               5 block diagonal + arrow                    */
    /* ---- ABI 9 ---- */
    int32_t band_levels;    /* parallel / block cyclic reduction: elimination
                               levels of one factorisation (0 otherwise)   */
    int32_t band_block;     /* ... and their block edge K                  */
    double chol_flops_alg;  /* algorithmic flops of one damped solve of the
                               reduced system: band n_b w^2 + 4 n_b w (+ the
                               arrow's n_b nG (2w + nG) + nG^3/3); block
                               diagonal sum pc^3/3 + 4 pc; dense n^3/3 + 4n^2
                               -- chol_flops is what the solver executes   */
    /* ---- ABI 10 ---- */
    int32_t pre_handbacks;  /* solves of this plan whose page-locked output
                               lists the speculative hand-back stored (one
                               kernel behind the trial the device decided
                               ends the solve)                            */
    int32_t reserved10;
} mmba_kernel_stats;
int mmba_plan_kernel_stats(mmba_plan *plan, int enable_timing,
                           mmba_kernel_stats *out);

/* Test hook (not part of the solver seam): pin a choice the plan builder
 * otherwise makes itself, for the plans (and in-process communicators)
 * this process creates afterwards; value -1 restores the builder's choice.
 * The seam's caller never needs it: the GPU tests use it to run every
 * solver path (it replaces the MMBA_* environment switches of ABI <= 5).
 * Returns MMBA_ERR_INVALID for an unknown key. */
#define MMBA_PATH_PCR 1            /* 0: block cyclic reduction instead of parallel cyclic
                                      reduction for band systems without an arrow */
#define MMBA_PATH_SHARD_BCR 2      /* 0: sharded plans factor with the partitioned band chain */
#define MMBA_PATH_BCR_DATAFLOW 3   /* 0: block cyclic reduction in per-level launches */
#define MMBA_PATH_BCR_GRID 4       /* n: the dataflow launches on at most n workgroups */
#define MMBA_PATH_DENSE 5          /* 1: dense reduced solve, 0: tiled sparse Cholesky */
#define MMBA_PATH_PERFRAME_BATCH 6 /* 0: per-frame mode with one plan per frame */
#define MMBA_PATH_LOCAL_RING 7     /* 1: in-process communicators sum in ring order */
#define MMBA_PATH_PROBE 8          /* 1: band / BCR phase probe, printed when the plan is destroyed */
#define MMBA_PATH_SHARD_SEP 9      /* 1 / 0: sharded plans without an arrow solve the reduced
                                      system in its separator form (each shard's interior
                                      eliminated, the separator system all-reduced) / by
                                      all-reducing it whole; default: whole while the whole
                                      band system fits one resident PCR grid */
#define MMBA_PATH_TRIAL_RECORDS 10 /* 0: the trial point's records in their own launch instead
                                      of inside the trial's back substitution (or, without a
                                      solved bundle, its parameter pass) */
#define MMBA_PATH_LENS_CF 11       /* 0: every lens coefficient a global parameter (an
                                      animated one read by one camera-frame's rows joins
                                      that camera-frame's block otherwise) */
#define MMBA_PATH_DEST_LANE 12     /* 0 / 1: small off-diagonal Schur destinations never /
                                      always by a lane each (default: where they are most
                                      of at least 16,384) */
#define MMBA_PATH_FAULT_SHARD 13   /* n >= 1: the shard of rank n - 1 of a sharded plan fails
                                      (MMBA_ERR_INVALID) at its first damped solve -- a test
                                      hook for a shard failing while its peers are inside a
                                      collective */
#define MMBA_PATH_COMM_TIMEOUT_MS 14 /* n > 0: collectives (and the host waits behind them)
                                        give up after n ms: the communicator is aborted and
                                        the call returns MMBA_ERR_COMM (default: environment
                                        MMBA_COMM_TIMEOUT_MS, else 120000) */
#define MMBA_PATH_STALL_SHARD 15   /* n >= 1: the shard of rank n - 1 of a sharded plan sleeps
                                      for twice the collective timeout before its first damped
                                      solve (a test hook for a shard that never reaches a
                                      collective) */
#define MMBA_PATH_PCR_CHAIN 16    /* pivot chain of parallel cyclic reduction's block
                                      factorisations: 0 one-pivot Cholesky (default); 1 the
                                      2 x 2-pivot chain without square roots (16 % faster,
                                      but 4.5e-6 off the oracle's one-step ||f|| on the
                                      160-frame C4-spec scene where Cholesky is 1.8e-8 off);
                                      2 LDL^T with 1 x 1 pivots */
#define MMBA_PATH_BACKSUB_ONEPASS 17 /* 1: the trial back substitution forms u_i = W_i^T x
                                         itself (no k_obs_wtx launch; same sums) */
#define MMBA_PATH_JB_RECOMPUTE 18  /* 1: the bundle pass re-evaluates each observation's bundle
                                      columns instead of reading the 64-B records the fused
                                      Jacobian pass stores (same bits; measured slower on C4) */
#define MMBA_PATH_NE_CF_SPLIT 19   /* 0: long camera-frame segments (C2) take one workgroup per
                                      camera-frame in the normal equations instead of four */
#define MMBA_PATH_RED_BD 20        /* 0: the Jacobian epilogue's scalar reduction runs as its own
                                      launch on block-diagonal plans without globals (C2) instead
                                      of riding in the one-launch damped solve */
#define MMBA_PATH_HANDBACK_DMA 21  /* 0: page-locked output lists come back through one kernel
                                      storing them at their host-mapped addresses instead of
                                      the DMA copies (one per list, on their own streams) */
#define MMBA_PATH_PRE_HANDBACK 22  /* with the kernel hand-back (21 = 0), 0: no speculative
                                      launch of it behind each decided trial */
#define MMBA_PATH_PRE_SCHUR 23     /* 1: the next damped solve's k_schur_obs is enqueued with the
                                      gated Jacobian ahead of the host's decision */
#define MMBA_PATH_NUM 24
int mmba_debug_set_path(int key, int value);

/* Test hook (not part of the solver seam): solve S x = r with the device
 * band + arrow Cholesky for a dense symmetric positive-definite S of order
 * nb + nG whose leading nb x nb block has half bandwidth w and whose last nG
 * rows are dense ("arrow").  P > 0 forces the number of band partitions
 * (nested dissection on the band rows), P <= 0 uses the solver's heuristic.
 * S is row-major, only its lower triangle is read.  ynorm2 = ||L^-1 r||^2 (the
 * quantity lmpar's Newton correction uses); parts_used = partitions run. */
int mmba_debug_band_solve(mmba_context *ctx, int nb, int w, int nG, int P, const double *S,
                          const double *r, double *x, double *ynorm2, int *parts_used);
/* Test hook (not part of the solver seam): the in-place all-reduce a sharded
 * plan issues, on a host buffer (copied to ctx's device, reduced on ctx's
 * stream through comm, copied back); op 0 = sum, 1 = max.  Collective: every
 * rank of comm calls it with the same count. */
int mmba_debug_comm_allreduce(mmba_context *ctx, mmba_comm *comm, double *buf, int count,
                              int op);
/* Test hook (not part of the solver seam): the dense reduced solve's fp64
 * MFMA GEMM / SYRK on host buffers, C = beta C + alpha A B^T (column-major;
 * A: M x K, lda; B: N x K, ldb; C: M x N, ldc; K a multiple of 16).  tri != 0:
 * lower triangle only (M == N, B is ignored and A is used for both).
 * in_place != 0: C = alpha A B^T computed in the array holding A (the
 * dense solver's panel solve: N == K <= 64, lda == ldc, beta 0). */
int mmba_debug_dgemm(mmba_context *ctx, int tri, int in_place, int M, int N, int K,
                     const double *A, int lda, const double *B, int ldb, double *C, int ldc,
                     double alpha, double beta);

/* Test hook (not part of the solver seam; ABI 9): on a plan whose reduced
 * system takes the dense solver (C3-class scenes), evaluate at internal x,
 * form the Jacobian's damped reduced system (S + lam D^2) and its right-hand
 * side r, keep them aside, solve with the plan's factorisation and return
 * ||S xR - r|| / ||r|| -- the full-size dense solve's own accuracy.
 * MMBA_ERR_UNSUPPORTED for other plans. */
int mmba_debug_reduced_residual(mmba_plan *plan, const double *x, double lam, double *relres);

#ifdef __cplusplus
}
#endif

#endif /* MMBA_H */
