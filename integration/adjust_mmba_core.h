// adjust_mmba_core.h -- the Maya-free core of the mmSolver plug-in shim for
// libmmba.so (include/mmba.h).
//
// The plug-in side of the drop-in has two halves:
//   adjust_mmba.cpp       the Maya layer: reads SolverData's Maya objects
//                         (Attr, MDagPath, the camera's lens node) through a
//                         SceneReader and copies SolverData's index vectors
//                         into SolverInputs; needs the Maya SDK.
//   adjust_mmba_core.cpp  this half: SolverInputs + SceneReader ->
//                         mmba_problem (what construct_scene_graph,
//                         maya_scene_graph.cpp:1114-1203, flattens for the MM
//                         Scene Graph), SolverOptions -> mmba_options, the
//                         device context and plan cache, the solve call and
//                         mmba_result -> SolverResult fields.  Plain C++17 on
//                         the C ABI: it builds and runs here
//                         (tests/shim/shim_core_test.cpp).
#ifndef MMBA_ADJUST_MMBA_CORE_H
#define MMBA_ADJUST_MMBA_CORE_H

#include <mmba.h>

#include <array>
#include <cstdint>
#include <list>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace mmba_shim {

// ---------------------------------------------------------------------------
// What the Maya layer reads from the scene.
// ---------------------------------------------------------------------------
// One attribute (Attr::getValue over the solve frames, maya_attr.cpp).
struct AttrRead {
    bool exists = false;          // the node has the plug (else the slot default)
    bool animated = false;        // animated / connected / solved per frame
    double value = 0.0;           // static value
    std::vector<double> frames;   // animated: one value per solve frame
};

// One transform node (check_transform_node, maya_scene_graph.cpp:571-742).
struct TransformRead {
    bool plain = true;            // no pivots / shear / rotate axis, inherits transform
    std::string parent;           // DAG path of the parent transform, "" = world
    int rotate_order = 0;         // Maya rotateOrder (= MMBA_ROO_*)
    bool rotate_order_animated = false;
};

// The lens node on camera.inLens (maya_lens_model_utils.cpp).
struct LensRead {
    bool connected = false;
    std::string node;
    std::string input;            // the lens node on this node's own inLens ("" = none)
    bool enabled = true;
    int model = 0;                // mmLensModel3de lensModel: 2 classic, 3 radial std deg 4,
                                  // 4 anamorphic std deg 4, 5 anamorphic rescaled
};

class SceneReader {
  public:
    virtual ~SceneReader() = default;
    // node.attr at every solve frame (force_animated: a parameter is keyed
    // per frame, so the flat scene holds it per frame)
    virtual AttrRead attr(const std::string &node, const std::string &attr,
                          bool force_animated) = 0;
    virtual TransformRead transform(const std::string &path) = 0;
    virtual LensRead lens(const std::string &camera_shape) = 0;
    // a lens node by name (the upstream layers of a layered lens)
    virtual LensRead lens_node(const std::string &node) = 0;
};

// ---------------------------------------------------------------------------
// SolverData (adjust_data.h:188-261) as plain data.
// ---------------------------------------------------------------------------
struct CameraDesc {
    std::string transform_path, shape_path;
    int film_fit = MMBA_FILM_FIT_HORIZONTAL;  // Camera::getFilmFitValue
    int render_width = 2048, render_height = 1556;
};

struct AttrDesc {            // attrList entry
    std::string node, attr;  // long name = node + "." + attr
    double min_value, max_value, offset = 0.0, scale = 1.0;  // Attr::get*Value
};

struct AttrRowDesc {         // stiffAttrsList / smoothAttrsList entry
    int attr_index = -1;     // into attrs
    double weight = 0.0, variance = 1.0, value = 0.0;
};

struct SolverInputs {
    int num_frames = 0;       // frameList.length()
    int current_frame = 0;    // frameList index of the current time (attribute rows)
    std::vector<CameraDesc> cameras;           // cameraList
    std::vector<std::string> bundles;          // bundleList (transform paths)
    std::vector<std::pair<int, int>> markers;  // markerList: (camera, bundle) indices
    std::vector<AttrDesc> attrs;               // attrList
    std::vector<std::pair<int, int>> paramToAttrList;
    std::vector<std::pair<int, int>> errorToMarkerList;
    std::vector<std::array<double, 2>> markerPosList;
    std::vector<double> markerWeightList;
    std::vector<double> paramWeightList;       // diag of mode 2 (empty = 1.0)
    std::vector<AttrRowDesc> stiff, smooth;
    std::vector<double> rolling_shutter;       // per camera, frames (ABI 3; empty = none)
    // ABI 8: every marker's x,y at every frame, marker-major
    // [markers * num_frames], overscan applied like markerPosList -- what
    // FlatScene's marker list holds; empty = taken from the observations
    std::vector<std::array<double, 2>> markerFramePos;
};

// ---------------------------------------------------------------------------
// The flat problem (AttrDataBlock + transforms + cameras + ... as arrays).
// ---------------------------------------------------------------------------
struct FlatScene {
    int32_t num_frames = 0;
    std::vector<int32_t> attr_animated;
    std::vector<int64_t> attr_offset;
    std::vector<double> attr_values;
    std::vector<int32_t> tfm_parent, tfm_roo, tfm_attrs;
    std::vector<int32_t> cam_tfm, cam_attrs, cam_fit, cam_size, cam_lens;
    std::vector<int32_t> lens_type, lens_attrs, lens_input;
    // every lens's 14 slot values at the current time (SolverInputs::
    // current_frame): the plug values the reference's input layers hold
    // for the whole solve (maya_lens_model_utils.cpp:433-446, mmba.h ABI 5)
    std::vector<double> lens_input_values;
    std::vector<int32_t> bnd_tfm, mkr_cam, mkr_bnd;
    std::vector<int32_t> obs_marker, obs_frame;
    std::vector<double> obs_xy, obs_weight;
    std::vector<double> mkr_frame_xy;  // ABI 8 (empty: NULL)
    std::vector<int32_t> param_attr, param_frame;
    // ABI 7: paramToAttrList[p].first and the lens of each
    // attrList entry (-1: not an attribute of a lens the cameras use)
    std::vector<int32_t> param_ref_attr, ref_attr_lens;
    std::vector<double> param_min, param_max, param_offset, param_scale, param_weight;
    std::vector<int32_t> stiff_attr, stiff_frame, smooth_attr, smooth_frame;
    std::vector<double> stiff_weight, stiff_variance, stiff_value;
    std::vector<double> smooth_weight, smooth_variance, smooth_value;
    std::vector<double> cam_rs;
    std::string why;  // set when the scene does not map

    bool build(const SolverInputs &in, SceneReader &rd);
    mmba_problem problem() const;
    // everything a plan captures at mmba_plan_create except attr_values
    std::vector<uint8_t> plan_key(const mmba_options &o) const;

  private:
    std::unordered_map<std::string, int32_t> attr_id, tfm_id, lens_id;
    std::unordered_map<std::string, bool> keyed;
    SceneReader *rd_ = nullptr;
    int32_t cur_frame_ = 0;  // SolverInputs::current_frame, clamped to the solve frames
    int32_t attr_of(const std::string &node, const char *attr);
    int32_t transform_of(const std::string &path, int depth = 0);
    int32_t lens_of(const std::string &camera_shape);
    int32_t lens_layer(const LensRead &l, int32_t below);
};

// SolverOptions (adjust_data.h:133-185) fields the LM path reads.
struct Options {
    int solverType = MMBA_SOLVER_CMINPACK_LMDER;  // SOLVER_TYPE_CMINPACK_* (same numbers)
    int iterMax = 100;
    double tau = 1.0, eps1 = 1e-6, eps2 = 1e-6, eps3 = 1e-6, delta = 1e-4;
    int autoDiffType = MMBA_AUTO_DIFF_FORWARD, autoParamScale = 1;
    int robustLossType = MMBA_ROBUST_LOSS_TRIVIAL;
    double robustLossScale = 1.0;
    bool mmSceneGraph = false;                    // SceneGraphMode::kMMSceneGraph
    double imageWidth = 2048.0;
    bool acceptOnlyBetter = true;
    bool solverSupportsRobustLoss = false;
};

// solve_3d_cminpack_lmder's call (adjust_cminpack_lmder.cpp:94-184) as
// mmba_options: solveFrames has measured the initial error and applies
// accept-only-better itself (adjust_base.cpp:1080-1103, 1208-1244) unless
// per_frame (each frame's solveFrames does both).
mmba_options options_of(const Options &so, bool per_frame = false);

// SolverResult fields (adjust_results.h:59-72) and solveFunc's counters.
struct Result {
    bool success = false;
    int reason_number = 0;
    std::string reason;
    int iterations = 0, functionEvals = 0, jacobianEvals = 0;
    double errorFinal = 0.0, errorAvg = 0.0, errorMin = 0.0, errorMax = 0.0;
    bool user_interrupted = false;
    // SolverData counters as the cminpack path leaves them
    int iterNum = 0, jacIterNum = 0, funcEvalNum = 0;
};
void fill_result(const mmba_result &r, Result &out);

// Device context + plan cache (a solve whose structure equals a cached
// plan's only refreshes the attribute values; the Python standard solver
// issues many such solves, solverstandardutils.py).
class Shim {
  public:
    ~Shim() { release(); }
    bool ready();              // false: no gfx950 device (the caller runs cminpack)
    const std::string &why() const { return why_; }
    mmba_plan *plan_for(const FlatScene &scene, const mmba_problem &prob, const mmba_options &o);
    void release();
    size_t cached_plans() const { return plans_.size(); }

  private:
    struct Entry {
        std::vector<uint8_t> key;
        mmba_plan *plan = nullptr;
    };
    mmba_context *ctx_ = nullptr;
    bool no_device_ = false;
    std::string why_;
    std::list<Entry> plans_;  // most recently used first
    static constexpr size_t kMaxPlans = 4;
};

// Outcome of a shim solve.
enum SolveStatus {
    kNotMapped = 0,  // no device / the scene does not map: run cminpack instead
    kSolved = 1,     // the device solve ran (solved or interrupted)
    kFailed = -1,    // the device solve ran and failed (do not run it again)
};

// solve_3d_cminpack_lmder's contract (adjust_cminpack_lmder.cpp:64-198):
// paramList in = x0 (internal), out = the solved x; errorList = fvec;
// errorListUser / errorDistanceList = SolverData::errorList /
// errorDistanceList as the last measureErrors left them.  `message` gets the
// reason for kNotMapped / kFailed.
SolveStatus solve(Shim &shim, const SolverInputs &in, SceneReader &rd, const Options &so,
                  int numberOfParameters, int numberOfErrors, double *paramList,
                  double *errorList, double *errorListUser, double *errorDistanceList,
                  const mmba_callbacks *cb, Result *out, std::string *message);

}  // namespace mmba_shim

#endif  // MMBA_ADJUST_MMBA_CORE_H
