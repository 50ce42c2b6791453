// adjust_mmba_core.cpp -- Maya-free half of the plug-in shim (see
// adjust_mmba_core.h).  SolverInputs + SceneReader -> mmba_problem:
//   attributes   every attribute the scene reads: transform TRS, camera shape
//                film back / focal / offsets / clips / scale, the lens
//                node's coefficients; a solved attribute keyed per frame
//                (paramToAttrList frame >= 0) or an animated / connected one
//                holds one value per solve frame, the rest one static value
//                (AttrDataBlock; get_translate_attrs / get_camera_attrs,
//                maya_scene_graph.cpp:255-416)
//   transforms   camera and bundle DAG chains, parents first (add_transforms,
//                :744-809); only plain TRS transforms map (:571-742)
//   cameras      add_cameras (:811-893) + the lens node on camera.inLens
//   bundles      add_bundles (:895-957)
//   markers      add_markers (:959-1067)
//   observations errorToMarkerList / markerPosList / markerWeightList as
//                solveFrames built them (adjust_relationships.cpp:124-182)
//   parameters   paramToAttrList + Attr min / max / offset / scale,
//                paramWeightList (:223-337)
//   rows         stiffAttrsList / smoothAttrsList (adjust_measureErrors.cpp
//                :311-387), read at the current time
#include "adjust_mmba_core.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace mmba_shim {

namespace {

template <class T>
void put(std::vector<uint8_t> &k, const std::vector<T> &v) {
    const uint64_t n = v.size();
    const uint8_t *pn = reinterpret_cast<const uint8_t *>(&n);
    k.insert(k.end(), pn, pn + sizeof(n));
    if (n) {
        const uint8_t *p = reinterpret_cast<const uint8_t *>(v.data());
        k.insert(k.end(), p, p + n * sizeof(T));
    }
}

std::string long_name(const std::string &node, const std::string &attr) {
    return node + "." + attr;
}

}  // namespace

int32_t FlatScene::attr_of(const std::string &node, const char *attr) {
    const std::string key = long_name(node, attr);
    auto it = attr_id.find(key);
    if (it != attr_id.end()) return it->second;
    const bool force = keyed.count(key) > 0;
    const AttrRead a = rd_->attr(node, attr, force);
    if (!a.exists) return -1;  // the node has no such plug: the slot default
    const int32_t id = static_cast<int32_t>(attr_animated.size());
    const bool anim = force || a.animated;
    attr_animated.push_back(anim ? 1 : 0);
    attr_offset.push_back(static_cast<int64_t>(attr_values.size()));
    if (anim) {
        if (static_cast<int32_t>(a.frames.size()) != num_frames) {
            why = "attribute sampled on " + std::to_string(a.frames.size()) + " of " +
                  std::to_string(num_frames) + " frames: " + key;
            attr_values.insert(attr_values.end(), num_frames, a.value);
        } else {
            attr_values.insert(attr_values.end(), a.frames.begin(), a.frames.end());
        }
    } else {
        attr_values.push_back(a.value);
    }
    attr_id.emplace(key, id);
    return id;
}

int32_t FlatScene::transform_of(const std::string &path, int depth) {
    auto it = tfm_id.find(path);
    if (it != tfm_id.end()) return it->second;
    if (depth > 16) {
        why = "transform hierarchy deeper than 16: " + path;
        return -1;
    }
    const TransformRead t = rd_->transform(path);
    if (!t.plain) {
        why = "transform with pivots / shear / rotate axis: " + path;
        return -1;
    }
    if (t.rotate_order_animated) {
        why = "animated rotate order: " + path;
        return -1;
    }
    int32_t parent = -1;
    if (!t.parent.empty()) {
        parent = transform_of(t.parent, depth + 1);
        if (parent < 0) return -1;
    }
    static const char *trs[9] = {"translateX", "translateY", "translateZ",
                                 "rotateX",    "rotateY",    "rotateZ",
                                 "scaleX",     "scaleY",     "scaleZ"};
    int32_t ids[9];
    for (int k = 0; k < 9; ++k) ids[k] = attr_of(path, trs[k]);
    const int32_t id = static_cast<int32_t>(tfm_parent.size());
    tfm_parent.push_back(parent);
    tfm_roo.push_back(t.rotate_order);  // Maya's rotateOrder enum is MMBA_ROO_* order
    tfm_attrs.insert(tfm_attrs.end(), ids, ids + 9);
    tfm_id.emplace(path, id);
    return id;
}

// The lens nodes on camera.inLens: the enabled nodes of the chain, top
// (camera-connected) first, as the reference collects them
// (maya_lens_model_utils.cpp:405-465); the first is the camera's lens, the
// others its input layers (mmba.h ABI 5: constants of the solve, evaluated
// with their attributes at the current time).  Each node's model and
// coefficients in the MMBA_LENS_* slots (mmlens LensModelType,
// _cxxbridge.h:414-421).
int32_t FlatScene::lens_of(const std::string &camera_shape) {
    LensRead l = rd_->lens(camera_shape);
    std::vector<LensRead> chain;
    for (int depth = 0; l.connected; ++depth) {
        if (depth > 16) {
            why = "lens input chain deeper than 16 nodes: " + l.node;
            return -2;
        }
        if (l.enabled) chain.push_back(l);
        if (l.input.empty()) break;
        l = rd_->lens_node(l.input);
    }
    int32_t below = -1;  // the layer under the current one
    for (auto it = chain.rbegin(); it != chain.rend(); ++it) {
        const int32_t id = lens_layer(*it, below);
        if (id == -2) return -2;
        if (id >= 0) below = id;  // a passthrough layer adds nothing to the chain
    }
    return below;
}

// One lens node as a lens of the flat scene, its input layer `below` (-1 none).
int32_t FlatScene::lens_layer(const LensRead &l, int32_t below) {
    auto it = lens_id.find(l.node);
    if (it != lens_id.end()) {
        if (lens_input[it->second] != below) {
            why = "lens node with two different input chains: " + l.node;
            return -2;
        }
        return it->second;
    }
    int32_t type;
    std::vector<const char *> slots;
    if (l.model == 2) {
        type = MMBA_LENS_3DE_CLASSIC;
        slots = {"tdeClassic_distortion", "tdeClassic_anamorphicSqueeze", "tdeClassic_curvatureX",
                 "tdeClassic_curvatureY", "tdeClassic_quarticDistortion"};
    } else if (l.model == 3) {
        type = MMBA_LENS_3DE_RADIAL_STD_DEG4;
        slots = {"tdeRadialStdDeg4_degree2_distortion", "tdeRadialStdDeg4_degree2_u",
                 "tdeRadialStdDeg4_degree2_v",          "tdeRadialStdDeg4_degree4_distortion",
                 "tdeRadialStdDeg4_degree4_u",          "tdeRadialStdDeg4_degree4_v",
                 "tdeRadialStdDeg4_cylindricDirection", "tdeRadialStdDeg4_cylindricBending"};
    } else if (l.model == 4 || l.model == 5) {
        type = l.model == 4 ? MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4
                            : MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED;
        slots = {"tdeAnamorphicStdDeg4_degree2_cx02", "tdeAnamorphicStdDeg4_degree2_cy02",
                 "tdeAnamorphicStdDeg4_degree2_cx22", "tdeAnamorphicStdDeg4_degree2_cy22",
                 "tdeAnamorphicStdDeg4_degree4_cx04", "tdeAnamorphicStdDeg4_degree4_cy04",
                 "tdeAnamorphicStdDeg4_degree4_cx24", "tdeAnamorphicStdDeg4_degree4_cy24",
                 "tdeAnamorphicStdDeg4_degree4_cx44", "tdeAnamorphicStdDeg4_degree4_cy44",
                 "tdeAnamorphicStdDeg4_lensRotation", "tdeAnamorphicStdDeg4_squeeze_x",
                 "tdeAnamorphicStdDeg4_squeeze_y"};
        if (l.model == 5) slots.push_back("tdeAnamorphicStdDeg4_rescale");
    } else {
        return -1;  // passthrough / uninitialised: no distortion of its own
    }
    int32_t ids[MMBA_LENS_NUM_ATTRS];
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) ids[k] = -1;
    for (size_t k = 0; k < slots.size(); ++k) ids[k] = attr_of(l.node, slots[k]);
    const int32_t id = static_cast<int32_t>(lens_type.size());
    lens_type.push_back(type);
    lens_attrs.insert(lens_attrs.end(), ids, ids + MMBA_LENS_NUM_ATTRS);
    lens_input.push_back(below);
    // the slot values at the current time: what an input layer's plug model
    // holds when the camera-connected node is read (the reference reads it
    // at the current Maya time, with no DG context, and clones it per frame,
    // maya_lens_model_utils.cpp:433-446, 655-662); absent slots take the
    // model's default (squeeze / rescale 1, the rest 0)
    const bool classic = type == MMBA_LENS_3DE_CLASSIC;
    const bool anam = type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4 ||
                      type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED;
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) {
        double v = ((classic && k == 1) || (anam && k >= 11)) ? 1.0 : 0.0;
        if (ids[k] >= 0) {
            const int64_t off = attr_offset[ids[k]];
            v = attr_values[off + (attr_animated[ids[k]] ? cur_frame_ : 0)];
        }
        lens_input_values.push_back(v);
    }
    lens_id.emplace(l.node, id);
    return id;
}

bool FlatScene::build(const SolverInputs &in, SceneReader &rd) {
    rd_ = &rd;
    num_frames = in.num_frames;
    if (num_frames <= 0) {
        why = "no solve frames";
        return false;
    }
    cur_frame_ = std::min(std::max(in.current_frame, 0), num_frames - 1);
    // attributes solved per frame are animated in the flat scene
    for (const auto &pa : in.paramToAttrList) {
        if (pa.first < 0 || pa.first >= static_cast<int>(in.attrs.size())) {
            why = "paramToAttrList attribute index";
            return false;
        }
        if (pa.second >= 0) keyed[long_name(in.attrs[pa.first].node, in.attrs[pa.first].attr)] = true;
    }

    // ---- cameras (add_cameras) ----
    for (const CameraDesc &cam : in.cameras) {
        const int32_t t = transform_of(cam.transform_path);
        if (t < 0) return false;
        const std::string &shape = cam.shape_path;
        int32_t ca[MMBA_CAM_NUM_ATTRS];
        ca[MMBA_CAM_FILM_BACK_W_INCH] = attr_of(shape, "horizontalFilmAperture");
        ca[MMBA_CAM_FILM_BACK_H_INCH] = attr_of(shape, "verticalFilmAperture");
        ca[MMBA_CAM_FOCAL_MM] = attr_of(shape, "focalLength");
        ca[MMBA_CAM_FILM_OFFSET_X_INCH] = attr_of(shape, "horizontalFilmOffset");
        ca[MMBA_CAM_FILM_OFFSET_Y_INCH] = attr_of(shape, "verticalFilmOffset");
        ca[MMBA_CAM_NEAR_CLIP] = attr_of(shape, "nearClipPlane");
        ca[MMBA_CAM_FAR_CLIP] = attr_of(shape, "farClipPlane");
        ca[MMBA_CAM_SCALE] = attr_of(shape, "cameraScale");
        cam_tfm.push_back(t);
        cam_attrs.insert(cam_attrs.end(), ca, ca + MMBA_CAM_NUM_ATTRS);
        cam_fit.push_back(cam.film_fit);  // Maya filmFit = MMBA_FILM_FIT_*
        cam_size.push_back(cam.render_width);
        cam_size.push_back(cam.render_height);
        const int32_t lens = lens_of(shape);
        if (lens == -2) return false;
        cam_lens.push_back(lens);
    }
    if (!in.rolling_shutter.empty()) {
        if (in.rolling_shutter.size() != in.cameras.size()) {
            why = "rolling_shutter: one value per camera";
            return false;
        }
        cam_rs = in.rolling_shutter;
    }

    // ---- bundles (add_bundles) ----
    for (const std::string &b : in.bundles) {
        const int32_t t = transform_of(b);
        if (t < 0) return false;
        bnd_tfm.push_back(t);
    }

    // ---- markers (add_markers) ----
    for (const auto &mk : in.markers) {
        if (mk.first < 0 || mk.first >= static_cast<int>(in.cameras.size()) || mk.second < 0 ||
            mk.second >= static_cast<int>(in.bundles.size())) {
            why = "marker without a solved camera / bundle";
            return false;
        }
        mkr_cam.push_back(mk.first);
        mkr_bnd.push_back(mk.second);
    }

    // ---- observations: errorToMarkerList as solveFrames built it ----
    const size_t no = in.errorToMarkerList.size();
    if (in.markerPosList.size() != no || in.markerWeightList.size() != no) {
        why = "errorToMarkerList / markerPosList / markerWeightList sizes";
        return false;
    }
    for (size_t k = 0; k < no; ++k) {
        obs_marker.push_back(in.errorToMarkerList[k].first);
        obs_frame.push_back(in.errorToMarkerList[k].second);
        obs_xy.push_back(in.markerPosList[k][0]);
        obs_xy.push_back(in.markerPosList[k][1]);
        obs_weight.push_back(in.markerWeightList[k]);
    }
    if (!in.markerFramePos.empty()) {
        if (in.markerFramePos.size() != in.markers.size() * static_cast<size_t>(num_frames)) {
            why = "markerFramePos size";
            return false;
        }
        for (const auto &xy : in.markerFramePos) {
            mkr_frame_xy.push_back(xy[0]);
            mkr_frame_xy.push_back(xy[1]);
        }
    }

    // ---- parameters: paramToAttrList ----
    for (size_t p = 0; p < in.paramToAttrList.size(); ++p) {
        const AttrDesc &attr = in.attrs[in.paramToAttrList[p].first];
        const std::string key = long_name(attr.node, attr.attr);
        auto it = attr_id.find(key);
        if (it == attr_id.end()) {
            why = "solved attribute the scene does not read: " + key;
            return false;
        }
        param_attr.push_back(it->second);
        param_frame.push_back(in.paramToAttrList[p].second);
        param_ref_attr.push_back(in.paramToAttrList[p].first);
        param_min.push_back(attr.min_value);
        param_max.push_back(attr.max_value);
        param_offset.push_back(attr.offset);
        param_scale.push_back(attr.scale);
        param_weight.push_back(p < in.paramWeightList.size() ? in.paramWeightList[p] : 1.0);
    }

    // the lens of every attrList entry: an attribute a lens slot reads
    // (attrFrameToLensModelList, maya_lens_model_utils.cpp:836-851)
    for (const AttrDesc &a : in.attrs) {
        int32_t l = -1;
        auto it = attr_id.find(long_name(a.node, a.attr));
        if (it != attr_id.end())
            for (size_t q = 0; q < lens_attrs.size() && l < 0; ++q)
                if (lens_attrs[q] == it->second) l = static_cast<int32_t>(q / MMBA_LENS_NUM_ATTRS);
        ref_attr_lens.push_back(l);
    }

    // ---- stiffness / smoothness rows, read at the current time ----
    auto rows = [&](const std::vector<AttrRowDesc> &src, std::vector<int32_t> &ra,
                    std::vector<int32_t> &rf, std::vector<double> &rw, std::vector<double> &rv,
                    std::vector<double> &rval) -> bool {
        for (const AttrRowDesc &r : src) {
            if (r.attr_index < 0 || r.attr_index >= static_cast<int>(in.attrs.size())) {
                why = "stiffness / smoothness attribute index";
                return false;
            }
            const AttrDesc &a = in.attrs[r.attr_index];
            const std::string key = long_name(a.node, a.attr);
            auto it = attr_id.find(key);
            if (it == attr_id.end()) {
                why = "stiffness / smoothness attribute the scene does not read: " + key;
                return false;
            }
            ra.push_back(it->second);
            rf.push_back(in.current_frame);
            rw.push_back(r.weight);
            rv.push_back(r.variance);
            rval.push_back(r.value);
        }
        return true;
    };
    if (!rows(in.stiff, stiff_attr, stiff_frame, stiff_weight, stiff_variance, stiff_value))
        return false;
    if (!rows(in.smooth, smooth_attr, smooth_frame, smooth_weight, smooth_variance, smooth_value))
        return false;
    return why.empty();
}

mmba_problem FlatScene::problem() const {
    mmba_problem p;
    std::memset(&p, 0, sizeof(p));
    p.num_frames = num_frames;
    p.num_attrs = static_cast<int32_t>(attr_animated.size());
    p.attr_animated = attr_animated.data();
    p.attr_offset = attr_offset.data();
    p.attr_values = attr_values.data();
    p.num_transforms = static_cast<int32_t>(tfm_parent.size());
    p.tfm_parent = tfm_parent.data();
    p.tfm_rotate_order = tfm_roo.data();
    p.tfm_attrs = tfm_attrs.data();
    p.num_cameras = static_cast<int32_t>(cam_tfm.size());
    p.cam_tfm = cam_tfm.data();
    p.cam_attrs = cam_attrs.data();
    p.cam_film_fit = cam_fit.data();
    p.cam_render_size = cam_size.data();
    p.cam_lens = cam_lens.data();
    p.num_lenses = static_cast<int32_t>(lens_type.size());
    p.lens_type = lens_type.data();
    p.lens_attrs = lens_attrs.data();
    bool layered = false;
    for (int32_t v : lens_input) layered = layered || v >= 0;
    p.lens_input = layered ? lens_input.data() : nullptr;
    // every lens's slots at the current time: the values the solver's lens
    // clones start from (input layers for the whole solve; a camera lens's
    // slots no parameter writes, B3 / B11)
    p.lens_input_values = lens_type.empty() ? nullptr : lens_input_values.data();
    p.num_bundles = static_cast<int32_t>(bnd_tfm.size());
    p.bnd_tfm = bnd_tfm.data();
    p.num_markers = static_cast<int32_t>(mkr_cam.size());
    p.mkr_cam = mkr_cam.data();
    p.mkr_bnd = mkr_bnd.data();
    p.num_obs = static_cast<int32_t>(obs_marker.size());
    p.obs_marker = obs_marker.data();
    p.obs_frame = obs_frame.data();
    p.obs_xy = obs_xy.data();
    p.obs_weight = obs_weight.data();
    p.num_params = static_cast<int32_t>(param_attr.size());
    p.param_attr = param_attr.data();
    p.param_frame = param_frame.data();
    p.param_min = param_min.data();
    p.param_max = param_max.data();
    p.param_offset = param_offset.data();
    p.param_scale = param_scale.data();
    p.param_weight = param_weight.data();
    p.param_ref_attr = param_ref_attr.data();
    p.num_ref_attrs = static_cast<int32_t>(ref_attr_lens.size());
    p.ref_attr_lens = ref_attr_lens.data();
    p.num_stiff = static_cast<int32_t>(stiff_attr.size());
    p.stiff_attr = stiff_attr.data();
    p.stiff_frame = stiff_frame.data();
    p.stiff_weight = stiff_weight.data();
    p.stiff_variance = stiff_variance.data();
    p.stiff_value = stiff_value.data();
    p.num_smooth = static_cast<int32_t>(smooth_attr.size());
    p.smooth_attr = smooth_attr.data();
    p.smooth_frame = smooth_frame.data();
    p.smooth_weight = smooth_weight.data();
    p.smooth_variance = smooth_variance.data();
    p.smooth_value = smooth_value.data();
    p.cam_rs_value = cam_rs.empty() ? nullptr : cam_rs.data();
    p.mkr_frame_xy = mkr_frame_xy.empty() ? nullptr : mkr_frame_xy.data();
    return p;
}

std::vector<uint8_t> FlatScene::plan_key(const mmba_options &o) const {
    std::vector<uint8_t> k;
    const uint8_t *po = reinterpret_cast<const uint8_t *>(&o);
    k.insert(k.end(), po, po + sizeof(o));
    put(k, std::vector<int32_t>{num_frames});
    put(k, attr_animated);
    put(k, attr_offset);
    put(k, tfm_parent);
    put(k, tfm_roo);
    put(k, tfm_attrs);
    put(k, cam_tfm);
    put(k, cam_attrs);
    put(k, cam_fit);
    put(k, cam_size);
    put(k, cam_lens);
    put(k, lens_type);
    put(k, lens_attrs);
    put(k, lens_input);
    // every lens's plug values are constants a plan captures (input layers,
    // and the camera lenses' slots no parameter writes, mmba.h ABI 7)
    put(k, lens_input_values);
    put(k, bnd_tfm);
    put(k, mkr_cam);
    put(k, mkr_bnd);
    put(k, obs_marker);
    put(k, obs_frame);
    put(k, obs_xy);
    put(k, obs_weight);
    put(k, mkr_frame_xy);
    put(k, param_attr);
    put(k, param_frame);
    put(k, param_ref_attr);
    put(k, ref_attr_lens);
    put(k, param_min);
    put(k, param_max);
    put(k, param_offset);
    put(k, param_scale);
    put(k, param_weight);
    put(k, stiff_attr);
    put(k, stiff_frame);
    put(k, stiff_weight);
    put(k, stiff_variance);
    put(k, stiff_value);
    put(k, smooth_attr);
    put(k, smooth_frame);
    put(k, smooth_weight);
    put(k, smooth_variance);
    put(k, smooth_value);
    put(k, cam_rs);
    return k;
}

mmba_options options_of(const Options &so, bool per_frame) {
    mmba_options o;
    mmba_options_default(&o, so.solverType == MMBA_SOLVER_CMINPACK_LMDIF
                                 ? MMBA_SOLVER_CMINPACK_LMDIF
                                 : MMBA_SOLVER_CMINPACK_LMDER);
    o.iter_max = so.iterMax;
    o.tau = so.tau;
    o.eps1 = so.eps1;
    o.eps2 = so.eps2;
    o.eps3 = so.eps3;
    o.delta = so.delta;
    o.auto_diff_type = so.autoDiffType;
    o.auto_param_scale = so.autoParamScale;
    o.scene_graph_mode = so.mmSceneGraph ? MMBA_SCENE_GRAPH_MM_SCENE_GRAPH
                                         : MMBA_SCENE_GRAPH_MAYA_DAG;
    o.image_width = so.imageWidth;
    o.robust_loss = so.solverSupportsRobustLoss ? 1 : 0;
    o.robust_loss_type = so.robustLossType;
    o.robust_loss_scale = so.robustLossScale;
    if (per_frame) {
        o.accept_only_better = so.acceptOnlyBetter ? 1 : 0;
        o.initial_error_given = 0;
    } else {
        o.accept_only_better = 0;
        o.initial_error_given = 1;
    }
    o.initial_error_avg = 0.0;
    return o;
}

void fill_result(const mmba_result &r, Result &out) {
    out.success = r.success != 0;
    out.reason_number = r.reason_number;  // the Maya layer maps it to cminpackReasons
    out.iterations = r.iterations;
    out.functionEvals = r.function_evals;
    out.jacobianEvals = r.jacobian_evals;
    out.errorFinal = r.error_final;
    out.errorAvg = r.error_avg;
    out.errorMin = r.error_min;
    out.errorMax = r.error_max;
    out.user_interrupted = r.user_interrupted != 0;
    out.iterNum = r.function_evals;
    out.jacIterNum = r.jacobian_evals;
    out.funcEvalNum = r.iterations;
}

bool Shim::ready() {
    if (ctx_) return true;
    if (no_device_) return false;
    if (mmba_device_count() < 1) {
        why_ = "no gfx950 device visible";
        no_device_ = true;
        return false;
    }
    // One device by default (device 0: the plain single-device context).
    // Sharding a solve over every visible GPU (mmba_context_create_multi,
    // ABI 9; Maya's main thread stays the only caller, adjust_base.cpp:
    // 1174-1183) is opt-in with MMSOLVER_MMBA_DEVICES=all (or a count): the
    // in-process RCCL group has no test on distinct devices yet,
    // and on one-device rehearsals the sharded forms measured slower than
    // the whole solve on one GPU.
    int devs[8];
    int nd = 1;
    if (const char *e = std::getenv("MMSOLVER_MMBA_DEVICES")) {
        const int avail = std::min(mmba_device_count(), 8);
        nd = std::string(e) == "all" ? avail : std::max(1, std::min(std::atoi(e), avail));
    }
    for (int d = 0; d < nd; ++d) devs[d] = d;
    const int rc = nd == 1 ? mmba_context_create(0, &ctx_) : mmba_context_create_multi(devs, nd, &ctx_);
    if (rc != MMBA_OK) {
        why_ = std::string("no gfx950 device: ") + mmba_last_error();
        no_device_ = true;
        ctx_ = nullptr;
        return false;
    }
    return true;
}

mmba_plan *Shim::plan_for(const FlatScene &scene, const mmba_problem &prob,
                          const mmba_options &o) {
    std::vector<uint8_t> key = scene.plan_key(o);
    for (auto it = plans_.begin(); it != plans_.end(); ++it) {
        if (it->key != key) continue;
        if (mmba_plan_set_attr_values(it->plan, prob.attr_values) != MMBA_OK) return nullptr;
        plans_.splice(plans_.begin(), plans_, it);
        return plans_.front().plan;
    }
    mmba_plan *plan = nullptr;
    if (mmba_plan_create(ctx_, &prob, &o, &plan) != MMBA_OK) return nullptr;
    plans_.push_front(Entry{std::move(key), plan});
    if (plans_.size() > kMaxPlans) {
        mmba_plan_destroy(plans_.back().plan);
        plans_.pop_back();
    }
    return plan;
}

void Shim::release() {
    for (Entry &e : plans_) mmba_plan_destroy(e.plan);
    plans_.clear();
    if (ctx_) mmba_context_destroy(ctx_);
    ctx_ = nullptr;
}

SolveStatus solve(Shim &shim, const SolverInputs &in, SceneReader &rd, const Options &so,
                  int numberOfParameters, int numberOfErrors, double *paramList,
                  double *errorList, double *errorListUser, double *errorDistanceList,
                  const mmba_callbacks *cb, Result *out, std::string *message) {
    auto say = [&](const std::string &m) {
        if (message) *message = m;
    };
    if (!shim.ready()) {
        say(shim.why());
        return kNotMapped;
    }
    FlatScene scene;
    if (!scene.build(in, rd)) {
        say("scene not mapped: " + scene.why);
        return kNotMapped;
    }
    const mmba_problem prob = scene.problem();
    if (prob.num_params != numberOfParameters ||
        2 * prob.num_obs + prob.num_stiff + prob.num_smooth != numberOfErrors) {
        say("parameter / error counts differ from solveFrames'");
        return kNotMapped;
    }
    const mmba_options o = options_of(so);
    mmba_plan *plan = shim.plan_for(scene, prob, o);
    if (!plan) {
        say(mmba_last_error());
        return kNotMapped;  // e.g. MMBA_ERR_UNSUPPORTED: cminpack runs it
    }
    mmba_result r;
    const int rc = mmba_plan_solve(plan, paramList, errorList, errorListUser, errorDistanceList,
                                   &r, cb, nullptr);
    if (rc != MMBA_OK && rc != MMBA_ERR_INTERRUPTED) {
        say(mmba_last_error());
        if (out) out->success = false;
        return kFailed;  // the solve ran and failed: do not run it again on the CPU
    }
    if (out) fill_result(r, *out);
    return kSolved;
}

}  // namespace mmba_shim
