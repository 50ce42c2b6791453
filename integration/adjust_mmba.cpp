// adjust_mmba.cpp -- mmSolver plug-in shim for libmmba.so (the MI355X
// bundle-adjustment core).  Flattens the solve objects of a prepared
// SolverData into an mmba_problem and runs the LM solve on the GPU in place
// of solve_3d_cminpack_lmder / _lmdif (adjust_base.cpp:1175-1184).
//
// Flattening (what construct_scene_graph, maya_scene_graph.cpp:1114-1203,
// builds for the MM Scene Graph, here as plain arrays):
//   attributes   every attribute the scene reads: transform TRS + rotate
//                order, camera shape film back / focal / offsets / clips /
//                scale, the lens node's coefficients; a solved attribute
//                keyed per frame (paramToAttrList frame >= 0) or any
//                animated / connected attribute is sampled at every solve
//                frame, the rest is one static value (AttrDataBlock,
//                get_translate_attrs / get_camera_attrs, :255-416)
//   transforms   camera and bundle DAG chains, parents first
//                (add_transforms, :744-809); only plain TRS transforms map
//                (check_transform_node, :571-742: no pivots, shear, axis)
//   cameras      add_cameras (:811-893) + the lens node on camera.inLens
//   bundles      add_bundles (:895-957)
//   markers      add_markers (:959-1067): camera / bundle by node name
//   observations errorToMarkerList / markerPosList / markerWeightList as
//                solveFrames built them (adjust_relationships.cpp:124-182)
//   parameters   paramToAttrList + Attr min / max / offset / scale,
//                paramWeightList (:223-337, adjust_base.cpp countUp...)
//   rows         stiffAttrsList / smoothAttrsList (adjust_measureErrors.cpp
//                :311-387)
//
// Plans are cached: a solve whose structure, observations, parameters and
// options equal a cached plan's only refreshes the attribute values
// (mmba_plan_set_attr_values); the Python standard solver issues many such
// solves (solverstandardutils.py).  Builds with the plug-in (Maya SDK); not
// compiled in this repository.
#include "adjust_mmba.h"

#include <mmba.h>

#include <maya/MAnimControl.h>
#include <maya/MDagPath.h>
#include <maya/MFn.h>
#include <maya/MFnDependencyNode.h>
#include <maya/MPlug.h>
#include <maya/MPlugArray.h>
#include <maya/MTime.h>

#include <algorithm>
#include <cfloat>
#include <cstdint>
#include <cstring>
#include <list>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "adjust_cminpack_base.h"
#include "adjust_defines.h"
#include "mmSolver/mayahelper/maya_attr.h"
#include "mmSolver/mayahelper/maya_bundle.h"
#include "mmSolver/mayahelper/maya_camera.h"
#include "mmSolver/mayahelper/maya_marker.h"
#include "mmSolver/utilities/debug_utils.h"

namespace {

// ---------------------------------------------------------------------------
// Flattened scene
// ---------------------------------------------------------------------------
struct FlatScene {
    int32_t num_frames = 0;
    // attributes
    std::vector<int32_t> attr_animated;
    std::vector<int64_t> attr_offset;
    std::vector<double> attr_values;
    std::unordered_map<std::string, int32_t> attr_id;  // Attr::getLongName()
    // transforms
    std::vector<int32_t> tfm_parent, tfm_roo, tfm_attrs;
    std::unordered_map<std::string, int32_t> tfm_id;  // DAG full path
    // cameras, lenses
    std::vector<int32_t> cam_tfm, cam_attrs, cam_fit, cam_size, cam_lens;
    std::vector<int32_t> lens_type, lens_attrs;
    std::unordered_map<std::string, int32_t> lens_id;  // lens node name
    // bundles, markers, observations
    std::vector<int32_t> bnd_tfm, mkr_cam, mkr_bnd;
    std::vector<int32_t> obs_marker, obs_frame;
    std::vector<double> obs_xy, obs_weight;
    // parameters
    std::vector<int32_t> param_attr, param_frame;
    std::vector<double> param_min, param_max, param_offset, param_scale, param_weight;
    // stiffness / smoothness rows
    std::vector<int32_t> stiff_attr, stiff_frame, smooth_attr, smooth_frame;
    std::vector<double> stiff_weight, stiff_variance, stiff_value;
    std::vector<double> smooth_weight, smooth_variance, smooth_value;

    std::string why;  // set when the scene does not map

    // solved attributes keyed per frame: forced animated
    std::unordered_map<std::string, bool> keyed;

    bool build(SolverData &ud, const SolverOptions &opts, const std::vector<double> &weights);
    mmba_problem problem() const;
    // everything a plan captures at mmba_plan_create except attr_values
    std::vector<uint8_t> plan_key(const mmba_options &o) const;

  private:
    int timeEvalMode = 0;
    const MTimeArray *frames = nullptr;
    int32_t attr_of(const MString &node, const char *attr_name, bool *ok = nullptr);
    int32_t transform_of(MDagPath path);
    bool plain_trs(const MString &node);
    int32_t lens_of(CameraPtr &cam);
};

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

// One attribute of the scene: static (one value) or animated (one value per
// solve frame, frameList order).
int32_t FlatScene::attr_of(const MString &node, const char *attr_name, bool *ok) {
    Attr a;
    a.setNodeName(node);
    a.setAttrName(MString(attr_name));
    const std::string key(a.getLongName().asChar());
    auto it = attr_id.find(key);
    if (it != attr_id.end()) return it->second;
    MPlug plug = a.getPlug();
    if (plug.isNull()) {  // the node has no such attribute: slot default
        if (ok) *ok = false;
        return -1;
    }
    const bool anim = keyed.count(key) > 0 || a.isAnimated() || a.isConnected();
    const int32_t id = static_cast<int32_t>(attr_animated.size());
    attr_animated.push_back(anim ? 1 : 0);
    attr_offset.push_back(static_cast<int64_t>(attr_values.size()));
    if (anim) {
        for (uint32_t f = 0; f < frames->length(); ++f) {
            double v = 0.0;
            a.getValue(v, (*frames)[f], timeEvalMode);
            attr_values.push_back(v);
        }
    } else {
        double v = 0.0;
        a.getValue(v, timeEvalMode);
        attr_values.push_back(v);
    }
    attr_id.emplace(key, id);
    return id;
}

// check_transform_node (maya_scene_graph.cpp:571-742): the core evaluates
// T * R(order) * S; pivots, pivot translations, rotate axis and shear must
// be zero and the transform must inherit its parent.
bool FlatScene::plain_trs(const MString &node) {
    static const char *zero_attrs[] = {
        "rotatePivotX", "rotatePivotY", "rotatePivotZ",
        "scalePivotX", "scalePivotY", "scalePivotZ",
        "rotatePivotTranslateX", "rotatePivotTranslateY", "rotatePivotTranslateZ",
        "scalePivotTranslateX", "scalePivotTranslateY", "scalePivotTranslateZ",
        "rotateAxisX", "rotateAxisY", "rotateAxisZ",
        "shearXY", "shearXZ", "shearYZ"};
    for (const char *n : zero_attrs) {
        Attr a;
        a.setNodeName(node);
        a.setAttrName(MString(n));
        if (a.getPlug().isNull()) continue;
        double v = 0.0;
        a.getValue(v, timeEvalMode);
        if (a.isAnimated() || a.isConnected() || v != 0.0) return false;
    }
    Attr inh;
    inh.setNodeName(node);
    inh.setAttrName("inheritsTransform");
    bool inherits = true;
    if (!inh.getPlug().isNull()) inh.getValue(inherits, timeEvalMode);
    return inherits;
}

// Transform of a DAG path, its parent chain first (parent index < child).
int32_t FlatScene::transform_of(MDagPath path) {
    MStatus status;
    const MString name = path.fullPathName(&status);
    const std::string key(name.asChar());
    auto it = tfm_id.find(key);
    if (it != tfm_id.end()) return it->second;
    if (!plain_trs(name)) {
        why = "transform with pivots / shear / rotate axis: " + key;
        return -1;
    }
    int32_t parent = -1;
    MDagPath up(path);
    if (up.pop() == MS::kSuccess && up.length() > 0 && up.hasFn(MFn::kTransform)) {
        parent = transform_of(up);
        if (parent < 0) return -1;
    }
    static const char *trs[9] = {"translateX", "translateY", "translateZ",
                                 "rotateX",    "rotateY",    "rotateZ",
                                 "scaleX",     "scaleY",     "scaleZ"};
    int32_t ids[9];
    for (int k = 0; k < 9; ++k) ids[k] = attr_of(name, trs[k]);
    Attr ro;
    ro.setNodeName(name);
    ro.setAttrName("rotateOrder");
    short roo = 0;
    ro.getValue(roo, timeEvalMode);
    if (ro.isAnimated() || ro.isConnected()) {
        why = "animated rotate order: " + key;
        return -1;
    }
    const int32_t id = static_cast<int32_t>(tfm_parent.size());
    tfm_parent.push_back(parent);
    tfm_roo.push_back(roo);  // Maya's rotateOrder enum is MMBA_ROO_* order
    tfm_attrs.insert(tfm_attrs.end(), ids, ids + 9);
    tfm_id.emplace(key, id);
    return id;
}

// The lens node on camera.inLens (mmLensModel3de), one layer: its model
// and its coefficients in the MMBA_LENS_* slots.
int32_t FlatScene::lens_of(CameraPtr &cam) {
    MStatus status;
    MFnDependencyNode shape(cam->getShapeObject(), &status);
    if (!status) return -1;
    MPlug in_lens = shape.findPlug("inLens", true, &status);
    if (!status || in_lens.isNull()) return -1;
    MPlugArray src;
    in_lens.connectedTo(src, /*asDst=*/true, /*asSrc=*/false, &status);
    if (src.length() == 0) return -1;
    MObject node = src[0].node();
    MFnDependencyNode lens_fn(node, &status);
    const MString lens_name = lens_fn.name();
    const std::string key(lens_name.asChar());
    auto it = lens_id.find(key);
    if (it != lens_id.end()) return it->second;
    // layered lenses (a lens feeding this lens) are not mapped
    MPlug up = lens_fn.findPlug("inLens", true, &status);
    MPlugArray up_src;
    if (status && !up.isNull()) up.connectedTo(up_src, true, false, &status);
    if (up_src.length() > 0) {
        why = "layered lens nodes: " + key;
        return -2;
    }
    Attr enable;
    enable.setNodeName(lens_name);
    enable.setAttrName("enable");
    bool on = true;
    enable.getValue(on, timeEvalMode);
    if (!on) return -1;
    Attr model;
    model.setNodeName(lens_name);
    model.setAttrName("lensModel");
    short m = 0;
    model.getValue(m, timeEvalMode);
    // mmlens LensModelType (_cxxbridge.h:414-421) -> MMBA_LENS_*
    int32_t type;
    std::vector<const char *> slots;
    if (m == 2) {
        type = MMBA_LENS_3DE_CLASSIC;
        slots = {"tdeClassic_distortion", "tdeClassic_anamorphicSqueeze", "tdeClassic_curvatureX",
                 "tdeClassic_curvatureY", "tdeClassic_quarticDistortion"};
    } else if (m == 3) {
        type = MMBA_LENS_3DE_RADIAL_STD_DEG4;
        slots = {"tdeRadialStdDeg4_degree2_distortion", "tdeRadialStdDeg4_degree2_u",
                 "tdeRadialStdDeg4_degree2_v",          "tdeRadialStdDeg4_degree4_distortion",
                 "tdeRadialStdDeg4_degree4_u",          "tdeRadialStdDeg4_degree4_v",
                 "tdeRadialStdDeg4_cylindricDirection", "tdeRadialStdDeg4_cylindricBending"};
    } else if (m == 4 || m == 5) {
        type = m == 4 ? MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4
                      : MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED;
        slots = {"tdeAnamorphicStdDeg4_degree2_cx02", "tdeAnamorphicStdDeg4_degree2_cy02",
                 "tdeAnamorphicStdDeg4_degree2_cx22", "tdeAnamorphicStdDeg4_degree2_cy22",
                 "tdeAnamorphicStdDeg4_degree4_cx04", "tdeAnamorphicStdDeg4_degree4_cy04",
                 "tdeAnamorphicStdDeg4_degree4_cx24", "tdeAnamorphicStdDeg4_degree4_cy24",
                 "tdeAnamorphicStdDeg4_degree4_cx44", "tdeAnamorphicStdDeg4_degree4_cy44",
                 "tdeAnamorphicStdDeg4_lensRotation", "tdeAnamorphicStdDeg4_squeeze_x",
                 "tdeAnamorphicStdDeg4_squeeze_y"};
        if (m == 5) slots.push_back("tdeAnamorphicStdDeg4_rescale");
    } else {
        return -1;  // passthrough / uninitialised: no distortion
    }
    int32_t ids[MMBA_LENS_NUM_ATTRS];
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) ids[k] = -1;
    for (size_t k = 0; k < slots.size(); ++k) ids[k] = attr_of(lens_name, slots[k]);
    const int32_t id = static_cast<int32_t>(lens_type.size());
    lens_type.push_back(type);
    lens_attrs.insert(lens_attrs.end(), ids, ids + MMBA_LENS_NUM_ATTRS);
    lens_id.emplace(key, id);
    return id;
}

bool FlatScene::build(SolverData &ud, const SolverOptions &opts,
                      const std::vector<double> &weights) {
    MStatus status;
    timeEvalMode = opts.timeEvalMode;
    frames = &ud.frameList;
    num_frames = static_cast<int32_t>(ud.frameList.length());

    // attributes solved per frame are animated in the flat scene
    for (const auto &pa : ud.paramToAttrList)
        if (pa.second >= 0) keyed[std::string(ud.attrList[pa.first]->getLongName().asChar())] = true;

    // ---- cameras (add_cameras) ----
    for (CameraPtr &cam : ud.cameraList) {
        MDagPath tfm_path, shp_path;
        if (MDagPath::getAPathTo(cam->getTransformObject(), tfm_path) != MS::kSuccess ||
            MDagPath::getAPathTo(cam->getShapeObject(), shp_path) != MS::kSuccess) {
            why = "camera DAG path";
            return false;
        }
        const int32_t t = transform_of(tfm_path);
        if (t < 0) return false;
        const MString shape = shp_path.fullPathName(&status);
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
        cam_fit.push_back(cam->getFilmFitValue());  // Maya filmFit = MMBA_FILM_FIT_*
        cam_size.push_back(cam->getRenderWidthValue());
        cam_size.push_back(cam->getRenderHeightValue());
        const int32_t lens = lens_of(cam);
        if (lens == -2) return false;
        cam_lens.push_back(lens);
    }

    // ---- bundles (add_bundles) ----
    for (BundlePtr &bnd : ud.bundleList) {
        MDagPath path;
        if (MDagPath::getAPathTo(bnd->getObject(), path) != MS::kSuccess) {
            why = "bundle DAG path";
            return false;
        }
        const int32_t t = transform_of(path);
        if (t < 0) return false;
        bnd_tfm.push_back(t);
    }

    // ---- markers (add_markers): camera / bundle by node name ----
    for (MarkerPtr &mkr : ud.markerList) {
        int32_t c = -1, b = -1;
        const MString cam_shape = mkr->getCamera()->getShapeNodeName();
        for (size_t j = 0; j < ud.cameraList.size() && c < 0; ++j)
            if (ud.cameraList[j]->getShapeNodeName() == cam_shape) c = static_cast<int32_t>(j);
        const MString bnd_name = mkr->getBundle()->getNodeName();
        for (size_t j = 0; j < ud.bundleList.size() && b < 0; ++j)
            if (ud.bundleList[j]->getNodeName() == bnd_name) b = static_cast<int32_t>(j);
        if (c < 0 || b < 0) {
            why = "marker without a solved camera / bundle";
            return false;
        }
        mkr_cam.push_back(c);
        mkr_bnd.push_back(b);
    }

    // ---- observations: errorToMarkerList as solveFrames built it ----
    const size_t no = ud.errorToMarkerList.size();
    for (size_t k = 0; k < no; ++k) {
        obs_marker.push_back(ud.errorToMarkerList[k].first);
        obs_frame.push_back(ud.errorToMarkerList[k].second);
        obs_xy.push_back(ud.markerPosList[k].x);
        obs_xy.push_back(ud.markerPosList[k].y);
        obs_weight.push_back(ud.markerWeightList[k]);
    }

    // ---- parameters: paramToAttrList ----
    for (size_t p = 0; p < ud.paramToAttrList.size(); ++p) {
        const AttrPtr &attr = ud.attrList[ud.paramToAttrList[p].first];
        const std::string key(attr->getLongName().asChar());
        auto it = attr_id.find(key);
        if (it == attr_id.end()) {
            why = "solved attribute the scene does not read: " + key;
            return false;
        }
        param_attr.push_back(it->second);
        param_frame.push_back(ud.paramToAttrList[p].second);
        param_min.push_back(attr->getMinimumValue());
        param_max.push_back(attr->getMaximumValue());
        param_offset.push_back(attr->getOffsetValue());
        param_scale.push_back(attr->getScaleValue());
        param_weight.push_back(p < weights.size() ? weights[p] : 1.0);
    }

    // ---- stiffness / smoothness rows (adjust_measureErrors.cpp:311-387):
    // the rows read the attribute at the current time ----
    int32_t now = 0;
    {
        const MTime t = MAnimControl::currentTime();
        for (uint32_t f = 0; f < ud.frameList.length(); ++f)
            if (ud.frameList[f] == t) now = static_cast<int32_t>(f);
    }
    auto row = [&](int attr_index, AttrPtr &w, AttrPtr &v, AttrPtr &val,
                   std::vector<int32_t> &ra, std::vector<int32_t> &rf, std::vector<double> &rw,
                   std::vector<double> &rv, std::vector<double> &rval) -> bool {
        const std::string key(ud.attrList[attr_index]->getLongName().asChar());
        auto it = attr_id.find(key);
        if (it == attr_id.end()) {
            why = "stiffness / smoothness attribute the scene does not read: " + key;
            return false;
        }
        double wv = 0.0, vv = 1.0, xv = 0.0;
        w->getValue(wv, timeEvalMode);
        v->getValue(vv, timeEvalMode);
        val->getValue(xv, timeEvalMode);
        ra.push_back(it->second);
        rf.push_back(now);
        rw.push_back(wv);
        rv.push_back(vv);
        rval.push_back(xv);
        return true;
    };
    for (int i = 0; i < ud.numberOfAttrStiffnessErrors; ++i) {
        StiffAttrsPtr &s = ud.stiffAttrsList[i];
        if (!row(s->attrIndex, s->weightAttr, s->varianceAttr, s->valueAttr, stiff_attr,
                 stiff_frame, stiff_weight, stiff_variance, stiff_value))
            return false;
    }
    for (int i = 0; i < ud.numberOfAttrSmoothnessErrors; ++i) {
        SmoothAttrsPtr &s = ud.smoothAttrsList[i];
        if (!row(s->attrIndex, s->weightAttr, s->varianceAttr, s->valueAttr, smooth_attr,
                 smooth_frame, smooth_weight, smooth_variance, smooth_value))
            return false;
    }
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
    put(k, bnd_tfm);
    put(k, mkr_cam);
    put(k, mkr_bnd);
    put(k, obs_marker);
    put(k, obs_frame);
    put(k, obs_xy);
    put(k, obs_weight);
    put(k, param_attr);
    put(k, param_frame);
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
    return k;
}

// ---------------------------------------------------------------------------
// Device context and plan cache
// ---------------------------------------------------------------------------
struct Shim {
    mmba_context *ctx = nullptr;
    bool no_device = false;
    struct Entry {
        std::vector<uint8_t> key;
        mmba_plan *plan = nullptr;
    };
    std::list<Entry> plans;  // most recently used first
    static constexpr size_t kMaxPlans = 4;

    ~Shim() { release(); }
    void release() {
        for (Entry &e : plans) mmba_plan_destroy(e.plan);
        plans.clear();
        if (ctx) mmba_context_destroy(ctx);
        ctx = nullptr;
    }
    bool ready() {
        if (ctx) return true;
        if (no_device) return false;
        if (mmba_context_create(0, &ctx) != MMBA_OK) {
            MMSOLVER_MAYA_WRN("mmba: " << mmba_last_error() << " (using cminpack)");
            no_device = true;
            ctx = nullptr;
            return false;
        }
        return true;
    }
    // A plan for this problem: a cached one with the same key gets the new
    // attribute values, otherwise a new plan (the oldest is dropped).
    mmba_plan *plan_for(const FlatScene &scene, const mmba_problem &prob, const mmba_options &o) {
        std::vector<uint8_t> key = scene.plan_key(o);
        for (auto it = plans.begin(); it != plans.end(); ++it) {
            if (it->key != key) continue;
            if (mmba_plan_set_attr_values(it->plan, prob.attr_values) != MMBA_OK) return nullptr;
            plans.splice(plans.begin(), plans, it);
            return plans.front().plan;
        }
        mmba_plan *plan = nullptr;
        if (mmba_plan_create(ctx, &prob, &o, &plan) != MMBA_OK) return nullptr;
        plans.push_front(Entry{std::move(key), plan});
        if (plans.size() > kMaxPlans) {
            mmba_plan_destroy(plans.back().plan);
            plans.pop_back();
        }
        return plan;
    }
};

Shim &shim() {
    static Shim s;
    return s;
}

mmba_options options_of(const SolverOptions &so) {
    mmba_options o;
    mmba_options_default(&o, so.solverType == SOLVER_TYPE_CMINPACK_LMDIF
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
    o.scene_graph_mode = so.sceneGraphMode == SceneGraphMode::kMMSceneGraph
                             ? MMBA_SCENE_GRAPH_MM_SCENE_GRAPH
                             : MMBA_SCENE_GRAPH_MAYA_DAG;
    o.image_width = so.imageWidth;
    o.robust_loss = so.solverSupportsRobustLoss ? 1 : 0;
    o.robust_loss_type = so.robustLossType;
    o.robust_loss_scale = so.robustLossScale;
    // solveFrames measured the initial error and applies accept-only-better
    // itself after the solve (adjust_base.cpp:1080-1103, 1208-1244)
    o.accept_only_better = 0;
    o.initial_error_given = 1;
    o.initial_error_avg = 0.0;
    return o;
}

struct Callbacks {
    mmba_callbacks cb;
    explicit Callbacks(SolverData &ud) {
        cb.interrupt = [](void *u) -> int {
            auto *d = static_cast<SolverData *>(u);
            return (d->computation && d->computation->isInterruptRequested()) ? 1 : 0;
        };
        cb.progress = [](void *u, int32_t it) {
            auto *d = static_cast<SolverData *>(u);
            if (d->computation) d->computation->setProgress(it);
        };
        cb.user = &ud;
    }
};

void fill_result(const mmba_result &r, SolverResult &out) {
    out.success = r.success != 0;
    out.reason_number = r.reason_number;
    out.reason = (r.reason_number >= 0 && r.reason_number <= 8)
                     ? cminpackReasons[r.reason_number]
                     : std::string("User interrupted.");
    out.iterations = r.iterations;
    out.functionEvals = r.function_evals;
    out.jacobianEvals = r.jacobian_evals;
    out.errorFinal = r.error_final;
    out.user_interrupted = r.user_interrupted != 0;
}

}  // namespace

bool solve_3d_mmba(SolverOptions &solverOptions, int numberOfParameters, int numberOfErrors,
                   std::vector<double> &paramList, std::vector<double> &errorList,
                   std::vector<double> &paramWeightList, SolverData &userData,
                   SolverResult &solveResult) {
    Shim &s = shim();
    if (!s.ready()) return false;
    FlatScene scene;
    if (!scene.build(userData, solverOptions, paramWeightList)) {
        MMSOLVER_MAYA_VRB("mmba: scene not mapped (" << scene.why << "), using cminpack");
        return false;
    }
    mmba_problem prob = scene.problem();
    if (prob.num_params != numberOfParameters ||
        2 * prob.num_obs + prob.num_stiff + prob.num_smooth != numberOfErrors)
        return false;
    const mmba_options o = options_of(solverOptions);
    mmba_plan *plan = s.plan_for(scene, prob, o);
    if (!plan) {
        MMSOLVER_MAYA_VRB("mmba: " << mmba_last_error() << ", using cminpack");
        return false;
    }
    Callbacks cb(userData);
    mmba_result r;
    const int rc = mmba_plan_solve(plan, paramList.data(), errorList.data(),
                                   userData.errorList.data(), userData.errorDistanceList.data(),
                                   &r, &cb.cb, nullptr);
    if (rc != MMBA_OK && rc != MMBA_ERR_INTERRUPTED) {
        MMSOLVER_MAYA_ERR("mmba: " << mmba_last_error());
        solveResult.success = false;
        return true;  // the solve ran and failed: do not run it again on the CPU
    }
    fill_result(r, solveResult);
    // solveFunc's counters, as the cminpack path leaves them
    userData.iterNum = r.function_evals;
    userData.jacIterNum = r.jacobian_evals;
    userData.funcEvalNum = r.iterations;
    userData.userInterrupted = r.user_interrupted != 0;
    return true;
}

bool solve_frames_mmba_per_frame(SolverOptions &solverOptions, std::vector<double> &paramList,
                                 std::vector<double> &paramWeightList, SolverData &userData,
                                 std::vector<SolverResult> &perFrameResults) {
    Shim &s = shim();
    if (!s.ready()) return false;
    for (const auto &pa : userData.paramToAttrList)
        if (pa.second < 0) return false;  // a static parameter chains the frames
    FlatScene scene;
    if (!scene.build(userData, solverOptions, paramWeightList)) return false;
    mmba_problem prob = scene.problem();
    mmba_options o = options_of(solverOptions);
    // every frame's solveFrames measures its own initial error and writes
    // back only when it got better (adjust_base.cpp:1080-1103, 1227-1244)
    o.accept_only_better = solverOptions.acceptOnlyBetter ? 1 : 0;
    o.initial_error_given = 0;
    mmba_plan *plan = s.plan_for(scene, prob, o);
    if (!plan) return false;
    Callbacks cb(userData);
    std::vector<mmba_result> res(static_cast<size_t>(prob.num_frames));
    const int rc = mmba_plan_solve_per_frame(plan, paramList.data(), res.data(), &cb.cb);
    if (rc == MMBA_ERR_UNSUPPORTED) return false;
    perFrameResults.assign(res.size(), SolverResult());
    for (size_t f = 0; f < res.size(); ++f) {
        fill_result(res[f], perFrameResults[f]);
        perFrameResults[f].errorAvg = res[f].error_avg;
        perFrameResults[f].errorMin = res[f].error_min;
        perFrameResults[f].errorMax = res[f].error_max;
    }
    if (rc != MMBA_OK) MMSOLVER_MAYA_ERR("mmba: " << mmba_last_error());
    return true;
}

void mmba_shim_release() { shim().release(); }
