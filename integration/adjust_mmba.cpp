// adjust_mmba.cpp -- the Maya layer of the mmSolver plug-in shim for
// libmmba.so.  It only reads: SolverData's Maya objects through a SceneReader
// (Attr::getValue over the solve frames, the DAG parents, the lens node on
// camera.inLens) and SolverData's index vectors into SolverInputs.
// Everything else -- flattening, plan cache, the solve call, the result
// mapping -- is the Maya-free core (adjust_mmba_core.cpp), which builds and is
// tested without Maya (tests/shim).  This file builds with the plug-in (Maya
// SDK) and dispatches from solveFrames (adjust_base.cpp:1175-1184,
// INTEGRATION.md section 2).
#include "adjust_mmba.h"

#include <maya/MAnimControl.h>
#include <maya/MDagPath.h>
#include <maya/MFn.h>
#include <maya/MFnDependencyNode.h>
#include <maya/MPlug.h>
#include <maya/MPlugArray.h>
#include <maya/MTime.h>

#include <string>
#include <vector>

#include "adjust_cminpack_base.h"
#include "adjust_defines.h"
#include "adjust_mmba_core.h"
#include "mmSolver/mayahelper/maya_attr.h"
#include "mmSolver/mayahelper/maya_bundle.h"
#include "mmSolver/mayahelper/maya_camera.h"
#include "mmSolver/mayahelper/maya_marker.h"
#include "mmSolver/utilities/debug_utils.h"

namespace {

using namespace mmba_shim;

// Scene reads through the reference's Maya helpers.
class MayaSceneReader : public SceneReader {
  public:
    MayaSceneReader(const MTimeArray &frames, int timeEvalMode)
        : frames_(frames), mode_(timeEvalMode) {}

    AttrRead attr(const std::string &node, const std::string &name, bool force) override {
        AttrRead r;
        Attr a;
        a.setNodeName(MString(node.c_str()));
        a.setAttrName(MString(name.c_str()));
        if (a.getPlug().isNull()) return r;
        r.exists = true;
        r.animated = force || a.isAnimated() || a.isConnected();
        if (r.animated) {
            r.frames.resize(frames_.length());
            for (uint32_t f = 0; f < frames_.length(); ++f)
                a.getValue(r.frames[f], frames_[f], mode_);
            r.value = r.frames.empty() ? 0.0 : r.frames[0];
        } else {
            a.getValue(r.value, mode_);
        }
        return r;
    }

    // check_transform_node (maya_scene_graph.cpp:571-742)
    TransformRead transform(const std::string &path) override {
        TransformRead t;
        const MString name(path.c_str());
        static const char *zero_attrs[] = {
            "rotatePivotX", "rotatePivotY", "rotatePivotZ",
            "scalePivotX", "scalePivotY", "scalePivotZ",
            "rotatePivotTranslateX", "rotatePivotTranslateY", "rotatePivotTranslateZ",
            "scalePivotTranslateX", "scalePivotTranslateY", "scalePivotTranslateZ",
            "rotateAxisX", "rotateAxisY", "rotateAxisZ",
            "shearXY", "shearXZ", "shearYZ"};
        for (const char *n : zero_attrs) {
            Attr a;
            a.setNodeName(name);
            a.setAttrName(MString(n));
            if (a.getPlug().isNull()) continue;
            double v = 0.0;
            a.getValue(v, mode_);
            if (a.isAnimated() || a.isConnected() || v != 0.0) t.plain = false;
        }
        Attr inh;
        inh.setNodeName(name);
        inh.setAttrName("inheritsTransform");
        bool inherits = true;
        if (!inh.getPlug().isNull()) inh.getValue(inherits, mode_);
        if (!inherits) t.plain = false;
        Attr ro;
        ro.setNodeName(name);
        ro.setAttrName("rotateOrder");
        short roo = 0;
        ro.getValue(roo, mode_);
        t.rotate_order = roo;
        t.rotate_order_animated = ro.isAnimated() || ro.isConnected();
        MSelectionList sel;
        MDagPath dag;
        if (sel.add(name) == MS::kSuccess && sel.getDagPath(0, dag) == MS::kSuccess) {
            MDagPath up(dag);
            if (up.pop() == MS::kSuccess && up.length() > 0 && up.hasFn(MFn::kTransform))
                t.parent = up.fullPathName().asChar();
        }
        return t;
    }

    // the lens node on camera.inLens (maya_lens_model_utils.cpp)
    LensRead lens(const std::string &camera_shape) override {
        MSelectionList sel;
        MObject shape_obj;
        if (sel.add(MString(camera_shape.c_str())) != MS::kSuccess ||
            sel.getDependNode(0, shape_obj) != MS::kSuccess)
            return LensRead{};
        return lens_on(shape_obj);
    }

    // a lens node by name: its own inLens is the next layer up the chain
    LensRead lens_node(const std::string &node) override {
        MSelectionList sel;
        MObject obj;
        if (sel.add(MString(node.c_str())) != MS::kSuccess || sel.getDependNode(0, obj) != MS::kSuccess)
            return LensRead{};
        LensRead l;
        read_lens(obj, l);
        return l;
    }

  private:
    // the lens node connected to node.inLens (connected = false when none)
    LensRead lens_on(const MObject &node) {
        LensRead l;
        MStatus status;
        MFnDependencyNode fn(node, &status);
        MPlug in_lens = fn.findPlug("inLens", true, &status);
        if (!status || in_lens.isNull()) return l;
        MPlugArray src;
        in_lens.connectedTo(src, /*asDst=*/true, /*asSrc=*/false, &status);
        if (src.length() == 0) return l;
        read_lens(src[0].node(), l);
        return l;
    }

    // the name of the node on obj.inLens ("" when none), not read further
    std::string upstream_name(const MObject &obj) {
        MStatus status;
        MFnDependencyNode fn(obj, &status);
        MPlug in_lens = fn.findPlug("inLens", true, &status);
        if (!status || in_lens.isNull()) return std::string();
        MPlugArray src;
        in_lens.connectedTo(src, /*asDst=*/true, /*asSrc=*/false, &status);
        if (src.length() == 0) return std::string();
        MFnDependencyNode up(src[0].node(), &status);
        return status ? std::string(up.name().asChar()) : std::string();
    }

    void read_lens(const MObject &obj, LensRead &l) {
        MStatus status;
        MFnDependencyNode lens_fn(obj, &status);
        if (!status) return;
        l.connected = true;
        l.node = lens_fn.name().asChar();
        l.input = upstream_name(obj);
        Attr enable;
        enable.setNodeName(lens_fn.name());
        enable.setAttrName("enable");
        enable.getValue(l.enabled, mode_);
        Attr model;
        model.setNodeName(lens_fn.name());
        model.setAttrName("lensModel");
        short m = 0;
        model.getValue(m, mode_);
        l.model = m;
    }

    const MTimeArray &frames_;
    int mode_;
};

std::string path_of(const MObject &obj) {
    MDagPath p;
    if (MDagPath::getAPathTo(obj, p) != MS::kSuccess) return std::string();
    return p.fullPathName().asChar();
}

// SolverData (adjust_data.h:188-261) -> SolverInputs.
bool inputs_of(SolverData &ud, const std::vector<double> &weights, SolverInputs &in,
               std::string &why) {
    in.num_frames = static_cast<int>(ud.frameList.length());
    const MTime now = MAnimControl::currentTime();
    for (uint32_t f = 0; f < ud.frameList.length(); ++f)
        if (ud.frameList[f] == now) in.current_frame = static_cast<int>(f);
    for (CameraPtr &cam : ud.cameraList) {
        CameraDesc c;
        c.transform_path = path_of(cam->getTransformObject());
        c.shape_path = path_of(cam->getShapeObject());
        if (c.transform_path.empty() || c.shape_path.empty()) {
            why = "camera DAG path";
            return false;
        }
        c.film_fit = cam->getFilmFitValue();  // Maya filmFit = MMBA_FILM_FIT_*
        c.render_width = cam->getRenderWidthValue();
        c.render_height = cam->getRenderHeightValue();
        in.cameras.push_back(c);
    }
    for (BundlePtr &bnd : ud.bundleList) {
        const std::string p = path_of(bnd->getObject());
        if (p.empty()) {
            why = "bundle DAG path";
            return false;
        }
        in.bundles.push_back(p);
    }
    for (MarkerPtr &mkr : ud.markerList) {  // camera / bundle by node name (add_markers)
        int c = -1, b = -1;
        const MString cam_shape = mkr->getCamera()->getShapeNodeName();
        for (size_t j = 0; j < ud.cameraList.size() && c < 0; ++j)
            if (ud.cameraList[j]->getShapeNodeName() == cam_shape) c = static_cast<int>(j);
        const MString bnd_name = mkr->getBundle()->getNodeName();
        for (size_t j = 0; j < ud.bundleList.size() && b < 0; ++j)
            if (ud.bundleList[j]->getNodeName() == bnd_name) b = static_cast<int>(j);
        in.markers.push_back({c, b});
    }
    for (AttrPtr &a : ud.attrList)
        in.attrs.push_back(AttrDesc{a->getNodeName().asChar(), a->getAttrName().asChar(),
                                    a->getMinimumValue(), a->getMaximumValue(),
                                    a->getOffsetValue(), a->getScaleValue()});
    in.paramToAttrList = ud.paramToAttrList;
    in.errorToMarkerList = ud.errorToMarkerList;
    for (const MPoint &p : ud.markerPosList) in.markerPosList.push_back({p.x, p.y});
    // MM Scene Graph with markers not grouped by camera: the flat
    // marker list the reference reads holds every marker at every frame
    bool grouped = true;
    for (size_t k = 1; k < in.markers.size(); ++k)
        grouped = grouped && in.markers[k].first >= in.markers[k - 1].first;
    if (!grouped && ud.solverOptions->sceneGraphMode == SceneGraphMode::kMMSceneGraph) {
        for (MarkerPtr &mkr : ud.markerList)
            for (uint32_t f = 0; f < ud.frameList.length(); ++f) {
                double px = 0.0, py = 0.0;
                mkr->getPosXY(px, py, ud.frameList[f], ud.solverOptions->timeEvalMode, true);
                in.markerFramePos.push_back({px, py});
            }
    }
    in.markerWeightList = ud.markerWeightList;
    in.paramWeightList = weights;
    auto rows = [&](auto &list, int count, std::vector<AttrRowDesc> &out) {
        for (int i = 0; i < count; ++i) {
            auto &s = list[i];
            AttrRowDesc r;
            r.attr_index = s->attrIndex;
            s->weightAttr->getValue(r.weight, ud.solverOptions->timeEvalMode);
            s->varianceAttr->getValue(r.variance, ud.solverOptions->timeEvalMode);
            s->valueAttr->getValue(r.value, ud.solverOptions->timeEvalMode);
            out.push_back(r);
        }
    };
    rows(ud.stiffAttrsList, ud.numberOfAttrStiffnessErrors, in.stiff);
    rows(ud.smoothAttrsList, ud.numberOfAttrSmoothnessErrors, in.smooth);
    return true;
}

Options options_of_maya(const SolverOptions &so) {
    Options o;
    o.solverType = so.solverType == SOLVER_TYPE_CMINPACK_LMDIF ? MMBA_SOLVER_CMINPACK_LMDIF
                                                              : MMBA_SOLVER_CMINPACK_LMDER;
    o.iterMax = so.iterMax;
    o.tau = so.tau;
    o.eps1 = so.eps1;
    o.eps2 = so.eps2;
    o.eps3 = so.eps3;
    o.delta = so.delta;
    o.autoDiffType = so.autoDiffType;
    o.autoParamScale = so.autoParamScale;
    o.robustLossType = so.robustLossType;
    o.robustLossScale = so.robustLossScale;
    o.mmSceneGraph = so.sceneGraphMode == SceneGraphMode::kMMSceneGraph;
    o.imageWidth = so.imageWidth;
    o.acceptOnlyBetter = so.acceptOnlyBetter;
    o.solverSupportsRobustLoss = so.solverSupportsRobustLoss;
    return o;
}

Shim &shim() {
    static Shim s;
    return s;
}

mmba_callbacks callbacks_of(SolverData &ud) {
    mmba_callbacks cb;
    cb.interrupt = [](void *u) -> int {
        auto *d = static_cast<SolverData *>(u);
        return (d->computation && d->computation->isInterruptRequested()) ? 1 : 0;
    };
    cb.progress = [](void *u, int32_t it) {
        auto *d = static_cast<SolverData *>(u);
        if (d->computation) d->computation->setProgress(it);
    };
    cb.user = &ud;
    return cb;
}

void to_solver_result(const Result &r, SolverResult &out) {
    out.success = r.success;
    out.reason_number = r.reason_number;
    out.reason = (r.reason_number >= 0 && r.reason_number <= 8)
                     ? cminpackReasons[r.reason_number]
                     : std::string("User interrupted.");
    out.iterations = r.iterations;
    out.functionEvals = r.functionEvals;
    out.jacobianEvals = r.jacobianEvals;
    out.errorFinal = r.errorFinal;
    out.user_interrupted = r.user_interrupted;
}

}  // namespace

bool solve_3d_mmba(SolverOptions &solverOptions, int numberOfParameters, int numberOfErrors,
                   std::vector<double> &paramList, std::vector<double> &errorList,
                   std::vector<double> &paramWeightList, SolverData &userData,
                   SolverResult &solveResult) {
    SolverInputs in;
    std::string why;
    if (!inputs_of(userData, paramWeightList, in, why)) {
        MMSOLVER_MAYA_VRB("mmba: " << why.c_str() << ", using cminpack");
        return false;
    }
    MayaSceneReader rd(userData.frameList, solverOptions.timeEvalMode);
    const mmba_callbacks cb = callbacks_of(userData);
    Result r;
    const SolveStatus st = mmba_shim::solve(
        shim(), in, rd, options_of_maya(solverOptions), numberOfParameters, numberOfErrors,
        paramList.data(), errorList.data(), userData.errorList.data(),
        userData.errorDistanceList.data(), &cb, &r, &why);
    if (st == kNotMapped) {
        MMSOLVER_MAYA_VRB("mmba: " << why.c_str() << ", using cminpack");
        return false;
    }
    if (st == kFailed) {
        MMSOLVER_MAYA_ERR("mmba: " << why.c_str());
        solveResult.success = false;
        return true;  // the solve ran and failed: do not run it again on the CPU
    }
    to_solver_result(r, solveResult);
    userData.iterNum = r.iterNum;  // solveFunc's counters as the cminpack path leaves them
    userData.jacIterNum = r.jacIterNum;
    userData.funcEvalNum = r.funcEvalNum;
    userData.userInterrupted = r.user_interrupted;
    return true;
}

bool solve_frames_mmba_per_frame(SolverOptions &solverOptions, std::vector<double> &paramList,
                                 std::vector<double> &paramWeightList, SolverData &userData,
                                 std::vector<SolverResult> &perFrameResults) {
    Shim &s = shim();
    if (!s.ready()) return false;
    for (const auto &pa : userData.paramToAttrList)
        if (pa.second < 0) return false;  // a static parameter chains the frames
    SolverInputs in;
    std::string why;
    if (!inputs_of(userData, paramWeightList, in, why)) return false;
    MayaSceneReader rd(userData.frameList, solverOptions.timeEvalMode);
    FlatScene scene;
    if (!scene.build(in, rd)) return false;
    const mmba_problem prob = scene.problem();
    // every frame's solveFrames measures its own initial error and writes
    // back only when it got better (adjust_base.cpp:1080-1103, 1227-1244)
    const mmba_options o = options_of(options_of_maya(solverOptions), /*per_frame=*/true);
    mmba_plan *plan = s.plan_for(scene, prob, o);
    if (!plan) return false;
    const mmba_callbacks cb = callbacks_of(userData);
    std::vector<mmba_result> res(static_cast<size_t>(prob.num_frames));
    const int rc = mmba_plan_solve_per_frame(plan, paramList.data(), res.data(), &cb);
    if (rc == MMBA_ERR_UNSUPPORTED) return false;
    perFrameResults.assign(res.size(), SolverResult());
    for (size_t f = 0; f < res.size(); ++f) {
        Result r;
        fill_result(res[f], r);
        to_solver_result(r, perFrameResults[f]);
        perFrameResults[f].errorAvg = r.errorAvg;
        perFrameResults[f].errorMin = r.errorMin;
        perFrameResults[f].errorMax = r.errorMax;
    }
    if (rc != MMBA_OK) MMSOLVER_MAYA_ERR("mmba: " << mmba_last_error());
    return true;
}

void mmba_shim_release() { shim().release(); }
