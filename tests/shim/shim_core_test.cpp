// shim_core_test.cpp -- drives the Maya-free shim core
// (integration/adjust_mmba_core.cpp) through the C ABI on known scenes.
//
// Each scene is what the Maya layer would hand the core: SolverData's index
// vectors (SolverInputs) and the scene reads (an in-memory SceneReader
// standing in for Attr / MDagPath / the lens node).  Scenes:
//   0  test1 (tests/test/test_solver/test1.py:52-122): bundle tx, ty solved,
//      known answer (-6.0, 3.6)
//   1  test3 (test3.py:55-124): camera rx, ry solved (delta 1e-5), known
//      answer (7.44014, -32.3891)
//   2  an animated camera over 4 frames with per-frame rotate solved, a 3DE
//      classic lens on camera.inLens (distortion solved) layered over a
//      static radial lens, and a rolling
//      shutter: keyed attributes, lens slots, rows of several frames
//   3  scene 2 without the rolling shutter, its input radial lens animated
//      (degree-2 / degree-4 distortion keyed per frame) and the current time
//      at solve frame 2: the input layer holds its frame-2 values for the
//      whole solve (maya_lens_model_utils.cpp:433-446)
//
// Built twice (tests/shim/Makefile): as an executable (main: every scene
// through mmba_shim::solve; without a gfx950 device the core must report the
// fallback to cminpack) and as libshimtest.so (the C entries below), which
// tests/test_shim_core.py loads to compare the flattened problem with the
// Python-built one through the CPU oracle.
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>

#include "adjust_mmba_core.h"

using namespace mmba_shim;

namespace {

struct MemReader : SceneReader {
    std::map<std::string, AttrRead> attrs;  // "node.attr"
    std::map<std::string, TransformRead> tfms;
    std::map<std::string, LensRead> lenses;  // by camera shape
    int F = 1;

    AttrRead attr(const std::string &node, const std::string &a, bool force) override {
        auto it = attrs.find(node + "." + a);
        if (it == attrs.end()) return AttrRead{};
        AttrRead r = it->second;
        if (force && !r.animated) {  // keyed per frame: one sample per solve frame
            r.animated = true;
            r.frames.assign(F, r.value);
        }
        return r;
    }
    TransformRead transform(const std::string &path) override {
        auto it = tfms.find(path);
        return it == tfms.end() ? TransformRead{} : it->second;
    }
    LensRead lens(const std::string &shape) override {
        auto it = lenses.find(shape);
        return it == lenses.end() ? LensRead{} : it->second;
    }
    std::map<std::string, LensRead> nodes;  // lens nodes by name (upstream layers)
    LensRead lens_node(const std::string &node) override {
        auto it = nodes.find(node);
        return it == nodes.end() ? LensRead{} : it->second;
    }

    void stat(const std::string &na, double v) {
        AttrRead r;
        r.exists = true;
        r.value = v;
        attrs[na] = r;
    }
    void anim(const std::string &na, std::vector<double> v) {
        AttrRead r;
        r.exists = true;
        r.animated = true;
        r.value = v.empty() ? 0.0 : v[0];
        r.frames = std::move(v);
        attrs[na] = r;
    }
    void trs(const std::string &path, const double t[3], const double r[3]) {
        static const char *n[6] = {"translateX", "translateY", "translateZ",
                                   "rotateX",    "rotateY",    "rotateZ"};
        for (int k = 0; k < 3; ++k) stat(path + "." + n[k], t[k]);
        for (int k = 0; k < 3; ++k) stat(path + "." + n[3 + k], r[k]);
        for (const char *s : {"scaleX", "scaleY", "scaleZ"}) stat(path + "." + s, 1.0);
        tfms[path] = TransformRead{};
    }
    void camera_shape(const std::string &shape) {
        stat(shape + ".horizontalFilmAperture", 36.0 / 25.4);
        stat(shape + ".verticalFilmAperture", 24.0 / 25.4);
        stat(shape + ".focalLength", 35.0);
        stat(shape + ".horizontalFilmOffset", 0.0);
        stat(shape + ".verticalFilmOffset", 0.0);
        stat(shape + ".nearClipPlane", 0.1);
        stat(shape + ".farClipPlane", 10000.0);
        stat(shape + ".cameraScale", 1.0);
    }
};

struct Scene {
    SolverInputs in;
    MemReader rd;
    Options so;
    std::vector<double> x0;       // internal values (unbounded: the attribute values)
    double expect[2] = {NAN, NAN};
    double tol = 0.0;
    FlatScene flat;               // kept alive for shim_demo_problem
};

AttrDesc solved(const std::string &node, const std::string &attr) {
    return AttrDesc{node, attr, -FLT_MAX, FLT_MAX, 0.0, 1.0};
}

// markers of scenes 2 / 3 (marker-major, frame-minor): the forward model at a
// true pose and lens (tests/shim/gen_scene2_markers.py)
const double kScene2Markers[20][2] = {
    {-0.23873034935799486, -0.050894781155829634},
    {-0.23181865466579299, -0.06415868658293411},
    {-0.22496889641796142, -0.048549320201375472},
    {-0.21805635698669693, -0.026341277304751515},
    {-0.12918474157362708, -0.021228432336373618},
    {-0.12170790356735069, -0.033055281860840904},
    {-0.11422490874317545, -0.018575519493559296},
    {-0.10638882977015819, -8.9621906492073043e-05},
    {-0.044956863564452644, 0.0016716474101909832},
    {-0.03722012829822597, -0.0093059329867673009},
    {-0.029069090752251482, 0.0046899590908291615},
    {-0.020263446930858117, 0.020251735335200423},
    {0.021639233221250404, 0.019727113220638085},
    {0.029532659655347186, 0.0096641178880656296},
    {0.038486605759479368, 0.023090849868926223},
    {0.047876170004553104, 0.0363256114043954},
    {0.075032417674294347, 0.034178340970243096},
    {0.083717764827209482, 0.024882861684639553},
    {0.092810152575285257, 0.038010888700753316},
    {0.10297730975261896, 0.049418792306458313},
};

std::unique_ptr<Scene> make_scene(int which) {
    auto sc = std::make_unique<Scene>();
    SolverInputs &in = sc->in;
    MemReader &rd = sc->rd;
    const CameraDesc cam{"|cam", "|cam|camShape", MMBA_FILM_FIT_HORIZONTAL, 2048, 1556};
    if (which == 0 || which == 1) {
        rd.F = 1;
        in.num_frames = 1;
        const double ct[3] = {-1.0, 1.0, -5.0}, cr[3] = {0.0, 0.0, 0.0};
        const double bt[3] = {5.5, 6.4, -25.0}, br[3] = {0.0, 0.0, 0.0};
        rd.trs("|cam", ct, cr);
        rd.camera_shape("|cam|camShape");
        rd.trs("|bundle", bt, br);
        in.cameras = {cam};
        in.bundles = {"|bundle"};
        in.markers = {{0, 0}};
        in.errorToMarkerList = {{0, 0}};
        in.markerPosList = {{-0.243056042, 0.189583713}};
        in.markerWeightList = {1.0};
        if (which == 0) {
            in.attrs = {solved("|bundle", "translateX"), solved("|bundle", "translateY")};
            sc->x0 = {5.5, 6.4};
            sc->expect[0] = -6.0;
            sc->expect[1] = 3.6;
            sc->tol = 1e-4;
            sc->so.iterMax = 1000;
        } else {
            in.attrs = {solved("|cam", "rotateX"), solved("|cam", "rotateY")};
            sc->x0 = {0.0, 0.0};
            sc->expect[0] = 7.44014;
            sc->expect[1] = -32.3891;
            sc->tol = 1e-3;
            sc->so.delta = 1e-5;
        }
        in.paramToAttrList = {{0, -1}, {1, -1}};
        return sc;
    }
    // scenes 2 / 3: 4 frames, per-frame camera rotate solved, classic lens
    // over a radial one (scene 2: static, rolling shutter; scene 3: animated
    // input layer, current time at frame 2)
    const int F = 4;
    rd.F = F;
    in.num_frames = F;
    in.current_frame = which == 3 ? 2 : 0;
    std::vector<double> tx(F), tz(F), rx(F), ry(F), rz(F);
    for (int f = 0; f < F; ++f) {
        tx[f] = 0.1 * f;
        tz[f] = -0.05 * f;
        rx[f] = 1.0 + 0.5 * f;
        ry[f] = -2.0 + 0.3 * f;
        rz[f] = 0.2 * f;
    }
    const double zero3[3] = {0.0, 0.0, 0.0};
    rd.trs("|cam", zero3, zero3);
    rd.anim("|cam.translateX", tx);
    rd.stat("|cam.translateY", 1.0);
    rd.anim("|cam.translateZ", tz);
    rd.anim("|cam.rotateX", rx);
    rd.anim("|cam.rotateY", ry);
    rd.anim("|cam.rotateZ", rz);
    rd.camera_shape("|cam|camShape");
    LensRead lens;
    lens.connected = true;
    lens.node = "lens1";
    lens.model = 2;  // 3DE classic
    lens.input = "lens0";  // layered over a radial lens (mmba.h ABI 5)
    rd.lenses["|cam|camShape"] = lens;
    LensRead lens0;
    lens0.connected = true;
    lens0.node = "lens0";
    lens0.model = 3;  // 3DE radial std deg 4
    rd.nodes["lens0"] = lens0;
    if (which == 3) {
        rd.anim("lens0.tdeRadialStdDeg4_degree2_distortion", {0.01, 0.02, 0.03, 0.05});
        rd.anim("lens0.tdeRadialStdDeg4_degree4_distortion", {0.0, 0.004, 0.012, 0.02});
    } else {
        rd.stat("lens0.tdeRadialStdDeg4_degree2_distortion", 0.03);
        rd.stat("lens0.tdeRadialStdDeg4_degree4_distortion", 0.008);
    }
    rd.stat("lens0.tdeRadialStdDeg4_degree2_u", 0.002);
    rd.stat("lens0.tdeRadialStdDeg4_degree2_v", -0.001);
    rd.stat("lens0.tdeRadialStdDeg4_degree4_u", 0.0);
    rd.stat("lens0.tdeRadialStdDeg4_degree4_v", 0.0);
    rd.stat("lens0.tdeRadialStdDeg4_cylindricDirection", 15.0);
    rd.stat("lens0.tdeRadialStdDeg4_cylindricBending", 0.02);
    rd.stat("lens1.tdeClassic_distortion", 0.02);
    rd.stat("lens1.tdeClassic_anamorphicSqueeze", 1.0);
    rd.stat("lens1.tdeClassic_curvatureX", 0.0);
    rd.stat("lens1.tdeClassic_curvatureY", 0.0);
    rd.stat("lens1.tdeClassic_quarticDistortion", 0.0);
    in.cameras = {cam};
    const int B = 5;
    for (int k = 0; k < B; ++k) {
        const std::string b = "|bundle" + std::to_string(k);
        const double bt[3] = {-4.0 + 2.0 * k, 1.0 + 0.5 * k, -20.0 - 3.0 * k};
        rd.trs(b, bt, zero3);
        in.bundles.push_back(b);
        in.markers.push_back({0, k});
    }
    for (int k = 0; k < B; ++k)
        for (int f = 0; f < F; ++f) {  // marker-major, frame-minor
            in.errorToMarkerList.push_back({k, f});
            in.markerPosList.push_back({kScene2Markers[k * F + f][0], kScene2Markers[k * F + f][1]});
            in.markerWeightList.push_back(1.0);
        }
    in.attrs = {solved("|cam", "rotateX"), solved("|cam", "rotateY"), solved("|cam", "rotateZ"),
                solved("lens1", "tdeClassic_distortion")};
    for (int a = 0; a < 3; ++a)
        for (int f = 0; f < F; ++f) {
            in.paramToAttrList.push_back({a, f});
            sc->x0.push_back(a == 0 ? rx[f] : (a == 1 ? ry[f] : rz[f]));
        }
    in.paramToAttrList.push_back({3, -1});
    sc->x0.push_back(0.02);
    if (which == 2) in.rolling_shutter = {0.5};
    if (which == 4)  // every marker's x,y at every frame (mmba.h ABI 8)
        for (int k = 0; k < B; ++k)
            for (int f = 0; f < F; ++f)
                in.markerFramePos.push_back({kScene2Markers[k * F + f][0], kScene2Markers[k * F + f][1]});
    sc->so.iterMax = 100;
    return sc;
}

constexpr int kScenes = 5;
std::unique_ptr<Scene> g_scene[kScenes];

Scene *scene(int which) {
    if (which < 0 || which >= kScenes) return nullptr;
    if (!g_scene[which]) {
        g_scene[which] = make_scene(which);
        Scene *sc = g_scene[which].get();
        if (!sc->flat.build(sc->in, sc->rd)) std::fprintf(stderr, "build: %s\n", sc->flat.why.c_str());
    }
    return g_scene[which].get();
}

Shim &shim() {
    static Shim s;
    return s;
}

}  // namespace

extern "C" {

// The flattened problem of scene `which` (valid until the library unloads).
int shim_demo_problem(int which, mmba_problem *out) {
    Scene *sc = scene(which);
    if (!sc || !sc->flat.why.empty()) return -1;
    *out = sc->flat.problem();
    return 0;
}

int shim_demo_num_params(int which) {
    Scene *sc = scene(which);
    return sc ? static_cast<int>(sc->x0.size()) : -1;
}

// x0 (internal) and the solver options as mmba_options.
int shim_demo_x0(int which, double *x0, mmba_options *opt) {
    Scene *sc = scene(which);
    if (!sc) return -1;
    std::memcpy(x0, sc->x0.data(), sizeof(double) * sc->x0.size());
    if (opt) *opt = options_of(sc->so);
    return 0;
}

// mmba_shim::solve on scene `which`: returns the SolveStatus; x_inout [n],
// fvec [m]; message gets the reason for a fallback / failure.
int shim_demo_solve(int which, double *x_out, double *fvec_out, int *reason, int *func_evals,
                    char *message, int message_len) {
    Scene *sc = scene(which);
    if (!sc) return -9;
    const mmba_problem p = sc->flat.problem();
    const int m = 2 * p.num_obs + p.num_stiff + p.num_smooth;
    std::vector<double> x = sc->x0, f(m), eu(m), ed(p.num_obs);
    Result r;
    std::string msg;
    const SolveStatus st = solve(shim(), sc->in, sc->rd, sc->so, (int)x.size(), m, x.data(),
                                 f.data(), eu.data(), ed.data(), nullptr, &r, &msg);
    if (message && message_len > 0) {
        std::strncpy(message, msg.c_str(), message_len - 1);
        message[message_len - 1] = 0;
    }
    if (st == kSolved) {
        std::memcpy(x_out, x.data(), sizeof(double) * x.size());
        std::memcpy(fvec_out, f.data(), sizeof(double) * f.size());
        *reason = r.reason_number;
        *func_evals = r.functionEvals;
    }
    return st;
}

int shim_demo_cached_plans() { return (int)shim().cached_plans(); }

}  // extern "C"

#ifdef SHIM_MAIN
int main() {
    int failures = 0;
    const bool device = mmba_device_count() > 0;
    for (int which = 0; which < kScenes; ++which) {
        Scene *sc = scene(which);
        if (!sc->flat.why.empty()) {
            std::printf("scene %d: not mapped: %s\n", which, sc->flat.why.c_str());
            ++failures;
            continue;
        }
        const mmba_problem p = sc->flat.problem();
        std::printf("scene %d: %d attrs, %d transforms, %d cameras, %d lenses, %d obs, %d params\n",
                    which, p.num_attrs, p.num_transforms, p.num_cameras, p.num_lenses, p.num_obs,
                    p.num_params);
        const int n = (int)sc->x0.size();
        std::vector<double> x(n), f(2 * p.num_obs);
        int reason = 0, fe = 0;
        char msg[256];
        const int st = shim_demo_solve(which, x.data(), f.data(), &reason, &fe, msg, sizeof msg);
        if (!device) {
            // no gfx950 device: the core must hand the solve back to cminpack
            const bool ok = st == kNotMapped && std::strstr(msg, "no gfx950 device");
            std::printf("  fallback to cminpack (%s): %s\n", msg, ok ? "ok" : "WRONG");
            failures += ok ? 0 : 1;
            continue;
        }
        if (st != kSolved) {
            std::printf("  solve status %d: %s\n", st, msg);
            ++failures;
            continue;
        }
        std::printf("  solved: reason %d, %d evaluations", reason, fe);
        if (!std::isnan(sc->expect[0])) {
            const bool ok = std::fabs(x[0] - sc->expect[0]) <= sc->tol &&
                            std::fabs(x[1] - sc->expect[1]) <= sc->tol;
            std::printf(", x = (%.6f, %.6f), known answer (%.6f, %.6f): %s", x[0], x[1],
                        sc->expect[0], sc->expect[1], ok ? "ok" : "WRONG");
            failures += ok ? 0 : 1;
        }
        std::printf("\n");
    }
    if (device) {
        // a second solve of every scene re-uses the cached plans
        for (int which = 0; which < kScenes; ++which) {
            Scene *sc = scene(which);
            std::vector<double> x(sc->x0.size()), f(2 * sc->flat.obs_marker.size());
            int reason = 0, fe = 0;
            char msg[256];
            if (shim_demo_solve(which, x.data(), f.data(), &reason, &fe, msg, sizeof msg) != kSolved)
                ++failures;
        }
        std::printf("cached plans: %d\n", shim_demo_cached_plans());
        // the shim caches at most 4 plans (Shim::kMaxPlans)
        if (shim_demo_cached_plans() != kScenes) ++failures;
    }
    shim().release();
    std::printf("%s\n", failures ? "FAILED" : "PASSED");
    return failures ? 1 : 0;
}
#endif
