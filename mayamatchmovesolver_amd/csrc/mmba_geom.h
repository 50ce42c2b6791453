// mmba_geom.h -- per-element geometry of the reference residual, as device code.
//
// Arithmetic follows (operation for operation, compiled with
// -ffp-contract=off so no FMA is introduced):
//   TRS matrix            lib/rust/mmscenegraph/src/math/transform.rs:338-452
//   world matrices        math/dag.rs:234-327 (parent_world * local)
//   projection matrix     math/camera.rs:153-327 (MMSG) /
//                         src/mmSolver/mayahelper/maya_camera.cpp:75-414 (Maya DAG)
//   reprojection          math/reprojection.rs:28-63 ((P * C^-1) * B, /w, *0.5)
//   marker film fit       scene/flat.rs:73-97, maya_camera.cpp:213-330
//   residual              src/mmSolver/adjust/adjust_measureErrors.cpp:231-292 (DAG),
//                         :444-499 (MMSG)
//   3DE classic distort   lib/cppbind/mmlens/src/lens_model_3de_classic.cpp:75-113,
//                         distortion_operations.h:34-96, include/mmlens/lib.h:36-75,
//                         LDPK classic_3de_mixed_distortion + generic map_inverse
#pragma once

#include "mmba_internal.h"

namespace mmba {

#define MMBA_DEV __device__ __forceinline__

constexpr double DEG2RAD = 0.017453292519943295;
constexpr double MM_TO_INCH = 0.03937007874015748;
constexpr double INCH_TO_MM = 25.4;
constexpr double MM_TO_CM = 0.1;
constexpr int MAX_DEPTH = 16;

// One attribute override: the perturbed parameter of an FD column.
struct Override {
    int attr;
    double value;
};

MMBA_DEV double attr_get(const DevProblem &P, int a, int f, double dflt,
                         const Override &ov) {
    if (a < 0) return dflt;
    if (a == ov.attr) return ov.value;
    return P.attr_anim[a] ? P.attr_val[P.attr_off[a] + f] : P.attr_val[P.attr_off[a]];
}

MMBA_DEV void mat4_mul(const double *a, const double *b, double *out) {
    double t[16];
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c)
            t[r * 4 + c] = a[r * 4 + 0] * b[0 * 4 + c] + a[r * 4 + 1] * b[1 * 4 + c] +
                           a[r * 4 + 2] * b[2 * 4 + c] + a[r * 4 + 3] * b[3 * 4 + c];
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = t[i];
}

MMBA_DEV void mat4_inverse(const double *m, double *out) {
    double inv[16];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] +
             m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] -
             m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] +
             m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] -
              m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] -
             m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] +
             m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] -
             m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] +
              m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] +
             m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] -
             m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] +
              m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] -
              m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] -
             m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] +
             m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] -
              m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] +
              m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    if (det == 0.) {
#pragma unroll
        for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1. : 0.;
        return;
    }
    double inv_det = 1.0 / det;
#pragma unroll
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * inv_det;
}

// R = (a * b) * c for 3x3 row-major rotation factors.
MMBA_DEV void rot3_chain(const double *a, const double *b, const double *c, double *R) {
    double AB[9];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            AB[r * 3 + k] = a[r * 3 + 0] * b[0 * 3 + k] + a[r * 3 + 1] * b[1 * 3 + k] +
                            a[r * 3 + 2] * b[2 * 3 + k];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            R[r * 3 + k] = AB[r * 3 + 0] * c[0 * 3 + k] + AB[r * 3 + 1] * c[1 * 3 + k] +
                           AB[r * 3 + 2] * c[2 * 3 + k];
}

MMBA_DEV void trs_matrix(double tx, double ty, double tz, double rx, double ry,
                         double rz, double sx, double sy, double sz, int roo,
                         double *out) {
    double srx, crx, sry, cry, srz, crz;
    // one shared argument reduction per angle (the camera-record chain is
    // one thread's serial fp64 stream: k_records is latency-bound)
    sincos(rx * DEG2RAD, &srx, &crx);
    sincos(ry * DEG2RAD, &sry, &cry);
    sincos(rz * DEG2RAD, &srz, &crz);
    // The reference forms T * (a * b * c) * S as 4x4 products. Every term that
    // 4x4 form adds beyond the 3x3 rotation block is an exact zero (x * 0,
    // added last), and T, S only place t and scale columns, so the 3x3
    // rotation products below, then column scaling, give the same doubles for
    // finite inputs at a quarter of the arithmetic.
    const double RX[9] = {1, 0, 0, 0, crx, -srx, 0, srx, crx};
    const double RY[9] = {cry, 0, sry, 0, 1, 0, -sry, 0, cry};
    const double RZ[9] = {crz, -srz, 0, srz, crz, 0, 0, 0, 1};
    // Each rotation order names its factors at compile time, so the factor
    // arrays stay in registers (a runtime-selected pointer put them in scratch).
    double R[9];
    switch (roo) {
        default:
        case MMBA_ROO_XYZ: rot3_chain(RZ, RY, RX, R); break;
        case MMBA_ROO_YZX: rot3_chain(RX, RZ, RY, R); break;
        case MMBA_ROO_ZXY: rot3_chain(RY, RX, RZ, R); break;
        case MMBA_ROO_XZY: rot3_chain(RY, RZ, RX, R); break;
        case MMBA_ROO_YXZ: rot3_chain(RZ, RX, RY, R); break;
        case MMBA_ROO_ZYX: rot3_chain(RX, RY, RZ, R); break;
    }
    const double s[3] = {sx, sy, sz};
    const double t[3] = {tx, ty, tz};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
#pragma unroll
        for (int k = 0; k < 3; ++k) out[r * 4 + k] = R[r * 3 + k] * s[k];
        out[r * 4 + 3] = t[r];
    }
    out[12] = 0.;
    out[13] = 0.;
    out[14] = 0.;
    out[15] = 1.;
}

MMBA_DEV void local_matrix(const DevProblem &P, int t, int f, const Override &ov,
                           double *out) {
    const int *ta = &P.tfm_attrs[9 * t];
    trs_matrix(attr_get(P, ta[0], f, 0., ov), attr_get(P, ta[1], f, 0., ov),
               attr_get(P, ta[2], f, 0., ov), attr_get(P, ta[3], f, 0., ov),
               attr_get(P, ta[4], f, 0., ov), attr_get(P, ta[5], f, 0., ov),
               attr_get(P, ta[6], f, 1., ov), attr_get(P, ta[7], f, 1., ov),
               attr_get(P, ta[8], f, 1., ov), P.tfm_roo[t], out);
}

// World matrix of transform t at frame f: root-first products (dag.rs:293-313).
MMBA_DEV void world_matrix(const DevProblem &P, int t, int f, const Override &ov,
                           double *W) {
    int chain[MAX_DEPTH];
    int d = 0;
    for (int u = t; u >= 0 && d < MAX_DEPTH; u = P.tfm_parent[u]) chain[d++] = u;
    local_matrix(P, chain[d - 1], f, ov, W);
    for (int j = d - 2; j >= 0; --j) {
        double L[16];
        local_matrix(P, chain[j], f, ov, L);
        mat4_mul(W, L, W);
    }
}

// Bundle world position = column 3 of world matrix (flat.rs:317-321 uses B[:,3]).
MMBA_DEV void bundle_position(const DevProblem &P, int b, int f, const Override &ov,
                              double *pos) {
    const int t = P.bnd_tfm[b];
    const int *ta = &P.tfm_attrs[9 * t];
    double tx = attr_get(P, ta[0], f, 0., ov);
    double ty = attr_get(P, ta[1], f, 0., ov);
    double tz = attr_get(P, ta[2], f, 0., ov);
    const int parent = P.tfm_parent[t];
    if (parent < 0) {
        pos[0] = tx;
        pos[1] = ty;
        pos[2] = tz;
        return;
    }
    double W[16];
    world_matrix(P, parent, f, ov, W);
#pragma unroll
    for (int r = 0; r < 3; ++r)
        pos[r] = W[r * 4 + 0] * tx + W[r * 4 + 1] * ty + W[r * 4 + 2] * tz + W[r * 4 + 3] * 1.0;
}

// Projection matrix in column-vector convention; see oracle/refcpu.c
// ref_projection_matrix for the mode differences (Appendix B5/B6).
MMBA_DEV void projection_matrix(int mode, double focal_mm, double fbw_inch,
                                double fbh_inch, double offx_inch, double offy_inch,
                                double image_w, double image_h, int film_fit,
                                double far_clip, double camera_scale, double *P) {
    const double near_clip = 0.1;
    double film_aspect = fbw_inch / fbh_inch;
    double image_aspect = image_w / image_h;
    double film_w_mm = fbw_inch * INCH_TO_MM, film_h_mm = fbh_inch * INCH_TO_MM;
    double off_x_mm = offx_inch * INCH_TO_MM, off_y_mm = offy_inch * INCH_TO_MM;
    double ftn = (near_clip / focal_mm) * camera_scale;
    double right = ftn * (0.5 * film_w_mm + off_x_mm);
    double left = ftn * (-0.5 * film_w_mm + off_x_mm);
    double top = ftn * (0.5 * film_h_mm + off_y_mm);
    double bottom = ftn * (-0.5 * film_h_mm + off_y_mm);
    double fsx = 1., fsy = 1., size_x = 0., size_y = 0.;
    const bool rust = (mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH);
    switch (film_fit) {
        default:
        case MMBA_FILM_FIT_HORIZONTAL:
            if (rust)
                fsx = image_aspect / film_aspect;
            else
                fsy = image_aspect / film_aspect;
            size_x = right - left;
            size_y = size_x / image_aspect;
            break;
        case MMBA_FILM_FIT_VERTICAL:
            fsx = 1.0 / (image_aspect / film_aspect);
            size_y = top - bottom;
            size_x = size_y * image_aspect;
            break;
        case MMBA_FILM_FIT_FILL:
            if (film_aspect > image_aspect) {
                fsx = film_aspect / image_aspect;
                size_y = top - bottom;
                size_x = size_y * image_aspect;
            } else {
                fsy = image_aspect / film_aspect;
                size_x = right - left;
                size_y = (size_x * (film_aspect / image_aspect)) / film_aspect;
            }
            break;
        case MMBA_FILM_FIT_OVERSCAN:
            if (film_aspect > image_aspect) {
                fsy = image_aspect / film_aspect;
                size_x = right - left;
                size_y = (right - left) / image_aspect;
            } else {
                fsx = film_aspect / image_aspect;
                size_x = (right - left) * (image_aspect / film_aspect);
                size_y = top - bottom;
            }
            break;
    }
    right *= fsx;
    left *= fsx;
    top *= fsy;
    bottom *= fsy;
    double p00 = 1.0 / (size_x * 0.5) * MM_TO_CM;
    double p11 = 1.0 / (size_y * 0.5) * MM_TO_CM;
    double ox = (right + left) / (right - left) * fsx;
    double oy = (top + bottom) / (top - bottom) * fsy;
    double zz = (far_clip + near_clip) / (far_clip - near_clip);
    double zw = 2.0 * far_clip * near_clip / (far_clip - near_clip);
#pragma unroll
    for (int i = 0; i < 16; ++i) P[i] = 0.;
    P[0] = p00;
    P[5] = p11;
    if (rust) {
        P[8] = ox;
        P[9] = oy;
        P[10] = zz;
        P[11] = zw;
        P[14] = -1.;
    } else {
        P[2] = ox;
        P[6] = oy;
        P[10] = zz;
        P[14] = -1.;
        P[11] = zw;
    }
}

// Camera-frame record from the camera's attribute values (cv: film back w/h,
// film offset x/y in inches, focal mm, far clip, camera scale) and its world
// matrix W.
MMBA_DEV void camera_record_tail(const DevProblem &P, int c, double w, double h, double ox,
                                 double oy, double focal, double far_clip, double cscale,
                                 const double *W, double *rec) {
    double fbw, fbh, offx, offy, fa;
    if (P.mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        double w_mm = w * 25.4, h_mm = h * 25.4;
        fbw = w_mm * MM_TO_INCH;
        fbh = h_mm * MM_TO_INCH;
        offx = (ox * 25.4) * MM_TO_INCH;
        offy = (oy * 25.4) * MM_TO_INCH;
        fa = w_mm / h_mm;
    } else {
        fbw = w;
        fbh = h;
        offx = ox;
        offy = oy;
        fa = w / h;
    }
    double iw = (double)P.cam_size[2 * c];
    double ih = (double)P.cam_size[2 * c + 1];
    double Pm[16];
    const int fit = P.cam_fit[c];
    projection_matrix(P.mode, focal, fbw, fbh, offx, offy, iw, ih, fit, far_clip, cscale, Pm);
    double ra = iw / ih;
    double Ci[16], PV[16];
    mat4_inverse(W, Ci);
    mat4_mul(Pm, Ci, PV);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rec[k] = PV[k];
        rec[4 + k] = PV[4 + k];
        rec[8 + k] = PV[12 + k];
    }
    rec[12] = W[3] / W[15];
    rec[13] = W[7] / W[15];
    rec[14] = W[11] / W[15];
    double cdir[3] = {-W[2], -W[6], -W[10]};
    double cl = sqrt(cdir[0] * cdir[0] + cdir[1] * cdir[1] + cdir[2] * cdir[2]);
    rec[15] = cdir[0] / cl;
    rec[16] = cdir[1] / cl;
    rec[17] = cdir[2] / cl;
    // marker film-fit factors (x *= rec[18], y *= rec[19])
    double sx = 1.0, sy = 1.0;
    switch (fit) {
        case MMBA_FILM_FIT_HORIZONTAL: sy = ra / fa; break;
        case MMBA_FILM_FIT_VERTICAL: sx = 1.0 / (ra / fa); break;
        case MMBA_FILM_FIT_FILL:
            if (fa > ra) sx = fa / ra; else sy = ra / fa;
            break;
        case MMBA_FILM_FIT_OVERSCAN:
            if (fa > ra) sy = ra / fa; else sx = fa / ra;
            break;
        default: break;
    }
    rec[18] = sx;
    rec[19] = sy;
}

// Camera-frame record: rows 0,1,3 of P*C^-1 (12), camera position (3),
// normalised forward direction (3), marker film-fit factors (2).
MMBA_DEV void camera_record(const DevProblem &P, int c, int f, const Override &ov,
                            double *rec) {
    const int *ca = &P.cam_attrs[MMBA_CAM_NUM_ATTRS * c];
    const double w = attr_get(P, ca[MMBA_CAM_FILM_BACK_W_INCH], f, 36.0 / 25.4, ov);
    const double h = attr_get(P, ca[MMBA_CAM_FILM_BACK_H_INCH], f, 24.0 / 25.4, ov);
    const double ox = attr_get(P, ca[MMBA_CAM_FILM_OFFSET_X_INCH], f, 0., ov);
    const double oy = attr_get(P, ca[MMBA_CAM_FILM_OFFSET_Y_INCH], f, 0., ov);
    const double focal = attr_get(P, ca[MMBA_CAM_FOCAL_MM], f, 35.0, ov);
    const double far_clip = attr_get(P, ca[MMBA_CAM_FAR_CLIP], f, 10000.0, ov);
    const double cscale = attr_get(P, ca[MMBA_CAM_SCALE], f, 1.0, ov);
    double W[16];
    world_matrix(P, P.cam_tfm[c], f, ov, W);
    camera_record_tail(P, c, w, h, ox, oy, focal, far_clip, cscale, W, rec);
}

// Same record for a camera transform without parent, gathered through the
// plan's per-camera-frame table of attribute-value indices
// (P.cf_aidx[17 cf + k]: 7 camera attributes, then tx ty tz rx ry rz sx sy sz;
// -1 = default): one dependent load level instead of the attribute-table walk.
// ov_idx is the perturbed attribute's value index (-1: none).
MMBA_DEV void camera_record_fast(const DevProblem &P, int cf, long long ov_idx, double ov_val,
                                 double *rec, int ov_attr = -1) {
    const int *ix = &P.cf_aidx[(size_t)CF_AIDX * cf];
    const double dflt[CF_AIDX] = {36.0 / 25.4, 24.0 / 25.4, 0., 0., 35.0, 10000.0, 1.0,
                                  0., 0., 0., 0., 0., 0., 1., 1., 1.};
    double v[CF_AIDX];
#pragma unroll
    for (int k = 0; k < CF_AIDX; ++k) {
        const int a = ix[k];
        v[k] = a < 0 ? dflt[k] : (a == ov_idx ? ov_val : P.attr_val[a]);
    }
    const int c = P.cf_cam[cf];
    double W[16];
    trs_matrix(v[7], v[8], v[9], v[10], v[11], v[12], v[13], v[14], v[15],
               P.tfm_roo[P.cam_tfm[c]], W);
    // a parented camera (the table exists for them in rolling-shutter plans):
    // world = parent world x local, world_matrix's order (ov_attr: the
    // overridden attribute, for a parent attribute's column)
    const int pt = P.tfm_parent[P.cam_tfm[c]];
    if (pt >= 0) {
        double Wp[16];
        world_matrix(P, pt, P.cf_frame[cf], Override{ov_attr, ov_val}, Wp);
        mat4_mul(Wp, W, W);
    }
    camera_record_tail(P, c, v[0], v[1], v[2], v[3], v[4], v[5], v[6], W, rec);
}

// Rolling shutter (mmba.h ABI 3): the camera-frame record as an observation
// at scanline time tau sees it -- the transform's translate / rotate values
// replaced by the 3DE exporter's three-frame blend (uvtrack_format.py:186-203,
// end frames extrapolated as at :311-314; the operations of oracle/refcpu.c
// rs_blend).  The override (ov_idx, ov_val) applies to every value read, the
// neighbouring frames' included.
// The same record for the FD columns of one observation, cheaper per column:
// RsCam holds what every column shares (the camera attribute values at the
// frame and their projection part, the translate / rotate values at f - 1, f,
// f + 1 with their value indices); rs_record then forms a column's record
// from the overridden values with the rigid inverse of T R S (the 3 x 3 block
// inverted as S^-1 R^T, the translation as -S^-1 R^T t) and only the non-zero
// entries of the projection (rows 0, 1, 3 of P C^-1).  Equal to
// camera_record_fast's arithmetic up to roundoff: the reference's general
// 4 x 4 inverse (oracle/refcpu.c) rounds differently, so RS residuals match
// the oracle to ~1e-15 relative, not bit for bit.
struct RsCam {
    int c, roo;
    int ptf, f;             // parent transform (-1: none) and the camera-frame's frame
    int ix[7];              // value indices of the 7 camera attributes (-1: default)
    int tx[6], px[6], nx[6];  // translate / rotate value indices at f, f - 1, f + 1
    double cam[7];          // camera attribute values
    double v[6][3];         // translate / rotate values at f - 1, f, f + 1 (raw)
    double s[3];            // scale at f
    double p00, p02, p11, p12, p32, sx, sy;  // projection part of the base record
};

MMBA_DEV void rs_proj(const DevProblem &P, int c, const double *cv, double &p00, double &p02,
                      double &p11, double &p12, double &p32, double &sx, double &sy) {
    double fbw, fbh, offx, offy, fa;
    if (P.mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        double w_mm = cv[0] * 25.4, h_mm = cv[1] * 25.4;
        fbw = w_mm * MM_TO_INCH;
        fbh = h_mm * MM_TO_INCH;
        offx = (cv[2] * 25.4) * MM_TO_INCH;
        offy = (cv[3] * 25.4) * MM_TO_INCH;
        fa = w_mm / h_mm;
    } else {
        fbw = cv[0];
        fbh = cv[1];
        offx = cv[2];
        offy = cv[3];
        fa = cv[0] / cv[1];
    }
    const double iw = (double)P.cam_size[2 * c], ih = (double)P.cam_size[2 * c + 1];
    double Pm[16];
    const int fit = P.cam_fit[c];
    projection_matrix(P.mode, cv[4], fbw, fbh, offx, offy, iw, ih, fit, cv[5], cv[6], Pm);
    p00 = Pm[0];
    p02 = Pm[2];
    p11 = Pm[5];
    p12 = Pm[6];
    p32 = Pm[14];
    const double ra = iw / ih;
    sx = 1.0;
    sy = 1.0;
    switch (fit) {
        case MMBA_FILM_FIT_HORIZONTAL: sy = ra / fa; break;
        case MMBA_FILM_FIT_VERTICAL: sx = 1.0 / (ra / fa); break;
        case MMBA_FILM_FIT_FILL:
            if (fa > ra) sx = fa / ra; else sy = ra / fa;
            break;
        case MMBA_FILM_FIT_OVERSCAN:
            if (fa > ra) sy = ra / fa; else sx = fa / ra;
            break;
        default: break;
    }
}

MMBA_DEV void rs_cam_load(const DevProblem &P, int cf, RsCam &R) {
    const int *ix = &P.cf_aidx[(size_t)CF_AIDX * cf];
    const int *nb = &P.cf_rs_vidx[(size_t)12 * cf];
    const double dflt[CF_AIDX] = {36.0 / 25.4, 24.0 / 25.4, 0., 0., 35.0, 10000.0, 1.0,
                                  0., 0., 0., 0., 0., 0., 1., 1., 1.};
    R.c = P.cf_cam[cf];
    R.roo = P.tfm_roo[P.cam_tfm[R.c]];
    R.ptf = P.tfm_parent[P.cam_tfm[R.c]];
    R.f = P.cf_frame[cf];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        R.ix[k] = ix[k];
        R.cam[k] = ix[k] < 0 ? dflt[k] : P.attr_val[ix[k]];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        R.tx[k] = ix[7 + k];
        R.px[k] = nb[k];
        R.nx[k] = nb[6 + k];
        R.v[k][1] = ix[7 + k] < 0 ? 0. : P.attr_val[ix[7 + k]];
        R.v[k][0] = nb[k] >= 0 ? P.attr_val[nb[k]] : 0.;
        R.v[k][2] = nb[6 + k] >= 0 ? P.attr_val[nb[6 + k]] : 0.;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) R.s[k] = ix[13 + k] < 0 ? 1. : P.attr_val[ix[13 + k]];
    rs_proj(P, R.c, R.cam, R.p00, R.p02, R.p11, R.p12, R.p32, R.sx, R.sy);
}

MMBA_DEV void rs_record(const DevProblem &P, const RsCam &R, double tau, long long ov_idx,
                        double ov_val, double *rec, int ov_attr = -1) {
    // projection part: recomputed only when a camera attribute is the override
    double p00 = R.p00, p02 = R.p02, p11 = R.p11, p12 = R.p12, p32 = R.p32, sx = R.sx, sy = R.sy;
    bool cam_ov = false;
#pragma unroll
    for (int k = 0; k < 7; ++k) cam_ov |= R.ix[k] >= 0 && R.ix[k] == ov_idx;
    if (cam_ov) {
        double cv[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) cv[k] = (R.ix[k] >= 0 && R.ix[k] == ov_idx) ? ov_val : R.cam[k];
        rs_proj(P, R.c, cv, p00, p02, p11, p12, p32, sx, sy);
    }
    // blended translate / rotate (rs_blend of oracle/refcpu.c)
    double b6[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double cv = (R.tx[k] >= 0 && R.tx[k] == ov_idx) ? ov_val : R.v[k][1];
        double pv = (R.px[k] >= 0 && R.px[k] == ov_idx) ? ov_val : R.v[k][0];
        double nv = (R.nx[k] >= 0 && R.nx[k] == ov_idx) ? ov_val : R.v[k][2];
        if (R.px[k] == -2) pv = cv + (cv - nv);
        if (R.nx[k] == -2) nv = cv + (cv - pv);
        const double b = (nv - pv) / 2.0;
        const double c = -cv + ((nv + pv) / 2.0);
        b6[k] = (cv + tau * b) + (tau * tau) * c;
    }
    double W[16];
    trs_matrix(b6[0], b6[1], b6[2], b6[3], b6[4], b6[5], R.s[0], R.s[1], R.s[2], R.roo, W);
    double Ci[16];
    if (R.ptf >= 0) {
        // a parented camera: the blend moves the camera's own translate /
        // rotate only; world = parent world at the frame (unblended; the
        // override reaches a parent attribute's column) x blended local, as
        // oracle/refcpu.c rs_camera_world, and the general inverse
        double Wp[16];
        world_matrix(P, R.ptf, R.f, Override{ov_attr, ov_val}, Wp);
        mat4_mul(Wp, W, W);
        mat4_inverse(W, Ci);
    } else {
        // C^-1 of W = T R S: rows k = (R S)^-1 = S^-1 R^T, column 3 = -S^-1 R^T t
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int r = 0; r < 3; ++r) Ci[k * 4 + r] = (W[r * 4 + k] / R.s[k]) / R.s[k];
            Ci[k * 4 + 3] = -(Ci[k * 4 + 0] * W[3] + Ci[k * 4 + 1] * W[7] + Ci[k * 4 + 2] * W[11]);
        }
    }
    // rows 0, 1, 3 of P C^-1 (P: p00 / p02 in row 0, p11 / p12 in row 1, p32
    // in row 3; row 3 of C^-1 is 0 0 0 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        rec[k] = p00 * Ci[k] + p02 * Ci[8 + k];
        rec[4 + k] = p11 * Ci[4 + k] + p12 * Ci[8 + k];
        rec[8 + k] = p32 * Ci[8 + k];
    }
    rec[12] = W[3];
    rec[13] = W[7];
    rec[14] = W[11];
    const double cdir[3] = {-W[2], -W[6], -W[10]};
    const double cl = sqrt(cdir[0] * cdir[0] + cdir[1] * cdir[1] + cdir[2] * cdir[2]);
    rec[15] = cdir[0] / cl;
    rec[16] = cdir[1] / cl;
    rec[17] = cdir[2] / cl;
    rec[18] = sx;
    rec[19] = sy;
}

// One observation's record at scanline time tau (residual / reprojection
// kernels): the same arithmetic as the FD columns of k_jacobian_rs, so fvec
// and the Jacobian's base point agree bit for bit.
MMBA_DEV void camera_record_rs(const DevProblem &P, int cf, double tau, long long ov_idx,
                               double ov_val, double *rec) {
    RsCam R;
    rs_cam_load(P, cf, R);
    rs_record(P, R, tau, ov_idx, ov_val, rec);
}

// ---- LDPK classic 3DE model (undistort polynomial + fixed-point inverse) ----
MMBA_DEV void lens_eval(const double *c, double px, double py, double &qx, double &qy) {
    const double ld = c[0], sq = c[1], cx = c[2], cy = c[3], qu = c[4];
    const double cxx = ld / sq, cxy = (ld + cx) / sq, cyx = ld + cy, cyy = ld;
    const double cxxx = qu / sq, cxxy = 2.0 * qu / sq, cxyy = qu / sq;
    const double cyxx = qu, cyyx = 2.0 * qu, cyyy = qu;
    double p0_2 = px * px, p1_2 = py * py;
    double p0_4 = p0_2 * p0_2, p1_4 = p1_2 * p1_2, p01_2 = p0_2 * p1_2;
    qx = px * (1 + cxx * p0_2 + cxy * p1_2 + cxxx * p0_4 + cxxy * p01_2 + cxyy * p1_4);
    qy = py * (1 + cyx * p0_2 + cyy * p1_2 + cyxx * p0_4 + cyyx * p01_2 + cyyy * p1_4);
}

// ---- LDPK radial decentered deg 4 + cylindric extender (3DE radial std
// deg 4; mmlens distortion_structs.h:108-150; ldpk_radial_decentered_
// distortion.h operator(), ldpk_cylindric_extender.h cylindric_extender_2)
// c: c2 u2 v2 c4 u4 v4 phi(degrees) b ----
MMBA_DEV void radial_eval(const double *c, double x, double y, double &qx, double &qy) {
    const double c2 = c[0], u2 = c[1], v2 = c[2], c4 = c[3], u4 = c[4], v4 = c[5];
    double x2 = x * x;
    double y2 = y * y;
    double xy = x * y;
    double r2 = x2 + y2;
    double r4 = r2 * r2;
    qx = x * (1.0 + c2 * r2 + c4 * r4) + (r2 + 2.0 * x2) * (u2 + u4 * r2) +
         2.0 * xy * (v2 + v4 * r2);
    qy = y * (1.0 + c2 * r2 + c4 * r4) + (r2 + 2.0 * y2) * (v2 + v4 * r2) +
         2.0 * xy * (u2 + u4 * r2);
}

// ---- LDPK anamorphic deg 4 (degree-4 specialisation of
// ldpk_generic_anamorphic_distortion.h: prepare() + operator()) ----
// c: cx02 cy02 cx22 cy22 cx04 cy04 cx24 cy24 cx44 cy44 rot(deg) sqx sqy rescale
MMBA_DEV void anam_eval(const double *c, double x, double y, double &qx, double &qy) {
    const double cx02 = c[0], cy02 = c[1], cx22 = c[2], cy22 = c[3], cx04 = c[4],
                 cy04 = c[5], cx24 = c[6], cy24 = c[7], cx44 = c[8], cy44 = c[9];
    double cx_x2 = cx02 + cx22, cx_y2 = cx02 - cx22, cx_x4 = cx04 + cx24 + cx44;
    double cx_x2y2 = 2.0 * cx04 - 6.0 * cx44, cx_y4 = cx04 - cx24 + cx44;
    double cy_x2 = cy02 + cy22, cy_y2 = cy02 - cy22, cy_x4 = cy04 + cy24 + cy44;
    double cy_x2y2 = 2.0 * cy04 - 6.0 * cy44, cy_y4 = cy04 - cy24 + cy44;
    double x2 = x * x, x4 = x2 * x2;
    double y2 = y * y, y4 = y2 * y2;
    qx = x * (1.0 + x2 * cx_x2 + y2 * cx_y2 + x4 * cx_x4 + x2 * y2 * cx_x2y2 + y4 * cx_y4);
    qy = y * (1.0 + x2 * cy_x2 + y2 * cy_y2 + x4 * cy_x4 + x2 * y2 * cy_x2y2 + y4 * cy_y4);
}

struct Mat2 {
    double a00, a01, a10, a11;
};
// LDPK mat2d product and inverse (ldpk_vec2d.h: row-major, invert = adj / det)
MMBA_DEV Mat2 m2_mul(const Mat2 &t, const Mat2 &a) {
    return Mat2{t.a00 * a.a00 + t.a01 * a.a10, t.a00 * a.a01 + t.a01 * a.a11,
                t.a10 * a.a00 + t.a11 * a.a10, t.a10 * a.a01 + t.a11 * a.a11};
}
MMBA_DEV Mat2 m2_inv(const Mat2 &a) {
    const double det = a.a00 * a.a11 - a.a01 * a.a10;
    return Mat2{a.a11 / det, -a.a01 / det, -a.a10 / det, a.a00 / det};
}

// p <- q - (f(q) - q), then p <- p + q - f(p): <= 20 iterations until
// ||f(p) - q|| < 1e-6, then 2 more (ldpk_generic_distortion_base.h map_inverse)
template <typename EVAL>
MMBA_DEV void fixed_point_inverse(EVAL f, double qx, double qy, double &px, double &py) {
    double fx, fy;
    f(qx, qy, fx, fy);
    px = qx - (fx - qx);
    py = qy - (fy - qy);
    for (int i = 0; i < 20; ++i) {
        double ix, iy;
        f(px, py, ix, iy);
        px = px + qx - ix;
        py = py + qy - iy;
        double dx = ix - qx, dy = iy - qy;
        if (sqrt(dx * dx + dy * dy) < 1e-6) break;
    }
    for (int i = 0; i < 2; ++i) {
        double ix, iy;
        f(px, py, ix, iy);
        px = px + qx - ix;
        py = py + qy - iy;
    }
}

// LT >= 0: the caller knows every lens it passes is of model LT (the plan's
// lens_uniform), so only that model's code is compiled in -- the generic
// form holds every model's inverse and their registers at once (C5's
// k_jacobian spilled 288 B per lane with it, round 6).
template <int LT = -1>
MMBA_DEV void lens_distort(int type, const double *coeff, double x, double y, double &ox,
                           double &oy) {
    if constexpr (LT >= 0) type = LT;
    const double w = 3.6, h = 2.4;  // LensModel defaults (lens_model.h:42)
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double qx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double qy = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    double px, py;
    if (type == MMBA_LENS_3DE_RADIAL_STD_DEG4) {
        // cylindric^-1 (invert(_m) * q, calc_m with M_PI), then the radial inverse
        const double pi = 3.14159265358979323846;
        const double phi = coeff[6], b = coeff[7];
        double q = sqrt(1.0 + b), cs = cos(phi * pi / 180.0), sn = sin(phi * pi / 180.0);
        const double m00 = cs * cs * q + sn * sn / q, m01 = (q - 1.0 / q) * cs * sn;
        const double m10 = (q - 1.0 / q) * cs * sn, m11 = cs * cs / q + sn * sn * q;
        const double det = m00 * m11 - m01 * m10;
        const double i00 = m11 / det, i01 = -m01 / det, i10 = -m10 / det, i11 = m00 / det;
        const double tx = i00 * qx + i01 * qy, ty = i10 * qx + i11 * qy;
        fixed_point_inverse(
            [&](double a, double bb, double &fa, double &fb) { radial_eval(coeff, a, bb, fa, fb); },
            tx, ty, px, py);
    } else if (type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4 ||
               type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED) {
        // PAR * anamorphic^-1(RSP^-1 q): RSP = R Sx Sy Rs PA, PAR = PA Rs R
        // (linear_extender::set, left-to-right products; PA = pixel aspect 1,
        // Rs = identity for the non-rescaled model: both leave products exact)
        const double pi = 3.14159265358979323846;
        const double phi = coeff[10] / 180.0 * pi;
        const Mat2 R{cos(phi), -sin(phi), sin(phi), cos(phi)};
        const Mat2 Sx{coeff[11], 0.0, 0.0, 1.0}, Sy{1.0, 0.0, 0.0, coeff[12]};
        const Mat2 Rs{coeff[13], 0.0, 0.0, 1.0}, PA{1.0, 0.0, 0.0, 1.0};
        const Mat2 rsp = m2_mul(m2_mul(m2_mul(m2_mul(R, Sx), Sy), Rs), PA);
        const Mat2 par = m2_mul(m2_mul(PA, Rs), R);
        const Mat2 ri = m2_inv(rsp);
        const double tx = ri.a00 * qx + ri.a01 * qy, ty = ri.a10 * qx + ri.a11 * qy;
        double ax, ay;
        fixed_point_inverse(
            [&](double a, double bb, double &fa, double &fb) { anam_eval(coeff, a, bb, fa, fb); },
            tx, ty, ax, ay);
        px = par.a00 * ax + par.a01 * ay;
        py = par.a10 * ax + par.a11 * ay;
    } else {
        fixed_point_inverse(
            [&](double a, double bb, double &fa, double &fb) { lens_eval(coeff, a, bb, fa, fb); },
            qx, qy, px, py);
    }
    double cxm = px * r + ((w / 2) + 0.0);
    double cym = py * r + ((h / 2) + 0.0);
    ox = cxm / w - 0.5;
    oy = cym / h - 0.5;
}

struct Resid {
    double ex, ey;    // weighted errors (fvec)
    double ux, uy;    // user deviation (errorList)
    double dist;      // errorDistanceList
};

// Reprojected point of a bundle position through a camera record
// (reprojection.rs:28-63: P C^-1 b, / w, x 0.5), before the lens.
MMBA_DEV void project_point(const double *rec, const double *bp, double &point_x,
                            double &point_y) {
    double sp0 = rec[0] * bp[0] + rec[1] * bp[1] + rec[2] * bp[2] + rec[3];
    double sp1 = rec[4] * bp[0] + rec[5] * bp[1] + rec[6] * bp[2] + rec[7];
    double sp3 = rec[8] * bp[0] + rec[9] * bp[1] + rec[10] * bp[2] + rec[11];
    point_x = (sp0 / sp3) * 0.5;
    point_y = (sp1 / sp3) * 0.5;
}

// Lens distortion of a reprojected point; a non-finite result keeps the
// undistorted coordinate (adjust_measureErrors.cpp:466-472).  chain: the
// lens's constant input layers, deepest first (mmba.h ABI 5), applied before
// the lens itself with no check between layers (each model's
// applyModelDistort runs its input's first, lens_model_3de_classic.cpp:82-88).
template <int LT = -1>
MMBA_DEV void distort_point(int lens_type, const double *lens, double &point_x,
                            double &point_y, const double *chain = nullptr, int nchain = 0) {
    if (lens_type != MMBA_LENS_NONE) {
        double ox, oy, ix = point_x, iy = point_y;
        for (int k = 0; k < nchain; ++k) {
            const double *ly = chain + (size_t)k * LENS_LAYER;
            lens_distort((int)ly[0], ly + 1, ix, iy, ix, iy);
        }
        lens_distort<LT>(lens_type, lens, ix, iy, ox, oy);
        if (isfinite(ox)) point_x = ox;
        if (isfinite(oy)) point_y = oy;
    }
}

// One observation's residual from a camera record and a bundle position.
template <int LT = -1>
MMBA_DEV Resid residual(const double *rec, const double *bp, double mkr_x, double mkr_y,
                        double sqrtw, int mode, double image_width, int lens_type,
                        const double *lens, const double *chain = nullptr, int nchain = 0) {
    double point_x, point_y;
    project_point(rec, bp, point_x, point_y);
    mkr_x *= rec[18];
    mkr_y *= rec[19];
    double factor = 1.0;
    if (mode != MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        double bd0 = bp[0] - rec[12], bd1 = bp[1] - rec[13], bd2 = bp[2] - rec[14];
        double bl = sqrt(bd0 * bd0 + bd1 * bd1 + bd2 * bd2);
        double dot = rec[15] * (bd0 / bl) + rec[16] * (bd1 / bl) + rec[17] * (bd2 / bl);
        if (dot < 0.0) factor = 1e+6;
    }
    distort_point<LT>(lens_type, lens, point_x, point_y, chain, nchain);
    double dx = fabs(mkr_x - point_x), dy = fabs(mkr_y - point_y);
    double dxp = dx * image_width, dyp = dy * image_width;
    Resid r;
    r.ex = dxp * sqrtw * factor;
    r.ey = dyp * sqrtw * factor;
    r.ux = dxp * factor;
    r.uy = dyp * factor;
    r.dist = sqrt((dx * dx) + (dy * dy)) * image_width;
    return r;
}

// The weighted errors of residual() only (same operations): the FD
// columns that do not leave errorList / errorDistanceList behind need no
// distance (one square root fewer per perturbed evaluation).
MMBA_DEV double2 residual_e(const double *rec, const double *bp, double mkr_x, double mkr_y,
                            double sqrtw, int mode, double image_width) {
    double point_x, point_y;
    project_point(rec, bp, point_x, point_y);
    mkr_x *= rec[18];
    mkr_y *= rec[19];
    double factor = 1.0;
    if (mode != MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        double bd0 = bp[0] - rec[12], bd1 = bp[1] - rec[13], bd2 = bp[2] - rec[14];
        double bl = sqrt(bd0 * bd0 + bd1 * bd1 + bd2 * bd2);
        double dot = rec[15] * (bd0 / bl) + rec[16] * (bd1 / bl) + rec[17] * (bd2 / bl);
        if (dot < 0.0) factor = 1e+6;
    }
    double dx = fabs(mkr_x - point_x), dy = fabs(mkr_y - point_y);
    double dxp = dx * image_width, dyp = dy * image_width;
    return make_double2(dxp * sqrtw * factor, dyp * sqrtw * factor);
}

// applyLossFunctionToErrors for one row (adjust_base.cpp:158-187), same
// operation order as the reference (pow, log1p).
MMBA_DEV double robust_loss(double f, int type, double scale) {
    double z = pow(f / scale, 2);
    double rho0 = z, rho1 = 1.0, rho2 = 0.0;
    if (type == MMBA_ROBUST_LOSS_SOFT_L_ONE) {
        double t = 1.0 + z;
        rho0 = 2.0 * (pow(t, 0.5 - 1.0));
        rho1 = pow(t, -0.5);
        rho2 = -0.5 * pow(t, -1.5);
    } else if (type == MMBA_ROBUST_LOSS_CAUCHY) {
        rho0 = log1p(z);
        double t = 1.0 + z;
        rho1 = 1.0 / t;
        rho2 = -1.0 / pow(t, 2.0);
    }
    (void)rho0;
    rho2 /= pow(scale, 2.0);
    double J_scale = rho1 + 2.0 * rho2 * pow(f, 2.0);
    const double eps = 2.220446049250313080847e-16;
    if (J_scale < eps) J_scale = eps;
    J_scale = pow(J_scale, 0.5);
    return f * (rho1 / J_scale);
}

// residual() with the robust loss applied to the weighted rows when the
// solver applies one (fvec only: errorList / errorDistanceList are unscaled).
template <int LT = -1>
MMBA_DEV Resid residual_l(const DevProblem &P, const double *rec, const double *bp, double mkr_x,
                          double mkr_y, double sqrtw, int lens_type, const double *lens) {
    Resid r = residual<LT>(rec, bp, mkr_x, mkr_y, sqrtw, P.mode, P.image_width, lens_type, lens,
                           P.lens_chain, P.lens_chain_n);
    if (P.loss_on) {
        r.ex = robust_loss(r.ex, P.loss_type, P.loss_scale);
        r.ey = robust_loss(r.ey, P.loss_type, P.loss_scale);
    }
    return r;
}

MMBA_DEV void lens_coeffs(const DevProblem &P, int lens, int f, const Override &ov,
                          double *c) {
    const int *la = &P.lens_attrs[MMBA_LENS_NUM_ATTRS * lens];
    const int type = P.lens_type[lens];
    const bool classic = type == MMBA_LENS_3DE_CLASSIC;
    const bool anam = type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4 ||
                      type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED;
    // absent slots take the model default (mmba.h): classic squeeze,
    // anamorphic squeeze x / y and rescale are 1, the rest 0
#pragma unroll
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k)
        c[k] = attr_get(P, la[k], f, ((classic && k == 1) || (anam && k >= 11)) ? 1. : 0., ov);
    if (type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4) c[13] = 1.;  // no rescale slot
}

// Box-constraint reparametrisation (adjust_base.cpp:194-220); the clamps
// keep std::max / std::min argument order (adjust_base.cpp:202-203,217-218).
__host__ __device__ inline double int_to_ext(double value, double xmin, double xmax,
                                             double offset, double scale) {
    const double float_max = 3.40282346638528859811704183484516925440e+38;
    if ((xmin <= -float_max) && (xmax >= float_max)) {
        value = (value / scale) - offset;
        value = (value < xmin) ? xmin : value;  // std::max<double>: NaN passes
        value = (xmax < value) ? xmax : value;  // std::min<double>
        return value;
    } else if (xmax >= float_max) {
        value = xmin - (1.0 + sqrt(value * value + 1.0));
    } else if (xmin <= -float_max) {
        value = xmax + (1.0 - sqrt(value * value + 1.0));
    } else {
        value = xmin + ((xmax - xmin) / 2.0) * (sin(value) + 1.0);
    }
    value = (value / scale) - offset;
    value = (value < xmin) ? xmin : value;
    value = (xmax < value) ? xmax : value;
    return value;
}

// Forward-difference point of one FD column at internal value v: lmder
// perturbs by +-delta and multiplies by inv_delta (adjust_solveFunc.cpp:
// 148-180, 395-402); lmdif's fdjac2 uses h = eps_dif |v| (eps_dif when v is
// 0) and divides.  Returns v + step, *step = inv_delta (lmder) or h (lmdif).
MMBA_DEV double fd_point(double v, double xmin, double xmax, int solver_type, double delta,
                         double eps_dif, double &step) {
    if (solver_type == MMBA_SOLVER_CMINPACK_LMDER) {
        double sign = 1.0;
        if ((v + delta) > xmax) sign = -1;
        if ((v - delta) < xmin) sign = 1;
        const double d = delta * sign;
        step = 1.0 / d;
        return v + d;
    }
    double h = eps_dif * fabs(v);
    if (h == 0.) h = eps_dif;
    step = h;
    return v + h;
}

// Lane-level helpers of the one-wave factorisations (mmba_bdiag.hip,
// mmba_batch.hip): fp64 rsqrt refined twice, v_readlane of a double.
MMBA_DEV double wave_rsq(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

MMBA_DEV double wave_rdlane(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// Unperturbed bundle position of observation (b, frame f): the bundle record
// of a fast bundle, else the transform chain.
MMBA_DEV void base_bundle(const DevProblem &P, int b, int f, double *bp) {
    if (P.bnd_p4[b].w >= 0) {
        const double *br = &P.brec[(size_t)b * BREC];
        bp[0] = br[0];
        bp[1] = br[1];
        bp[2] = br[2];
    } else {
        const Override none{-1, 0.};
        bundle_position(P, b, f, none, bp);
    }
}

// Lens model type of the camera's lens (MMBA_LENS_*), 0 without one.
MMBA_DEV int obs_lens(const DevProblem &P, int cam, int &lens) {
    if (!P.cam_lens) return MMBA_LENS_NONE;
    lens = P.cam_lens[cam];
    return lens >= 0 ? P.lens_type[lens] : MMBA_LENS_NONE;
}

// Lens model type of observation i's lens instance (mmba.h ABI 7: the
// instance markerFrameToLensModelList[markerIndex + frameIndex] names), 0
// without one.
MMBA_DEV int obs_lens_inst(const DevProblem &P, int i, int &inst) {
    if (!P.obs_inst) return MMBA_LENS_NONE;
    inst = P.obs_inst[i];
    return inst >= 0 ? P.lens_type[P.inst_lens[inst]] : MMBA_LENS_NONE;
}

// The coefficients lens instance `inst` holds (absent slots: the plug
// model's value, which is the model default for a slot without attribute).
MMBA_DEV void inst_coeffs(const DevProblem &P, int inst, const Override &ov, double *c) {
    const int *ia = &P.inst_attr[MMBA_LENS_NUM_ATTRS * inst];
    const int *fa = &P.inst_frame[MMBA_LENS_NUM_ATTRS * inst];
    const double *va = &P.inst_val[MMBA_LENS_NUM_ATTRS * inst];
#pragma unroll
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k)
        c[k] = ia[k] < 0 ? va[k] : attr_get(P, ia[k], fa[k], 0., ov);
    if (P.lens_type[P.inst_lens[inst]] == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4) c[13] = 1.;  // no rescale slot
}

}  // namespace mmba
