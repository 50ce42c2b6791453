/*
 * refcpu.h -- CPU restatement of mmSolver's LM bundle-adjustment hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the shipped product links or calls
 * this; it is the parity checker for tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py.
 *
 * It restates (file:line in the reference, bpatchasaheb/mayaMatchMoveSolver):
 *   - MM Scene Graph evaluation: lib/rust/mmscenegraph/src/scene/flat.rs:172-358,
 *     math/dag.rs:36-327, math/transform.rs:338-452, math/camera.rs:153-327,
 *     math/reprojection.rs:28-63
 *   - Maya DAG projection: src/mmSolver/mayahelper/maya_camera.cpp:75-414,863-894
 *   - residuals: src/mmSolver/adjust/adjust_measureErrors.cpp:118-309 (DAG),
 *     :392-521 (MMSG)
 *   - FD Jacobian: src/mmSolver/adjust/adjust_solveFunc.cpp:148-525
 *   - bound transforms: src/mmSolver/adjust/adjust_base.cpp:194-258
 *   - lens distort (3DE classic): lib/cppbind/mmlens/src/lens_model_3de_classic.cpp:75-113,
 *     distortion_operations.h:34-96, include/mmlens/lib.h:36-75 and the LDPK 2.8
 *     classic model / generic fixed-point inverse (text of the vendored headers)
 *   - LM: MINPACK-1 lmder/lmdif/lmpar/qrfac/qrsolv/enorm/fdjac2 as used through
 *     cminpack 1.3.8 (third-party, not vendored; call sites
 *     adjust_cminpack_lmder.cpp:94-184, adjust_cminpack_lmdif.cpp:95-189).
 *
 * Pinning: MINPACK restatement checked against scipy.optimize._minpack
 * (scipy 1.15.3) on identical callbacks; geometry checked against the Rust
 * unit-test golden values; full solves against the Maya test known answers
 * (see tests/test_oracle_*.py).
 */
#ifndef MMBA_REFCPU_H
#define MMBA_REFCPU_H

#include "../include/mmba.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- MINPACK restatement ---- */
typedef int (*ref_fcn_der)(void *p, int m, int n, const double *x,
                           double *fvec, double *fjac, int ldfjac, int iflag);
typedef int (*ref_fcn_dif)(void *p, int m, int n, const double *x,
                           double *fvec, int iflag);

double ref_enorm(int n, const double *x);
int ref_lmder(ref_fcn_der fcn, void *p, int m, int n, double *x, double *fvec,
              double *fjac, int ldfjac, double ftol, double xtol, double gtol,
              int maxfev, double *diag, int mode, double factor, int nprint,
              int *nfev, int *njev, int *ipvt, double *qtf, double *wa1,
              double *wa2, double *wa3, double *wa4);
int ref_lmdif(ref_fcn_dif fcn, void *p, int m, int n, double *x, double *fvec,
              double ftol, double xtol, double gtol, int maxfev, double epsfcn,
              double *diag, int mode, double factor, int nprint, int *nfev,
              double *fjac, int ldfjac, int *ipvt, double *qtf, double *wa1,
              double *wa2, double *wa3, double *wa4);

/* ---- geometry hooks (row-major 4x4, column-vector convention p' = M p) ---- */
void ref_trs_matrix(double tx, double ty, double tz, double rx, double ry,
                    double rz, double sx, double sy, double sz, int roo,
                    double out[16]);
void ref_projection_matrix(int scene_graph_mode, double focal_mm,
                           double fbw_inch, double fbh_inch, double offx_inch,
                           double offy_inch, double image_w, double image_h,
                           int film_fit, double far_clip, double camera_scale,
                           double out[16]);
void ref_reproject(const double cam_world[16], const double proj[16],
                   const double point[3], double out_xy[2]);
void ref_lens_3de_classic_distort(const double coeff[5], double x, double y,
                                  double *out_x, double *out_y);
void ref_lens_3de_classic_undistort(const double coeff[5], double x, double y,
                                    double *out_x, double *out_y);
/* 3DE radial decentered deg 4 cylindric: coeff = c2 u2 v2 c4 u4 v4 phi(deg) b */
void ref_lens_3de_radial_distort(const double coeff[8], double x, double y,
                                 double *out_x, double *out_y);
void ref_lens_3de_radial_undistort(const double coeff[8], double x, double y,
                                   double *out_x, double *out_y);
/* 3DE anamorphic deg 4 rotate squeeze xy (+ rescaled): coeff = cx02 cy02 cx22
 * cy22 cx04 cy04 cx24 cy24 cx44 cy44 rotation(deg) squeeze_x squeeze_y rescale
 * (rescale 1 for the non-rescaled model) */
void ref_lens_3de_anamorphic_distort(const double coeff[14], double x, double y,
                                     double *out_x, double *out_y);
void ref_lens_3de_anamorphic_undistort(const double coeff[14], double x, double y,
                                       double *out_x, double *out_y);

/* ---- full solve through the same mmba_problem layout ---- */
int ref_reproject_obs(const mmba_problem *prob, const mmba_options *opt, const double *x,
                      double *point_xy, double *marker_xy);
int ref_measure(const mmba_problem *prob, const mmba_options *opt,
                const double *x /* NULL = initial attr values */,
                double *fvec, double *err_user, double *err_dist,
                double *avg_min_max);
int ref_solve(const mmba_problem *prob, const mmba_options *opt,
              double *x_inout, double *fvec, double *err_user,
              double *err_dist, mmba_result *res, mmba_trace *trace);

/* Jacobian (m x n, column-major, ldfjac = m) of the reference FD scheme at x. */
int ref_jacobian(const mmba_problem *prob, const mmba_options *opt,
                 const double *x, double *fvec, double *fjac);

/* Test hook for the interrupt path (MComputation::isInterruptRequested): the
 * k-th poll (0-based) and every later one report an interrupt; k < 0 never. */
void ref_set_interrupt_after(int k);

double ref_param_external_to_internal(double value, double xmin, double xmax,
                                      double offset, double scale);
double ref_param_internal_to_external(double value, double xmin, double xmax,
                                      double offset, double scale);

#ifdef __cplusplus
}
#endif

#endif /* MMBA_REFCPU_H */
