// mmba_kernels.h -- host launch wrappers for the kernels in mmba_kernels.hip.
#pragma once

#include <vector>

#include "mmba_internal.h"

namespace mmba {

// threads per workgroup of k_ne_bnd_jb: one epilogue partial column per
// workgroup (the bundle columns of the reductions after the Jacobian)
constexpr int NE_BND_TPB = 64;

void launch_param_prep(hipStream_t s, const DevProblem &P, const double *x, double *ext,
                       double *ext_pert, double *step, int solver_type, double delta,
                       double eps_dif);
void launch_set_attrs(hipStream_t s, const DevProblem &P, const double *ext);
// launch_param_prep + launch_set_attrs in one launch
void launch_param_set(hipStream_t s, const DevProblem &P, const double *x, double *ext,
                      double *ext_pert, double *step, int solver_type, double delta,
                      double eps_dif);
// Partial rows -> scalar slots in one launch (row r: partial[off, off + n),
// sum or max, -> scalar[slot]); flag (nullable) -> scalar[flag_slot], cleared.
struct RedRow {
    int off, n, is_max, slot;
};
struct RedSpec {
    int nrows;
    int flag_slot;
    RedRow row[8];
};
// LmDec (mmba_internal.h): the decision after a trial point, restated on the device.
// host (optional): the last block copies scalar[0, host_n) into that
// page-locked mirror and then stores seq into *host_seq (system scope,
// release): the LM thread polls that word instead of a stream event.
void launch_reduce_multi(hipStream_t s, const double *partial, const RedSpec &spec,
                         double *scalar, int *flag = nullptr, double *host = nullptr,
                         int host_n = 0, unsigned *ticket = nullptr,
                         unsigned *host_seq = nullptr, unsigned seq = 0,
                         const LmDec &dec = LmDec());
// lmder bookkeeping after the normal equations (column norms, rank test, diag
// update, ||D x||, gnorm): partial rows 0 / 1 / 2 (rstride apart, nparts each)
void launch_jac_epilogue(hipStream_t s, const DevProblem &P, const double *Acc,
                         const double *Abb, const double *aggbuf, double *acnorm, double *g,
                         double *diag, const double *x, int first, int mode, double fnorm,
                         const double *fnorm_sq, int do_xn, int do_gn, const int *mask,
                         double *partial, int nparts, int rstride, const double *c15 = nullptr,
                         const double *s15 = nullptr, double *gfull = nullptr,
                         const double *adiag15 = nullptr, const double *u15 = nullptr);
// lmder trial point x - xs with setParameters at it; partial rows 0 (pnorm^2)
// and 1 (||D x_new||^2)
void launch_trial_prep(hipStream_t s, const DevProblem &P, const double *xs, const double *x,
                       const double *diag, double *wa1, double *wa2, double *wa3, double *ext,
                       double *ext_pert, double *step, int solver_type, double delta,
                       double eps_dif, const int *mask, double *partial, int nparts,
                       int rstride);
// Camera-frame records (variant 0 only when base_only) and bundle records,
// one launch.
void launch_records(hipStream_t s, const DevProblem &P, const int *var_cf,
                    const double *ext_pert, const double *step, double *recs, int nvar,
                    double *brec, int base_only);
int residual_blocks(const DevProblem &P);
// Partial count of the trial point's residual pass (launch_residual_jp):
// one per camera-frame where trial_cf_fusable, else residual_blocks.
bool &trial_cf_off();
bool trial_cf_fusable(const DevProblem &P);
int trial_blocks(const DevProblem &P);
// Reductions: with a ticket (a zero-initialised device counter) the partial
// sums are combined inside the same launch, otherwise by a second kernel.
void launch_reproject(hipStream_t s, const DevProblem &P, const double *recs, double *pts,
                      double *mkr);
void launch_residual(hipStream_t s, const DevProblem &P, const double *recs, double *f, double *eu,
                     double *ed, double *partial, double *out = nullptr,
                     unsigned int *ticket = nullptr, double *dist = nullptr);
// errorDistanceList statistics (compute_error_stats) of ed: out[0] = sum of
// the finite entries, out[1] = -min, out[2] = max (partial rows rstride apart)
void launch_dist_stats(hipStream_t s, const DevProblem &P, const double *ed, double *partial,
                       int nparts, int rstride, double *out);
// launch_residual (partials only) plus ||J p||^2 partials of the same blocks
// into partial_jp (k_jp_sumsq's sum, one launch)
// Reduction launch folded into a producer (unsharded trial point): the
// producer's last workgroup (ticket) runs k_reduce_multi's work -- the rows
// of spec (offsets into partial), the fail flag and the host mirror.
struct RedTail {
    int on = 0;
    RedSpec spec{};
    const double *partial = nullptr;
    double *scalar = nullptr;
    int *flag = nullptr;
    double *host = nullptr;
    int host_n = 0;
    unsigned *ticket = nullptr;
};
void launch_residual_jp(hipStream_t s, const DevProblem &P, const double *recs, double *f,
                        double *eu, double *ed, double *partial, const double *J,
                        const int *jcol, const int *nloc, const double *pstep,
                        double *partial_jp, double *dist = nullptr, const RedTail &T = RedTail());
// Second evaluation of central FD columns (lmder, autoDiffType central):
// records / bundle records / perturbed values at x + deltaB and the column
// factor 0.5 / (|dA| + |dB|) (0: forward column).  recs == nullptr: forward.
struct CentralB {
    const double *recs = nullptr, *brec = nullptr, *ext_pert = nullptr, *step = nullptr;
    // B15 (Plan::b15): camera-frame block columns stored in the basis Q_cf
    // (q15: ncf x PCMAX x PCMAX) less f kappa_cf on the first (kap15)
    const double *q15 = nullptr, *kap15 = nullptr;
};
// c15 (optional): c_p = 0.5 / (|dA| + |dB|) of animated central columns, else 0
void launch_param_central(hipStream_t s, const DevProblem &P, const double *x, double *ext_pertB,
                          double *stepB, double delta, double *count, double *c15 = nullptr);
// B15 rank-one Jacobian term J = J_s + f c^T (Plan::b15): s = ||f||^2 at the
// Jacobian's point (*fsq, or fn^2) -> *out
void launch_b15_s(hipStream_t s, const double *fsq, double fn, double *out);
// xs = (M + U B U^T)^-1 (u + s c) from z_u = M^-1 u, z_c = M^-1 c (Woodbury,
// U = [u c], B = [0 1; 1 s]); K^-1 -> kinv[0..3]; scalar[fail_slot] =
// max(itself, *fail_prev, singular K)
void launch_b15_combine(hipStream_t s, int n, const double *u, const double *c, const double *zu,
                        const double *zc, const double *sp, double *xs, double *kinv,
                        double *scalar, int fail_slot, const double *fail_prev);
// per camera-frame Householder basis Q (Q c_cf = kappa e_0) -> q15, kap15;
// c in that basis -> cr
void launch_b15_q(hipStream_t s, const DevProblem &P, const double *c, double *q15, double *kap15,
                  double *cr);
// out = Q x on camera-frame parameters (its own inverse), copy elsewhere
void launch_b15_rot(hipStream_t s, const DevProblem &P, const double *q15, const double *x,
                    double *out);
// AccL = Acc + lam Q D^2 Q per camera-frame block; diagL = diag, 0 on
// camera-frame parameters
void launch_b15_accl(hipStream_t s, const DevProblem &P, const double *Acc, const double *q15,
                     const double *diag, double lam, double *AccL, double *diagL);
// diag(Q A Q) -> adiag and Q g -> u on camera-frame parameters (g copied elsewhere)
void launch_b15_unrot(hipStream_t s, const DevProblem &P, const double *Acc, const double *g,
                      const double *q15, double *adiag, double *u);
void launch_b15_unrot_J(hipStream_t s, const DevProblem &P, double *J, const double *q15);
// ||D x||^2 -> *out (one workgroup, fixed order)
void launch_b15_dnorm(hipStream_t s, int n, const double *x, const double *diag, double *out);
// *out -= w^T K^-1 w, w = [z_u . v, z_c . v] (lmpar's v^T (A + lam D^2)^-1 v)
void launch_b15_newton(hipStream_t s, int n, const double *v, const double *zu, const double *zc,
                       const double *kinv, double *out);
// *out += 2 (c . xs)(u . xs) + s (c . xs)^2 (||J p||^2 of the rank-one term)
void launch_b15_jp(hipStream_t s, int n, const double *xs, const double *u, const double *c,
                   const double *sp, double *out);
void launch_jacobian(hipStream_t s, const DevProblem &P, const double *recs,
                     const double *ext_pert, const double *step, int solver_type, double *J,
                     int *jcol, int *nloc, const int *stale_param, double *eu, double *ed,
                     int ncv = 0,  // ncv 6 / 7: uniform fast kernels (Plan::jac_ncv)
                     const double *f = nullptr,  // residuals at x (column-parallel kernel)
                     const CentralB &CB = CentralB());
// Attribute stiffness / smoothness rows (mmba_rows.hip): fr / eur point at
// row 0 of the rows (f + 2M); partial[slot] gets the rows' sum of squares
// (slot = nblk(M, 256): the entry after the residual blocks).
void launch_rows_eval(hipStream_t s, const DevProblem &P, double *fr, double *eur,
                      double *partial, int slot, const double *Jrow = nullptr,
                      const double *pstep = nullptr, double *partial_jp = nullptr);
void launch_rows_jac(hipStream_t s, const DevProblem &P, const double *ext,
                     const double *ext_pert, const double *step, const double *ext_pertB,
                     const double *stepB, int lmder, double *Jrow, double *eur, int last_param);
void launch_rows_ne(hipStream_t s, const DevProblem &P, const double *Jrow, const double *fr,
                    const int *p_own, double *Acc, double *Abb, double *aggbuf, double *g);
// aggbuf = [Agg (NGMAX^2) | g_G (NGMAX)]: the global-parameter normal
// equations, all-reduced across shards before launch_colnorms.
// lmder's bookkeeping after the normal equations (k_jac_epilogue's column
// norms, rank test, diag update, ||D x||, gnorm) fused into the uniform
// normal-equation kernels: each camera-frame / bundle block writes one
// partial per quantity at column cf_base + cf / bnd_base + block of the rows
// partial[0 | rstride | 2 rstride] (max, sum, max).
constexpr int NE_CF_SPLIT = 4;  // workgroups per camera-frame of k_ne_cf_split
constexpr int NE_CF_NT = 36;    // partial sums per workgroup (PC <= 7: 28 + 7)
struct NeEpi {
    int on = 0;
    int first = 0, mode = 1, do_xn = 0, do_gn = 0;
    double fnorm = 0.;
    const double *fnorm_sq = nullptr;  // non-null: fnorm = sqrt(*fnorm_sq) (device slot)
    const double *x = nullptr;
    double *diag = nullptr, *acnorm = nullptr, *partial = nullptr;
    int rstride = 0, cf_base = 0, bnd_base = 0;
    // fold (unsharded k_ne_bnd_jb): the bundle pass's last workgroup (ticket)
    // reduces the epilogue rows of spec into scalar with k_reduce_multi's
    // arithmetic -- no separate reduction launch
    int fold = 0;
    RedSpec spec{};
    double *scalar = nullptr;
    unsigned *ticket = nullptr;
    // jb_recs != nullptr (MMBA_PATH_JB_RECOMPUTE, the fused path only): the
    // bundle pass re-evaluates each observation's three bundle columns and f
    // from the base camera record (jb_recs) and the bundle record -- the
    // arithmetic of jac_obs_u, so the same bits -- instead of reading the
    // 64-B JB record k_jac_ne_u would have written
    const double *jb_recs = nullptr;
    int jb_lmder = 1;
    // cf_part != nullptr (C2-like long segments, no global parameter): each
    // camera-frame's observations are split over NE_CF_SPLIT workgroups,
    // which store their partial sums write-through; the last of them (per
    // camera-frame ticket, monotonic) adds them in part order and writes
    // Acc / g and the epilogue (k_ne_cf_split)
    double *cf_part = nullptr;
    unsigned *cf_ticket = nullptr;
    // Lb != nullptr: the bundle pass also factors Abb at lam = 0
    // (k_bundle_factor's arithmetic) for the undamped solve that follows
    double *Lb = nullptr, *tb = nullptr;
    int *fail = nullptr;
    // gate != nullptr: the launch runs only when *gate != 0 (a Jacobian
    // enqueued ahead of the host's decision, LmDec)
    const int *gate = nullptr;
    // MMBA_PATH_PROBE = 2: k_jac_ne_u stores, per workgroup (logical
    // camera-frame), the wall clock at entry, after staging, after its
    // observations and at exit, and its XCC id
    long long *probe = nullptr;
};
// Fused K2 (k_jac_ne_u): FD Jacobian + camera-frame normal equations in one
// pass for uniform fast plans without global parameters (ncv = jac_ncv).
bool jac_ne_fusable(const DevProblem &P, int ncv);
void launch_jac_ne(hipStream_t s, const DevProblem &P, const double *recs, const double *step,
                   int solver_type, double *J, int *jcol, int *nloc, const int *stale_param,
                   double *eu, double *ed, double *Acc, double *g, const NeEpi &E);
// Whether launch_ne can fuse the bookkeeping (uniform camera blocks, fast
// bundles, no global parameters).
bool ne_epilogue_fusable(const DevProblem &P);
void launch_ne(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
               const int *nloc, const double *f, double *Acc, double *Acg, double *Abb,
               double *Abg, double *aggbuf, double *g, double *glob_partial, int glob_chunk,
               const NeEpi &epi = NeEpi(), bool cf_done = false);
void launch_colnorms(hipStream_t s, const DevProblem &P, const double *Acc, const double *Abb,
                     const double *aggbuf, double *acnorm, double *g);
void launch_bundle_factor(hipStream_t s, const DevProblem &P, const double *Abb,
                          const double *Abg, const double *g, const double *diag, double lam,
                          double *Lb, double *tb, double *Wg, int *fail);
void launch_schur_obs(hipStream_t s, const DevProblem &P, const double *J, const double *Lb,
                      double *W, const RedSpec *red = nullptr, const double *partial = nullptr,
                      double *scalar = nullptr, const int *gate = nullptr);
// rolling shutter with solved bundles: W rows of the virtual observations
// (Plan::build, PV)
void launch_schur_obs_rs(hipStream_t s, const DevProblem &PV, int Mr, const int *nloc,
                         const int *vobs, const int *vcoff, const double *J, const double *Lb,
                         double *W);
// red (optional): row reductions of k_reduce_multi's plain form (no flag,
// mirror or decision) run by extra workgroups of the same launch
void launch_schur_init(hipStream_t s, const DevProblem &P, const double *Acc, const double *Acg,
                       const double *Agg, const double *g, const double *diag, double lam,
                       const SView &V, int npad, double *rhs, const RedSpec *red = nullptr,
                       const double *partial = nullptr, double *scalar = nullptr);
void launch_schur_pairs(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                        const double *tb, const SView &V, double *rhs);
void launch_chol_panel(hipStream_t s, double *S, const int *slot, int NT, int k, const int *rows,
                       int nrows, double *Linv, int *fail);
void launch_chol_update(hipStream_t s, double *S, const int *slot, int NT, int k,
                        const int2 *pairs, int npairs);
void launch_trsv_fwd(hipStream_t s, const double *S, const int *slot, int NT, int k,
                     const int *rows, int nrows, const double *Linv, double *r, double *y);
void launch_trsv_bwd(hipStream_t s, const double *S, const int *slot, int NT, int k,
                     const int *cols, int ncols, const double *Linv, double *y, double *x);
void launch_trsv_fwd_all(hipStream_t s, const double *S, const int *slot, int NT,
                         const int *rows_off, const int *rows, const double *Linv, double *r,
                         double *y);
void launch_trsv_bwd_all(hipStream_t s, const double *S, const int *slot, int NT,
                         const int *cols_off, const int *cols, const double *Linv, double *y,
                         double *x);
// Returns true when the right-hand side update rhs_R -= sum W_i t_b(i) was
// fused into the diagonal destinations (uniform path; else launch_schur_rhs).
// k_schur_init's camera-frame rows folded into the diagonal destinations
// (unsharded, nG == 0, every solved camera-frame has a diagonal destination):
// those blocks are assigned Acc + lam D^2 - sum W W^T and rhs = g - sum W t.
struct SchurInitFold {
    int on;
    const double *Acc, *g, *diag;
    double lam;
};
bool launch_schur_dest(hipStream_t s, const DevProblem &P, const double *W, const int2 *dest,
                       const int *dest_off, int ndest, const int2 *pairs, const SView &V,
                       int pc_uniform, int assign_off, const double *tb = nullptr,
                       double *rhs = nullptr, SchurInitFold fold = SchurInitFold{},
                       const int *wave_list = nullptr, int n_wave = 0,
                       const int *lane_list = nullptr, int n_lane = 0);
void launch_schur_rhs(hipStream_t s, const DevProblem &P, const double *W, const double *tb,
                      const int *row_cf, double *rhs);
void launch_schur_glob(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                       const double *tb, const SView &V, double *rhs);
void launch_backsub_bundle(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                           const double *tb, const double *Lb, const double *xR, double *U,
                           double *x);
// The trial point's parameter pass (k_trial_prep's operations) fused into
// the bundle back substitution: bundle parameters as their step is formed,
// the other parameters (other[0, nother)) by extra workgroups; partial rows
// pn / xn (rstride apart) get one entry per workgroup (trial_fold_parts).
struct TrialFold {
    const double *x = nullptr, *diag = nullptr;
    double *wa1 = nullptr, *wa2 = nullptr, *wa3 = nullptr;
    double *ext = nullptr, *ext_pert = nullptr, *step = nullptr;
    int solver_type = 0;
    double delta = 0., eps_dif = 0.;
    const int *other = nullptr;
    int nother = 0;
    double *partial = nullptr;
    int rstride = 0;
    // sharded: the parameters this shard counts in ||D p||^2, ||D x_new||^2
    const int *own = nullptr;
    // rec (trial_records_ok): the trial point's record set is built here too
    // -- bundle records by the bundle's thread, camera-frame records by the
    // camera-frame's workgroup after its parameters -- and k_records is not
    // launched; the other parameters are then exactly the camera-frames'
    int rec = 0;
    double *recs = nullptr, *brec = nullptr;
};
// Whether the trial's records can be built inside the back substitution: no
// global parameter (every non-bundle parameter belongs to one camera-frame),
// camera records from the per-camera-frame table, no rolling shutter.
bool trial_records_ok(const DevProblem &P);
int trial_fold_parts(const DevProblem &P, int nother, bool rec = false);
// Plans without a solved bundle (Plan::trial_prep_rec): the trial's parameter
// pass and its records in one launch (T.other: the parameters outside every
// camera-frame block); partial rows of trial_prep_rec_parts entries.
int trial_prep_rec_parts(const DevProblem &P, int nother);
void launch_trial_prep_rec(hipStream_t s, const DevProblem &P, const double *xs, const TrialFold &T);
void launch_obs_wtx(hipStream_t s, const DevProblem &P, const double *W, const double *xR,
                    double *U);
void launch_backsub_trial(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                          const double *tb, const double *Lb, const double *xR, const double *U,
                          double *x, const TrialFold &T);
void launch_scatter_xR(hipStream_t s, const DevProblem &P, const double *xR, double *x);
void launch_newton_bundle(hipStream_t s, const DevProblem &P, const double *W, const double *Wg,
                          const double *Lb, const double *v, double *wR, double *usq,
                          double *un, double *gp);
void launch_gather_R(hipStream_t s, const DevProblem &P, const double *v, double *vR, int nRpad);
// Band + arrow reduced system (mmba_band.hip): factorisation in place, then
// L y = r (band_forward; keeps the separator part of y for band_backward) and
// L^T x = y.  r, y, x are in reduced-system order (length nb + nG).
void band_factor(hipStream_t s, const BandSolver &B, int *fail, long long *probe);
// Factorisation followed by the forward solve y = L^-1 r (fused into the
// factorisation launches when B.use_bcr).
void band_factor_forward(hipStream_t s, const BandSolver &B, int *fail, long long *probe,
                         const double *r, double *y);
// (sharded: the partitions p_lo..p_hi run here, the separator system and its
// right-hand side are all-reduced over B.comm)
void band_forward(hipStream_t s, const BandSolver &B, const double *r, double *y);
void band_backward(hipStream_t s, const BandSolver &B, const double *y, double *x);
// Block cyclic reduction variant (mmba_bcr.hip), same contract; used by the
// band_* entry points when B.use_bcr.
void bcr_factor(hipStream_t s, const BandSolver &B, int *fail, long long *probe,
                const double *r = nullptr, double *y = nullptr);
void bcr_forward(hipStream_t s, const BandSolver &B, const double *r, double *y);
void bcr_backward(hipStream_t s, const BandSolver &B, const double *y, double *x);
// Parallel cyclic reduction (mmba_pcr.hip): x = S^-1 r in one launch (x also
// scattered to parameter order into xs when non-null); the Newton pass
// part[j] = sum over block j's rows (mask) of w (S^-1 w) with the factors of
// the last pcr_solve; workgroups of the solve kernel resident at once.
void pcr_solve(hipStream_t s, const PcrDev &P, const double *r, double *x, double *xs, int *fail);
void pcr_rhs_dot(hipStream_t s, const PcrDev &P, const double *w, const int *mask, int *fail);
// Z = S^-1 R for nc <= PCR_NCMAX column-major right-hand sides, with the
// factors of the last pcr_solve on P (mmba_pcr.hip)
void pcr_rhs_mc(hipStream_t s, const PcrDev &P, const double *R, int ldr, int nc, double *Z,
                int ldz, int *fail);
// contexts open on a device (mmba_context_create / _destroy): PCR launches
// are ordered across streams while there is more than one
void pcr_note_context(int dev, int delta);
int pcr_max_resident(int K);
int pcr_resident_wide(int K);  // the 512-thread form's bound
// workgroups of one k_pcr_solve launch over nblk blocks (the XCD map)
int pcr_grid(int nblk);
// Block-diagonal + arrow solver (mmba_bdiag.hip): factor S, y = L^-1 r and,
// with x, the solution (scattered to parameter order into xs when non-null).
void bd_direct(hipStream_t s, const DevProblem &P, const BdDev &D, const double *Acc,
               const double *g, const double *diag, double lam, double *xR, double *xs,
               int *fail, double *scalar, int dn_slot, int fail_slot,
               const RedSpec *red = nullptr, const double *partial = nullptr);
void bd_factor_solve(hipStream_t s, const BdDev &D, int *fail, const double *r, double *y,
                     double *x, double *xs);
// y = L^-1 w with the stored factor (lmpar's Newton term)
void bd_forward(hipStream_t s, const BdDev &D, const double *w, double *y);
// mask (nullable): entries this shard owns
void launch_sumsq(hipStream_t s, const double *a, const double *d, int n, double *partial,
                  int nparts, double *out, const int *mask = nullptr,
                  unsigned int *ticket = nullptr);
void launch_sumsq_div(hipStream_t s, const double *a, const double *d, int n, double *partial,
                      int nparts, double *out, const int *mask = nullptr,
                      unsigned int *ticket = nullptr);
// sum of y^2 over mask-1 rows and y v over mask-2 rows (separator form's
// Newton term)
void launch_sumsq_mix(hipStream_t s, const double *y, const double *v, int n, double *partial,
                      int nparts, double *out, const int *mask);
void launch_reduce_sum(hipStream_t s, const double *partial, int n, double *out);
void launch_gnorm(hipStream_t s, const double *g, const double *acnorm, int n, double fnorm,
                  double *partial, int nparts, double *out, const int *mask = nullptr,
                  unsigned int *ticket = nullptr);
void launch_jp_sumsq(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
                     const int *nloc, const double *p, double *partial, int nparts,
                     double *out, unsigned int *ticket = nullptr);
void launch_zero_flag(hipStream_t s, const double *acnorm, int n, const int *mask,
                      double *partial, int nparts, double *out, unsigned int *ticket = nullptr);
// *out = (*flag != 0) as a double (fail flags joining the scalar reads);
// the flag is cleared for the next use
void launch_flag_to_scalar(hipStream_t s, int *flag, double *out);
void launch_keep_rows(hipStream_t s, double *v, int lo, int hi, int nCF, int nR, int root);
void launch_keep_mask(hipStream_t s, const double *src, const int *mask, int n, double *dst);
void launch_lm_step(hipStream_t s, int n, const double *xs, const double *x, const double *diag,
                    double *wa1, double *wa2, double *wa3);
void launch_diag_init(hipStream_t s, int n, const double *acnorm, double *diag, int first,
                      int mode);
void launch_newton_v(hipStream_t s, int n, const double *diag, const double *x, double dxnorm,
                     double *v);
// unsharded hand-back into host-mapped page-locked lists (k_handback_host)
void launch_handback_host(hipStream_t s, int Mg, int nrows, const int *dev_of_ref,
                          const double *f2, const double *eu2, const double *ed, double *hf,
                          double *heu, double *hed, const double *dec = nullptr,
                          const double *f2_trial = nullptr);
void launch_unpermute(hipStream_t s, int M, const int *ref_of_dev, const int *obs_own,
                      const double *f2,
                      const double *eu2, const double *ed, double *f2o, double *eu2o,
                      double *edo);

// Sharded Jacobian scalars: [ZERO, XN2, gnorm per rank] -> SL_ZERO.. (max fold).
void launch_fold_ranks(hipStream_t s, const double *t, int nranks, double *out, int do_xn,
                       int do_gn);

// Per-frame solve mode, one workgroup per frame (mmba_batch.hip).
void launch_batch_lm(hipStream_t s, const DevProblem &P, const BatchArgs &B, int nf_max);

// mmba_gemm.hip: C = beta C + alpha A B^T (fp64 MFMA; tri: lower triangle,
// A == B, M == N); column-major, K a multiple of 16.
void launch_dgemm_nt(hipStream_t s, bool tri, int M, int N, int Kd, const double *A, int lda,
                     const double *B, int ldb, double *C, int ldc, double alpha, double beta);

// rolling shutter (mmba_rs.hip)
void launch_jacobian_rs(hipStream_t s, const DevProblem &P, const double *ext_pert,
                        const double *step, int solver_type, double *J, int *jcol, int *nloc,
                        const int *stale_param, double *eu, double *ed);
void launch_ne_rs(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
                  const int *nloc, const double *f, double *Acc, double *Acg, double *g);
void launch_rs_offdiag(hipStream_t s, const DevProblem &P, const SView &V);

}  // namespace mmba
