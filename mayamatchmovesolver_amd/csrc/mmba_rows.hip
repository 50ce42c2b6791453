// mmba_rows.hip -- attribute stiffness / smoothness error rows
// (src/mmSolver/adjust/adjust_measureErrors.cpp:311-387).
//
// Each row depends on one attribute value, so it touches at most one
// parameter: in the normal equations it only adds J_r^2 to that parameter's
// diagonal and J_r f_r to its gradient ("arrowhead" rows that do not change
// the block structure).  Rows are few (one per stiff / smooth attribute), so
// each kernel is one workgroup.  In MM Scene Graph mode the reference never
// writes them (:518), so they stay 0 there (rows_live == 0).
#include "mmba_geom.h"
#include "mmba_kernels.h"

namespace mmba {

// ((1 / gaussian(v, value, variance)) - 1) * weight, gaussian(x, mean, sigma) =
// exp(-((x - mean)^2 / (2 sigma^2))) (adjust_measureErrors.cpp:106-109,342-346).
MMBA_DEV double row_raw(const DevProblem &P, int r, double v) {
    const double g =
        exp(-(pow((v - P.row_val[r]), 2.0) / (2.0 * (pow(P.row_var[r], 2.0)))));
    return ((1.0 / g) - 1.0) * P.row_w[r];
}

MMBA_DEV double row_fvec(const DevProblem &P, double raw) {
    return P.loss_on ? robust_loss(raw, P.loss_type, P.loss_scale) : raw;
}

// Current value of the row's attribute (at the row's frame when animated).
MMBA_DEV double row_value(const DevProblem &P, int r) {
    const int a = P.row_attr[r];
    if (a < 0) return 0.;
    return P.attr_anim[a] ? P.attr_val[P.attr_off[a] + P.row_frame[r]] : P.attr_val[P.attr_off[a]];
}

// measureErrors' row part at the current attribute values: f rows (loss
// applied), errorList rows, sum f^2 -> partial[slot]; with Jrow / pstep the
// trial point's (J p)_r = J_r p_{param(r)}, sum -> partial_jp[slot].  Only
// the root shard counts the rows.
__global__ void __launch_bounds__(64) k_rows_eval(DevProblem P, double *fr, double *eur,
                                                  double *partial, int slot,
                                                  const double *__restrict__ Jrow,
                                                  const double *__restrict__ pstep,
                                                  double *partial_jp) {
    __shared__ double red[2][64];
    double s = 0., sj = 0.;
    for (int r = threadIdx.x; r < P.nrows; r += 64) {
        double raw = 0.;
        if (P.rows_live) raw = row_raw(P, r, row_value(P, r));
        const double f = row_fvec(P, raw);
        fr[r] = f;
        if (eur) eur[r] = raw;
        s += f * f;
        if (Jrow) {
            const int p = P.row_param[r];
            const double jp = p >= 0 ? Jrow[r] * pstep[p] : 0.;
            sj += jp * jp;
        }
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = sj;
    __syncthreads();
    for (int w = 32; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            red[0][threadIdx.x] += red[0][threadIdx.x + w];
            red[1][threadIdx.x] += red[1][threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partial[slot] = P.root ? red[0][0] : 0.;
        if (Jrow) partial_jp[slot] = P.root ? red[1][0] : 0.;
    }
}

// FD Jacobian of the rows (solveFunc_calculateJacobianMatrixForParameter
// re-measures every row for every column): the row's only non-zero column
// is its own parameter.  lmder forward: (f(x + dA) - f(x)) / dA; central
// (stepB != 0): (f(x + dA) - f(x + dB)) * 0.5 / (|dA| + |dB|); lmdif: fdjac2's
// (f(x + h) - f(x)) / h.  errorList rows as the last column (parameter
// last_param, normally n - 1) left them (Appendix B13).
__global__ void __launch_bounds__(64) k_rows_jac(DevProblem P, const double *__restrict__ ext,
                                                 const double *__restrict__ ext_pert,
                                                 const double *__restrict__ step,
                                                 const double *__restrict__ ext_pertB,
                                                 const double *__restrict__ stepB, int lmder,
                                                 double *Jrow, double *eur, int last_param) {
    for (int r = threadIdx.x; r < P.nrows; r += 64) {
        const int p = P.row_param[r];
        if (!P.rows_live || p < 0) {
            Jrow[r] = 0.;
            continue;
        }
        const double f0 = row_fvec(P, row_raw(P, r, ext[p]));
        const double rawA = row_raw(P, r, ext_pert[p]);
        const double fA = row_fvec(P, rawA);
        double J, raw_last = rawA;
        if (!lmder) {
            J = (fA - f0) / step[p];
        } else if (stepB && stepB[p] != 0.) {
            const double rawB = row_raw(P, r, ext_pertB[p]);
            J = (fA - row_fvec(P, rawB)) * stepB[p];
            raw_last = rawB;
        } else {
            J = (fA - f0) * step[p];
        }
        Jrow[r] = J;
        if (eur && p == last_param) eur[r] = raw_last;
    }
}

// Rows into the normal equations (after launch_ne, before the column norms):
// A_pp += J_r^2, g_p += J_r f_r, in row order (one thread: rows sharing a
// parameter add in a fixed order).  Global parameters go to the [Agg | gG]
// block, whose g entries are copied out by the column-norm kernels.
__global__ void k_rows_ne(DevProblem P, const double *__restrict__ Jrow,
                          const double *__restrict__ fr, const int *__restrict__ p_own,
                          double *Acc, double *Abb, double *aggbuf, double *g) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int nCF = P.nR - P.nG;
    for (int r = 0; r < P.nrows; ++r) {
        const int p = P.row_param[r];
        if (p < 0 || (p_own && !p_own[p])) continue;
        const double J = Jrow[r], f = fr[r];
        const int cls = P.p_class[p];
        if (cls == PC_CF) {
            const int cf = P.p_blk[p];
            const int a = P.p_pos[p] - P.cf_roff[cf];
            Acc[(size_t)cf * PCMAX * PCMAX + a * PCMAX + a] += J * J;
            g[p] += J * f;
        } else if (cls == PC_B) {
            const int b = P.p_blk[p];
            const int a = P.p_pos[p];
            Abb[(size_t)b * 9 + a * 3 + a] += J * J;
            g[p] += J * f;
        } else {
            const int gi = P.p_pos[p] - nCF;
            aggbuf[gi * NGMAX + gi] += J * J;
            aggbuf[NGMAX * NGMAX + gi] += J * f;
        }
    }
}

void launch_rows_eval(hipStream_t s, const DevProblem &P, double *fr, double *eur,
                      double *partial, int slot, const double *Jrow, const double *pstep,
                      double *partial_jp) {
    if (P.nrows <= 0) return;
    k_rows_eval<<<1, 64, 0, s>>>(P, fr, eur, partial, slot, Jrow, pstep, partial_jp);
}

void launch_rows_jac(hipStream_t s, const DevProblem &P, const double *ext,
                     const double *ext_pert, const double *step, const double *ext_pertB,
                     const double *stepB, int lmder, double *Jrow, double *eur, int last_param) {
    if (P.nrows <= 0) return;
    k_rows_jac<<<1, 64, 0, s>>>(P, ext, ext_pert, step, ext_pertB, stepB, lmder, Jrow, eur,
                                last_param);
}

void launch_rows_ne(hipStream_t s, const DevProblem &P, const double *Jrow, const double *fr,
                    const int *p_own, double *Acc, double *Abb, double *aggbuf, double *g) {
    if (P.nrows <= 0) return;
    k_rows_ne<<<1, 64, 0, s>>>(P, Jrow, fr, p_own, Acc, Abb, aggbuf, g);
}

}  // namespace mmba
