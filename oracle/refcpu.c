/*
 * refcpu.c -- CPU restatement of mmSolver's LM bundle-adjustment hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker and cpu_baseline); see refcpu.h
 * for the list of reference files restated here.  The structure is kept
 * cost-faithful to the reference MM Scene Graph path: every residual call
 * re-evaluates every transform at every frame and re-projects every
 * marker x frame pair, rebuilding the projection matrix and the 4x4 camera
 * inverse per pair (flat.rs:172-358); the Jacobian is one full evaluation
 * per parameter (adjust_solveFunc.cpp:482-525); the LM is dense MINPACK QR.
 */
#include "refcpu.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define RMIN(a, b) ((a) < (b) ? (a) : (b))
#define RMAX(a, b) ((a) > (b) ? (a) : (b))
/* std::max<double>(v, lo) / std::min<double>(v, hi) as the reference clamps
 * (adjust_base.cpp:202-203,217-218,232-233): a NaN value passes through. */
#define CLAMP_LO(v, lo) (((v) < (lo)) ? (lo) : (v))
#define CLAMP_HI(v, hi) (((hi) < (v)) ? (hi) : (v))

/* lib/rust/mmscenegraph/src/constant.rs */
static const double DEGREES_TO_RADIANS = 0.017453292519943295;
static const double MM_TO_INCH = 0.03937007874015748;
static const double INCH_TO_MM = 25.4;
static const double MM_TO_CM = 0.1;

/* ======================================================================
 * MINPACK-1 restatement (public algorithm; cminpack 1.3.8 call pattern).
 * ====================================================================== */

double ref_enorm(int n, const double *x) {
    const double rdwarf = 3.834e-20, rgiant = 1.304e19;
    double s1 = 0., s2 = 0., s3 = 0., x1max = 0., x3max = 0.;
    const double agiant = rgiant / (double)n;
    for (int i = 0; i < n; ++i) {
        double xabs = fabs(x[i]);
        if (xabs > rdwarf && xabs < agiant) {
            s2 += xabs * xabs;
        } else if (xabs > rdwarf) {
            if (xabs > x1max) {
                double d = x1max / xabs;
                s1 = 1. + s1 * (d * d);
                x1max = xabs;
            } else {
                double d = xabs / x1max;
                s1 += d * d;
            }
        } else {
            if (xabs > x3max) {
                double d = x3max / xabs;
                s3 = 1. + s3 * (d * d);
                x3max = xabs;
            } else if (xabs != 0.) {
                double d = xabs / x3max;
                s3 += d * d;
            }
        }
    }
    if (s1 != 0.) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
    if (s2 != 0.) {
        if (s2 >= x3max) return sqrt(s2 * (1. + (x3max / s2) * (x3max * s3)));
        return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
    }
    return x3max * sqrt(s3);
}

static void qrfac(int m, int n, double *a, int lda, int pivot, int *ipvt,
                  double *rdiag, double *acnorm, double *wa) {
    const double p05 = .05;
    const double epsmch = DBL_EPSILON;
    for (int j = 0; j < n; ++j) {
        acnorm[j] = ref_enorm(m, &a[(size_t)j * lda]);
        rdiag[j] = acnorm[j];
        wa[j] = rdiag[j];
        if (pivot) ipvt[j] = j;
    }
    const int minmn = RMIN(m, n);
    for (int j = 0; j < minmn; ++j) {
        if (pivot) {
            int kmax = j;
            for (int k = j; k < n; ++k)
                if (rdiag[k] > rdiag[kmax]) kmax = k;
            if (kmax != j) {
                for (int i = 0; i < m; ++i) {
                    double temp = a[i + (size_t)j * lda];
                    a[i + (size_t)j * lda] = a[i + (size_t)kmax * lda];
                    a[i + (size_t)kmax * lda] = temp;
                }
                rdiag[kmax] = rdiag[j];
                wa[kmax] = wa[j];
                int k = ipvt[j];
                ipvt[j] = ipvt[kmax];
                ipvt[kmax] = k;
            }
        }
        double *aj = &a[(size_t)j * lda];
        double ajnorm = ref_enorm(m - j, &aj[j]);
        if (ajnorm != 0.) {
            if (aj[j] < 0.) ajnorm = -ajnorm;
            for (int i = j; i < m; ++i) aj[i] /= ajnorm;
            aj[j] += 1.;
            for (int k = j + 1; k < n; ++k) {
                double *ak = &a[(size_t)k * lda];
                double sum = 0.;
                for (int i = j; i < m; ++i) sum += aj[i] * ak[i];
                double temp = sum / aj[j];
                for (int i = j; i < m; ++i) ak[i] -= temp * aj[i];
                if (pivot && rdiag[k] != 0.) {
                    temp = ak[j] / rdiag[k];
                    double d1 = 1. - temp * temp;
                    rdiag[k] *= sqrt(RMAX(0., d1));
                    d1 = rdiag[k] / wa[k];
                    if (p05 * (d1 * d1) <= epsmch) {
                        rdiag[k] = ref_enorm(m - (j + 1), &ak[j + 1]);
                        wa[k] = rdiag[k];
                    }
                }
            }
        }
        rdiag[j] = -ajnorm;
    }
}

static void qrsolv(int n, double *r, int ldr, const int *ipvt,
                   const double *diag, const double *qtb, double *x,
                   double *sdiag, double *wa) {
    const double p5 = .5, p25 = .25;
    for (int j = 0; j < n; ++j) {
        for (int i = j; i < n; ++i) r[i + (size_t)j * ldr] = r[j + (size_t)i * ldr];
        x[j] = r[j + (size_t)j * ldr];
        wa[j] = qtb[j];
    }
    for (int j = 0; j < n; ++j) {
        int l = ipvt[j];
        if (diag[l] != 0.) {
            for (int k = j; k < n; ++k) sdiag[k] = 0.;
            sdiag[j] = diag[l];
            double qtbpj = 0.;
            for (int k = j; k < n; ++k) {
                if (sdiag[k] == 0.) continue;
                double *rk = &r[(size_t)k * ldr];
                double sn, cs;
                if (fabs(rk[k]) < fabs(sdiag[k])) {
                    double cotan = rk[k] / sdiag[k];
                    sn = p5 / sqrt(p25 + p25 * (cotan * cotan));
                    cs = sn * cotan;
                } else {
                    double tn = sdiag[k] / rk[k];
                    cs = p5 / sqrt(p25 + p25 * (tn * tn));
                    sn = cs * tn;
                }
                rk[k] = cs * rk[k] + sn * sdiag[k];
                double temp = cs * wa[k] + sn * qtbpj;
                qtbpj = -sn * wa[k] + cs * qtbpj;
                wa[k] = temp;
                for (int i = k + 1; i < n; ++i) {
                    temp = cs * rk[i] + sn * sdiag[i];
                    sdiag[i] = -sn * rk[i] + cs * sdiag[i];
                    rk[i] = temp;
                }
            }
        }
        sdiag[j] = r[j + (size_t)j * ldr];
        r[j + (size_t)j * ldr] = x[j];
    }
    int nsing = n;
    for (int j = 0; j < n; ++j) {
        if (sdiag[j] == 0. && nsing == n) nsing = j;
        if (nsing < n) wa[j] = 0.;
    }
    for (int k = 1; k <= nsing; ++k) {
        int j = nsing - k;
        double sum = 0.;
        for (int i = j + 1; i < nsing; ++i) sum += r[i + (size_t)j * ldr] * wa[i];
        wa[j] = (wa[j] - sum) / sdiag[j];
    }
    for (int j = 0; j < n; ++j) x[ipvt[j]] = wa[j];
}

static void lmpar(int n, double *r, int ldr, const int *ipvt,
                  const double *diag, const double *qtb, double delta,
                  double *par, double *x, double *sdiag, double *wa1,
                  double *wa2) {
    const double p1 = .1, p001 = .001;
    const double dwarf = DBL_MIN;
    int nsing = n;
    for (int j = 0; j < n; ++j) {
        wa1[j] = qtb[j];
        if (r[j + (size_t)j * ldr] == 0. && nsing == n) nsing = j;
        if (nsing < n) wa1[j] = 0.;
    }
    for (int k = 1; k <= nsing; ++k) {
        int j = nsing - k;
        wa1[j] /= r[j + (size_t)j * ldr];
        double temp = wa1[j];
        for (int i = 0; i <= j - 1; ++i) wa1[i] -= r[i + (size_t)j * ldr] * temp;
    }
    for (int j = 0; j < n; ++j) x[ipvt[j]] = wa1[j];

    int iter = 0;
    for (int j = 0; j < n; ++j) wa2[j] = diag[j] * x[j];
    double dxnorm = ref_enorm(n, wa2);
    double fp = dxnorm - delta;
    if (fp <= p1 * delta) goto TERMINATE;

    {
        double parl = 0.;
        if (nsing >= n) {
            for (int j = 0; j < n; ++j) {
                int l = ipvt[j];
                wa1[j] = diag[l] * (wa2[l] / dxnorm);
            }
            for (int j = 0; j < n; ++j) {
                double sum = 0.;
                for (int i = 0; i <= j - 1; ++i) sum += r[i + (size_t)j * ldr] * wa1[i];
                wa1[j] = (wa1[j] - sum) / r[j + (size_t)j * ldr];
            }
            double temp = ref_enorm(n, wa1);
            parl = fp / delta / temp / temp;
        }
        for (int j = 0; j < n; ++j) {
            double sum = 0.;
            for (int i = 0; i <= j; ++i) sum += r[i + (size_t)j * ldr] * qtb[i];
            wa1[j] = sum / diag[ipvt[j]];
        }
        double gnorm = ref_enorm(n, wa1);
        double paru = gnorm / delta;
        if (paru == 0.) paru = dwarf / RMIN(delta, p1);
        *par = RMAX(*par, parl);
        *par = RMIN(*par, paru);
        if (*par == 0.) *par = gnorm / dxnorm;

        for (;;) {
            ++iter;
            if (*par == 0.) *par = RMAX(dwarf, p001 * paru);
            double temp = sqrt(*par);
            for (int j = 0; j < n; ++j) wa1[j] = temp * diag[j];
            qrsolv(n, r, ldr, ipvt, wa1, qtb, x, sdiag, wa2);
            for (int j = 0; j < n; ++j) wa2[j] = diag[j] * x[j];
            dxnorm = ref_enorm(n, wa2);
            temp = fp;
            fp = dxnorm - delta;
            if (fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) ||
                iter == 10)
                goto TERMINATE;
            for (int j = 0; j < n; ++j) {
                int l = ipvt[j];
                wa1[j] = diag[l] * (wa2[l] / dxnorm);
            }
            for (int j = 0; j < n; ++j) {
                wa1[j] /= sdiag[j];
                temp = wa1[j];
                for (int i = j + 1; i < n; ++i) wa1[i] -= r[i + (size_t)j * ldr] * temp;
            }
            temp = ref_enorm(n, wa1);
            double parc = fp / delta / temp / temp;
            if (fp > 0.) parl = RMAX(parl, *par);
            if (fp < 0.) paru = RMIN(paru, *par);
            *par = RMAX(parl, *par + parc);
        }
    }
TERMINATE:
    if (iter == 0) *par = 0.;
}

/* The shared LM outer/inner loop of lmder and lmdif.  `jac` computes the
 * Jacobian at x (returns iflag, adds to *nfev / *njev as the reference does). */
typedef int (*lm_jac_fn)(void *ctx, int m, int n, double *x, double *fvec,
                         double *fjac, int ldfjac, int *nfev, int *njev);
typedef int (*lm_fun_fn)(void *ctx, int m, int n, const double *x, double *fvec);

#include <stdio.h>
static int g_debug = 0;
void ref_set_debug(int d) { g_debug = d; }

static int lm_core(lm_fun_fn fun, lm_jac_fn jac, void *ctx, int m, int n,
                   double *x, double *fvec, double *fjac, int ldfjac,
                   double ftol, double xtol, double gtol, int maxfev,
                   double *diag, int mode, double factor, int *nfev, int *njev,
                   int *ipvt, double *qtf, double *wa1, double *wa2,
                   double *wa3, double *wa4) {
    const double p1 = .1, p5 = .5, p25 = .25, p75 = .75, p0001 = 1e-4;
    const double epsmch = DBL_EPSILON;
    int info = 0, iflag = 0;
    *nfev = 0;
    if (njev) *njev = 0;
    double delta = 0., xnorm = 0., par, fnorm, gnorm, ratio;

    if (n <= 0 || m < n || ldfjac < m || ftol < 0. || xtol < 0. || gtol < 0. ||
        maxfev <= 0 || factor <= 0.)
        goto TERMINATE;
    if (mode == 2) {
        for (int j = 0; j < n; ++j)
            if (diag[j] <= 0.) goto TERMINATE;
    }
    iflag = fun(ctx, m, n, x, fvec);
    *nfev = 1;
    if (iflag < 0) goto TERMINATE;
    fnorm = ref_enorm(m, fvec);
    par = 0.;
    int iter = 1;
    for (;;) {
        iflag = jac(ctx, m, n, x, fvec, fjac, ldfjac, nfev, njev);
        if (iflag < 0) goto TERMINATE;
        qrfac(m, n, fjac, ldfjac, 1, ipvt, wa1, wa2, wa3);
        if (iter == 1) {
            if (mode != 2) {
                for (int j = 0; j < n; ++j) {
                    diag[j] = wa2[j];
                    if (wa2[j] == 0.) diag[j] = 1.;
                }
            }
            for (int j = 0; j < n; ++j) wa3[j] = diag[j] * x[j];
            xnorm = ref_enorm(n, wa3);
            delta = factor * xnorm;
            if (delta == 0.) delta = factor;
        }
        for (int i = 0; i < m; ++i) wa4[i] = fvec[i];
        for (int j = 0; j < n; ++j) {
            double *fj = &fjac[(size_t)j * ldfjac];
            if (fj[j] != 0.) {
                double sum = 0.;
                for (int i = j; i < m; ++i) sum += fj[i] * wa4[i];
                double temp = -sum / fj[j];
                for (int i = j; i < m; ++i) wa4[i] += fj[i] * temp;
            }
            fj[j] = wa1[j];
            qtf[j] = wa4[j];
        }
        gnorm = 0.;
        if (fnorm != 0.) {
            for (int j = 0; j < n; ++j) {
                int l = ipvt[j];
                if (wa2[l] != 0.) {
                    double sum = 0.;
                    for (int i = 0; i <= j; ++i)
                        sum += fjac[i + (size_t)j * ldfjac] * (qtf[i] / fnorm);
                    gnorm = RMAX(gnorm, fabs(sum / wa2[l]));
                }
            }
        }
        if (gnorm <= gtol) info = 4;
        if (info != 0) goto TERMINATE;
        if (mode != 2)
            for (int j = 0; j < n; ++j) diag[j] = RMAX(diag[j], wa2[j]);

        do {
            lmpar(n, fjac, ldfjac, ipvt, diag, qtf, delta, &par, wa1, wa2, wa3,
                  wa4);
            for (int j = 0; j < n; ++j) {
                wa1[j] = -wa1[j];
                wa2[j] = x[j] + wa1[j];
                wa3[j] = diag[j] * wa1[j];
            }
            double pnorm = ref_enorm(n, wa3);
            if (g_debug) fprintf(stderr, "ref trial: delta=%.17g par=%.17g pnorm=%.17g\n", delta, par, pnorm);
            if (iter == 1) delta = RMIN(delta, pnorm);
            iflag = fun(ctx, m, n, wa2, wa4);
            ++(*nfev);
            if (iflag < 0) goto TERMINATE;
            double fnorm1 = ref_enorm(m, wa4);
            double actred = -1.;
            if (p1 * fnorm1 < fnorm) {
                double d1 = fnorm1 / fnorm;
                actred = 1. - d1 * d1;
            }
            for (int j = 0; j < n; ++j) {
                wa3[j] = 0.;
                double temp = wa1[ipvt[j]];
                for (int i = 0; i <= j; ++i) wa3[i] += fjac[i + (size_t)j * ldfjac] * temp;
            }
            double temp1 = ref_enorm(n, wa3) / fnorm;
            double temp2 = (sqrt(par) * pnorm) / fnorm;
            double prered = temp1 * temp1 + temp2 * temp2 / p5;
            double dirder = -(temp1 * temp1 + temp2 * temp2);
            ratio = 0.;
            if (prered != 0.) ratio = actred / prered;
            if (ratio <= p25) {
                double temp;
                if (actred >= 0.)
                    temp = p5;
                else
                    temp = p5 * dirder / (dirder + p5 * actred);
                if (p1 * fnorm1 >= fnorm || temp < p1) temp = p1;
                delta = temp * RMIN(delta, pnorm / p1);
                par /= temp;
            } else if (par == 0. || ratio >= p75) {
                delta = pnorm / p5;
                par = p5 * par;
            }
            if (ratio >= p0001) {
                for (int j = 0; j < n; ++j) {
                    x[j] = wa2[j];
                    wa2[j] = diag[j] * x[j];
                }
                for (int i = 0; i < m; ++i) fvec[i] = wa4[i];
                xnorm = ref_enorm(n, wa2);
                fnorm = fnorm1;
                ++iter;
            }
            if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1.) info = 1;
            if (delta <= xtol * xnorm) info = 2;
            if (fabs(actred) <= ftol && prered <= ftol && p5 * ratio <= 1. && info == 2)
                info = 3;
            if (info != 0) goto TERMINATE;
            if (*nfev >= maxfev) info = 5;
            if (fabs(actred) <= epsmch && prered <= epsmch && p5 * ratio <= 1.) info = 6;
            if (delta <= epsmch * xnorm) info = 7;
            if (gnorm <= epsmch) info = 8;
            if (info != 0) goto TERMINATE;
        } while (ratio < p0001);
    }
TERMINATE:
    if (iflag < 0) info = iflag;
    return info;
}

/* ---- generic lmder / lmdif entry points (for the scipy cross-check) ---- */
typedef struct {
    ref_fcn_der fder;
    ref_fcn_dif fdif;
    void *p;
    double epsfcn;
    double *wa;
} generic_ctx;

static int gen_fun_der(void *c, int m, int n, const double *x, double *fvec) {
    generic_ctx *g = (generic_ctx *)c;
    return g->fder(g->p, m, n, x, fvec, NULL, m, 1);
}
static int gen_jac_der(void *c, int m, int n, double *x, double *fvec,
                       double *fjac, int ldfjac, int *nfev, int *njev) {
    generic_ctx *g = (generic_ctx *)c;
    (void)nfev;
    int iflag = g->fder(g->p, m, n, x, fvec, fjac, ldfjac, 2);
    ++(*njev);
    return iflag;
}
static int gen_fun_dif(void *c, int m, int n, const double *x, double *fvec) {
    generic_ctx *g = (generic_ctx *)c;
    return g->fdif(g->p, m, n, x, fvec, 1);
}
/* fdjac2 */
static int gen_jac_dif(void *c, int m, int n, double *x, double *fvec,
                       double *fjac, int ldfjac, int *nfev, int *njev) {
    generic_ctx *g = (generic_ctx *)c;
    (void)njev;
    const double epsmch = DBL_EPSILON;
    const double eps = sqrt(RMAX(g->epsfcn, epsmch));
    for (int j = 0; j < n; ++j) {
        double temp = x[j];
        double h = eps * fabs(temp);
        if (h == 0.) h = eps;
        x[j] = temp + h;
        int iflag = g->fdif(g->p, m, n, x, g->wa, 2);
        x[j] = temp;
        if (iflag < 0) return iflag;
        for (int i = 0; i < m; ++i) fjac[i + (size_t)j * ldfjac] = (g->wa[i] - fvec[i]) / h;
    }
    *nfev += n;
    return 0;
}

int ref_lmder(ref_fcn_der fcn, void *p, int m, int n, double *x, double *fvec,
              double *fjac, int ldfjac, double ftol, double xtol, double gtol,
              int maxfev, double *diag, int mode, double factor, int nprint,
              int *nfev, int *njev, int *ipvt, double *qtf, double *wa1,
              double *wa2, double *wa3, double *wa4) {
    (void)nprint;
    generic_ctx g = {fcn, NULL, p, 0., NULL};
    return lm_core(gen_fun_der, gen_jac_der, &g, m, n, x, fvec, fjac, ldfjac,
                   ftol, xtol, gtol, maxfev, diag, mode, factor, nfev, njev,
                   ipvt, qtf, wa1, wa2, wa3, wa4);
}

int ref_lmdif(ref_fcn_dif fcn, void *p, int m, int n, double *x, double *fvec,
              double ftol, double xtol, double gtol, int maxfev, double epsfcn,
              double *diag, int mode, double factor, int nprint, int *nfev,
              double *fjac, int ldfjac, int *ipvt, double *qtf, double *wa1,
              double *wa2, double *wa3, double *wa4) {
    (void)nprint;
    generic_ctx g = {NULL, fcn, p, epsfcn, wa4};
    /* fdjac2 uses wa4 as scratch while lm_core's wa4 is idle at that point. */
    int njev = 0;
    return lm_core(gen_fun_dif, gen_jac_dif, &g, m, n, x, fvec, fjac, ldfjac,
                   ftol, xtol, gtol, maxfev, diag, mode, factor, nfev, &njev,
                   ipvt, qtf, wa1, wa2, wa3, wa4);
}

/* ======================================================================
 * Bound transforms (adjust_base.cpp:194-258), bug-compatible (Appendix B2).
 * ====================================================================== */
double ref_param_internal_to_external(double value, const double xmin,
                                      const double xmax, const double offset,
                                      const double scale) {
    const double float_max = FLT_MAX;
    if ((xmin <= -float_max) && (xmax >= float_max)) {
        value = (value / scale) - offset;
        value = CLAMP_LO(value, xmin);
        value = CLAMP_HI(value, xmax);
        return value;
    } else if (xmax >= float_max) {
        value = xmin - (1.0 + sqrt(value * value + 1.0));
    } else if (xmin <= -float_max) {
        value = xmax + (1.0 - sqrt(value * value + 1.0));
    } else {
        value = xmin + ((xmax - xmin) / 2.0) * (sin(value) + 1.0);
    }
    value = (value / scale) - offset;
    value = CLAMP_LO(value, xmin);
    value = CLAMP_HI(value, xmax);
    return value;
}

double ref_param_external_to_internal(double value, double xmin, double xmax,
                                      const double offset, const double scale) {
    value = CLAMP_LO(value, xmin);
    value = CLAMP_HI(value, xmax);
    value = (value * scale) + offset;
    xmin = (xmin * scale) + offset;
    xmax = (xmax * scale) + offset;
    const double float_max = FLT_MAX;
    if ((xmin <= float_max) && (xmax >= float_max)) {
        return value; /* "No bounds!" branch (also taken for lower-only, B2) */
    } else if (xmax >= float_max) {
        value = sqrt(pow(((value - xmin) + 1.0), 2.0) - 1.0);
    } else if (xmin <= -float_max) {
        value = sqrt(pow((xmax - value) + 1.0, 2.0) - 1.0);
    } else {
        value = asin((2.0 * (value - xmin) / (xmax - xmin)) - 1.0);
    }
    return value;
}

/* ======================================================================
 * Geometry.  Row-major 4x4, column-vector convention (nalgebra semantics).
 * ====================================================================== */
static void mat4_mul(const double *a, const double *b, double *out) {
    double t[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c)
            t[r * 4 + c] = a[r * 4 + 0] * b[0 * 4 + c] + a[r * 4 + 1] * b[1 * 4 + c] +
                           a[r * 4 + 2] * b[2 * 4 + c] + a[r * 4 + 3] * b[3 * 4 + c];
    memcpy(out, t, sizeof(t));
}

/* General 4x4 inverse by cofactors (nalgebra try_inverse / MESA form). */
static int mat4_inverse(const double *m, double *out) {
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
        /* reprojection.rs:35-38 falls back to identity scaling. */
        for (int i = 0; i < 16; ++i) out[i] = (i % 5 == 0) ? 1. : 0.;
        return 0;
    }
    double inv_det = 1.0 / det;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * inv_det;
    return 1;
}

/* transform.rs:338-452 calculate_matrix_with_values: T * R(roo) * S. */
void ref_trs_matrix(double tx, double ty, double tz, double rx, double ry,
                    double rz, double sx, double sy, double sz, int roo,
                    double out[16]) {
    const double S[16] = {sx, 0, 0, 0, 0, sy, 0, 0, 0, 0, sz, 0, 0, 0, 0, 1};
    double srx = sin(rx * DEGREES_TO_RADIANS), crx = cos(rx * DEGREES_TO_RADIANS);
    double sry = sin(ry * DEGREES_TO_RADIANS), cry = cos(ry * DEGREES_TO_RADIANS);
    double srz = sin(rz * DEGREES_TO_RADIANS), crz = cos(rz * DEGREES_TO_RADIANS);
    const double RX[16] = {1, 0, 0, 0, 0, crx, -srx, 0, 0, srx, crx, 0, 0, 0, 0, 1};
    const double RY[16] = {cry, 0, sry, 0, 0, 1, 0, 0, -sry, 0, cry, 0, 0, 0, 0, 1};
    const double RZ[16] = {crz, -srz, 0, 0, srz, crz, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const double *a, *b, *c;
    switch (roo) {
        default:
        case MMBA_ROO_XYZ: a = RZ; b = RY; c = RX; break;
        case MMBA_ROO_YZX: a = RX; b = RZ; c = RY; break;
        case MMBA_ROO_ZXY: a = RY; b = RX; c = RZ; break;
        case MMBA_ROO_XZY: a = RY; b = RZ; c = RX; break;
        case MMBA_ROO_YXZ: a = RZ; b = RX; c = RY; break;
        case MMBA_ROO_ZYX: a = RX; b = RY; c = RZ; break;
    }
    double R[16], T[16] = {1, 0, 0, tx, 0, 1, 0, ty, 0, 0, 1, tz, 0, 0, 0, 1};
    mat4_mul(a, b, R);
    mat4_mul(R, c, R);
    mat4_mul(T, R, out);
    mat4_mul(out, S, out);
}

/* camera.rs:153-327 (MMSG) or maya_camera.cpp:75-414 (Maya DAG).  The output
 * is always in column-vector convention (clip = P * p_cam).  In Maya DAG mode
 * the row-vector matrix is transposed, so film offsets land in P[0][2] and
 * P[1][2] and shift x/y; in MMSG mode they sit in the z row (Appendix B6). */
void ref_projection_matrix(int mode, double focal_mm, double fbw_inch,
                           double fbh_inch, double offx_inch, double offy_inch,
                           double image_w, double image_h, int film_fit,
                           double far_clip, double camera_scale, double P[16]) {
    const double near_clip = 0.1; /* forced: camera.rs dag.rs:140, maya_camera.cpp:789 */
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
    int rust = (mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH);
    switch (film_fit) {
        default:
        case MMBA_FILM_FIT_HORIZONTAL:
            if (rust)
                fsx = image_aspect / film_aspect; /* camera.rs:200 (B5) */
            else
                fsy = image_aspect / film_aspect; /* maya_camera.cpp:161 */
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
    for (int i = 0; i < 16; ++i) P[i] = 0.;
    P[0] = p00;
    P[5] = p11;
    if (rust) {
        /* Matrix4::new row-major: third row = [ox, oy, zz, zw], fourth = [0,0,-1,0] */
        P[8] = ox;
        P[9] = oy;
        P[10] = zz;
        P[11] = zw;
        P[14] = -1.;
    } else {
        /* Maya row-vector matrix M; column-vector P = M^T. */
        P[2] = ox;
        P[6] = oy;
        P[10] = zz;
        P[14] = -1.;
        P[11] = zw;
    }
}

/* reprojection.rs:28-63 as called from flat.rs:317-321: (P * C^-1) * B. */
void ref_reproject(const double cam_world[16], const double proj[16],
                   const double point[3], double out_xy[2]) {
    double cinv[16], pv[16];
    mat4_inverse(cam_world, cinv);
    mat4_mul(proj, cinv, pv);
    double sp[4];
    for (int r = 0; r < 4; ++r)
        sp[r] = pv[r * 4 + 0] * point[0] + pv[r * 4 + 1] * point[1] +
                pv[r * 4 + 2] * point[2] + pv[r * 4 + 3];
    out_xy[0] = (sp[0] / sp[3]) * 0.5;
    out_xy[1] = (sp[1] / sp[3]) * 0.5;
}

/* ---- LDPK classic_3de_mixed_distortion + generic fixed-point inverse ---- */
static void lens_eval(const double c[5], double px, double py, double *qx,
                      double *qy) {
    const double ld = c[0], sq = c[1], cx = c[2], cy = c[3], qu = c[4];
    const double cxx = ld / sq, cxy = (ld + cx) / sq, cyx = ld + cy, cyy = ld;
    const double cxxx = qu / sq, cxxy = 2.0 * qu / sq, cxyy = qu / sq;
    const double cyxx = qu, cyyx = 2.0 * qu, cyyy = qu;
    double p0_2 = px * px, p1_2 = py * py;
    double p0_4 = p0_2 * p0_2, p1_4 = p1_2 * p1_2, p01_2 = p0_2 * p1_2;
    *qx = px * (1 + cxx * p0_2 + cxy * p1_2 + cxxx * p0_4 + cxxy * p01_2 + cxyy * p1_4);
    *qy = py * (1 + cyx * p0_2 + cyy * p1_2 + cyxx * p0_4 + cyyx * p01_2 + cyyy * p1_4);
}

static void lens_map_inverse(const double c[5], double qx, double qy,
                             double *px_out, double *py_out) {
    double fx, fy;
    lens_eval(c, qx, qy, &fx, &fy);
    double px = qx - (fx - qx), py = qy - (fy - qy);
    for (int i = 0; i < 20; ++i) {
        double ix, iy;
        lens_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
        double dx = ix - qx, dy = iy - qy;
        double diff = sqrt(dx * dx + dy * dy);
        if (diff < 1e-6) break;
    }
    for (int i = 0; i < 2; ++i) {
        double ix, iy;
        lens_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
    }
    *px_out = px;
    *py_out = py;
}

/* LensModel defaults (lens_model.h:42): film back 3.6 x 2.4 cm, no offset. */
static const double LENS_FB_W_CM = 3.6, LENS_FB_H_CM = 2.4;

void ref_lens_3de_classic_distort(const double coeff[5], double x, double y,
                                  double *out_x, double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    double px, py;
    lens_map_inverse(coeff, dnx, dny, &px, &py);
    double cxm = px * r + ((w / 2) + 0.0);
    double cym = py * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

void ref_lens_3de_classic_undistort(const double coeff[5], double x, double y,
                                    double *out_x, double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    double px, py;
    lens_eval(coeff, dnx, dny, &px, &py);
    double cxm = px * r + ((w / 2) + 0.0);
    double cym = py * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

/* 3DE radial decentered deg 4 cylindric (mmlens
 * lens_model_3de_radial_decentered_deg_4_cylindric.cpp:58-92 ->
 * distortion_structs.h:108-150 Distortion3deRadialStdDeg4): undistort =
 * cylindric(radial(p)); distort = radial.map_inverse(cylindric^-1(q)), the
 * fixed-point inverse of ldpk_generic_distortion_base.h (20 + 2 iterations,
 * 1e-6).  Restated from the LDPK 2.8 header text
 * (ldpk_radial_decentered_distortion.h operator(), ldpk_cylindric_extender.h
 * cylindric_extender_2::calc_m / eval / eval_inv, ldpk_vec2d.h invert / mat*vec).
 * c: degree-2 c2 u2 v2, degree-4 c4 u4 v4, phi (degrees), b. */
static void radial_eval(const double c[8], double x, double y, double *qx, double *qy) {
    const double c2 = c[0], u2 = c[1], v2 = c[2], c4 = c[3], u4 = c[4], v4 = c[5];
    double x2 = x * x;
    double y2 = y * y;
    double xy = x * y;
    double r2 = x2 + y2;
    double r4 = r2 * r2;
    *qx = x * (1.0 + c2 * r2 + c4 * r4) + (r2 + 2.0 * x2) * (u2 + u4 * r2) +
          2.0 * xy * (v2 + v4 * r2);
    *qy = y * (1.0 + c2 * r2 + c4 * r4) + (r2 + 2.0 * y2) * (v2 + v4 * r2) +
          2.0 * xy * (u2 + u4 * r2);
}

static void cylindric_mats(const double c[8], double m[4], double mi[4]) {
    const double phi = c[6], b = c[7];
    const double pi = 3.14159265358979323846; /* M_PI, as ldpk_cylindric_extender.h */
    double q = sqrt(1.0 + b), cs = cos(phi * pi / 180.0), sn = sin(phi * pi / 180.0);
    m[0] = cs * cs * q + sn * sn / q;
    m[1] = (q - 1.0 / q) * cs * sn;
    m[2] = (q - 1.0 / q) * cs * sn;
    m[3] = cs * cs / q + sn * sn * q;
    double det = m[0] * m[3] - m[1] * m[2];
    mi[0] = m[3] / det;
    mi[1] = -m[1] / det;
    mi[2] = -m[2] / det;
    mi[3] = m[0] / det;
}

static void radial_map_inverse(const double c[8], double qx, double qy, double *px_out,
                               double *py_out) {
    double fx, fy;
    radial_eval(c, qx, qy, &fx, &fy);
    double px = qx - (fx - qx), py = qy - (fy - qy);
    for (int i = 0; i < 20; ++i) {
        double ix, iy;
        radial_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
        double dx = ix - qx, dy = iy - qy;
        double diff = sqrt(dx * dx + dy * dy);
        if (diff < 1e-6) break;
    }
    for (int i = 0; i < 2; ++i) {
        double ix, iy;
        radial_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
    }
    *px_out = px;
    *py_out = py;
}

void ref_lens_3de_radial_distort(const double coeff[8], double x, double y, double *out_x,
                                 double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    double m[4], mi[4];
    cylindric_mats(coeff, m, mi);
    double tx = mi[0] * dnx + mi[1] * dny;
    double ty = mi[2] * dnx + mi[3] * dny;
    double px, py;
    radial_map_inverse(coeff, tx, ty, &px, &py);
    double cxm = px * r + ((w / 2) + 0.0);
    double cym = py * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

void ref_lens_3de_radial_undistort(const double coeff[8], double x, double y, double *out_x,
                                   double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    double m[4], mi[4];
    cylindric_mats(coeff, m, mi);
    double qx, qy;
    radial_eval(coeff, dnx, dny, &qx, &qy);
    double px = m[0] * qx + m[1] * qy;
    double py = m[2] * qx + m[3] * qy;
    double cxm = px * r + ((w / 2) + 0.0);
    double cym = py * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

/* 3DE anamorphic deg 4 rotate squeeze xy (+ rescaled) (mmlens
 * lens_model_3de_anamorphic_deg_4_rotate_squeeze_xy[_rescaled].cpp ->
 * distortion_structs.h:152-301 Distortion3deAnamorphicStdDeg4[Rescaled]):
 *   undistort = RSP * anamorphic(PAR^-1 * p),
 *   distort   = PAR * anamorphic.map_inverse(RSP^-1 * q),
 * RSP = R Sx Sy [Rs] PA and PAR = PA [Rs] R (ldpk_linear_extender.h set(),
 * left-to-right 2x2 products), R = rotation by value / 180 * pi
 * (ldpk_rotation_extender.h), Sx / Sy / Rs / PA squeeze-x / squeeze-y
 * extenders (ldpk_squeeze_extender.h; PA = the LensModel pixel aspect 1.0,
 * lens_model.h:41), the anamorphic polynomial of the degree-4
 * specialisation of ldpk_generic_anamorphic_distortion.h (prepare(),
 * operator()).  A missing rescale factor (non-rescaled model) is the
 * identity, which leaves every product exactly unchanged.
 * c: cx02 cy02 cx22 cy22 cx04 cy04 cx24 cy24 cx44 cy44 rot(deg) sqx sqy rescale */
typedef struct {
    double a00, a01, a10, a11;
} ref_m2;

static ref_m2 m2_mul(ref_m2 t, ref_m2 a) {
    ref_m2 r = {t.a00 * a.a00 + t.a01 * a.a10, t.a00 * a.a01 + t.a01 * a.a11,
                t.a10 * a.a00 + t.a11 * a.a10, t.a10 * a.a01 + t.a11 * a.a11};
    return r;
}

static ref_m2 m2_inv(ref_m2 a) {
    double det = a.a00 * a.a11 - a.a01 * a.a10;
    ref_m2 r = {a.a11 / det, -a.a01 / det, -a.a10 / det, a.a00 / det};
    return r;
}

static void anam_mats(const double c[14], ref_m2 *rsp, ref_m2 *par) {
    const double pi = 3.14159265358979323846;
    double phi = c[10] / 180.0 * pi;
    ref_m2 R = {cos(phi), -sin(phi), sin(phi), cos(phi)};
    ref_m2 Sx = {c[11], 0.0, 0.0, 1.0};
    ref_m2 Sy = {1.0, 0.0, 0.0, c[12]};
    ref_m2 Rs = {c[13], 0.0, 0.0, 1.0};
    ref_m2 PA = {1.0, 0.0, 0.0, 1.0};
    *rsp = m2_mul(m2_mul(m2_mul(m2_mul(R, Sx), Sy), Rs), PA);
    *par = m2_mul(m2_mul(PA, Rs), R);
}

static void anam_eval(const double c[14], double x, double y, double *qx, double *qy) {
    const double cx02 = c[0], cy02 = c[1], cx22 = c[2], cy22 = c[3], cx04 = c[4],
                 cy04 = c[5], cx24 = c[6], cy24 = c[7], cx44 = c[8], cy44 = c[9];
    double cx_x2 = cx02 + cx22, cx_y2 = cx02 - cx22, cx_x4 = cx04 + cx24 + cx44;
    double cx_x2y2 = 2.0 * cx04 - 6.0 * cx44, cx_y4 = cx04 - cx24 + cx44;
    double cy_x2 = cy02 + cy22, cy_y2 = cy02 - cy22, cy_x4 = cy04 + cy24 + cy44;
    double cy_x2y2 = 2.0 * cy04 - 6.0 * cy44, cy_y4 = cy04 - cy24 + cy44;
    double x2 = x * x, x4 = x2 * x2;
    double y2 = y * y, y4 = y2 * y2;
    *qx = x * (1.0 + x2 * cx_x2 + y2 * cx_y2 + x4 * cx_x4 + x2 * y2 * cx_x2y2 + y4 * cx_y4);
    *qy = y * (1.0 + x2 * cy_x2 + y2 * cy_y2 + x4 * cy_x4 + x2 * y2 * cy_x2y2 + y4 * cy_y4);
}

static void anam_map_inverse(const double c[14], double qx, double qy, double *px_out,
                             double *py_out) {
    double fx, fy;
    anam_eval(c, qx, qy, &fx, &fy);
    double px = qx - (fx - qx), py = qy - (fy - qy);
    for (int i = 0; i < 20; ++i) {
        double ix, iy;
        anam_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
        double dx = ix - qx, dy = iy - qy;
        double diff = sqrt(dx * dx + dy * dy);
        if (diff < 1e-6) break;
    }
    for (int i = 0; i < 2; ++i) {
        double ix, iy;
        anam_eval(c, px, py, &ix, &iy);
        px = px + qx - ix;
        py = py + qy - iy;
    }
    *px_out = px;
    *py_out = py;
}

void ref_lens_3de_anamorphic_distort(const double coeff[14], double x, double y,
                                     double *out_x, double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    ref_m2 rsp, par;
    anam_mats(coeff, &rsp, &par);
    ref_m2 ri = m2_inv(rsp);
    double tx = ri.a00 * dnx + ri.a01 * dny;
    double ty = ri.a10 * dnx + ri.a11 * dny;
    double px, py;
    anam_map_inverse(coeff, tx, ty, &px, &py);
    double ox = par.a00 * px + par.a01 * py;
    double oy = par.a10 * px + par.a11 * py;
    double cxm = ox * r + ((w / 2) + 0.0);
    double cym = oy * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

void ref_lens_3de_anamorphic_undistort(const double coeff[14], double x, double y,
                                       double *out_x, double *out_y) {
    const double w = LENS_FB_W_CM, h = LENS_FB_H_CM;
    const double r = sqrt(w * w + h * h) / 2.0;
    double ux = x + 0.5, uy = y + 0.5;
    double dnx = ((ux - 1.0 / 2.0) * w - 0.0) / r;
    double dny = ((uy - 1.0 / 2.0) * h - 0.0) / r;
    ref_m2 rsp, par;
    anam_mats(coeff, &rsp, &par);
    ref_m2 pi_ = m2_inv(par);
    double tx = pi_.a00 * dnx + pi_.a01 * dny;
    double ty = pi_.a10 * dnx + pi_.a11 * dny;
    double qx, qy;
    anam_eval(coeff, tx, ty, &qx, &qy);
    double ox = rsp.a00 * qx + rsp.a01 * qy;
    double oy = rsp.a10 * qx + rsp.a11 * qy;
    double cxm = ox * r + ((w / 2) + 0.0);
    double cym = oy * r + ((h / 2) + 0.0);
    *out_x = cxm / w - 0.5;
    *out_y = cym / h - 0.5;
}

/* ======================================================================
 * Scene state + measureErrors.
 * ====================================================================== */
typedef struct {
    const mmba_problem *p;
    const mmba_options *o;
    double *attr;      /* mutable attribute block */
    double *tfm_world; /* [T * F * 16] */
    double *pts;       /* MMSG out_point_list [K * F * 2] */
    double *err_user;  /* ud->errorList   [m] */
    double *err_dist;  /* ud->errorDistanceList [M] */
    char *frame_all;   /* all-ones frame mask */
    char *frame_mask;  /* per-parameter mask */
    /* LM bookkeeping, mirrors SolverData counters (adjust_solveFunc.cpp:146-200) */
    int func_evals, jac_evals;
    double *xa, *xb, *ea, *eb; /* FD scratch */
    mmba_trace *trace;
    int interrupted;
    double *obs_pts, *obs_mkr; /* optional: reprojected point / corrected marker [2M] */
    int m;                     /* residual rows: 2M + stiffness + smoothness */
    int rs_any;                /* some camera has a rolling shutter (mmba.h ABI 3) */
    /* B3 (mmba.h ABI 7): lens_src[(l * F + f) * 14 + k] = the parameter whose
     * value slot k of lens instance (l, f) holds, -1: the plug model's value */
    int *lens_src;
    int lens_set; /* setParameters has run: the clones hold the parameters'
                     values (before it, every slot is the plug model's value:
                     solveFrames' initial measureErrors, adjust_base.cpp:
                     1002-1004 then 1076-1089) */
    /* B4 (mmba.h ABI 8): the marker whose flat entry observation i reads in
     * MMSG mode, and that entry's x,y (before film fit) */
    int *geo_mkr;      /* [M] */
    double *geo_xy;    /* [2M] */
} ref_scene;

/* Test hook standing in for MComputation::isInterruptRequested: the poll
 * returns true from the `g_interrupt_after`-th poll on (sticky, like the Maya
 * flag); < 0 never interrupts. */
static int g_interrupt_after = -1;
static int g_interrupt_polls = 0;
void ref_set_interrupt_after(int k) {
    g_interrupt_after = k;
    g_interrupt_polls = 0;
}
static int interrupt_requested(ref_scene *s) {
    const int k = g_interrupt_polls++;
    if (g_interrupt_after >= 0 && k >= g_interrupt_after) {
        s->interrupted = 1;
        return 1;
    }
    return 0;
}

/* applyLossFunctionToErrors (adjust_base.cpp:132-187), over every row of the
 * buffer measureErrors was handed (adjust_measureErrors.cpp:553-558). */
static void apply_loss(int m, double *f, int type, double scale) {
    for (int i = 0; i < m; ++i) {
        double z = pow(f[i] / scale, 2);
        double rho0 = z, rho1 = 1.0, rho2 = 0.0;
        if (type == MMBA_ROBUST_LOSS_TRIVIAL) {
            rho0 = z;
            rho1 = 1.0;
            rho2 = 0.0;
        } else if (type == MMBA_ROBUST_LOSS_SOFT_L_ONE) {
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
        rho0 *= pow(scale, 2.0);
        rho2 /= pow(scale, 2.0);
        double J_scale = rho1 + 2.0 * rho2 * pow(f[i], 2.0);
        const double eps = DBL_EPSILON;
        if (J_scale < eps) J_scale = eps;
        J_scale = pow(J_scale, 0.5);
        f[i] *= rho1 / J_scale;
    }
}

/* gaussian() of adjust_measureErrors.cpp:106-109. */
static double gaussian(double x, double mean, double sigma) {
    return exp(-(pow((x - mean), 2.0) / (2.0 * (pow(sigma, 2.0)))));
}

static double attr_value(const ref_scene *s, int a, int f, double dflt) {
    if (a < 0) return dflt;
    const mmba_problem *p = s->p;
    return p->attr_animated[a] ? s->attr[p->attr_offset[a] + f]
                               : s->attr[p->attr_offset[a]];
}

static void eval_world_matrices(ref_scene *s) {
    const mmba_problem *p = s->p;
    const int F = p->num_frames;
    for (int t = 0; t < p->num_transforms; ++t) {
        const int *ta = &p->tfm_attrs[9 * t];
        for (int f = 0; f < F; ++f) {
            double local[16];
            ref_trs_matrix(attr_value(s, ta[0], f, 0.), attr_value(s, ta[1], f, 0.),
                           attr_value(s, ta[2], f, 0.), attr_value(s, ta[3], f, 0.),
                           attr_value(s, ta[4], f, 0.), attr_value(s, ta[5], f, 0.),
                           attr_value(s, ta[6], f, 1.), attr_value(s, ta[7], f, 1.),
                           attr_value(s, ta[8], f, 1.), p->tfm_rotate_order[t], local);
            double *w = &s->tfm_world[((size_t)t * F + f) * 16];
            int parent = p->tfm_parent[t];
            if (parent >= 0)
                mat4_mul(&s->tfm_world[((size_t)parent * F + f) * 16], local, w);
            else
                memcpy(w, local, sizeof(local));
        }
    }
}

/* Film back values as each mode sees them: MMSG holds mm in the data block
 * (maya_scene_graph.cpp:359-375) and converts back to inch in
 * compute_projection_matrix_with_attrs (dag.rs:135-145). */
static void camera_film(const ref_scene *s, int c, int f, double *fbw_in,
                        double *fbh_in, double *offx_in, double *offy_in,
                        double *aspect) {
    const int *ca = &s->p->cam_attrs[MMBA_CAM_NUM_ATTRS * c];
    double w = attr_value(s, ca[MMBA_CAM_FILM_BACK_W_INCH], f, 36.0 / 25.4);
    double h = attr_value(s, ca[MMBA_CAM_FILM_BACK_H_INCH], f, 24.0 / 25.4);
    double ox = attr_value(s, ca[MMBA_CAM_FILM_OFFSET_X_INCH], f, 0.);
    double oy = attr_value(s, ca[MMBA_CAM_FILM_OFFSET_Y_INCH], f, 0.);
    if (s->o->scene_graph_mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        double w_mm = w * 25.4, h_mm = h * 25.4;
        *fbw_in = w_mm * MM_TO_INCH;
        *fbh_in = h_mm * MM_TO_INCH;
        *offx_in = (ox * 25.4) * MM_TO_INCH;
        *offy_in = (oy * 25.4) * MM_TO_INCH;
        *aspect = w_mm / h_mm; /* flat.rs:327-331 */
    } else {
        *fbw_in = w;
        *fbh_in = h;
        *offx_in = ox;
        *offy_in = oy;
        *aspect = w / h; /* adjust_measureErrors.cpp:196-198 */
    }
}

static void camera_projection(const ref_scene *s, int c, int f, double P[16],
                              double *film_aspect, double *render_aspect) {
    const int *ca = &s->p->cam_attrs[MMBA_CAM_NUM_ATTRS * c];
    double fbw, fbh, ox, oy;
    camera_film(s, c, f, &fbw, &fbh, &ox, &oy, film_aspect);
    double focal = attr_value(s, ca[MMBA_CAM_FOCAL_MM], f, 35.0);
    double far_clip = attr_value(s, ca[MMBA_CAM_FAR_CLIP], f, 10000.0);
    double cscale = attr_value(s, ca[MMBA_CAM_SCALE], f, 1.0);
    double iw = (double)s->p->cam_render_size[2 * c];
    double ih = (double)s->p->cam_render_size[2 * c + 1];
    ref_projection_matrix(s->o->scene_graph_mode, focal, fbw, fbh, ox, oy, iw,
                          ih, s->p->cam_film_fit[c], far_clip, cscale, P);
    *render_aspect = iw / ih;
}

/* flat.rs:73-97 / maya_camera.cpp:213-330 (backward direction). */
static void film_fit_marker(int film_fit, double film_aspect,
                            double render_aspect, double *x, double *y) {
    switch (film_fit) {
        case MMBA_FILM_FIT_HORIZONTAL:
            *y *= render_aspect / film_aspect;
            break;
        case MMBA_FILM_FIT_VERTICAL:
            *x *= 1.0 / (render_aspect / film_aspect);
            break;
        case MMBA_FILM_FIT_FILL:
            if (film_aspect > render_aspect)
                *x *= film_aspect / render_aspect;
            else
                *y *= render_aspect / film_aspect;
            break;
        case MMBA_FILM_FIT_OVERSCAN:
            if (film_aspect > render_aspect)
                *y *= render_aspect / film_aspect;
            else
                *x *= film_aspect / render_aspect;
            break;
        default:
            break;
    }
}

/* Default of lens attribute slot k (mmba.h): classic squeeze, anamorphic
 * squeeze x / y and rescale are 1, everything else 0. */
static double lens_default(int type, int k) {
    if (type == MMBA_LENS_3DE_CLASSIC) return k == 1 ? 1. : 0.;
    if (type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4 ||
        type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED)
        return k >= 11 ? 1. : 0.;
    return 0.;
}

static void lens_model_distort(int type, const double *c, double x, double y, double *ox,
                               double *oy) {
    if (type == MMBA_LENS_3DE_CLASSIC)
        ref_lens_3de_classic_distort(c, x, y, ox, oy);
    else if (type == MMBA_LENS_3DE_RADIAL_STD_DEG4)
        ref_lens_3de_radial_distort(c, x, y, ox, oy);
    else
        ref_lens_3de_anamorphic_distort(c, x, y, ox, oy);
}

/* An input layer of a layered lens (mmba.h ABI 5): the values read with the
 * camera-connected node's plug (lens_input_values), or each slot's
 * attribute at frame 0 -- constants of the solve (the reference never
 * re-points the clones' input chain, maya_lens_model_utils.cpp:715). */
static void lens_layer_values(const ref_scene *s, int l, double c[MMBA_LENS_NUM_ATTRS]) {
    const mmba_problem *p = s->p;
    const int type = p->lens_type[l];
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) {
        if (p->lens_input_values) {
            c[k] = p->lens_input_values[MMBA_LENS_NUM_ATTRS * l + k];
        } else {
            const int a = p->lens_attrs[MMBA_LENS_NUM_ATTRS * l + k];
            c[k] = a >= 0 ? p->attr_values[p->attr_offset[a]] : lens_default(type, k);
        }
    }
    if (type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4) c[13] = 1.;
}

/* The model's applyModelDistort: its input model's first (recursively, so
 * the deepest layer runs first), no check in between
 * (lens_model_3de_classic.cpp:82-88 and the other models alike). */
static void lens_chain_distort(const ref_scene *s, int l, int depth, double x, double y,
                               double *ox, double *oy) {
    const mmba_problem *p = s->p;
    const int in = p->lens_input ? p->lens_input[l] : -1;
    if (in >= 0 && depth < 8) lens_chain_distort(s, in, depth + 1, x, y, &x, &y);
    double c[MMBA_LENS_NUM_ATTRS];
    lens_layer_values(s, l, c);
    lens_model_distort(p->lens_type[l], c, x, y, ox, oy);
}

/* ---- the reference's lens lists and the index
 * arithmetic that reads them (mmba.h ABI 7).
 *   lensModelList[l*F + f]: clone f of lens l's plug model
 *     (maya_lens_model_utils.cpp:654-661: lensIndex = the list's size before
 *     the lens's F clones are appended);
 *   markerFrameToLensModelList[i*F + f] = lensModelList[lens(marker i)*F + f]
 *     (:782-799, the camera's first lens node);
 *   attrFrameToLensModelList[a*F + f] = lensModelList[lens(attr a)*F + f]
 *     (:836-851, lens attributes only; null otherwise);
 * measureErrors reads markerFrameToLensModelList[markerIndex + frameIndex]
 * (adjust_measureErrors.cpp:244, 463); setParameters writes an animated lens
 * attribute's value into attrFrameToLensModelList[attrIndex + frameIndex] and
 * a static one's into [attrIndex + j] for every frame j
 * (adjust_setParameters.cpp:113-121, 206-214), a null entry being ignored
 * (setLensModelAttributeValue, maya_lens_model_utils.cpp:87-93).  Each
 * evaluation sets every parameter in order, so a slot holds the value of the
 * LAST parameter that writes it; a slot no parameter writes keeps the plug
 * model's value (lens attributes are never read per frame, B11). ---- */

/* The attribute's index in the solver's attrList (paramToAttrList[p].first):
 * param_ref_attr, or the attributes numbered in order of first appearance. */
static int b3_ref_attrs(const mmba_problem *p, int *par_ref) {
    if (p->param_ref_attr) {
        for (int q = 0; q < p->num_params; ++q) par_ref[q] = p->param_ref_attr[q];
        return p->num_ref_attrs;
    }
    int n = 0;
    for (int q = 0; q < p->num_params; ++q) {
        par_ref[q] = -1;
        for (int r = 0; r < q; ++r)
            if (p->param_attr[r] == p->param_attr[q]) par_ref[q] = par_ref[r];
        if (par_ref[q] < 0) par_ref[q] = n++;
    }
    return n;
}

/* (lens, slot) of an attribute id, or -1 */
static int b3_lens_slot(const mmba_problem *p, int a, int *slot) {
    for (int l = 0; l < p->num_lenses; ++l)
        for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k)
            if (p->lens_attrs[MMBA_LENS_NUM_ATTRS * l + k] == a) {
                *slot = k;
                return l;
            }
    return -1;
}

/* The lens of attrList entry r: ref_attr_lens, or the lens of the first
 * parameter's attribute that is entry r. */
static int b3_ref_lens(const mmba_problem *p, const int *par_ref, int r) {
    if (p->ref_attr_lens) return p->ref_attr_lens[r];
    int k;
    for (int q = 0; q < p->num_params; ++q)
        if (par_ref[q] == r) return b3_lens_slot(p, p->param_attr[q], &k);
    return -1;
}

/* Fills s->lens_src by running setParameters' lens writes once.  Returns
 * MMBA_ERR_UNSUPPORTED where the reference's behaviour is undefined: a write
 * into a lens of another model type (a reinterpret_cast of the model,
 * maya_lens_model_utils.cpp:160-170) or an attrList index out of range. */
static int b3_build(ref_scene *s) {
    const mmba_problem *p = s->p;
    const int F = p->num_frames, nL = p->num_lenses, n = p->num_params;
    if (!p->cam_lens || nL <= 0) return MMBA_OK;
    s->lens_src = (int *)malloc(sizeof(int) * (size_t)nL * F * MMBA_LENS_NUM_ATTRS);
    for (size_t q = 0; q < (size_t)nL * F * MMBA_LENS_NUM_ATTRS; ++q) s->lens_src[q] = -1;
    int *par_ref = (int *)malloc(sizeof(int) * (n ? n : 1));
    const int n_ref = b3_ref_attrs(p, par_ref);
    int rc = MMBA_OK;
    for (int q = 0; q < n && rc == MMBA_OK; ++q) {
        int k;
        const int la = b3_lens_slot(p, p->param_attr[q], &k);
        if (la < 0) continue; /* not a lens attribute: the DG / AttrDataBlock path */
        const int g0 = p->param_frame[q] >= 0 ? p->param_frame[q] : 0;
        const int g1 = p->param_frame[q] >= 0 ? p->param_frame[q] + 1 : F;
        for (int g = g0; g < g1; ++g) {
            const int t = par_ref[q] + g; /* attrIndex + frameIndex / + j */
            if (par_ref[q] < 0 || t / F >= n_ref) {
                rc = MMBA_ERR_UNSUPPORTED;
                break;
            }
            const int lt = b3_ref_lens(p, par_ref, t / F);
            if (lt < 0) continue; /* a null model: nothing is set */
            if (p->lens_type[lt] != p->lens_type[la]) {
                rc = MMBA_ERR_UNSUPPORTED;
                break;
            }
            s->lens_src[((size_t)lt * F + t % F) * MMBA_LENS_NUM_ATTRS + k] = q;
        }
    }
    free(par_ref);
    return rc;
}

/* Distortion of observation i: the instance markerFrameToLensModelList
 * [markerIndex + frameIndex] names, with its input layers first. */
static void apply_lens_obs(const ref_scene *s, int i, double *px, double *py) {
    const mmba_problem *p = s->p;
    if (!s->lens_src) return;
    const int F = p->num_frames;
    const int t = p->obs_marker[i] + p->obs_frame[i];
    const int lens = p->cam_lens[p->mkr_cam[t / F]];
    const int fi = t % F;
    if (lens < 0) return;
    const int type = p->lens_type[lens];
    if (type < MMBA_LENS_3DE_CLASSIC || type > MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4_RESCALED) return;
    double c[MMBA_LENS_NUM_ATTRS], plug[MMBA_LENS_NUM_ATTRS];
    lens_layer_values(s, lens, plug); /* the plug model the clones copy */
    for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) {
        const int q = s->lens_set ? s->lens_src[((size_t)lens * F + fi) * MMBA_LENS_NUM_ATTRS + k]
                                  : -1;
        c[k] = q < 0 ? plug[k]
                     : attr_value(s, p->param_attr[q], p->param_frame[q] >= 0 ? p->param_frame[q] : 0,
                                  0.);
    }
    if (type == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4) c[13] = 1.; /* no rescale slot */
    double ox = *px, oy = *py, ix = *px, iy = *py;
    const int in = p->lens_input ? p->lens_input[lens] : -1;
    if (in >= 0) lens_chain_distort(s, in, 1, ix, iy, &ix, &iy);
    lens_model_distort(type, c, ix, iy, &ox, &oy);
    if (isfinite(ox)) *px = ox; /* adjust_measureErrors.cpp:466-472 */
    if (isfinite(oy)) *py = oy;
}

/* Rolling shutter (mmba.h ABI 3; an extension with no solver counterpart in
 * the reference -- "parity unpinned against the reference").  The arithmetic
 * is the 3DE exporter's (share/3dequalizer/python/uvtrack_format.py):
 * rs = time shift x fps (:269-270), scanline time from the point's vertical
 * position (:318, 3DE y in [0, 1] bottom-up = 0.5 + y here), the end-frame
 * extrapolation (:311-314) and the three-frame quadratic blend
 * _apply_rs_correction (:186-203), applied to the camera transform's
 * translate / rotate attribute values at the observation's time f + tau. */
static int rs_on(const ref_scene *s, int c) {
    return s->p->cam_rs_value && s->p->cam_rs_value[c] != 0.0 && s->p->num_frames > 1;
}

static double rs_blend(const ref_scene *s, int a, int f, double tau) {
    const int F = s->p->num_frames;
    const double cv = attr_value(s, a, f, 0.);
    double pv = f > 0 ? attr_value(s, a, f - 1, 0.) : 0.;
    double nv = f < F - 1 ? attr_value(s, a, f + 1, 0.) : 0.;
    if (f == 0) pv = cv + (cv - nv);
    if (f == F - 1) nv = cv + (cv - pv);
    const double b = (nv - pv) / 2.0;
    const double c = -cv + ((nv + pv) / 2.0);
    return (cv + tau * b) + (tau * tau) * c;
}

/* World matrix of camera c's transform as observation (f, y) sees it. */
static void rs_camera_world(const ref_scene *s, int c, int f, double y, double W[16]) {
    const mmba_problem *p = s->p;
    const int t = p->cam_tfm[c];
    const int *ta = &p->tfm_attrs[9 * t];
    const double tau = p->cam_rs_value[c] * (0.5 - y);
    double local[16];
    ref_trs_matrix(rs_blend(s, ta[0], f, tau), rs_blend(s, ta[1], f, tau),
                   rs_blend(s, ta[2], f, tau), rs_blend(s, ta[3], f, tau),
                   rs_blend(s, ta[4], f, tau), rs_blend(s, ta[5], f, tau),
                   attr_value(s, ta[6], f, 1.), attr_value(s, ta[7], f, 1.),
                   attr_value(s, ta[8], f, 1.), p->tfm_rotate_order[t], local);
    const int parent = p->tfm_parent[t];
    if (parent >= 0)
        mat4_mul(&s->tfm_world[((size_t)parent * p->num_frames + f) * 16], local, W);
    else
        memcpy(W, local, sizeof(local));
}

/* Writes errors for observations whose frame is enabled (mask). */
static void measure(ref_scene *s, const char *frame_mask, double *errors) {
    const mmba_problem *p = s->p;
    const int F = p->num_frames;
    const double image_width = s->o->image_width;
    eval_world_matrices(s);
    if (s->o->scene_graph_mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        /* FlatScene::evaluate: camera -> marker -> frame, every pair
         * (flat.rs:271-356), projection matrix rebuilt per pair. */
        size_t pos = 0;
        for (int c = 0; c < p->num_cameras; ++c) {
            for (int k = 0; k < p->num_markers; ++k) {
                if (p->mkr_cam[k] != c) continue;
                const int bt = p->bnd_tfm[p->mkr_bnd[k]];
                const int ct = p->cam_tfm[c];
                for (int f = 0; f < F; ++f) {
                    double P[16], fa, ra;
                    camera_projection(s, c, f, P, &fa, &ra);
                    const double *cw = &s->tfm_world[((size_t)ct * F + f) * 16];
                    const double *bw = &s->tfm_world[((size_t)bt * F + f) * 16];
                    double bp[3] = {bw[3], bw[7], bw[11]};
                    ref_reproject(cw, P, bp, &s->pts[pos * 2]);
                    ++pos;
                }
            }
        }
    }
    for (int i = 0; i < p->num_obs; ++i) {
        const int k = p->obs_marker[i];
        const int f = p->obs_frame[i];
        if (frame_mask && !frame_mask[f]) continue;
        const int g = s->geo_mkr[i]; /* B4: the flat entry's marker */
        const int c = p->mkr_cam[g];
        double mkr_x = s->geo_xy[2 * i], mkr_y = s->geo_xy[2 * i + 1];
        double point_x, point_y, factor = 1.0;
        double P[16], fa, ra;
        camera_projection(s, c, f, P, &fa, &ra);
        film_fit_marker(p->cam_film_fit[c], fa, ra, &mkr_x, &mkr_y);
        const int ct = p->cam_tfm[c];
        const int bt = p->bnd_tfm[p->mkr_bnd[g]];
        const double *cw = &s->tfm_world[((size_t)ct * F + f) * 16];
        const double *bw = &s->tfm_world[((size_t)bt * F + f) * 16];
        double bp[3] = {bw[3], bw[7], bw[11]};
        double cw_rs[16];
        const int rs = rs_on(s, c);
        if (rs) { /* this observation's scanline pose (both modes) */
            rs_camera_world(s, c, f, p->obs_xy[2 * i + 1], cw_rs);
            cw = cw_rs;
        }
        if (rs && s->o->scene_graph_mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
            double xy[2];
            ref_reproject(cw, P, bp, xy);
            point_x = xy[0];
            point_y = xy[1];
        } else if (s->o->scene_graph_mode == MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
            const double *pt = &s->pts[((size_t)k * F + f) * 2];
            point_x = pt[0];
            point_y = pt[1];
        } else {
            double xy[2];
            ref_reproject(cw, P, bp, xy);
            point_x = xy[0];
            point_y = xy[1];
            /* Behind-camera factor (adjust_measureErrors.cpp:262-270). */
            double cam_pos[3] = {cw[3] / cw[15], cw[7] / cw[15], cw[11] / cw[15]};
            double cdir[3] = {-cw[2], -cw[6], -cw[10]};
            double cl = sqrt(cdir[0] * cdir[0] + cdir[1] * cdir[1] + cdir[2] * cdir[2]);
            double bdir[3] = {bp[0] - cam_pos[0], bp[1] - cam_pos[1], bp[2] - cam_pos[2]};
            double bl = sqrt(bdir[0] * bdir[0] + bdir[1] * bdir[1] + bdir[2] * bdir[2]);
            double dot = (cdir[0] / cl) * (bdir[0] / bl) + (cdir[1] / cl) * (bdir[1] / bl) +
                         (cdir[2] / cl) * (bdir[2] / bl);
            if (dot < 0.0) factor = 1e+6;
        }
        apply_lens_obs(s, i, &point_x, &point_y);
        if (s->obs_pts) {
            s->obs_pts[2 * i] = point_x;
            s->obs_pts[2 * i + 1] = point_y;
            s->obs_mkr[2 * i] = mkr_x;
            s->obs_mkr[2 * i + 1] = mkr_y;
        }
        double w = sqrt(p->obs_weight[i]);
        double dx = fabs(mkr_x - point_x), dy = fabs(mkr_y - point_y);
        double dxp = dx * image_width, dyp = dy * image_width;
        errors[2 * i] = dxp * w * factor;
        errors[2 * i + 1] = dyp * w * factor;
        s->err_user[2 * i] = dxp * factor;
        s->err_user[2 * i + 1] = dyp * factor;
        s->err_dist[i] = sqrt((dx * dx) + (dy * dy)) * image_width;
    }
    /* Stiffness then smoothness rows (adjust_measureErrors.cpp:311-387), Maya
     * DAG path only (the MM Scene Graph path leaves them untouched, :518);
     * every call re-measures them, whatever the frame mask. */
    if (s->o->scene_graph_mode != MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) {
        const int base = 2 * p->num_obs;
        for (int i = 0; i < p->num_stiff; ++i) {
            const int a = p->stiff_attr[i];
            const double v = attr_value(s, a, p->stiff_frame ? p->stiff_frame[i] : 0, 0.);
            const double e = ((1.0 / gaussian(v, p->stiff_value[i], p->stiff_variance[i])) - 1.0);
            s->err_user[base + i] = e * p->stiff_weight[i];
            errors[base + i] = e * p->stiff_weight[i];
        }
        const int base2 = base + p->num_stiff;
        for (int i = 0; i < p->num_smooth; ++i) {
            const int a = p->smooth_attr[i];
            const double v = attr_value(s, a, p->smooth_frame ? p->smooth_frame[i] : 0, 0.);
            const double e =
                ((1.0 / gaussian(v, p->smooth_value[i], p->smooth_variance[i])) - 1.0);
            s->err_user[base2 + i] = e * p->smooth_weight[i];
            errors[base2 + i] = e * p->smooth_weight[i];
        }
    }
    if (s->o->robust_loss)
        apply_loss(s->m, errors, s->o->robust_loss_type, s->o->robust_loss_scale);
}

/* setParameters (adjust_setParameters.cpp:174-276). */
static void set_parameters(ref_scene *s, const double *x) {
    const mmba_problem *p = s->p;
    for (int i = 0; i < p->num_params; ++i) {
        double v = ref_param_internal_to_external(x[i], p->param_min[i], p->param_max[i],
                                                  p->param_offset[i], p->param_scale[i]);
        int a = p->param_attr[i];
        int f = p->param_frame[i];
        size_t idx = p->attr_offset[a] + (p->attr_animated[a] ? (f < 0 ? 0 : f) : 0);
        s->attr[idx] = v;
    }
    s->lens_set = 1;
}

/* calculateParameterDelta (adjust_solveFunc.cpp:148-180). */
static double param_delta(double value, double delta, double sign, double xmin,
                          double xmax) {
    double new_sign = sign;
    if ((value + delta) > xmax) new_sign = -1;
    if ((value - delta) < xmin) new_sign = 1;
    return delta * new_sign;
}

static void trace_push(ref_scene *s, int m, const double *fvec) {
    if (s->trace && s->trace->count < s->trace->capacity)
        s->trace->fnorm[s->trace->count] = ref_enorm(m, fvec);
    if (s->trace) s->trace->count++;
}

/* solveFunc iflag=1 (adjust_solveFunc.cpp:262-303). */
static int scene_fun(void *c, int m, int n, const double *x, double *fvec) {
    ref_scene *s = (ref_scene *)c;
    (void)n;
    s->func_evals++;
    if (interrupt_requested(s)) return -1; /* adjust_solveFunc.cpp:567-571 */
    set_parameters(s, x);
    measure(s, NULL, fvec);
    trace_push(s, m, fvec);
    return 0;
}

/* solveFunc_calculateJacobianMatrix (adjust_solveFunc.cpp:305-525). */
static int scene_jac_der(void *c, int m, int n, double *x, double *fvec,
                         double *fjac, int ldfjac, int *nfev, int *njev) {
    ref_scene *s = (ref_scene *)c;
    const mmba_problem *p = s->p;
    (void)nfev;
    const double delta = s->o->delta;
    const int F = p->num_frames;
    if (interrupt_requested(s)) { /* solveFunc entry, adjust_solveFunc.cpp:567-571 */
        ++(*njev);
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        if (interrupt_requested(s)) { /* per column, adjust_solveFunc.cpp:321-325 */
            ++(*njev);
            return -1;
        }
        memcpy(s->xa, x, sizeof(double) * n);
        memcpy(s->ea, fvec, sizeof(double) * m);
        const double value = x[i];
        const double xmin = p->param_min[i], xmax = p->param_max[i];
        const double deltaA = param_delta(value, delta, 1, xmin, xmax);
        const char *mask = s->frame_all;
        if (p->param_frame[i] >= 0) {
            memset(s->frame_mask, 0, F);
            s->frame_mask[p->param_frame[i]] = 1;
            if (s->rs_any) { /* the blend reaches the neighbouring frames */
                if (p->param_frame[i] > 0) s->frame_mask[p->param_frame[i] - 1] = 1;
                if (p->param_frame[i] < F - 1) s->frame_mask[p->param_frame[i] + 1] = 1;
            }
            mask = s->frame_mask;
        }
        s->jac_evals++;
        s->xa[i] = s->xa[i] + deltaA;
        set_parameters(s, s->xa);
        measure(s, mask, s->ea);
        double *col = &fjac[(size_t)i * ldfjac];
        if (s->o->auto_diff_type == MMBA_AUTO_DIFF_CENTRAL) {
            const double deltaB = param_delta(value, delta, -1, xmin, xmax);
            if (deltaA == deltaB) {
                const double inv_delta = 1.0 / deltaA;
                for (int j = 0; j < m; ++j) col[j] = (s->ea[j] - fvec[j]) * inv_delta;
            } else {
                memcpy(s->xb, x, sizeof(double) * n);
                memset(s->eb, 0, sizeof(double) * m); /* errorListB(numberOfErrors, 0) */
                s->jac_evals++;
                s->xb[i] = s->xb[i] + deltaB;
                set_parameters(s, s->xb);
                measure(s, mask, s->eb);
                const double inv_delta = 0.5 / (fabs(deltaA) + fabs(deltaB));
                for (int j = 0; j < m; ++j) col[j] = (s->ea[j] - s->eb[j]) * inv_delta;
            }
        } else {
            const double inv_delta = 1.0 / deltaA;
            for (int j = 0; j < m; ++j) col[j] = (s->ea[j] - fvec[j]) * inv_delta;
        }
    }
    ++(*njev);
    return 0;
}

/* lmdif: fdjac2 calls fcn with iflag=2 -> counted as Jacobian calls. */
static int scene_jac_dif(void *c, int m, int n, double *x, double *fvec,
                         double *fjac, int ldfjac, int *nfev, int *njev) {
    ref_scene *s = (ref_scene *)c;
    const double epsmch = DBL_EPSILON;
    const double eps = sqrt(RMAX(fabs(s->o->delta), epsmch));
    for (int j = 0; j < n; ++j) {
        double temp = x[j];
        double h = eps * fabs(temp);
        if (h == 0.) h = eps;
        x[j] = temp + h;
        s->jac_evals++;
        if (interrupt_requested(s)) { /* every fdjac2 call is a solveFunc call */
            x[j] = temp;
            *nfev += n;
            return -1;
        }
        set_parameters(s, x);
        measure(s, NULL, s->ea);
        x[j] = temp;
        for (int i = 0; i < m; ++i) fjac[i + (size_t)j * ldfjac] = (s->ea[i] - fvec[i]) / h;
    }
    *nfev += n;
    ++(*njev);
    return 0;
}

static int validate(const mmba_problem *p, const mmba_options *o) {
    if (!p || !o) return MMBA_ERR_INVALID;
    if (p->num_frames <= 0 || p->num_obs <= 0 || p->num_params <= 0) return MMBA_ERR_INVALID;
    for (int i = 0; i < p->num_params; ++i) {
        int a = p->param_attr[i];
        if (a < 0 || a >= p->num_attrs) return MMBA_ERR_INVALID;
        if (p->attr_animated[a] && p->param_frame[i] < 0) return MMBA_ERR_INVALID;
    }
    return MMBA_OK;
}

static void scene_init(ref_scene *s, const mmba_problem *p,
                       const mmba_options *o) {
    memset(s, 0, sizeof(*s));
    s->p = p;
    s->o = o;
    size_t nvals = 0;
    for (int a = 0; a < p->num_attrs; ++a) {
        size_t end = p->attr_offset[a] + (p->attr_animated[a] ? p->num_frames : 1);
        if (end > nvals) nvals = end;
    }
    s->attr = (double *)malloc(sizeof(double) * (nvals ? nvals : 1));
    memcpy(s->attr, p->attr_values, sizeof(double) * nvals);
    s->tfm_world = (double *)malloc(sizeof(double) * 16 * (size_t)p->num_transforms * p->num_frames);
    s->pts = (double *)malloc(sizeof(double) * 2 * ((size_t)p->num_markers * p->num_frames + 1));
    s->m = 2 * p->num_obs + p->num_stiff + p->num_smooth;
    s->err_user = (double *)calloc((size_t)s->m, sizeof(double));
    s->err_dist = (double *)calloc((size_t)p->num_obs, sizeof(double));
    s->frame_all = (char *)malloc(p->num_frames);
    memset(s->frame_all, 1, p->num_frames);
    s->frame_mask = (char *)malloc(p->num_frames);
    s->xa = (double *)malloc(sizeof(double) * p->num_params);
    s->xb = (double *)malloc(sizeof(double) * p->num_params);
    s->ea = (double *)calloc((size_t)s->m, sizeof(double));
    s->eb = (double *)calloc((size_t)s->m, sizeof(double));
    for (int c = 0; c < p->num_cameras; ++c) s->rs_any |= rs_on(s, c);
}

/* B4: FlatScene::evaluate lists markers camera by camera, each camera's in
 * marker order (flat.rs:271-356), and measureErrors_mmSceneGraph reads the
 * point and marker lists at markerIndex * F + frameIndex
 * (adjust_measureErrors.cpp:454-459): observation (marker i, frame f) sees
 * the i-th marker of that listing at f.  Its x,y there: mkr_frame_xy, else the
 * observation of that marker at f (none: refused). */
static int b4_build(ref_scene *s) {
    const mmba_problem *p = s->p;
    const int K = p->num_markers, F = p->num_frames, M = p->num_obs;
    s->geo_mkr = (int *)malloc(sizeof(int) * (size_t)(M > 0 ? M : 1));
    s->geo_xy = (double *)malloc(sizeof(double) * 2 * (size_t)(M > 0 ? M : 1));
    for (int i = 0; i < M; ++i) {
        s->geo_mkr[i] = p->obs_marker[i];
        s->geo_xy[2 * i] = p->obs_xy[2 * i];
        s->geo_xy[2 * i + 1] = p->obs_xy[2 * i + 1];
    }
    if (s->o->scene_graph_mode != MMBA_SCENE_GRAPH_MM_SCENE_GRAPH) return MMBA_OK;
    int *flat = (int *)malloc(sizeof(int) * (size_t)(K > 0 ? K : 1));
    int n = 0, moved = 0;
    for (int c = 0; c < p->num_cameras; ++c)
        for (int k = 0; k < K; ++k)
            if (p->mkr_cam[k] == c) flat[n++] = k;
    for (int k = 0; k < K; ++k) moved |= flat[k] != k;
    int rc = MMBA_OK;
    if (moved && s->rs_any) rc = MMBA_ERR_UNSUPPORTED;
    for (int i = 0; moved && rc == MMBA_OK && i < M; ++i) {
        const int k = flat[p->obs_marker[i]], f = p->obs_frame[i];
        s->geo_mkr[i] = k;
        if (k == p->obs_marker[i]) continue;
        const double *xy = NULL;
        if (p->mkr_frame_xy) {
            xy = &p->mkr_frame_xy[2 * ((size_t)k * F + f)];
        } else {
            for (int j = 0; j < M && !xy; ++j)
                if (p->obs_marker[j] == k && p->obs_frame[j] == f) xy = &p->obs_xy[2 * j];
            if (!xy) rc = MMBA_ERR_UNSUPPORTED;
        }
        if (xy) {
            s->geo_xy[2 * i] = xy[0];
            s->geo_xy[2 * i + 1] = xy[1];
        }
    }
    free(flat);
    return rc;
}

/* scene_init + the B3 lens table and the B4 listing (the parts that can refuse) */
static int scene_open(ref_scene *s, const mmba_problem *p, const mmba_options *o) {
    scene_init(s, p, o);
    const int rc = b3_build(s);
    return rc != MMBA_OK ? rc : b4_build(s);
}

static void scene_free(ref_scene *s) {
    free(s->lens_src);
    free(s->geo_mkr);
    free(s->geo_xy);
    free(s->attr);
    free(s->tfm_world);
    free(s->pts);
    free(s->err_user);
    free(s->err_dist);
    free(s->frame_all);
    free(s->frame_mask);
    free(s->xa);
    free(s->xb);
    free(s->ea);
    free(s->eb);
}

/* compute_error_stats (adjust_base.cpp:346-372). */
static void error_stats(const double *dist, int M, double *avg, double *mn,
                        double *mx) {
    double a = 0., lo = DBL_MAX, hi = -0.0;
    for (int i = 0; i < M; ++i) {
        double e = dist[i];
        if (!isfinite(e)) continue;
        a += e;
        if (e < lo) lo = e;
        if (e > hi) hi = e;
    }
    a /= M;
    *avg = a;
    *mn = lo;
    *mx = hi;
}

int ref_measure(const mmba_problem *prob, const mmba_options *opt,
                const double *x, double *fvec, double *err_user,
                double *err_dist, double *avg_min_max) {
    int rc = validate(prob, opt);
    if (rc) return rc;
    ref_scene s;
    rc = scene_open(&s, prob, opt);
    if (rc) {
        scene_free(&s);
        return rc;
    }
    const int m = s.m;
    double *f = (double *)calloc((size_t)m, sizeof(double));
    if (x) set_parameters(&s, x);
    measure(&s, NULL, f);
    if (fvec) memcpy(fvec, f, sizeof(double) * m);
    if (err_user) memcpy(err_user, s.err_user, sizeof(double) * m);
    if (err_dist) memcpy(err_dist, s.err_dist, sizeof(double) * prob->num_obs);
    if (avg_min_max)
        error_stats(s.err_dist, prob->num_obs, &avg_min_max[0], &avg_min_max[1], &avg_min_max[2]);
    free(f);
    scene_free(&s);
    return MMBA_OK;
}

/* Per-observation reprojection (the out_point_list / out_marker_list of
 * FlatScene::evaluate, flat.rs:271-356, and the point / marker pair
 * measureErrors compares, adjust_measureErrors.cpp:444-472), lens applied. */
int ref_reproject_obs(const mmba_problem *prob, const mmba_options *opt, const double *x,
                      double *point_xy, double *marker_xy) {
    int rc = validate(prob, opt);
    if (rc) return rc;
    ref_scene s;
    rc = scene_open(&s, prob, opt);
    if (rc) {
        scene_free(&s);
        return rc;
    }
    const int m = s.m;
    double *f = (double *)calloc((size_t)m, sizeof(double));
    s.obs_pts = point_xy;
    s.obs_mkr = marker_xy;
    if (x) set_parameters(&s, x);
    measure(&s, NULL, f);
    free(f);
    s.obs_pts = s.obs_mkr = NULL;
    scene_free(&s);
    return MMBA_OK;
}

int ref_jacobian(const mmba_problem *prob, const mmba_options *opt,
                 const double *x, double *fvec, double *fjac) {
    int rc = validate(prob, opt);
    if (rc) return rc;
    ref_scene s;
    rc = scene_open(&s, prob, opt);
    if (rc) {
        scene_free(&s);
        return rc;
    }
    const int m = s.m, n = prob->num_params;
    double *xx = (double *)malloc(sizeof(double) * n);
    memcpy(xx, x, sizeof(double) * n);
    scene_fun(&s, m, n, xx, fvec);
    int nfev = 0, njev = 0;
    if (opt->solver_type == MMBA_SOLVER_CMINPACK_LMDIF)
        scene_jac_dif(&s, m, n, xx, fvec, fjac, m, &nfev, &njev);
    else
        scene_jac_der(&s, m, n, xx, fvec, fjac, m, &nfev, &njev);
    free(xx);
    scene_free(&s);
    return MMBA_OK;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* solveFrames (adjust_base.cpp:713-1287) from the initial measurement to
 * accept-only-better, with solve_3d_cminpack_lmder|lmdif in the middle. */
int ref_solve(const mmba_problem *prob, const mmba_options *opt,
              double *x_inout, double *fvec_out, double *err_user_out,
              double *err_dist_out, mmba_result *res, mmba_trace *trace) {
    int rc = validate(prob, opt);
    if (rc) return rc;
    const int m = 2 * prob->num_obs + prob->num_stiff + prob->num_smooth;
    const int n = prob->num_params, M = prob->num_obs;
    if (n > m) return MMBA_ERR_INVALID; /* adjust_base.cpp:864-881 */
    double t0 = now_s();
    ref_scene s;
    rc = scene_open(&s, prob, opt);
    if (rc) {
        scene_free(&s);
        return rc;
    }
    if (trace) trace->count = 0;
    mmba_result r;
    memset(&r, 0, sizeof(r));

    double *fvec = (double *)calloc(m, sizeof(double));
    double init_avg = 0., init_min = 0., init_max = 0.;
    if (opt->accept_only_better && !opt->initial_error_given) {
        measure(&s, NULL, fvec); /* scene values, before parameters are set */
        error_stats(s.err_dist, M, &init_avg, &init_min, &init_max);
    } else if (opt->accept_only_better) {
        init_avg = opt->initial_error_avg; /* measured by the caller */
    }
    r.error_initial_avg = init_avg;
    r.error_avg = init_avg;
    r.error_min = init_min;
    r.error_max = init_max;

    double *x0 = (double *)malloc(sizeof(double) * n);
    memcpy(x0, x_inout, sizeof(double) * n);
    double *x = (double *)malloc(sizeof(double) * n);
    memcpy(x, x_inout, sizeof(double) * n);
    const int ldfjac = m;
    double *fjac = (double *)calloc((size_t)m * n, sizeof(double));
    double *diag = (double *)malloc(sizeof(double) * n);
    for (int j = 0; j < n; ++j) /* paramWeightList */
        diag[j] = prob->param_weight ? prob->param_weight[j] : 1.0;
    int *ipvt = (int *)malloc(sizeof(int) * n);
    double *qtf = (double *)malloc(sizeof(double) * n);
    double *wa1 = (double *)malloc(sizeof(double) * n);
    double *wa2 = (double *)malloc(sizeof(double) * n);
    double *wa3 = (double *)malloc(sizeof(double) * n);
    double *wa4 = (double *)calloc((size_t)m, sizeof(double));
    s.trace = trace;
    const int mode = opt->auto_param_scale == 1 ? 1 : 2;
    const double factor = opt->tau * 100.0;
    int nfev = 0, njev = 0;
    int info = lm_core(scene_fun,
                       opt->solver_type == MMBA_SOLVER_CMINPACK_LMDIF ? scene_jac_dif : scene_jac_der,
                       &s, m, n, x, fvec, fjac, ldfjac, opt->eps1, opt->eps2, opt->eps3,
                       opt->iter_max, diag, mode, factor, &nfev, &njev, ipvt, qtf, wa1,
                       wa2, wa3, wa4);
    r.error_final = ref_enorm(m, fvec);
    r.reason_number = info;
    r.iterations = nfev;
    r.function_evals = s.func_evals;
    r.jacobian_evals = s.jac_evals;
    r.outer_iterations = njev;
    r.success = s.func_evals > 0;
    r.user_interrupted = s.interrupted; /* out_cmdResult.solverResult.user_interrupted */

    /* Stats from the last measurement (B13), then accept-only-better. */
    double avg, mn, mx;
    error_stats(s.err_dist, M, &avg, &mn, &mx);
    r.error_avg = avg;
    r.error_min = mn;
    r.error_max = mx;
    int better = 1;
    if (opt->accept_only_better) better = avg <= init_avg;
    r.error_is_better = better;
    if (err_user_out) memcpy(err_user_out, s.err_user, sizeof(double) * m);
    if (err_dist_out) memcpy(err_dist_out, s.err_dist, sizeof(double) * M);
    if (fvec_out) memcpy(fvec_out, fvec, sizeof(double) * m);
    /* lmder leaves the solved x in paramList (adjust_cminpack_lmder.cpp:128);
     * solveFrames writes it back only when error_is_better (:1231-1244) */
    memcpy(x_inout, x, sizeof(double) * n);
    (void)x0;

    /* RMS at the returned parameters (build's own metric). */
    {
        ref_scene s2;
        scene_open(&s2, prob, opt);
        set_parameters(&s2, x_inout);
        measure(&s2, NULL, wa4);
        double acc = 0.;
        for (int i = 0; i < M; ++i) acc += s2.err_dist[i] * s2.err_dist[i];
        r.error_rms = sqrt(acc / M);
        scene_free(&s2);
    }
    r.num_trace = trace ? trace->count : 0;
    r.time_solve_s = now_s() - t0;
    if (res) *res = r;

    free(fvec); free(x0); free(x); free(fjac); free(diag); free(ipvt); free(qtf);
    free(wa1); free(wa2); free(wa3); free(wa4);
    scene_free(&s);
    return MMBA_OK;
}
