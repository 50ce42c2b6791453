// mmba_batch.hip -- per-frame solve mode as ONE launch: one workgroup per
// frame runs that frame's whole MINPACK solve (FrameSolveMode::kPerFrame,
// adjust_base.cpp:1430-1484, each frame a solveFrames call through
// solve_3d_cminpack_lmder / _lmdif).
//
// Without a static parameter the frames share nothing: frame f's sub-problem
// is its observations and its camera-frames' parameters (<= 32), so its
// normal equations are a few small dense blocks and every LM decision is a
// scalar.  Running each frame as a stream of tiny launches leaves the GPU
// launch-bound (the C2 scene: 120 frames x 7 parameters x ~1,650
// observations); here the workgroup keeps the frame's state in LDS and
// loops:
//   evaluation   setParameters (the frame's attribute values), camera
//                records, measureErrors over the frame's observations
//                (errorList / errorDistanceList, ||f||^2, ||J p||^2)
//   Jacobian     the perturbed records of every column, forward differences
//                per observation, per-block J^T J and J^T f (one block
//                reduction per camera-frame), Jacobian rows kept for ||J p||
//   lmpar        wave 0: lane k holds row k of (A + par D^2); augmented
//                Cholesky with register broadcasts, back substitution, the
//                Newton correction -- the same decisions as lmpar_ne
//                (mmba_lm.cpp) and oracle/refcpu.c lmpar
// The control flow of lmder (oracle/refcpu.c ref_solve; mmba_lm.cpp
// Plan::solve) is evaluated identically by every thread from LDS scalars.
#include <cfloat>

#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

namespace {

constexpr int BT = 256;  // threads per frame workgroup

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return wave_rdlane(v, 0);
}

__device__ __forceinline__ double wmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return wave_rdlane(v, 0);
}

// Augmented Cholesky of one wave (mmba_bdiag.hip bd_chol_aug with NF rows):
// lane i < NF holds row i, lane NF the right-hand side; afterwards rows
// hold C (diagonal sqrt(d), rsl = 1/sqrt(d)) and lane NF holds C^-1 b.
template <int NF>
__device__ __forceinline__ void chol_aug(double (&a)[NF], double &rsl, bool &bad) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        double d = wave_rdlane(a[j], j);
        if (!(d > 0.) || !isfinite(d)) {
            bad = true;
            d = 1.;
        }
        const double rs = wave_rsq(d);
        const double l = (lane > j) ? a[j] * rs : 0.;
        a[j] = (lane == j) ? d * rs : (lane > j ? l : a[j]);
        if (lane == j) rsl = rs;
#pragma unroll
        for (int c = j + 1; c < NF; ++c) a[c] = fma(-l, wave_rdlane(l, c), a[c]);
    }
}

struct EvalR {
    double fsq, jp, dsum, dmin, dmax;
};

}  // namespace

template <int NF, int PCT>
__global__ void __launch_bounds__(BT) k_batch_lm(DevProblem P, BatchArgs B) {
    constexpr int KA = PCT * (PCT + 1) / 2;  // lower triangle of one block
    constexpr int K = KA + PCT;              // + J^T f
    constexpr int NREC = BATCH_CFMAX + NF;
    __shared__ double s_rec[NREC * CAMREC];
    __shared__ double s_A[NF * NF];
    __shared__ double s_g[NF], s_x[NF], s_diag[NF], s_wa1[NF], s_wa2[NF], s_extp[NF], s_step[NF];
    __shared__ int s_p[NF];
    __shared__ long long s_vidx[NF];
    __shared__ double s_red[4 * (K > 8 ? K : 8)];
    __shared__ double s_sc[8];
    __shared__ int s_flag;

    const int f = blockIdx.x;
    if (f >= B.nf) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int cf0 = B.fr_cf_off[f], ncl = B.fr_cf_off[f + 1] - cf0;
    const int kp0 = B.fr_par_off[f], nl = B.fr_par_off[f + 1] - kp0;
    const int roff0 = ncl > 0 ? P.cf_roff[cf0] : 0;
    const int plast = B.fr_last[f];
    const double Mf = (double)B.fr_nobs[f];
    const bool lmder = B.solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const double eps_dif = sqrt(fmax(fabs(B.delta), DBL_EPSILON));
    const Override none{-1, 0.};
    const size_t M = (size_t)P.M;

    if (tid < nl) {
        const int p = B.fr_par[kp0 + tid];
        const int a = P.p_attr[p];
        s_p[tid] = p;
        s_vidx[tid] = P.attr_off[a] + (P.attr_anim[a] ? P.p_frame[p] : 0);
        s_x[tid] = B.x[p];
        s_diag[tid] = B.mode == 2 ? B.pweight[p] : 0.;
    }
    __syncthreads();

    // camera record of local camera-frame c (k < 0) or of parameter k's
    // perturbed value (k >= 0) into s_rec slot
    auto record = [&](int c, int k, int slot) {
        const int cf = cf0 + c;
        double *rec = &s_rec[slot * CAMREC];
        if (P.cf_aidx) {
            camera_record_fast(P, cf, k < 0 ? -1ll : s_vidx[k], k < 0 ? 0. : s_extp[k], rec);
        } else {
            const Override ov = k < 0 ? none : Override{P.p_attr[s_p[k]], s_extp[k]};
            camera_record(P, P.cf_cam[cf], P.cf_frame[cf], ov, rec);
        }
    };
    auto resid_at = [&](int i, const double *rec) {
        const int b = P.obs_bnd[i], fr = P.obs_frame[i], cam = P.obs_cam[i];
        double bp[3];
        base_bundle(P, b, fr, bp);
        double lc[MMBA_LENS_NUM_ATTRS];
        int lens = -1;
        const int hl = obs_lens(P, cam, lens);
        if (hl) lens_coeffs(P, lens, fr, none, lc);
        return residual_l(P, rec, bp, P.obs_xy[2 * i], P.obs_xy[2 * i + 1], P.obs_sqrtw[i], hl,
                          lc);
    };
    // attribute writes of this workgroup -> visible to its record threads
    auto publish = [&]() {
        __threadfence();
        __syncthreads();
        __threadfence();
    };
    // block sums of up to 5 scalars (identical on every thread)
    auto block_red5 = [&](double (&v)[5], const bool (&is_max)[5]) {
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const double r = is_max[j] ? wmax(v[j]) : wsum(v[j]);
            if (lane == 0) s_red[wv * 5 + j] = r;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 5; ++j) {
            const double a0 = s_red[j], a1 = s_red[5 + j], a2 = s_red[10 + j], a3 = s_red[15 + j];
            v[j] = is_max[j] ? fmax(fmax(a0, a1), fmax(a2, a3)) : (a0 + a1) + (a2 + a3);
        }
        __syncthreads();
    };

    // measureErrors at xv (set: setParameters first); pv: ||J p||^2 with the
    // last Jacobian's rows; distances -> dist[buf]; stats: sum / min / max
    auto eval = [&](bool set, const double *xv, const double *pv, int buf,
                    bool write_ed = true) -> EvalR {
        if (set) {
            if (tid < nl) {
                const int p = s_p[tid];
                P.attr_val[s_vidx[tid]] =
                    int_to_ext(xv[tid], P.p_min[p], P.p_max[p], P.p_off[p], P.p_scale[p]);
            }
            publish();
        }
        if (tid < ncl) record(tid, -1, tid);
        __syncthreads();
        double v[5] = {0., 0., 0., DBL_MAX, -DBL_MAX};
        double *dist = B.dist + (size_t)buf * M;
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
            const int kc = P.cf_roff[cf] - roff0, pc = P.cf_pc[cf];
            for (int i = o0 + tid; i < o1; i += BT) {
                const Resid r = resid_at(i, &s_rec[c * CAMREC]);
                v[0] += r.ex * r.ex + r.ey * r.ey;
                if (write_ed) B.ed[i] = r.dist;
                dist[i] = r.dist;
                v[2] += r.dist;
                v[3] = fmin(v[3], r.dist);
                v[4] = fmax(v[4], r.dist);
                if (pv) {
                    const double *Jr = &B.J[(size_t)i * 2 * PCMAX];
                    double ax = 0., ay = 0.;
                    for (int a = 0; a < pc; ++a) {
                        ax += Jr[2 * a] * pv[kc + a];
                        ay += Jr[2 * a + 1] * pv[kc + a];
                    }
                    v[1] += ax * ax + ay * ay;
                }
            }
        }
        v[3] = -v[3];
        const bool mx[5] = {false, false, false, true, true};
        block_red5(v, mx);
        return EvalR{v[0], v[1], v[2], -v[3], v[4]};
    };

    // FD Jacobian at s_x: J^T J blocks -> s_A, J^T f -> s_g, rows -> B.J;
    // errorDistanceList as the last column's measureErrors left it (B13)
    auto jacobian = [&]() {
        if (tid < nl) {
            const int p = s_p[tid];
            const double v = s_x[tid], xmin = P.p_min[p], xmax = P.p_max[p];
            const double off = P.p_off[p], sc = P.p_scale[p];
            double st;
            const double xp = fd_point(v, xmin, xmax, B.solver_type, B.delta, eps_dif, st);
            s_step[tid] = st;
            s_extp[tid] = int_to_ext(xp, xmin, xmax, off, sc);
            P.attr_val[s_vidx[tid]] = int_to_ext(v, xmin, xmax, off, sc);
        }
        publish();
        if (tid < ncl) {
            record(tid, -1, tid);
        } else if (tid >= BATCH_CFMAX && tid < BATCH_CFMAX + nl) {
            const int k = tid - BATCH_CFMAX;
            record(P.p_blk[s_p[k]] - cf0, k, tid);
        }
        for (int t = tid; t < NF * NF; t += BT) s_A[t] = 0.;
        if (tid < NF) s_g[tid] = 0.;
        __syncthreads();
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            const int o0 = P.cf_obs_off[cf], o1 = P.cf_obs_off[cf + 1];
            const int kc = P.cf_roff[cf] - roff0, pc = P.cf_pc[cf];
            double acc[K];
#pragma unroll
            for (int q = 0; q < K; ++q) acc[q] = 0.;
            for (int i = o0 + tid; i < o1; i += BT) {
                const Resid r0 = resid_at(i, &s_rec[c * CAMREC]);
                Resid rs = r0;
                double jx[PCT], jy[PCT];
#pragma unroll
                for (int a = 0; a < PCT; ++a) {
                    jx[a] = 0.;
                    jy[a] = 0.;
                    if (a < pc) {
                        const int k = kc + a;
                        const Resid r = resid_at(i, &s_rec[(BATCH_CFMAX + k) * CAMREC]);
                        const double st = s_step[k];
                        if (lmder) {  // inv_delta, multiplied
                            jx[a] = (r.ex - r0.ex) * st;
                            jy[a] = (r.ey - r0.ey) * st;
                        } else {      // h, divided (fdjac2)
                            jx[a] = (r.ex - r0.ex) / st;
                            jy[a] = (r.ey - r0.ey) / st;
                        }
                        if (s_p[k] == plast) rs = r;
                    }
                }
                double *Jr = &B.J[(size_t)i * 2 * PCMAX];
#pragma unroll
                for (int a = 0; a < PCT; ++a) {
                    if (a < pc) {
                        Jr[2 * a] = jx[a];
                        Jr[2 * a + 1] = jy[a];
                    }
#pragma unroll
                    for (int b2 = 0; b2 <= a; ++b2)
                        acc[a * (a + 1) / 2 + b2] += jx[a] * jx[b2] + jy[a] * jy[b2];
                    acc[KA + a] += jx[a] * r0.ex + jy[a] * r0.ey;
                }
                B.ed[i] = rs.dist;
            }
#pragma unroll
            for (int q = 0; q < K; ++q) {
                const double r = wsum(acc[q]);
                if (lane == 0) s_red[wv * K + q] = r;
            }
            __syncthreads();
            if (tid < K) {
                const double v = (s_red[tid] + s_red[K + tid]) + (s_red[2 * K + tid] + s_red[3 * K + tid]);
                if (tid < KA) {
                    int a = 0, t = tid;
                    while (t > a) {
                        t -= a + 1;
                        ++a;
                    }
                    if (a < pc) {
                        s_A[(kc + a) * NF + kc + t] = v;
                        s_A[(kc + t) * NF + kc + a] = v;
                    }
                } else if (tid - KA < pc) {
                    s_g[kc + tid - KA] = v;
                }
            }
            __syncthreads();
        }
    };

    auto poll = [&]() -> bool {
        if (!B.interrupt) return false;
        if (tid == 0) s_flag = __hip_atomic_load(B.interrupt, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        const bool r = s_flag != 0;
        __syncthreads();
        return r;
    };

    int info = 0, nfev = 0, njev = 0, fe = 0, je = 0;
    bool intr = false, failed = false, measured = false, dist_ok = false;
    int dsel = 0;
    double init_avg = 0., init_fnorm = 0.;
    if (B.accept_only_better && !B.initial_error_given) {
        // measureErrors before any parameter is set (adjust_base.cpp:1080-1103)
        const EvalR e = eval(false, s_x, nullptr, 0);
        init_avg = e.dsum / Mf;
        init_fnorm = sqrt(e.fsq);
        measured = true;
    } else if (B.accept_only_better) {
        init_avg = B.initial_error_avg;
    }
    const double p1 = .1, p5 = .5, p25 = .25, p75 = .75, p0001 = 1e-4;
    const double epsmch = DBL_EPSILON;
    double delta = 0., xnorm = 0., par = 0., fnorm = init_fnorm, gnorm = 0., ratio = 0.;
    bool ok = !(nl <= 0 || 2. * Mf < nl || B.ftol < 0. || B.xtol < 0. || B.gtol < 0. ||
                B.maxfev <= 0 || B.factor <= 0.);
    if (ok && B.mode == 2)
        for (int k = 0; k < nl; ++k) ok &= s_diag[k] > 0.;
    if (ok) {
        nfev = 1;
        fe = 1;
        if (poll()) {
            intr = true;
            info = -1;
        }
    }
    if (ok && !intr) {
        // the first evaluation repeats the initial measurement when x0
        // writes back the scene's values bit for bit
        bool same = measured;
        for (int k = 0; k < nl && same; ++k) {
            const int p = s_p[k];
            same = int_to_ext(s_x[k], P.p_min[p], P.p_max[p], P.p_off[p], P.p_scale[p]) ==
                   P.attr_val[s_vidx[k]];
        }
        __syncthreads();
        if (!same) fnorm = sqrt(eval(true, s_x, nullptr, 0).fsq);
        dist_ok = true;
        int iter = 1;
        bool stop = false;
        while (!stop) {
            if (poll()) {  // the Jacobian request (first FD column)
                intr = true;
                info = -1;
                if (lmder) {
                    ++njev;
                } else {
                    je += 1;
                    nfev += nl;
                }
                break;
            }
            jacobian();
            ++njev;
            je += nl;
            if (!lmder) nfev += nl;
            const bool first = iter == 1;
            if (wv == 0) {
                // lmder after qrfac: column norms, diag, ||D x||, gnorm
                double an = 0., dg = 0., xn = 0., gm = 0., zf = 0.;
                if (lane < nl) {
                    an = sqrt(s_A[lane * NF + lane]);
                    dg = s_diag[lane];
                    if (B.mode != 2) {
                        if (first) dg = an == 0. ? 1. : an;
                        dg = fmax(dg, an);
                        s_diag[lane] = dg;
                    }
                    const double v = dg * s_x[lane];
                    xn = v * v;
                    if (an == 0.) zf = 1.;
                    if (fnorm != 0. && an != 0.) gm = fabs((s_g[lane] / fnorm) / an);
                }
                xn = wsum(xn);
                gm = wmax(gm);
                zf = wmax(zf);
                if (lane == 0) {
                    s_sc[0] = xn;
                    s_sc[1] = gm;
                    s_sc[2] = zf;
                }
            }
            __syncthreads();
            const bool rank_def = s_sc[2] != 0.;
            if (first) {
                xnorm = sqrt(s_sc[0]);
                delta = B.factor * xnorm;
                if (delta == 0.) delta = B.factor;
            }
            gnorm = fnorm != 0. ? s_sc[1] : 0.;
            __syncthreads();
            if (gnorm <= B.gtol) info = 4;
            if (info != 0) break;
            do {
                if (wv == 0) {
                    // lmpar on (A + par D^2), lanes = the frame's parameters
                    const double dk = lane < nl ? s_diag[lane] : 0.;
                    double a[NF];
                    double rsl = 0., xsl = 0.;
                    auto factor_solve = [&](double lam) -> bool {
#pragma unroll
                        for (int c = 0; c < NF; ++c) {
                            double v = 0.;
                            if (lane < nl) {
                                if (c < nl && c <= lane) {
                                    v = s_A[lane * NF + c];
                                    if (c == lane) {
                                        v += lam * (dk * dk);
                                        if (v == 0.) v = 1.;  // zero column: component 0
                                    }
                                }
                            } else if (lane < NF) {
                                v = c == lane ? 1. : 0.;
                            } else if (lane == NF && c < nl) {
                                v = (s_A[c * NF + c] == 0. && lam == 0.) ? 0. : s_g[c];
                            }
                            a[c] = v;
                        }
                        bool bad = false;
                        chol_aug<NF>(a, rsl, bad);
                        // x = C^-T y, y = C^-1 b in lane NF
                        double acc = 0.;
#pragma unroll
                        for (int j = 0; j < NF; ++j) {
                            const double y = wave_rdlane(a[j], NF);
                            if (lane == j) acc = y;
                        }
#pragma unroll
                        for (int i = NF - 1; i >= 0; --i) {
                            const double xi = wave_rdlane(acc, i) * wave_rdlane(rsl, i);
                            if (lane == i) acc = xi;
#pragma unroll
                            for (int j = 0; j < i; ++j) {
                                const double cij = wave_rdlane(a[j], i);
                                if (lane == j) acc -= cij * xi;
                            }
                        }
                        xsl = lane < nl ? acc : 0.;
                        return bad;
                    };
                    auto dnorm = [&]() {
                        const double v = dk * xsl;
                        return sqrt(wsum(lane < nl ? v * v : 0.));
                    };
                    // ||C^-1 v||^2, v = D (D xs / dxnorm), with the current factor
                    auto newton = [&](double dxn) {
                        double acc = lane < nl ? dk * ((dk * xsl) / dxn) : 0.;
#pragma unroll
                        for (int j = 0; j < NF; ++j) {
                            const double yj = wave_rdlane(acc, j) * wave_rdlane(rsl, j);
                            if (lane == j)
                                acc = yj;
                            else if (lane > j && lane < NF)
                                acc -= a[j] * yj;
                        }
                        return wsum(lane < NF ? acc * acc : 0.);
                    };
                    const double dwarf = DBL_MIN;
                    double lpar = par;
                    bool fail = false;
                    int it = 0;
                    const bool bad0 = factor_solve(0.);
                    double dxnorm = bad0 ? HUGE_VAL : dnorm();
                    double fp = dxnorm - delta;
                    if (fp <= p1 * delta) {
                        lpar = 0.;
                    } else {
                        double parl = 0.;
                        if (!rank_def && !bad0) {
                            const double t = sqrt(newton(dxnorm));
                            parl = fp / delta / t / t;
                        }
                        const double gk = lane < nl ? s_g[lane] / dk : 0.;
                        const double gdn = sqrt(wsum(gk * gk));
                        double paru = gdn / delta;
                        if (paru == 0.) paru = dwarf / fmin(delta, p1);
                        lpar = fmax(lpar, parl);
                        lpar = fmin(lpar, paru);
                        if (lpar == 0.) lpar = gdn / dxnorm;
                        for (;;) {
                            ++it;
                            if (lpar == 0.) lpar = fmax(dwarf, .001 * paru);
                            bool bad = factor_solve(lpar);
                            for (int retry = 0; bad && !fail; ++retry) {
                                if (retry == 8) {
                                    fail = true;
                                } else {
                                    lpar *= 10.;
                                    bad = factor_solve(lpar);
                                }
                            }
                            if (fail) break;
                            dxnorm = dnorm();
                            const double temp = fp;
                            fp = dxnorm - delta;
                            if (fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) ||
                                it == 10)
                                break;
                            const double t = sqrt(newton(dxnorm));
                            const double parc = fp / delta / t / t;
                            if (fp > 0.) parl = fmax(parl, lpar);
                            if (fp < 0.) paru = fmin(paru, lpar);
                            lpar = fmax(parl, lpar + parc);
                        }
                    }
                    // trial point: p = -xs, wa2 = x + p, ||D p||, ||D wa2||
                    double pn = 0., xn = 0.;
                    if (lane < nl) {
                        const double st = -xsl;
                        const double w2 = s_x[lane] + st;
                        s_wa1[lane] = st;
                        s_wa2[lane] = w2;
                        pn = dk * st;
                        pn *= pn;
                        xn = dk * w2;
                        xn *= xn;
                    }
                    pn = wsum(pn);
                    xn = wsum(xn);
                    if (lane == 0) {
                        s_sc[3] = lpar;
                        s_sc[4] = pn;
                        s_sc[5] = xn;
                        s_sc[6] = fail ? 1. : 0.;
                    }
                }
                __syncthreads();
                par = s_sc[3];
                const double pnorm = sqrt(s_sc[4]), xn2t = s_sc[5];
                failed = s_sc[6] != 0.;
                __syncthreads();
                if (failed) {
                    stop = true;
                    break;
                }
                ++nfev;
                ++fe;
                if (poll()) {
                    intr = true;
                    info = -1;
                    stop = true;
                    break;
                }
                const EvalR e = eval(true, s_wa2, s_wa1, 1 - dsel);
                if (iter == 1) delta = fmin(delta, pnorm);
                const double fnorm1 = sqrt(e.fsq);
                double actred = -1.;
                if (p1 * fnorm1 < fnorm) {
                    const double d1 = fnorm1 / fnorm;
                    actred = 1. - d1 * d1;
                }
                const double temp1 = sqrt(e.jp) / fnorm;
                const double temp2 = (sqrt(par) * pnorm) / fnorm;
                const double prered = temp1 * temp1 + temp2 * temp2 / p5;
                const double dirder = -(temp1 * temp1 + temp2 * temp2);
                ratio = 0.;
                if (prered != 0.) ratio = actred / prered;
                if (ratio <= p25) {
                    double temp;
                    if (actred >= 0.)
                        temp = p5;
                    else
                        temp = p5 * dirder / (dirder + p5 * actred);
                    if (p1 * fnorm1 >= fnorm || temp < p1) temp = p1;
                    delta = temp * fmin(delta, pnorm / p1);
                    par /= temp;
                } else if (par == 0. || ratio >= p75) {
                    delta = pnorm / p5;
                    par = p5 * par;
                }
                if (ratio >= p0001) {
                    if (tid < nl) s_x[tid] = s_wa2[tid];
                    __syncthreads();
                    dsel = 1 - dsel;
                    xnorm = sqrt(xn2t);
                    fnorm = fnorm1;
                    ++iter;
                }
                if (fabs(actred) <= B.ftol && prered <= B.ftol && p5 * ratio <= 1.) info = 1;
                if (delta <= B.xtol * xnorm) info = 2;
                if (fabs(actred) <= B.ftol && prered <= B.ftol && p5 * ratio <= 1. && info == 2)
                    info = 3;
                if (info != 0) {
                    stop = true;
                    break;
                }
                if (nfev >= B.maxfev) info = 5;
                if (fabs(actred) <= epsmch && prered <= epsmch && p5 * ratio <= 1.) info = 6;
                if (delta <= epsmch * xnorm) info = 7;
                if (gnorm <= epsmch) info = 8;
                if (info != 0) {
                    stop = true;
                    break;
                }
            } while (ratio < p0001);
        }
    }
    // TERMINATE: RMS at the returned x, compute_error_stats of the last
    // measured errorDistanceList (B13)
    if (!dist_ok) eval(true, s_x, nullptr, dsel, false);  // distances at x only
    {
        double v[5] = {0., 0., 0., DBL_MAX, -DBL_MAX};
        const double *dist = B.dist + (size_t)dsel * M;
        // errorList / errorDistanceList never written by this solve
        const bool zero_ed = !measured && (nfev == 0 || (intr && nfev <= 1));
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            for (int i = P.cf_obs_off[cf] + tid; i < P.cf_obs_off[cf + 1]; i += BT) {
                double d = B.ed[i];
                if (zero_ed) {
                    d = 0.;
                    B.ed[i] = 0.;
                }
                v[0] += dist[i] * dist[i];
                v[2] += d;
                v[3] = fmin(v[3], d);
                v[4] = fmax(v[4], d);
            }
        }
        v[3] = -v[3];
        const bool mx[5] = {false, false, false, true, true};
        block_red5(v, mx);
        const double rms_sq = v[0];
        const double avg = v[2] / Mf;
        const bool better = B.accept_only_better ? (avg <= init_avg) : true;
        if (better && tid < nl) B.x[s_p[tid]] = s_x[tid];
        if (tid == 0) {
            BatchOut o;
            o.fnorm = fnorm;
            o.init_avg = init_avg;
            o.avg = avg;
            o.mn = -v[3];
            o.mx = v[4];
            o.rms = sqrt(rms_sq / Mf);
            o.info = info;
            o.nfev = nfev;
            o.njev = njev;
            o.func_evals = fe;
            o.jac_evals = je;
            o.interrupted = intr ? 1 : 0;
            o.better = better ? 1 : 0;
            o.failed = failed ? 1 : 0;
            o.measured = measured ? 1 : 0;
            o.pad = 0;
            B.out[f] = o;
        }
    }
}

void launch_batch_lm(hipStream_t s, const DevProblem &P, const BatchArgs &B, int nf_max) {
    if (B.nf <= 0) return;
    if (nf_max <= 8)
        k_batch_lm<8, 8><<<B.nf, BT, 0, s>>>(P, B);
    else if (nf_max <= 16)
        k_batch_lm<16, PCMAX><<<B.nf, BT, 0, s>>>(P, B);
    else
        k_batch_lm<32, PCMAX><<<B.nf, BT, 0, s>>>(P, B);
}

}  // namespace mmba
