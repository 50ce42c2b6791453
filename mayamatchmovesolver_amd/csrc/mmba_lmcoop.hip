// mmba_lmcoop.hip -- the whole lmder / lmdif solve as ONE cooperative launch
// for block-diagonal plans (every parameter belongs to one camera-frame, no
// solved bundle, no global parameter: the C2 scene, 120 frames x 7
// parameters x ~1,650 observations).
//
// The host-driven Plan::solve spends ~10 launches and one host
// synchronisation per outer iteration on such a plan (~195 us per LM
// iteration, almost all of it launch and decision latency).  Here workgroup
// g owns a contiguous range of camera-frames: their parameters, records,
// J^T J / J^T f blocks and damped solves stay in its LDS, and every scalar
// the MINPACK control flow needs (||f||, ||D x||, gnorm, ||D xs||, the
// Newton correction, ||J p||, the pivot flag) is a grid reduction: each
// workgroup stores its partials write-through, counts itself in on one
// agent-scope counter, polls it, and then every workgroup sums the G
// partials in the same fixed order -- so every workgroup takes identical
// decisions (the lmder / lmpar control flow of Plan::solve and lmpar_ne,
// mmba_lm.cpp; oracle/refcpu.c lm_core / lmpar; MINPACK-1 lmder.f).
//
// Hand-off (MI355X guide, "Valid forms", first table row): partial stores
// sc1 (write-through), every storing wave drained (vmcnt 0) behind a
// workgroup barrier, one lane's agent-scope atomic add, an sc1 poll of the
// counter, a workgroup barrier, sc1 loads of every partial.  The launch is
// cooperative (hipLaunchCooperativeKernel), so every workgroup is resident
// and every poll ends; each poll is also bounded (a timeout aborts the
// solve on every workgroup through an abort word and is reported).
#include <cfloat>

#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

namespace {

constexpr int CT = 256;    // threads per workgroup
constexpr int CPB = 4;     // camera-frames per workgroup (one wave each in lmpar)
constexpr int NFC = 8;     // parameters per camera-frame (lanes of the solve)
constexpr int NRED = 8;    // values per grid reduction

typedef __attribute__((address_space(1))) unsigned long long cg_u64;
typedef __attribute__((address_space(1))) unsigned int cg_u32;

__device__ __forceinline__ void cg_st(double *p, double v) {
    __hip_atomic_store((cg_u64 *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double cg_ld(const double *p) {
    return __longlong_as_double((long long)__hip_atomic_load(
        (cg_u64 *)const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ unsigned cg_ldu(const unsigned *p) {
    return __hip_atomic_load((cg_u32 *)const_cast<unsigned *>(p), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double cg_wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return wave_rdlane(v, 0);
}
__device__ __forceinline__ double cg_wmax(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return wave_rdlane(v, 0);
}

// Augmented Cholesky of one wave (lane i < NF: row i; lane NF: the
// right-hand side), k_batch_lm's chol_aug.
__device__ __forceinline__ void cg_chol_aug(double (&a)[NFC], double &rsl, bool &bad) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < NFC; ++j) {
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
        for (int c = j + 1; c < NFC; ++c) a[c] = fma(-l, wave_rdlane(l, c), a[c]);
    }
}

// Block sums (sum, or max where bit j of MAXMASK is set) of per-thread
// values into gv[0, NV); red: [4][>= NV] scratch.  Static indices only.
template <int NV, unsigned MAXMASK>
__device__ __forceinline__ void cg_block_reduce(const double (&v)[NV], double (*red)[4 * NRED + 12],
                                                double *gv) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
        const bool mx = (MAXMASK >> j) & 1u;
        const double r = mx ? cg_wmax(v[j]) : cg_wsum(v[j]);
        if (lane == 0) red[wv][j] = r;
    }
    __syncthreads();
    if (threadIdx.x < NV) {
        const int t = threadIdx.x;
        const bool mx = (MAXMASK >> t) & 1u;
        const double a0 = red[0][t], a1 = red[1][t], a2 = red[2][t], a3 = red[3][t];
        gv[t] = mx ? fmax(fmax(a0, a1), fmax(a2, a3)) : (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
}

}  // namespace

// One cooperative launch: the solve of Plan::solve from x0's evaluation to
// termination.  The caller has reset the attribute block, built the bundle
// records and (accept-only-better) enqueued the initial measurement.
__global__ void __launch_bounds__(CT) k_lm_coop(DevProblem P, CoopArgs A) {
    constexpr int KA = NFC * (NFC + 1) / 2, KJ = KA + NFC;
    __shared__ double s_rec[CPB][NFC + 1][CAMREC];
    __shared__ double s_A[CPB][NFC * NFC];
    __shared__ double s_g[CPB * NFC], s_x[CPB * NFC], s_diag[CPB * NFC], s_xs[CPB * NFC];
    __shared__ double s_wa1[CPB * NFC], s_wa2[CPB * NFC], s_extp[CPB * NFC], s_step[CPB * NFC];
    __shared__ int s_p[CPB * NFC];
    __shared__ long long s_vidx[CPB * NFC];
    static_assert(KJ <= 4 * NRED + 12, "reduction scratch");
    __shared__ double s_red[4][4 * NRED + 12];
    __shared__ double s_gv[NRED];  // this workgroup's grid-reduction partials, then the totals
    __shared__ int s_abort;

    const int G = gridDim.x, g = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int cf0 = A.cf_off[g], ncl = A.cf_off[g + 1] - cf0;  // ncl <= CPB
    const bool lmder = A.solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const double eps_dif = sqrt(fmax(fabs(A.delta), DBL_EPSILON));
    const Override none{-1, 0.};

    // local parameter k = c * NFC + a: parameter a of camera-frame cf0 + c
    if (tid < CPB * NFC) {
        const int c = tid / NFC, a = tid % NFC;
        int p = -1;
        if (c < ncl && a < P.cf_pc[cf0 + c]) p = P.cf_var_param[P.cf_var_off[cf0 + c] + 1 + a];
        s_p[tid] = p;
        if (p >= 0) {
            const int at = P.p_attr[p];
            s_vidx[tid] = P.attr_off[at] + (P.attr_anim[at] ? P.p_frame[p] : 0);
            s_x[tid] = A.x[p];
            s_diag[tid] = A.mode == 2 ? A.pweight[p] : 0.;
        } else {
            s_vidx[tid] = -1;
            s_x[tid] = 0.;
            s_diag[tid] = 0.;
        }
    }
    if (tid == 0) s_abort = 0;
    __syncthreads();

    // ---- grid reduction: nv values in s_gv (sum, or max where is_max) ----
    unsigned round = 0;
    auto grid_reduce = [&](int nv, unsigned maxmask) {
        double *part = A.part + (size_t)(round & 1) * G * NRED;
        if (tid < nv) cg_st(&part[(size_t)g * NRED + tid], s_gv[tid]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(A.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = (round + 1) * (unsigned)G;
            for (unsigned spins = 0;; ++spins) {
                if (cg_ldu(A.ctr) >= target) break;
                if (cg_ldu(A.abort) != 0u || spins > (1u << 24)) {
                    __hip_atomic_store((cg_u32 *)A.abort, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    s_abort = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        // wave v < nv sums value v over the G workgroups: lane l takes
        // workgroups l, l + 64, ... in order, then a fixed xor tree (the
        // same bits on every workgroup)
        for (int v = wv; v < nv; v += CT / 64) {
            const bool mx = (maxmask >> v) & 1u;
            double a = mx ? -DBL_MAX : 0.;
            for (int b = lane; b < G; b += 64) {
                const double q = cg_ld(&part[(size_t)b * NRED + v]);
                a = mx ? fmax(a, q) : a + q;
            }
            a = mx ? cg_wmax(a) : cg_wsum(a);
            if (lane == 0) s_red[0][v] = a;
        }
        __syncthreads();
        if (tid < nv) s_gv[tid] = s_red[0][tid];
        __syncthreads();
        ++round;
        return s_abort != 0;
    };
    auto record = [&](int c, int k, double *rec) {
        const int cf = cf0 + c;
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
    // setParameters of this workgroup's parameters at xv (its records read
    // them next; no other workgroup reads them)
    auto set_params = [&](const double *xv) {
        if (tid < CPB * NFC && s_p[tid] >= 0) {
            const int p = s_p[tid];
            P.attr_val[s_vidx[tid]] =
                int_to_ext(xv[tid], P.p_min[p], P.p_max[p], P.p_off[p], P.p_scale[p]);
        }
        __threadfence();
        __syncthreads();
        __threadfence();
    };

    // measureErrors at xv: fvec -> fo, errorList -> eu / ed, distances -> dist;
    // partials [||f||^2, ||J p||^2 (pv)] -> s_gv[0, 1]
    auto eval = [&](const double *xv, const double *pv, double *fo, double *dist) {
        set_params(xv);
        if (tid < ncl) record(tid, -1, s_rec[tid][0]);
        __syncthreads();
        double v[2] = {0., 0.};
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            const int pc = P.cf_pc[cf];
            for (int i = P.cf_obs_off[cf] + tid; i < P.cf_obs_off[cf + 1]; i += CT) {
                const Resid r = resid_at(i, s_rec[c][0]);
                fo[2 * i] = r.ex;
                fo[2 * i + 1] = r.ey;
                A.eu[2 * i] = r.ux;
                A.eu[2 * i + 1] = r.uy;
                A.ed[i] = r.dist;
                dist[i] = r.dist;
                v[0] += r.ex * r.ex + r.ey * r.ey;
                if (pv) {
                    const double *Jr = &A.J[(size_t)i * 2 * NFC];
                    double ax = 0., ay = 0.;
                    for (int a = 0; a < pc; ++a) {
                        ax += Jr[2 * a] * pv[c * NFC + a];
                        ay += Jr[2 * a + 1] * pv[c * NFC + a];
                    }
                    v[1] += ax * ax + ay * ay;
                }
            }
        }
        cg_block_reduce<2, 0u>(v, s_red, s_gv);
    };

    // FD Jacobian at s_x: J^T J blocks -> s_A, J^T f -> s_g, rows -> A.J;
    // errorList / errorDistanceList of the frame's stale column (B13)
    auto jacobian = [&]() {
        if (tid < CPB * NFC && s_p[tid] >= 0) {
            const int p = s_p[tid];
            const double v = s_x[tid], xmin = P.p_min[p], xmax = P.p_max[p];
            const double off = P.p_off[p], sc = P.p_scale[p];
            double st;
            const double xp = fd_point(v, xmin, xmax, A.solver_type, A.delta, eps_dif, st);
            s_step[tid] = st;
            s_extp[tid] = int_to_ext(xp, xmin, xmax, off, sc);
            P.attr_val[s_vidx[tid]] = int_to_ext(v, xmin, xmax, off, sc);
        }
        __threadfence();
        __syncthreads();
        __threadfence();
        // records: thread c (1 + NFC) + k: camera-frame c, k = 0 base, k > 0 variant k - 1
        if (tid < CPB * (NFC + 1)) {
            const int c = tid / (NFC + 1), k = tid % (NFC + 1);
            if (c < ncl && (k == 0 || s_p[c * NFC + k - 1] >= 0))
                record(c, k == 0 ? -1 : c * NFC + k - 1, s_rec[c][k]);
        }
        for (int t = tid; t < CPB * NFC * NFC; t += CT) s_A[t / (NFC * NFC)][t % (NFC * NFC)] = 0.;
        if (tid < CPB * NFC) s_g[tid] = 0.;
        __syncthreads();
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            const int pc = P.cf_pc[cf];
            const int pstale = A.stale[P.cf_frame[cf]];
            double acc[KJ];
#pragma unroll
            for (int q = 0; q < KJ; ++q) acc[q] = 0.;
            for (int i = P.cf_obs_off[cf] + tid; i < P.cf_obs_off[cf + 1]; i += CT) {
                const Resid r0 = resid_at(i, s_rec[c][0]);
                Resid rs = r0;
                double jx[NFC], jy[NFC];
#pragma unroll
                for (int a = 0; a < NFC; ++a) {
                    jx[a] = 0.;
                    jy[a] = 0.;
                    if (a < pc) {
                        const int k = c * NFC + a;
                        const Resid r = resid_at(i, s_rec[c][1 + a]);
                        const double st = s_step[k];
                        if (lmder) {  // inv_delta, multiplied (adjust_solveFunc.cpp:395-402)
                            jx[a] = (r.ex - r0.ex) * st;
                            jy[a] = (r.ey - r0.ey) * st;
                        } else {      // h, divided (fdjac2)
                            jx[a] = (r.ex - r0.ex) / st;
                            jy[a] = (r.ey - r0.ey) / st;
                        }
                        if (s_p[k] == pstale) rs = r;
                    }
                }
                double *Jr = &A.J[(size_t)i * 2 * NFC];
#pragma unroll
                for (int a = 0; a < NFC; ++a) {
                    if (a < pc) {
                        Jr[2 * a] = jx[a];
                        Jr[2 * a + 1] = jy[a];
                    }
#pragma unroll
                    for (int b2 = 0; b2 <= a; ++b2)
                        acc[a * (a + 1) / 2 + b2] += jx[a] * jx[b2] + jy[a] * jy[b2];
                    acc[KA + a] += jx[a] * r0.ex + jy[a] * r0.ey;
                }
                // errorList / errorDistanceList as the frame's last FD column
                // left them (the others hold the values at x already)
                A.eu[2 * i] = rs.ux;
                A.eu[2 * i + 1] = rs.uy;
                A.ed[i] = rs.dist;
            }
#pragma unroll
            for (int q = 0; q < KJ; ++q) {
                const double r = cg_wsum(acc[q]);
                if (lane == 0) s_red[wv][q] = r;
            }
            __syncthreads();
            if (tid < KJ) {
                const double v = (s_red[0][tid] + s_red[1][tid]) + (s_red[2][tid] + s_red[3][tid]);
                if (tid < KA) {
                    int a = 0, t = tid;
                    while (t > a) {
                        t -= a + 1;
                        ++a;
                    }
                    if (a < pc) {
                        s_A[c][a * NFC + t] = v;
                        s_A[c][t * NFC + a] = v;
                    }
                } else if (tid - KA < pc) {
                    s_g[c * NFC + tid - KA] = v;
                }
            }
            __syncthreads();
        }
    };

    // damped solve of every local camera-frame block (wave c): (A_c + lam
    // D_c^2) xs_c = g_c; partials [||D xs||^2, pivot failure] -> s_gv[0, 1].
    // The factor stays in the wave's registers for newton().
    double fa[NFC];
    double frs = 0., fxs = 0.;
    auto solve = [&](double lam) {
        bool bad = false;
        double dn = 0.;
        if (wv < ncl) {
            const int c = wv;
            const int pc = P.cf_pc[cf0 + c];
            const double dk = lane < pc ? s_diag[c * NFC + lane] : 0.;
#pragma unroll
            for (int col = 0; col < NFC; ++col) {
                double v = 0.;
                if (lane < pc) {
                    if (col < pc && col <= lane) {
                        v = s_A[c][lane * NFC + col];
                        if (col == lane) {
                            v += lam * (dk * dk);
                            if (v == 0.) v = 1.;  // zero column: component 0
                        }
                    }
                } else if (lane < NFC) {
                    v = col == lane ? 1. : 0.;
                } else if (lane == NFC && col < pc) {
                    v = (s_A[c][col * NFC + col] == 0. && lam == 0.) ? 0. : s_g[c * NFC + col];
                }
                fa[col] = v;
            }
            cg_chol_aug(fa, frs, bad);
            double acc = 0.;
#pragma unroll
            for (int j = 0; j < NFC; ++j) {
                const double y = wave_rdlane(fa[j], NFC);
                if (lane == j) acc = y;
            }
#pragma unroll
            for (int i = NFC - 1; i >= 0; --i) {
                const double xi = wave_rdlane(acc, i) * wave_rdlane(frs, i);
                if (lane == i) acc = xi;
#pragma unroll
                for (int j = 0; j < i; ++j) {
                    const double cij = wave_rdlane(fa[j], i);
                    if (lane == j) acc -= cij * xi;
                }
            }
            fxs = lane < pc ? acc : 0.;
            if (lane < NFC) s_xs[c * NFC + lane] = fxs;
            const double v = dk * fxs;
            dn = cg_wsum(lane < pc ? v * v : 0.);
            bad = __builtin_amdgcn_ballot_w64(bad) != 0;
        }
        if (lane == 0) {
            s_red[wv][0] = dn;
            s_red[wv][1] = bad ? 1. : 0.;
        }
        __syncthreads();
        if (tid == 0) {
            double d = 0., b = 0.;
            for (int w = 0; w < CT / 64; ++w)
                if (w < ncl) {
                    d += s_red[w][0];
                    b = fmax(b, s_red[w][1]);
                }
            s_gv[0] = d;
            s_gv[1] = b;
        }
        __syncthreads();
    };
    // sum over local blocks of ||C^-1 v||^2, v = D (D xs / dxnorm), with the
    // factors of the last solve -> s_gv[0]
    auto newton = [&](double dxn) {
        double nsq = 0.;
        if (wv < ncl) {
            const int c = wv;
            const int pc = P.cf_pc[cf0 + c];
            const double dk = lane < pc ? s_diag[c * NFC + lane] : 0.;
            double acc = lane < pc ? dk * ((dk * fxs) / dxn) : 0.;
#pragma unroll
            for (int j = 0; j < NFC; ++j) {
                const double yj = wave_rdlane(acc, j) * wave_rdlane(frs, j);
                if (lane == j)
                    acc = yj;
                else if (lane > j && lane < NFC)
                    acc -= fa[j] * yj;
            }
            nsq = cg_wsum(lane < NFC ? acc * acc : 0.);
        }
        if (lane == 0) s_red[wv][0] = nsq;
        __syncthreads();
        if (tid == 0) {
            double d = 0.;
            for (int w = 0; w < CT / 64; ++w)
                if (w < ncl) d += s_red[w][0];
            s_gv[0] = d;
        }
        __syncthreads();
    };

    int info = 0, nfev = 0, njev = 0, fe = 0, je = 0, ntr = 0;
    bool failed = false, aborted = false;
    int fsel = 0;  // 0: fvec / distances at x in A.f / A.dist; 1: in A.ft / A.distt
    const double p1 = .1, p5 = .5, p25 = .25, p75 = .75, p0001 = 1e-4;
    const double epsmch = DBL_EPSILON;
    double delta = 0., xnorm = 0., par = 0., fnorm = 0., gnorm = 0., ratio = 0.;
    auto trace = [&](double fn) {
        if (g == 0 && tid == 0 && ntr < A.trace_cap) A.trace[ntr] = fn;
        ++ntr;
    };

    nfev = 1;
    fe = 1;
    eval(s_x, nullptr, A.f, A.dist);  // x0 (lmder's first fcn call)
    aborted = grid_reduce(1, 0u);
    fnorm = sqrt(s_gv[0]);
    trace(fnorm);
    int iter = 1;
    while (!aborted) {
        jacobian();
        ++njev;
        je += P.n;
        if (!lmder) nfev += P.n;
        const bool first = iter == 1;
        {
            // lmder after qrfac: column norms, diag, ||D x||, gnorm, rank flag
            double xn = 0., gm = 0., zf = 0.;
            if (tid < CPB * NFC && s_p[tid] >= 0) {
                const int c = tid / NFC, a = tid % NFC;
                const double an = sqrt(s_A[c][a * NFC + a]);
                double dg = s_diag[tid];
                if (A.mode != 2) {
                    if (first) dg = an == 0. ? 1. : an;
                    dg = fmax(dg, an);
                    s_diag[tid] = dg;
                }
                const double v = dg * s_x[tid];
                xn = v * v;
                if (an == 0.) zf = 1.;
                if (fnorm != 0. && an != 0.) gm = fabs((s_g[tid] / fnorm) / an);
            }
            const double vv[3] = {xn, gm, zf};
            cg_block_reduce<3, 6u>(vv, s_red, s_gv);
            aborted = grid_reduce(3, 6u);
        }
        if (aborted) break;
        const bool rank_def = s_gv[2] != 0.;
        if (first) {
            xnorm = sqrt(s_gv[0]);
            delta = A.factor * xnorm;
            if (delta == 0.) delta = A.factor;
        }
        gnorm = fnorm != 0. ? s_gv[1] : 0.;
        __syncthreads();
        if (gnorm <= A.gtol) info = 4;
        if (info != 0) break;
        do {
            // ---- lmpar (lmpar_ne, mmba_lm.cpp) ----
            const double dwarf = DBL_MIN;
            int it = 0;
            solve(0.);
            aborted = grid_reduce(2, 2u);
            if (aborted) break;
            const bool ok0 = s_gv[1] == 0.;
            double dxnorm = ok0 ? sqrt(s_gv[0]) : HUGE_VAL;
            double fp = dxnorm - delta;
            if (fp <= p1 * delta) {
                par = 0.;
            } else {
                double parl = 0.;
                const bool newton0 = !rank_def && ok0;
                // [Newton correction, ||g / D||^2] in one reduction
                double nsq = 0.;
                if (newton0) {
                    newton(dxnorm);
                    nsq = s_gv[0];
                }
                double gd = 0.;
                if (tid < CPB * NFC && s_p[tid] >= 0) {
                    const double q = s_g[tid] / s_diag[tid];
                    gd = q * q;
                }
                const double vv[1] = {gd};
                cg_block_reduce<1, 0u>(vv, s_red, s_gv);
                if (tid == 0) {
                    s_gv[1] = s_gv[0];
                    s_gv[0] = nsq;
                }
                __syncthreads();
                aborted = grid_reduce(2, 0u);
                if (aborted) break;
                if (newton0) {
                    const double temp = sqrt(s_gv[0]);
                    parl = fp / delta / temp / temp;
                }
                const double gdn = sqrt(s_gv[1]);
                double paru = gdn / delta;
                if (paru == 0.) paru = dwarf / fmin(delta, p1);
                par = fmax(par, parl);
                par = fmin(par, paru);
                if (par == 0.) par = gdn / dxnorm;
                for (;;) {
                    ++it;
                    if (par == 0.) par = fmax(dwarf, .001 * paru);
                    solve(par);
                    aborted = grid_reduce(2, 2u);
                    for (int retry = 0; !aborted && s_gv[1] != 0.; ++retry) {
                        // (A + par D^2) is positive definite for par > 0: a
                        // failed factorisation is a breakdown; raise par a
                        // few times, then give up (Plan::solve throws)
                        if (retry == 8) {
                            failed = true;
                            break;
                        }
                        par *= 10.;
                        solve(par);
                        aborted = grid_reduce(2, 2u);
                    }
                    if (aborted || failed) break;
                    dxnorm = sqrt(s_gv[0]);
                    const double temp = fp;
                    fp = dxnorm - delta;
                    if (fabs(fp) <= p1 * delta || (parl == 0. && fp <= temp && temp < 0.) ||
                        it == 10)
                        break;
                    newton(dxnorm);
                    aborted = grid_reduce(1, 0u);
                    if (aborted) break;
                    const double t = sqrt(s_gv[0]);
                    const double parc = fp / delta / t / t;
                    if (fp > 0.) parl = fmax(parl, par);
                    if (fp < 0.) paru = fmin(paru, par);
                    par = fmax(parl, par + parc);
                }
                if (aborted || failed) break;
                if (it == 0) par = 0.;
            }
            // ---- trial point: p = -xs, wa2 = x + p ----
            double pn = 0., xn = 0.;
            if (tid < CPB * NFC && s_p[tid] >= 0) {
                const double st = -s_xs[tid];
                const double w2 = s_x[tid] + st;
                const double dk = s_diag[tid];
                s_wa1[tid] = st;
                s_wa2[tid] = w2;
                pn = dk * st;
                pn *= pn;
                xn = dk * w2;
                xn *= xn;
            }
            {
                const double vv[2] = {pn, xn};
                cg_block_reduce<2, 0u>(vv, s_red, s_gv);
            }
            const double bpn = s_gv[0], bxn = s_gv[1];
            __syncthreads();
            ++nfev;
            ++fe;
            eval(s_wa2, s_wa1, fsel ? A.f : A.ft, fsel ? A.dist : A.distt);
            // [||f||^2, ||J p||^2, ||D p||^2, ||D wa2||^2]
            if (tid == 0) {
                s_gv[2] = bpn;
                s_gv[3] = bxn;
            }
            __syncthreads();
            aborted = grid_reduce(4, 0u);
            if (aborted) break;
            const double fnorm1 = sqrt(s_gv[0]);
            const double pnorm = sqrt(s_gv[2]);
            trace(fnorm1);
            if (iter == 1) delta = fmin(delta, pnorm);
            double actred = -1.;
            if (p1 * fnorm1 < fnorm) {
                const double d1 = fnorm1 / fnorm;
                actred = 1. - d1 * d1;
            }
            const double temp1 = sqrt(s_gv[1]) / fnorm;
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
                if (tid < CPB * NFC) s_x[tid] = s_wa2[tid];
                fsel = 1 - fsel;
                xnorm = sqrt(s_gv[3]);
                fnorm = fnorm1;
                ++iter;
            }
            __syncthreads();
            if (fabs(actred) <= A.ftol && prered <= A.ftol && p5 * ratio <= 1.) info = 1;
            if (delta <= A.xtol * xnorm) info = 2;
            if (fabs(actred) <= A.ftol && prered <= A.ftol && p5 * ratio <= 1. && info == 2)
                info = 3;
            if (info != 0) break;
            if (nfev >= A.maxfev) info = 5;
            if (fabs(actred) <= epsmch && prered <= epsmch && p5 * ratio <= 1.) info = 6;
            if (delta <= epsmch * xnorm) info = 7;
            if (gnorm <= epsmch) info = 8;
            if (info != 0) break;
        } while (ratio < p0001);
        if (aborted || failed || info != 0) break;
    }
    // the accepted point's fvec and distances end in A.f / A.dist, x in A.x
    if (fsel) {
        for (int c = 0; c < ncl; ++c) {
            const int cf = cf0 + c;
            for (int i = P.cf_obs_off[cf] + tid; i < P.cf_obs_off[cf + 1]; i += CT) {
                A.f[2 * i] = A.ft[2 * i];
                A.f[2 * i + 1] = A.ft[2 * i + 1];
                A.dist[i] = A.distt[i];
            }
        }
    }
    if (tid < CPB * NFC && s_p[tid] >= 0) A.x[s_p[tid]] = s_x[tid];
    if (g == 0 && tid == 0) {
        CoopOut o;
        o.fnorm = fnorm;
        o.info = info;
        o.nfev = nfev;
        o.njev = njev;
        o.func_evals = fe;
        o.jac_evals = je;
        o.ntrace = ntr;
        o.failed = failed ? 1 : 0;
        o.aborted = aborted ? 1 : 0;
        *A.out = o;
    }
}

// Camera-frame ranges of the workgroups (<= CPB each, G <= 256); false when
// the plan does not fit the cooperative launch.
bool lm_coop_layout(int ncf, std::vector<int> &cf_off) {
    if (ncf <= 0) return false;
    const int per = (ncf + 255) / 256;
    if (per > CPB) return false;
    const int G = (ncf + per - 1) / per;
    cf_off.resize(G + 1);
    for (int g = 0; g <= G; ++g) cf_off[g] = std::min(ncf, g * per);
    return true;
}

int lm_coop_nfc() { return NFC; }

bool launch_lm_coop(hipStream_t s, const DevProblem &P, const CoopArgs &A, int G) {
    // every workgroup must be resident (grid reductions): a cooperative
    // launch fails instead of deadlocking when they are not
    DevProblem Pc = P;
    CoopArgs Ac = A;
    void *args[] = {&Pc, &Ac};
    const hipError_t e = hipLaunchCooperativeKernel(reinterpret_cast<const void *>(&k_lm_coop),
                                                    dim3(G), dim3(CT), args, 0, s);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

}  // namespace mmba
