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
#include <cstdio>
#include <cstdlib>

#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

namespace {

constexpr int CT = 256;    // threads per workgroup
constexpr int CPB = 4;     // camera-frames owned per workgroup (one wave each in lmpar)
constexpr int SLM = 8;     // camera-frames touched by one workgroup's observation slice
constexpr int NFC = 8;     // parameters per camera-frame (lanes of the solve)
constexpr int NRED = 8;    // values per grid reduction
constexpr int KJC = NFC * (NFC + 1) / 2 + NFC;  // J^T J lower triangle + J^T f

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
//
// Two roles per workgroup g:
//   slice  observations [slice_off[g], slice_off[g + 1]) (balanced, cut
//          anywhere; <= SLM camera-frames: C2's frames hold 63 to 2,643
//          observations): setParameters of their
//          camera-frames, their camera records, residuals, FD Jacobian rows,
//          and J^T J / J^T f partials per camera-frame slot -> A.nep
//   owner  camera-frames g, g + G, ... (<= CPB): sums the slots of each
//          (A.cf_src, in workgroup order), the lmder epilogue of its
//          parameters and the damped solves (one wave per camera-frame);
//          its steps xs go to A.xs for the slices' trial points.
// Both roles keep their own copy of the parameters they touch and update it
// with the same operations, so no owner-to-slice hand-off of x is needed.
template <bool LENS>
__global__ void __launch_bounds__(CT) k_lm_coop(DevProblem P, CoopArgs A) {
    constexpr int KA = NFC * (NFC + 1) / 2, KJ = KJC;
    // slice role
    __shared__ double s_rec[SLM][NFC + 1][CAMREC];
    __shared__ double s_sx[SLM * NFC], s_swa2[SLM * NFC], s_swa1[SLM * NFC];
    __shared__ double s_extp[SLM * NFC], s_step[SLM * NFC];
    __shared__ int s_sp[SLM * NFC];
    __shared__ long long s_vidx[SLM * NFC];
    // owner role
    __shared__ double s_A[CPB][NFC * NFC];
    __shared__ double s_g[CPB * NFC], s_ox[CPB * NFC], s_diag[CPB * NFC], s_xs[CPB * NFC];
    __shared__ double s_owa2[CPB * NFC];
    __shared__ int s_op[CPB * NFC];
    static_assert(KJ <= 4 * NRED + 12, "reduction scratch");
    __shared__ double s_red[4][4 * NRED + 12];
    __shared__ double s_gv[NRED];  // this workgroup's grid-reduction partials, then the totals
    __shared__ int s_abort;

    const int G = gridDim.x, g = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int scf0 = A.slice_cf[g], nsl = A.slice_ncf[g];  // slice camera-frames
    const int so0 = A.slice_off[g], so1 = A.slice_off[g + 1];
    const int ncf = P.ncf;
    int nown = 0;  // owned camera-frames g, g + G, ...
    for (int c = g; c < ncf && nown < CPB; c += G) ++nown;
    const bool lmder = A.solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const double eps_dif = sqrt(fmax(fabs(A.delta), DBL_EPSILON));
    const Override none{-1, 0.};

    // parameter a of local camera-frame c at index c * NFC + a (both roles)
    if (tid < SLM * NFC) {
        const int c = tid / NFC, a = tid % NFC;
        int p = -1;
        if (c < nsl && a < P.cf_pc[scf0 + c]) p = P.cf_var_param[P.cf_var_off[scf0 + c] + 1 + a];
        s_sp[tid] = p;
        s_vidx[tid] = -1;
        s_sx[tid] = 0.;
        if (p >= 0) {
            const int at = P.p_attr[p];
            s_vidx[tid] = P.attr_off[at] + (P.attr_anim[at] ? P.p_frame[p] : 0);
            s_sx[tid] = A.x[p];
        }
    } else if (tid >= 64 && tid < 64 + CPB * NFC) {
        const int k = tid - 64, c = k / NFC, a = k % NFC;
        const int cf = g + c * G;
        int p = -1;
        if (c < nown && a < P.cf_pc[cf]) p = P.cf_var_param[P.cf_var_off[cf] + 1 + a];
        s_op[k] = p;
        s_ox[k] = p >= 0 ? A.x[p] : 0.;
        s_diag[k] = (p >= 0 && A.mode == 2) ? A.pweight[p] : 0.;
    }
    if (tid == 0) s_abort = 0;
    __syncthreads();

    // ---- grid reduction of nv values in s_gv (sum, or max where bit v of
    // maxmask); nv = 0: a plain grid barrier ----
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
        const int cf = scf0 + c;
        if (P.cf_aidx) {
            camera_record_fast(P, cf, k < 0 ? -1ll : s_vidx[k], k < 0 ? 0. : s_extp[k], rec);
        } else {
            const Override ov = k < 0 ? none : Override{P.p_attr[s_sp[k]], s_extp[k]};
            camera_record(P, P.cf_cam[cf], P.cf_frame[cf], ov, rec);
        }
    };
    auto resid_at = [&](int i, const double *rec) {
        const int b = P.obs_bnd[i], fr = P.obs_frame[i];
        double bp[3];
        base_bundle(P, b, fr, bp);
        if constexpr (LENS) {
            double lc[MMBA_LENS_NUM_ATTRS];
            int lens = -1;
            const int hl = obs_lens(P, P.obs_cam[i], lens);
            if (hl) lens_coeffs(P, lens, fr, none, lc);
            return residual_l(P, rec, bp, P.obs_xy[2 * i], P.obs_xy[2 * i + 1], P.obs_sqrtw[i],
                              hl, lc);
        } else {
            return residual_l(P, rec, bp, P.obs_xy[2 * i], P.obs_xy[2 * i + 1], P.obs_sqrtw[i],
                              MMBA_LENS_NONE, nullptr);
        }
    };
    // the slice's observations of local camera-frame c
    auto obs_lo = [&](int c) { return max(so0, P.cf_obs_off[scf0 + c]); };
    auto obs_hi = [&](int c) { return min(so1, P.cf_obs_off[scf0 + c + 1]); };
    // setParameters of the slice's camera-frames at xv (its own records read
    // them next; other workgroups write the same values for shared ones)
    auto set_params = [&](const double *xv) {
        if (tid < SLM * NFC && s_sp[tid] >= 0) {
            const int p = s_sp[tid];
            P.attr_val[s_vidx[tid]] =
                int_to_ext(xv[tid], P.p_min[p], P.p_max[p], P.p_off[p], P.p_scale[p]);
        }
        __threadfence();
        __syncthreads();
        __threadfence();
    };

    // measureErrors of the slice at xv: fvec -> fo, errorList -> eu / ed,
    // distances -> dist; partials [||f||^2, ||J p||^2 (pv)] -> s_gv[0, 1]
    auto eval = [&](const double *xv, const double *pv, double *fo, double *dist) {
        set_params(xv);
        if (tid < nsl) record(tid, -1, s_rec[tid][0]);
        __syncthreads();
        double v[2] = {0., 0.};
        for (int c = 0; c < nsl; ++c) {
            const int pc = P.cf_pc[scf0 + c];
            for (int i = obs_lo(c) + tid; i < obs_hi(c); i += CT) {
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

    // FD Jacobian rows of the slice at s_sx -> A.J; J^T J / J^T f of each
    // slice camera-frame -> A.nep[g * SLM + c] (write-through: the owners read
    // them after the next grid barrier); errorList / errorDistanceList of the
    // frame's stale column (B13)
    auto jacobian = [&]() {
        if (tid < SLM * NFC && s_sp[tid] >= 0) {
            const int p = s_sp[tid];
            const double v = s_sx[tid], xmin = P.p_min[p], xmax = P.p_max[p];
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
        if (tid < SLM * (NFC + 1)) {
            const int c = tid / (NFC + 1), k = tid % (NFC + 1);
            if (c < nsl && (k == 0 || s_sp[c * NFC + k - 1] >= 0))
                record(c, k == 0 ? -1 : c * NFC + k - 1, s_rec[c][k]);
        }
        __syncthreads();
        for (int c = 0; c < nsl; ++c) {
            const int cf = scf0 + c;
            const int pc = P.cf_pc[cf];
            const int pstale = A.stale[P.cf_frame[cf]];
            double acc[KJ];
#pragma unroll
            for (int q = 0; q < KJ; ++q) acc[q] = 0.;
            for (int i = obs_lo(c) + tid; i < obs_hi(c); i += CT) {
                // the records stay in LDS (an opaque zero offset keeps the
                // compiler from hoisting 180 loop-invariant doubles into
                // registers)
                int z = 0;
                asm volatile("" : "+s"(z));
                const double *rc = &s_rec[c][0][0] + z;
                const Resid r0 = resid_at(i, rc);
                Resid rs = r0;
                double jx[NFC], jy[NFC];
#pragma unroll
                for (int a = 0; a < NFC; ++a) {
                    jx[a] = 0.;
                    jy[a] = 0.;
                    if (a < pc) {
                        const int k = c * NFC + a;
                        const Resid r = resid_at(i, rc + (1 + a) * CAMREC);
                        const double st = s_step[k];
                        if (lmder) {  // inv_delta, multiplied (adjust_solveFunc.cpp:395-402)
                            jx[a] = (r.ex - r0.ex) * st;
                            jy[a] = (r.ey - r0.ey) * st;
                        } else {      // h, divided (fdjac2)
                            jx[a] = (r.ex - r0.ex) / st;
                            jy[a] = (r.ey - r0.ey) / st;
                        }
                        if (s_sp[k] == pstale) rs = r;
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
                cg_st(&A.nep[((size_t)g * SLM + c) * KJ + tid], v);
            }
            __syncthreads();
        }
    };

    // owner: J^T J / J^T f of the owned camera-frames from the slices' slots
    // (in workgroup order) -> s_A, s_g
    auto assemble = [&]() {
        for (int t = tid; t < CPB * NFC * NFC; t += CT) s_A[t / (NFC * NFC)][t % (NFC * NFC)] = 0.;
        __syncthreads();
        if (tid < CPB * KJ) {
            const int c = tid / KJ, q = tid % KJ;
            if (c < nown) {
                const int cf = g + c * G, pc = P.cf_pc[cf];
                double v = 0.;
                for (int u = A.cf_src_off[cf]; u < A.cf_src_off[cf + 1]; ++u)
                    v += cg_ld(&A.nep[(size_t)A.cf_src[u] * KJ + q]);
                if (q < KA) {
                    int a = 0, t = q;
                    while (t > a) {
                        t -= a + 1;
                        ++a;
                    }
                    if (a < pc) {
                        s_A[c][a * NFC + t] = v;
                        s_A[c][t * NFC + a] = v;
                    }
                } else if (q - KA < pc) {
                    s_g[c * NFC + q - KA] = v;
                }
            }
        }
        __syncthreads();
    };

    // owner: damped solve of every owned camera-frame block (wave c):
    // (A_c + lam D_c^2) xs_c = g_c -> s_xs and A.xs (write-through);
    // partials [||D xs||^2, pivot failure] -> s_gv[0, 1].  The factor stays
    // in the wave's registers for newton().
    double fa[NFC];
    double frs = 0., fxs = 0.;
    auto solve = [&](double lam) {
        bool bad = false;
        double dn = 0.;
        if (wv < nown) {
            const int c = wv;
            const int pc = P.cf_pc[g + c * G];
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
            if (lane < NFC) {
                s_xs[c * NFC + lane] = fxs;
                if (lane < pc) cg_st(&A.xs[s_op[c * NFC + lane]], fxs);
            }
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
                if (w < nown) {
                    d += s_red[w][0];
                    b = fmax(b, s_red[w][1]);
                }
            s_gv[0] = d;
            s_gv[1] = b;
        }
        __syncthreads();
    };
    // owner: sum over owned blocks of ||C^-1 v||^2, v = D (D xs / dxnorm),
    // with the factors of the last solve -> s_gv[0]
    auto newton = [&](double dxn) {
        double nsq = 0.;
        if (wv < nown) {
            const int c = wv;
            const int pc = P.cf_pc[g + c * G];
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
                if (w < nown) d += s_red[w][0];
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

    int npr = 0;
    auto stamp = [&]() {
        if (A.probe && g == 0 && tid == 0 && npr < 64) A.probe[npr] = (long long)wall_clock64();
        ++npr;
    };
    stamp();
    nfev = 1;
    fe = 1;
    eval(s_sx, nullptr, A.f, A.dist);  // x0 (lmder's first fcn call)
    aborted = grid_reduce(1, 0u);
    fnorm = sqrt(s_gv[0]);
    trace(fnorm);
    int iter = 1;
    while (!aborted) {
        stamp();
        jacobian();
        stamp();
        ++njev;
        je += P.n;
        if (!lmder) nfev += P.n;
        const bool first = iter == 1;
        aborted = grid_reduce(0, 0u);  // every slot stored
        stamp();
        if (aborted) break;
        assemble();
        {
            // lmder after qrfac: column norms, diag, ||D x||, gnorm, rank
            // flag -- and the undamped solve lmpar starts from, in the same
            // reduction
            double xn = 0., gm = 0., zf = 0.;
            if (tid < CPB * NFC && s_op[tid] >= 0) {
                const int c = tid / NFC, a = tid % NFC;
                const double an = sqrt(s_A[c][a * NFC + a]);
                double dg = s_diag[tid];
                if (A.mode != 2) {
                    if (first) dg = an == 0. ? 1. : an;
                    dg = fmax(dg, an);
                    s_diag[tid] = dg;
                }
                const double v = dg * s_ox[tid];
                xn = v * v;
                if (an == 0.) zf = 1.;
                if (fnorm != 0. && an != 0.) gm = fabs((s_g[tid] / fnorm) / an);
            }
            const double vv[3] = {xn, gm, zf};
            cg_block_reduce<3, 6u>(vv, s_red, s_gv);
            const double b0 = s_gv[0], b1 = s_gv[1], b2 = s_gv[2];
            __syncthreads();
            solve(0.);
            if (tid == 0) {
                s_gv[3] = s_gv[0];  // ||D xs||^2 of the undamped step
                s_gv[4] = s_gv[1];  // its pivot flag
                s_gv[0] = b0;
                s_gv[1] = b1;
                s_gv[2] = b2;
            }
            __syncthreads();
            stamp();
            aborted = grid_reduce(5, 2u | 4u | 16u);
            stamp();
        }
        if (aborted) break;
        const bool rank_def = s_gv[2] != 0.;
        if (first) {
            xnorm = sqrt(s_gv[0]);
            delta = A.factor * xnorm;
            if (delta == 0.) delta = A.factor;
        }
        gnorm = fnorm != 0. ? s_gv[1] : 0.;
        double dn0 = s_gv[3], bad0 = s_gv[4];
        bool pre = true;  // the undamped solve of this Jacobian is current
        __syncthreads();
        if (gnorm <= A.gtol) info = 4;
        if (info != 0) break;
        do {
            // ---- lmpar (lmpar_ne, mmba_lm.cpp) ----
            const double dwarf = DBL_MIN;
            int it = 0;
            if (!pre) {
                solve(0.);
                aborted = grid_reduce(2, 2u);
                if (aborted) break;
                dn0 = s_gv[0];
                bad0 = s_gv[1];
            }
            pre = false;
            const bool ok0 = bad0 == 0.;
            double dxnorm = ok0 ? sqrt(dn0) : HUGE_VAL;
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
                if (tid < CPB * NFC && s_op[tid] >= 0) {
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
            }
            // ---- trial point: p = -xs, wa2 = x + p ----
            // owners: ||D p||^2, ||D wa2||^2 of their parameters
            double pn = 0., xn = 0.;
            if (tid < CPB * NFC && s_op[tid] >= 0) {
                const double st = -s_xs[tid];
                const double w2 = s_ox[tid] + st;
                const double dk = s_diag[tid];
                s_owa2[tid] = w2;
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
            // slices: the same trial point from the owners' steps (stored
            // write-through before the last grid reduction)
            if (tid < SLM * NFC) {
                double st = 0.;
                if (s_sp[tid] >= 0) st = -cg_ld(&A.xs[s_sp[tid]]);
                s_swa1[tid] = st;
                s_swa2[tid] = s_sx[tid] + st;
            }
            __syncthreads();
            ++nfev;
            ++fe;
            stamp();
            eval(s_swa2, s_swa1, fsel ? A.f : A.ft, fsel ? A.dist : A.distt);
            stamp();
            // [||f||^2, ||J p||^2, ||D p||^2, ||D wa2||^2]
            if (tid == 0) {
                s_gv[2] = bpn;
                s_gv[3] = bxn;
            }
            __syncthreads();
            aborted = grid_reduce(4, 0u);
            stamp();
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
                if (tid < SLM * NFC) s_sx[tid] = s_swa2[tid];
                if (tid < CPB * NFC) s_ox[tid] = s_owa2[tid];
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
        for (int i = so0 + tid; i < so1; i += CT) {
            A.f[2 * i] = A.ft[2 * i];
            A.f[2 * i + 1] = A.ft[2 * i + 1];
            A.dist[i] = A.distt[i];
        }
    }
    if (tid < CPB * NFC && s_op[tid] >= 0) A.x[s_op[tid]] = s_ox[tid];
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
        o.nprobe = npr;
        *A.out = o;
    }
}

// Observation slices (balanced, one per workgroup, <= SLM camera-frames
// each), camera-frame owners (g, g + G, ...: <= CPB per workgroup) and the
// normal-equation slots of every camera-frame in workgroup order; false when
// the plan does not fit the cooperative launch.
bool lm_coop_layout(int ncf, const std::vector<int> &cf_obs_off, int gmax, CoopLayout &L) {
    const int M = cf_obs_off[ncf];
    if (ncf <= 0 || M <= 0 || gmax <= 0) return false;
    // slices of ~M / G observations, also cut where a slice would touch a
    // (SLM + 1)-th camera-frame; fewer, longer slices when that needs more
    // workgroups than fit
    const int gmin = (ncf + CPB - 1) / CPB;  // owners: <= CPB camera-frames each
    if (gmin > gmax) return false;
    for (int target = std::max(512, (M + gmax - 1) / gmax);; target += target / 4 + 1) {
        std::vector<int> off{0}, first{0}, cnt;
        int cf = 0, n = 0;  // current slice: first camera-frame, camera-frames touched
        for (int o = 0; o < M;) {
            while (cf_obs_off[cf + 1] <= o) ++cf;
            const int start = off.back();
            if (n == 0) first.back() = cf;
            ++n;
            const int end = std::min(cf_obs_off[cf + 1], start + target);
            o = end;
            if (end == start + target || n == SLM || o == M) {
                off.push_back(o);
                cnt.push_back(n);
                if (o < M) first.push_back(0);
                n = 0;
            }
        }
        int G = (int)cnt.size();
        if (G > gmax) {
            if (target >= M) return false;
            continue;
        }
        // every owner slot exists: pad with empty slices up to gmin
        while (G < gmin) {
            off.push_back(M);
            first.push_back(ncf - 1);
            cnt.push_back(0);
            ++G;
        }
        L.G = G;
        L.slice_off = off;
        L.slice_cf = first;
        L.slice_ncf = cnt;
        std::vector<std::vector<int>> src(ncf);
        for (int g = 0; g < G; ++g)
            for (int c = 0; c < cnt[g]; ++c) src[first[g] + c].push_back(g * SLM + c);
        L.cf_src_off.assign(ncf + 1, 0);
        L.cf_src.clear();
        for (int c = 0; c < ncf; ++c) {
            L.cf_src_off[c] = (int)L.cf_src.size();
            for (int u : src[c]) L.cf_src.push_back(u);
        }
        L.cf_src_off[ncf] = (int)L.cf_src.size();
        return true;
    }
}

// Workgroups a cooperative launch of k_lm_coop can keep resident on the
// current device (occupancy x compute units), 0 when it cannot launch.
int lm_coop_max_grid(bool lens) {
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const void *fn = lens ? reinterpret_cast<const void *>(&k_lm_coop<true>)
                          : reinterpret_cast<const void *>(&k_lm_coop<false>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, CT, 0) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    if (std::getenv("MMBA_COOP_DEBUG"))
        std::fprintf(stderr, "[mmba coop] %d compute units x %d resident workgroups\n", cus, per);
    return std::min(256, per * cus);
}

int lm_coop_nfc() { return NFC; }
int lm_coop_slots() { return SLM; }
int lm_coop_kj() { return KJC; }

bool launch_lm_coop(hipStream_t s, const DevProblem &P, const CoopArgs &A, int G, bool lens) {
    // every workgroup must be resident (grid reductions): a cooperative
    // launch fails instead of deadlocking when they are not
    DevProblem Pc = P;
    CoopArgs Ac = A;
    void *args[] = {&Pc, &Ac};
    const void *fn = lens ? reinterpret_cast<const void *>(&k_lm_coop<true>)
                          : reinterpret_cast<const void *>(&k_lm_coop<false>);
    const hipError_t e = hipLaunchCooperativeKernel(fn, dim3(G), dim3(CT), args, 0, s);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        if (std::getenv("MMBA_COOP_DEBUG"))
            std::fprintf(stderr, "[mmba coop] cooperative launch of %d workgroups failed: %s\n", G,
                         hipGetErrorString(e));
        return false;
    }
    return true;
}

}  // namespace mmba
