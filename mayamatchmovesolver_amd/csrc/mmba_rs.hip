// mmba_rs.hip -- rolling shutter (mmba.h ABI 3; BASELINE configs[4]
// "rolling-shutter per-scanline pose").
//
// The reference solver has no rolling-shutter model (its only rolling-shutter
// arithmetic is the 3DE exporter's 2D correction,
// share/3dequalizer/python/uvtrack_format.py:243-330); this is an extension
// whose arithmetic follows that exporter (camera_record_rs, mmba_geom.h) and
// whose parity is pinned against oracle/refcpu.c (rs_blend), not against the
// reference.
//
// Structure: an observation at frame f sees its camera's pose blended over
// the camera-frames f-1, f, f+1, so its Jacobian row has three camera-frame
// blocks (plus the lens / global columns) and the camera-frame normal
// equations couple each camera-frame with the next two of the same camera:
// the reduced system is a band (+ arrow) factored by the band solvers
// (block cyclic reduction for C5's 2 cameras x 6 parameters: half bandwidth
// 29).  Restricted to camera transforms without a parent, no solved bundle,
// forward differences, one shard (Plan::build refuses the rest).
#include <hip/hip_runtime.h>

#include "mmba_geom.h"
#include "mmba_kernels.h"

namespace mmba {

static inline int nblk_rs(long n, int bs) { return (int)((n + bs - 1) / bs); }

__device__ __forceinline__ long long param_vidx(const DevProblem &P, int p) { return P.p_vidx[p]; }

// ---------------------------------------------------------------------------
// FD Jacobian rows (solveFunc_calculateJacobianMatrixForParameter restated per
// observation): columns = the camera-frame's variants, the previous frame's
// CF parameters, the next frame's CF parameters, the lens parameters.  A
// neighbouring-frame parameter that is not one of the blended translate /
// rotate values leaves the observation unchanged: its entry is exactly 0
// (what f(x + d e_p) - f(x) gives), written without an evaluation.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(128) k_jacobian_rs(DevProblem P, const double *__restrict__ ext_pert,
                                                     const double *__restrict__ step,
                                                     int solver_type, double *J, int *jcol,
                                                     int *nloc, const int *__restrict__ stale_param,
                                                     double *eu, double *ed) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P.M) return;
    const int M = P.M;
    const int cf = P.obs_cf[i];
    const int b = P.obs_bnd[i];
    const int fr = P.obs_frame[i];
    const int cam = P.obs_cam[i];
    const double mx = P.obs_xy[2 * i], my = P.obs_xy[2 * i + 1], sw = P.obs_sqrtw[i];
    const double tau = P.obs_tau[i];
    const Override none{-1, 0.};
    double bp0[3];
    base_bundle(P, b, fr, bp0);
    double lc0[MMBA_LENS_NUM_ATTRS];
    int lens = -1;
    const int hl = obs_lens(P, cam, lens);
    if (hl) lens_coeffs(P, lens, fr, none, lc0);
    double rec[CAMREC];
    camera_record_rs(P, cf, tau, -1, 0., rec);
    const Resid r0 = residual_l(P, rec, bp0, mx, my, sw, hl, lc0);
    const bool lmder = solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const int pstale = stale_param[fr];
    Resid rs = r0;
    int l = 0;
    auto emit = [&](int p, double jx, double jy) {
        J[(size_t)(2 * l) * M + i] = jx;
        J[(size_t)(2 * l + 1) * M + i] = jy;
        jcol[(size_t)l * M + i] = p;
        ++l;
    };
    auto fd = [&](int p, const Resid &r) {
        const double st = step[p];
        if (p == pstale) rs = r;
        if (lmder)  // st = 1/delta, multiplied (adjust_solveFunc.cpp:395-402)
            emit(p, (r.ex - r0.ex) * st, (r.ey - r0.ey) * st);
        else        // st = h, divided (fdjac2)
            emit(p, (r.ex - r0.ex) / st, (r.ey - r0.ey) / st);
    };
    auto cam_col = [&](int p) {
        camera_record_rs(P, cf, tau, param_vidx(P, p), ext_pert[p], rec);
        fd(p, residual_l(P, rec, bp0, mx, my, sw, hl, lc0));
    };
    // this camera-frame's variants (its CF parameters, camera-side globals)
    const int voff = P.cf_var_off[cf];
    const int nvar = P.cf_var_off[cf + 1] - voff;
    for (int v = 1; v < nvar && l < LMAX; ++v) cam_col(P.cf_var_param[voff + v]);
    // the neighbouring frames' CF parameters
    const int *nx = &P.cf_rs_vidx[(size_t)12 * cf];
    for (int side = 0; side < 2; ++side) {
        const int cn = P.cf_rs_nb[2 * cf + side];
        if (cn < 0) continue;
        const int vo = P.cf_var_off[cn] + 1;
        for (int a = 0; a < P.cf_pc[cn] && l < LMAX; ++a) {
            const int p = P.cf_var_param[vo + a];
            const long long vi = param_vidx(P, p);
            bool blended = false;
#pragma unroll
            for (int k = 0; k < 6; ++k) blended |= nx[6 * side + k] == vi;
            if (blended) {
                cam_col(p);
            } else {
                emit(p, 0., 0.);  // f(x + d e_p) = f(x): the column's entry is 0
            }
        }
    }
    // lens parameters of this camera's lens
    if (hl) {
        camera_record_rs(P, cf, tau, -1, 0., rec);
        for (int q = P.cam_lpar_off[cam]; q < P.cam_lpar_off[cam + 1] && l < LMAX; ++q) {
            const int p = P.cam_lpar[q];
            if (P.p_frame[p] >= 0 && P.p_frame[p] != fr) continue;
            double lc[MMBA_LENS_NUM_ATTRS];
            lens_coeffs(P, lens, fr, Override{P.p_attr[p], ext_pert[p]}, lc);
            fd(p, residual_l(P, rec, bp0, mx, my, sw, hl, lc));
        }
    }
    nloc[i] = l;
    // errorList / errorDistanceList as left by the last FD column (B13)
    if (eu) {
        eu[2 * i] = rs.ux;
        eu[2 * i + 1] = rs.uy;
        ed[i] = rs.dist;
    }
}

// ---------------------------------------------------------------------------
// Camera-frame normal equations: one workgroup per (camera-frame cf, offset
// d = 0, 1, 2), block A(cf, next^d(cf)) summed over the observation segments
// whose rows reach both blocks, in segment order (deterministic, no atomics):
//   d = 0: segments prev(cf), cf, next(cf); also g_cf and Acg(cf)
//   d = 1: segments cf, next(cf)
//   d = 2: segment next(cf)
// Column offset of block X in the rows of segment s: 0 (X = s), nvar(s)
// (X = prev(s)), nvar(s) + pc(prev(s)) (X = next(s)).
// ---------------------------------------------------------------------------
constexpr int RS_CHUNK = 64;

__device__ __forceinline__ int rs_block_off(const DevProblem &P, int s, int X) {
    if (X == s) return 0;
    const int nvs = P.cf_var_off[s + 1] - P.cf_var_off[s] - 1;
    const int pp = P.cf_rs_nb[2 * s], nn = P.cf_rs_nb[2 * s + 1];
    if (X == pp) return nvs;
    if (X == nn) return nvs + (pp >= 0 ? P.cf_pc[pp] : 0);
    return -1;
}

__global__ void __launch_bounds__(256) k_ne_rs(DevProblem P, const double *__restrict__ J,
                                               const int *__restrict__ jcol,
                                               const int *__restrict__ nloc,
                                               const double *__restrict__ f, double *Acc,
                                               double *Acg, double *g, double *Aoff) {
    __shared__ double sJ[2 * LMAX][RS_CHUNK];
    __shared__ int sG[NGMAX][RS_CHUNK];
    __shared__ double sF[2][RS_CHUNK];
    const int cf = blockIdx.x / 3, d = blockIdx.x % 3;
    const int pc = P.cf_pc[cf];
    if (pc == 0) return;
    const int n1 = P.cf_rs_nb[2 * cf + 1];
    int B = cf;
    if (d >= 1) B = n1;
    if (d == 2 && B >= 0) B = P.cf_rs_nb[2 * B + 1];
    if (B < 0) return;
    const int pcB = P.cf_pc[B];
    if (pcB == 0) return;
    const int nG = d == 0 ? P.nG : 0;
    const int nCF = P.nR - P.nG;
    const int M = P.M;
    const int lm = P.lmax;
    const int ncc = pc * (pc + 1) / 2;
    const int e = threadIdx.x;
    int ea = 0, eb = 0, kind = -1;
    if (d == 0) {
        if (e < ncc) {
            int rem = e, r = 0;
            while (rem >= pc - r) {
                rem -= pc - r;
                ++r;
            }
            ea = r;
            eb = r + rem;
            kind = 0;
        } else if (e < ncc + pc) {
            ea = e - ncc;
            kind = 1;
        } else if (e < ncc + pc + pc * nG) {
            ea = (e - ncc - pc) / nG;
            eb = (e - ncc - pc) % nG;
            kind = 2;
        }
    } else if (e < pc * pcB) {
        ea = e / pcB;
        eb = e % pcB;
        kind = 3;
    }
    int segs[3], ns = 0;
    if (d == 0) {
        segs[ns++] = P.cf_rs_nb[2 * cf];
        segs[ns++] = cf;
        segs[ns++] = n1;
    } else if (d == 1) {
        segs[ns++] = cf;
        segs[ns++] = n1;
    } else {
        segs[ns++] = n1;
    }
    double acc = 0.;
    for (int q = 0; q < ns; ++q) {
        const int sg = segs[q];
        if (sg < 0) continue;
        const int oA = rs_block_off(P, sg, cf), oB = rs_block_off(P, sg, B);
        const int o0 = P.cf_obs_off[sg], o1 = P.cf_obs_off[sg + 1];
        for (int c0 = o0; c0 < o1; c0 += RS_CHUNK) {
            const int cnt = min(RS_CHUNK, o1 - c0);
            __syncthreads();
            for (int t = threadIdx.x; t < 2 * lm * RS_CHUNK; t += blockDim.x) {
                const int row = t / RS_CHUNK, o = t % RS_CHUNK;
                sJ[row][o] = (o < cnt) ? J[(size_t)row * M + c0 + o] : 0.;
            }
            if (nG > 0) {
                for (int t = threadIdx.x; t < NGMAX * RS_CHUNK; t += blockDim.x)
                    sG[t / RS_CHUNK][t % RS_CHUNK] = -1;
                __syncthreads();
                for (int t = threadIdx.x; t < lm * RS_CHUNK; t += blockDim.x) {
                    const int l = t / RS_CHUNK, o = t % RS_CHUNK;
                    if (o >= cnt || l >= nloc[c0 + o]) continue;
                    const int p = jcol[(size_t)l * M + c0 + o];
                    if (P.p_class[p] == PC_G) sG[P.p_pos[p] - nCF][o] = l;
                }
            }
            for (int t = threadIdx.x; t < RS_CHUNK; t += blockDim.x) {
                sF[0][t] = (t < cnt) ? f[2 * (c0 + t)] : 0.;
                sF[1][t] = (t < cnt) ? f[2 * (c0 + t) + 1] : 0.;
            }
            __syncthreads();
            if (kind == 0 || kind == 3) {
                const int la = oA + ea, lb = oB + eb;
                for (int o = 0; o < cnt; ++o)
                    acc += sJ[2 * la][o] * sJ[2 * lb][o] + sJ[2 * la + 1][o] * sJ[2 * lb + 1][o];
            } else if (kind == 1) {
                const int la = oA + ea;
                for (int o = 0; o < cnt; ++o)
                    acc += sJ[2 * la][o] * sF[0][o] + sJ[2 * la + 1][o] * sF[1][o];
            } else if (kind == 2) {
                const int la = oA + ea;
                for (int o = 0; o < cnt; ++o) {
                    const int lg = sG[eb][o];
                    if (lg >= 0)
                        acc += sJ[2 * la][o] * sJ[2 * lg][o] + sJ[2 * la + 1][o] * sJ[2 * lg + 1][o];
                }
            }
        }
    }
    if (kind == 0) {
        double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
        A[ea * PCMAX + eb] = acc;
        A[eb * PCMAX + ea] = acc;
    } else if (kind == 1) {
        g[P.cf_var_param[P.cf_var_off[cf] + 1 + ea]] = acc;
    } else if (kind == 2) {
        Acg[((size_t)cf * PCMAX + ea) * NGMAX + eb] = acc;
    } else if (kind == 3) {
        Aoff[((size_t)(2 * cf + d - 1) * PCMAX + ea) * PCMAX + eb] = acc;
    }
}

// The coupling blocks into the reduced system (after k_schur_init):
// S(roff(B) + b, roff(cf) + a) = A(cf, B)_ab, B = next^d(cf), d = 1, 2.
__global__ void __launch_bounds__(256) k_rs_offdiag(DevProblem P, const double *__restrict__ Aoff,
                                                    const SView V) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int per = 2 * PCMAX * PCMAX;
    const int cf = t / per;
    if (cf >= P.ncf) return;
    const int r = t % per;
    const int d = 1 + r / (PCMAX * PCMAX);
    const int a = (r / PCMAX) % PCMAX, b = r % PCMAX;
    const int pc = P.cf_pc[cf];
    if (a >= pc) return;
    int B = P.cf_rs_nb[2 * cf + 1];
    if (d == 2 && B >= 0) B = P.cf_rs_nb[2 * B + 1];
    if (B < 0 || b >= P.cf_pc[B]) return;
    *s_at(V, P.cf_roff[B] + b, P.cf_roff[cf] + a) =
        Aoff[((size_t)(2 * cf + d - 1) * PCMAX + a) * PCMAX + b];
}

void launch_jacobian_rs(hipStream_t s, const DevProblem &P, const double *ext_pert,
                        const double *step, int solver_type, double *J, int *jcol, int *nloc,
                        const int *stale_param, double *eu, double *ed) {
    k_jacobian_rs<<<nblk_rs(P.M, 128), 128, 0, s>>>(P, ext_pert, step, solver_type, J, jcol, nloc,
                                                    stale_param, eu, ed);
}

void launch_ne_rs(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
                  const int *nloc, const double *f, double *Acc, double *Acg, double *g) {
    if (P.ncf > 0) k_ne_rs<<<3 * P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, P.rs_Aoff);
}

void launch_rs_offdiag(hipStream_t s, const DevProblem &P, const SView &V) {
    const long n = (long)P.ncf * 2 * PCMAX * PCMAX;
    if (n > 0) k_rs_offdiag<<<nblk_rs(n, 256), 256, 0, s>>>(P, P.rs_Aoff, V);
}

}  // namespace mmba
