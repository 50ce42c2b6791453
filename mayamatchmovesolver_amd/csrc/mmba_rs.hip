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
// 29).  A parented camera blends its own translate / rotate under the
// parent's world matrix at the frame.  Solved bundles: the Schur
// complement runs over virtual observations, one per (observation,
// camera-frame block it reaches) (Plan::build, k_schur_obs_rs).  Restricted
// to forward differences, one shard (Plan::build refuses the rest).
#include <hip/hip_runtime.h>

#include "mmba_geom.h"
#include "mmba_kernels.h"

namespace mmba {

#ifndef MMBA_RS_WAVES
#define MMBA_RS_WAVES 1
#endif

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
// The columns are listed first (parameter, kind), then evaluated by one code
// site: kind 0 = a camera-side value (this frame or a blended neighbour),
// 1 = a neighbouring frame's parameter the blend does not read (entry 0,
// no evaluation), 2 = a lens coefficient, 3 = a parameter of the
// observation's bundle (the bundle moved, the base record).  One evaluation site keeps the
// inlined record + lens code (the register-heavy part) once.
template <int TPB>
__global__ void __launch_bounds__(TPB, MMBA_RS_WAVES) k_jacobian_rs(DevProblem P, const double *__restrict__ ext_pert,
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
    const double mx = P.obs_xy[2 * i], my = P.obs_xy[2 * i + 1], sw = P.obs_sqrtw[i];
    const double tau = P.obs_tau[i];
    const Override none{-1, 0.};
    double bp0[3];
    base_bundle(P, b, fr, bp0);
    int inst = -1;
    const int hl = obs_lens_inst(P, i, inst);
    // the column list
    int cp[LMAX];
    unsigned char ck[LMAX];
    int nl = 0;
    const int voff = P.cf_var_off[cf];
    const int nvar = P.cf_var_off[cf + 1] - voff;
    for (int v = 1; v < nvar && nl < LMAX; ++v) {
        cp[nl] = P.cf_var_param[voff + v];
        ck[nl++] = 0;
    }
    const int *nx = &P.cf_rs_vidx[(size_t)12 * cf];
    for (int side = 0; side < 2; ++side) {
        const int cn = P.cf_rs_nb[2 * cf + side];
        if (cn < 0) continue;
        const int vo = P.cf_var_off[cn] + 1;
        for (int a = 0; a < P.cf_pc[cn] && nl < LMAX; ++a) {
            const int p = P.cf_var_param[vo + a];
            const long long vi = param_vidx(P, p);
            bool blended = false;
#pragma unroll
            for (int k = 0; k < 6; ++k) blended |= nx[6 * side + k] == vi;
            cp[nl] = p;
            ck[nl++] = blended ? 0 : 1;
        }
    }
    if (hl)
        for (int q = P.inst_lpar_off[inst]; q < P.inst_lpar_off[inst + 1] && nl < LMAX; ++q) {
            const int p = P.inst_lpar[q];
            if (P.p_frame[p] >= 0 && P.p_frame[p] != fr) continue;  // (plain instances: none)
            cp[nl] = p;
            ck[nl++] = 2;
        }
    // the observation's bundle parameters last (k_ne_bnd / k_schur_obs_rs
    // find them at nloc - pb): the base record with the bundle moved
    for (int q = P.bnd_par_off[b]; q < P.bnd_par_off[b] + P.bnd_pb[b] && nl < LMAX; ++q) {
        cp[nl] = P.bnd_par[q];
        ck[nl++] = 3;
    }
    const bool lmder = solver_type == MMBA_SOLVER_CMINPACK_LMDER;
    const int pstale = stale_param[fr];
    RsCam RC;
    rs_cam_load(P, cf, RC);
    // the lens coefficients at x once; a lens column replaces its slot(s)
    // (inst_coeffs with the override, without re-reading the table)
    double lc0[MMBA_LENS_NUM_ATTRS];
    int la[MMBA_LENS_NUM_ATTRS];
    int ltype = MMBA_LENS_NONE;
    if (hl) {
        inst_coeffs(P, inst, none, lc0);
        ltype = hl;
#pragma unroll
        for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k) la[k] = P.inst_attr[MMBA_LENS_NUM_ATTRS * inst + k];
    }
    // column -1: the base point; then every column that needs an evaluation
    Resid r0{}, rs{};
    for (int l = -1; l < nl; ++l) {
        const int kind = l < 0 ? 0 : ck[l];
        const int p = l < 0 ? -1 : cp[l];
        double jx = 0., jy = 0.;
        if (kind != 1) {
            double rec[CAMREC];
            rs_record(P, RC, tau, kind == 0 && p >= 0 ? param_vidx(P, p) : -1,
                      p >= 0 ? ext_pert[p] : 0., rec, kind == 0 && p >= 0 ? P.p_attr[p] : -1);
            double bq[3] = {bp0[0], bp0[1], bp0[2]};
            if (kind == 3) bundle_position(P, b, fr, Override{P.p_attr[p], ext_pert[p]}, bq);
            double lc[MMBA_LENS_NUM_ATTRS];
            if (hl) {
                const int oa = kind == 2 ? P.p_attr[p] : -2;
                const double ov = kind == 2 ? ext_pert[p] : 0.;
#pragma unroll
                for (int k = 0; k < MMBA_LENS_NUM_ATTRS; ++k)
                    lc[k] = (la[k] >= 0 && la[k] == oa) ? ov : lc0[k];
                if (ltype == MMBA_LENS_3DE_ANAMORPHIC_STD_DEG4) lc[13] = 1.;  // inst_coeffs' rule
            }
            const Resid r = residual_l(P, rec, bq, mx, my, sw, hl, lc);
            if (l < 0) {
                r0 = r;
                rs = r;
                continue;
            }
            if (p == pstale) rs = r;
            const double st = step[p];
            if (lmder) {  // st = 1/delta, multiplied (adjust_solveFunc.cpp:395-402)
                jx = (r.ex - r0.ex) * st;
                jy = (r.ey - r0.ey) * st;
            } else {      // st = h, divided (fdjac2)
                jx = (r.ex - r0.ex) / st;
                jy = (r.ey - r0.ey) / st;
            }
        }
        J[(size_t)(2 * l) * M + i] = jx;
        J[(size_t)(2 * l + 1) * M + i] = jy;
        jcol[(size_t)l * M + i] = p;
    }
    nloc[i] = nl;
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
    // rows padded to RS_CHUNK + 1: the threads of a wave read different rows
    // at one column (a 512-B row stride put them all on one LDS bank)
    __shared__ double sJ[2 * LMAX][RS_CHUNK + 1];
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

// Uniform block size PC and at most NG global parameters: the same blocks
// with per-lane accumulators (lane o takes the segment's observations o, o +
// 256, ...), a fixed xor-shuffle tree per wave and the 4 wave sums added in
// wave order -- deterministic, no LDS staging of J.  The global columns of an
// observation are its camera-side globals (variant columns pc .. nvar) and
// its lens columns (after the neighbours' blocks), found through jcol.
template <int PC, int NG>
__global__ void __launch_bounds__(256) k_ne_rs_u(DevProblem P, const double *__restrict__ J,
                                                 const int *__restrict__ jcol,
                                                 const int *__restrict__ nloc,
                                                 const double *__restrict__ f, double *Acc,
                                                 double *Acg, double *g, double *Aoff) {
    constexpr int NCC = PC * (PC + 1) / 2, N0 = NCC + PC + PC * NG, N1 = PC * PC;
    constexpr int NA = N0 > N1 ? N0 : N1;
    __shared__ double wsum[4][NA];
    const int cf = blockIdx.x / 3, d = blockIdx.x % 3;
    if (P.cf_pc[cf] != PC) return;
    const int n1 = P.cf_rs_nb[2 * cf + 1];
    int B = cf;
    if (d >= 1) B = n1;
    if (d == 2 && B >= 0) B = P.cf_rs_nb[2 * B + 1];
    if (B < 0 || P.cf_pc[B] != PC) return;
    const size_t M = P.M;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double acc[NA];
#pragma unroll
    for (int e = 0; e < NA; ++e) acc[e] = 0.;
    int segs[3] = {-1, -1, -1};
    if (d == 0) {
        segs[0] = P.cf_rs_nb[2 * cf];
        segs[1] = cf;
        segs[2] = n1;
    } else if (d == 1) {
        segs[0] = cf;
        segs[1] = n1;
    } else {
        segs[0] = n1;
    }
    for (int q = 0; q < 3; ++q) {
        const int sg = segs[q];
        if (sg < 0) continue;
        const int oA = rs_block_off(P, sg, cf), oB = rs_block_off(P, sg, B);
        // this segment's global columns (the same for all its observations)
        int gl[NG > 0 ? NG : 1], gi[NG > 0 ? NG : 1];
        const int ngc = NG > 0 ? min(P.cf_rs_gcnt[sg], NG) : 0;
#pragma unroll
        for (int t = 0; t < (NG > 0 ? NG : 1); ++t) {
            gl[t] = t < ngc ? P.cf_rs_gcol[(size_t)NGMAX * sg + t] : 0;
            gi[t] = t < ngc ? P.cf_rs_gidx[(size_t)NGMAX * sg + t] : -1;
        }
        const int o0 = P.cf_obs_off[sg], o1 = P.cf_obs_off[sg + 1];
        for (int i = o0 + tid; i < o1; i += 256) {
            double ax[PC], ay[PC];
#pragma unroll
            for (int a = 0; a < PC; ++a) {
                ax[a] = J[(size_t)(2 * (oA + a)) * M + i];
                ay[a] = J[(size_t)(2 * (oA + a) + 1) * M + i];
            }
            if (d != 0) {
                double bx[PC], by[PC];
#pragma unroll
                for (int c = 0; c < PC; ++c) {
                    bx[c] = J[(size_t)(2 * (oB + c)) * M + i];
                    by[c] = J[(size_t)(2 * (oB + c) + 1) * M + i];
                }
#pragma unroll
                for (int a = 0; a < PC; ++a)
#pragma unroll
                    for (int c = 0; c < PC; ++c) acc[a * PC + c] += ax[a] * bx[c] + ay[a] * by[c];
                continue;
            }
            const double fx = f[2 * i], fy = f[2 * i + 1];
            int e = 0;
#pragma unroll
            for (int a = 0; a < PC; ++a)
#pragma unroll
                for (int c = a; c < PC; ++c) acc[e++] += ax[a] * ax[c] + ay[a] * ay[c];
#pragma unroll
            for (int a = 0; a < PC; ++a) acc[NCC + a] += ax[a] * fx + ay[a] * fy;
            if constexpr (NG > 0) {
                double gx[NG], gy[NG];
#pragma unroll
                for (int t = 0; t < NG; ++t) gx[t] = gy[t] = 0.;
#pragma unroll
                for (int t = 0; t < NG; ++t) {
                    if (t >= ngc) break;
                    const int l = gl[t];
                    const double ux = J[(size_t)(2 * l) * M + i], uy = J[(size_t)(2 * l + 1) * M + i];
#pragma unroll
                    for (int u = 0; u < NG; ++u) {
                        gx[u] = (gi[t] == u) ? ux : gx[u];
                        gy[u] = (gi[t] == u) ? uy : gy[u];
                    }
                }
#pragma unroll
                for (int a = 0; a < PC; ++a)
#pragma unroll
                    for (int t = 0; t < NG; ++t) acc[NCC + PC + a * NG + t] += ax[a] * gx[t] + ay[a] * gy[t];
            }
        }
    }
    const int ne = d == 0 ? N0 : N1;
#pragma unroll
    for (int e = 0; e < NA; ++e) {
        double v = acc[e];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) wsum[wv][e] = v;
    }
    __syncthreads();
    for (int e = tid; e < ne; e += 256) {
        const double v = (wsum[0][e] + wsum[1][e]) + (wsum[2][e] + wsum[3][e]);
        if (d != 0) {
            Aoff[(size_t)(2 * cf + d - 1) * PCMAX * PCMAX + (e / PC) * PCMAX + e % PC] = v;
        } else if (e < NCC) {
            int a = 0, rem = e;
            while (rem >= PC - a) {
                rem -= PC - a;
                ++a;
            }
            const int c = a + rem;
            double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
            A[a * PCMAX + c] = v;
            A[c * PCMAX + a] = v;
        } else if (e < NCC + PC) {
            g[P.cf_var_param[P.cf_var_off[cf] + 1 + (e - NCC)]] = v;
        } else {
            constexpr int NGd = NG > 0 ? NG : 1;
            const int a = (e - NCC - PC) / NGd, t = (e - NCC - PC) % NGd;
            if (t < P.nG) Acg[((size_t)cf * PCMAX + a) * NGMAX + t] = v;
        }
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
    k_jacobian_rs<64><<<nblk_rs(P.M, 64), 64, 0, s>>>(P, ext_pert, step, solver_type, J, jcol,
                                                      nloc, stale_param, eu, ed);
}

void launch_ne_rs(hipStream_t s, const DevProblem &P, const double *J, const int *jcol,
                  const int *nloc, const double *f, double *Acc, double *Acg, double *g) {
    if (P.ncf == 0) return;
    const int pcu = P.pc_uniform;
    if (pcu == 6 && P.nG == 0)
        k_ne_rs_u<6, 0><<<3 * P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, P.rs_Aoff);
    else if (pcu == 6 && P.nG <= 2)
        k_ne_rs_u<6, 2><<<3 * P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, P.rs_Aoff);
    else if (pcu == 6 && P.nG <= 4)
        k_ne_rs_u<6, 4><<<3 * P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, P.rs_Aoff);
    else
        k_ne_rs<<<3 * P.ncf, 256, 0, s>>>(P, J, jcol, nloc, f, Acc, Acg, g, P.rs_Aoff);
}

void launch_rs_offdiag(hipStream_t s, const DevProblem &P, const SView &V) {
    const long n = (long)P.ncf * 2 * PCMAX * PCMAX;
    if (n > 0) k_rs_offdiag<<<nblk_rs(n, 256), 256, 0, s>>>(P, P.rs_Aoff, V);
}

}  // namespace mmba
