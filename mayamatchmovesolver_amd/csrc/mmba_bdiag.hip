// mmba_bdiag.hip -- block-diagonal + arrow reduced system (no bundle is
// solved: C2 pose + focal per frame, C5 poses + a shared lens, and every
// per-frame solve).  Without a solved bundle no term couples two
// camera-frames, so S is block diagonal in the camera-frame blocks (pc <= 10
// rows each) plus nG dense arrow rows (global parameters).  The Cholesky of
// such a matrix needs no cyclic reduction: each block is factored on its own
// (one wave per block, all blocks at once), the arrow's Schur complement
//   T = S_GG - sum_b Y_b^T Y_b,  Y_b = C_b^-1 S_bG
// is one small dense factorisation, and the back substitution is again one
// wave per block.  Without global parameters the whole damped solve
// (A + lam D^2) x = g is ONE launch.  Same contract as the band solvers
// (band_factor_forward / band_forward / band_backward): reduced-order
// vectors, y = L^-1 r of the permuted factor, ||y|| as lmpar's Newton term.
#include "mmba_geom.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"
#include "mmba_red_dev.h"

namespace mmba {

// Lane roles of one block's wave: rows 0..PC-1 of the block, then one
// right-hand-side lane per arrow row (Y_b columns), then the rhs lane.
constexpr int BD_G0 = PCMAX;  // first arrow lane (12 + NGMAX 48 + rhs: 61 lanes)
constexpr int BD_R = BD_G0 + NGMAX;  // right-hand-side lane (after the widest arrow)
static_assert(BD_R < 64, "arrow and right-hand-side lanes exceed the wave");

// Augmented Cholesky of one block by one wave (bcr_chol_aug_wave's scheme
// with a register-only column broadcast: PC <= 12 is short enough for
// v_readlane per entry): lane i < PC holds row i of [S_b], every
// right-hand-side lane holds its column; afterwards rows hold C and the
// right-hand-side lanes (C^-1 b)^T.  Rows >= pc are identity padding.
template <int PC>
__device__ __forceinline__ void bd_chol_aug(double (&a)[PC], double &rsl, bool &bad) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int j = 0; j < PC; ++j) {
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
        for (int c = j + 1; c < PC; ++c) a[c] = fma(-l, wave_rdlane(l, c), a[c]);
    }
}

// Block b (camera-frame cf = B.blk_cf[b]) of S from the band layout, its
// arrow columns and rhs; factor; store C (diagonal = 1/C_jj), Y_b and y_b;
// the arrow partials Y_b^T Y_b, Y_b^T y_b.  One wave per block, four blocks
// per workgroup.
template <int PC>
__global__ void __launch_bounds__(256) k_bd_factor(BdDev B, const double *__restrict__ r,
                                                   double *y, int *fail) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B.nblk) return;
    const int r0 = B.roff[b], pc = B.pc[b], nG = B.nG, w = B.w, W1 = w + 1;
    double a[PC];
#pragma unroll
    for (int c = 0; c < PC; ++c) {
        double v = 0.;
        if (lane < PC) {
            if (lane < pc) {
                if (c < pc && c <= lane) v = B.Bd[(size_t)(r0 + lane) * W1 + (c - lane + w)];
            } else if (c == lane) {
                v = 1.;  // identity padding
            }
        } else if (lane >= BD_G0 && lane < BD_G0 + nG) {
            v = c < pc ? B.Ga[(size_t)(lane - BD_G0) * B.nb + r0 + c] : 0.;
        } else if (lane == BD_R) {
            v = c < pc ? r[r0 + c] : 0.;
        }
        a[c] = v;
    }
    double rsl = 0.;
    bool bad = false;
    bd_chol_aug<PC>(a, rsl, bad);
    if (bad && lane == 0) atomicOr(fail, 1);
    double *FC = B.FC + (size_t)b * PC * PC;
    if (lane < PC) {
#pragma unroll
        for (int c = 0; c < PC; ++c) FC[lane * PC + c] = (c == lane) ? rsl : (c < lane ? a[c] : 0.);
    } else if (lane >= BD_G0 && lane < BD_G0 + nG) {
#pragma unroll
        for (int c = 0; c < PC; ++c) B.FY[((size_t)b * NGMAX + (lane - BD_G0)) * PC + c] = a[c];
    } else if (lane == BD_R) {
#pragma unroll
        for (int c = 0; c < PC; ++c)
            if (c < pc) y[r0 + c] = a[c];
    }
    if (nG > 0) {
        // arrow partials (Y^T Y)[q][q2] and (Y^T y)[q], one entry per lane,
        // from the wave's Y / y staged in LDS (row NGMAX = y)
        __shared__ double sy[4][(NGMAX + 1) * PC];
        double *my = sy[threadIdx.x >> 6];
        if (lane >= BD_G0 && lane < BD_G0 + nG) {
#pragma unroll
            for (int c = 0; c < PC; ++c) my[(lane - BD_G0) * PC + c] = a[c];
        } else if (lane == BD_R) {
#pragma unroll
            for (int c = 0; c < PC; ++c) my[NGMAX * PC + c] = a[c];
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (int e = lane; e < nG * nG + nG; e += 64) {
            double acc = 0.;
            const int q = e < nG * nG ? e / nG : e - nG * nG;
            const int q2 = e < nG * nG ? e % nG : NGMAX;
            for (int c = 0; c < pc; ++c) acc = fma(my[q * PC + c], my[q2 * PC + c], acc);
            if (q2 < NGMAX)
                B.Zc[(size_t)b * NGMAX * NGMAX + q * NGMAX + q2] = acc;
            else
                B.gpart[(size_t)b * NGMAX + q] = acc;
        }
    }
}

// Back substitution x_b = C_b^-T (y_b - Y_b x_G) from the stored factor;
// with xs the solution is also scattered to parameter order.  One wave per
// block; lane i < pc owns row i.
template <int PC>
__global__ void __launch_bounds__(256) k_bd_back(BdDev B, const double *__restrict__ y, double *x,
                                                 double *xs) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B.nblk) return;
    const int r0 = B.roff[b], pc = B.pc[b], nG = B.nG, nb = B.nb;
    const double *FC = B.FC + (size_t)b * PC * PC;
    double cc[PC];  // column lane of C (diagonal 1/C_jj)
    double v = 0.;
    if (lane < PC) {
#pragma unroll
        for (int u = 0; u < PC; ++u) cc[u] = u >= lane ? FC[u * PC + lane] : 0.;
        if (lane < pc) {
            v = y[r0 + lane];
            for (int q = 0; q < nG; ++q)
                v = fma(-B.FY[((size_t)b * NGMAX + q) * PC + lane], x[nb + q], v);
        }
    } else {
#pragma unroll
        for (int u = 0; u < PC; ++u) cc[u] = 0.;
    }
#pragma unroll
    for (int u = PC - 1; u >= 0; --u) {
        if (lane == u) v *= cc[u];
        const double xu = wave_rdlane(v, u);
        if (lane < u) v = fma(-cc[u], xu, v);
    }
    if (lane < pc) {
        const int R = r0 + lane;
        x[R] = v;
        if (xs) xs[B.row_param[R]] = v;
    }
}

// Forward solve only (lmpar's Newton term): y_b = C_b^-1 w_b from the stored
// factor, the arrow partials Y_b^T y_b.  One wave per block.
template <int PC>
__global__ void __launch_bounds__(256) k_bd_fwd(BdDev B, const double *__restrict__ wv,
                                                double *y) {
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= B.nblk) return;
    const int r0 = B.roff[b], pc = B.pc[b], nG = B.nG;
    const double *FC = B.FC + (size_t)b * PC * PC;
    double cr[PC];  // row lane of C (diagonal 1/C_ii)
    double v = 0.;
    if (lane < PC) {
#pragma unroll
        for (int u = 0; u < PC; ++u) cr[u] = u <= lane ? FC[lane * PC + u] : 0.;
        if (lane < pc) v = wv[r0 + lane];
    } else {
#pragma unroll
        for (int u = 0; u < PC; ++u) cr[u] = 0.;
    }
#pragma unroll
    for (int u = 0; u < PC; ++u) {
        if (lane == u) v *= cr[u];
        const double yu = wave_rdlane(v, u);
        if (lane > u) v = fma(-cr[u], yu, v);
    }
    if (lane < pc) y[r0 + lane] = v;
    if (nG > 0) {
        double yv[PC];
#pragma unroll
        for (int c = 0; c < PC; ++c) yv[c] = wave_rdlane(v, c);
        if (lane < nG) {
            double acc = 0.;
            const double *Yq = B.FY + ((size_t)b * NGMAX + lane) * PC;
            for (int c = 0; c < pc; ++c) acc = fma(Yq[c], yv[c], acc);
            B.gpart[(size_t)b * NGMAX + lane] = acc;
        }
    }
}

// Arrow corner: T = S_GG - sum_b Y_b^T Y_b = Ct Ct^T (dense, one wave, lane =
// row), y_G = Ct^-1 (r_G - sum_b Y_b^T y_b); with back: x_G = Ct^-T y_G (the
// back kernel then needs it).  factor = false: forward with the stored Ct.
// NGT: the arrow width this instantiation carries in registers (nG <= NGT;
// the identity padding beyond nG changes no entry, so the bits do not depend
// on NGT)
template <int NGT>
__global__ void __launch_bounds__(64) k_bd_root(BdDev B, const double *__restrict__ r, double *y,
                                                double *x, double *xs, int factor, int *fail) {
    __shared__ double zs[NGMAX * NGMAX], gs[NGMAX];
    const int lane = threadIdx.x, nG = B.nG, nb = B.nb;
    // sums over blocks: lane l adds blocks l, l + 64, ... in that order, then
    // a fixed xor tree.  Entries are taken RB at a time and each lane's loads
    // of a round (BK blocks per entry) are issued before its adds: one memory
    // round trip per round instead of one per block (the additions and their
    // order are unchanged, so are the bits)
    constexpr int RB = 4, BK = 8;
    const int nmat = factor ? nG * nG : 0, ntot = nmat + nG;
    for (int e0 = 0; e0 < ntot; e0 += RB) {
        double v[RB];
#pragma unroll
        for (int k = 0; k < RB; ++k) v[k] = 0.;
        for (int b0 = 0; b0 < B.nblk; b0 += 64 * BK) {
            double q[RB][BK];
#pragma unroll
            for (int k = 0; k < RB; ++k) {
                const int e = e0 + k;
                const double *src = e >= ntot ? nullptr
                                  : e < nmat ? B.Zc + (e / nG) * NGMAX + e % nG
                                             : B.gpart + (e - nmat);
                const size_t st = e < nmat ? (size_t)NGMAX * NGMAX : (size_t)NGMAX;
#pragma unroll
                for (int t = 0; t < BK; ++t) {
                    const int b = b0 + lane + 64 * t;
                    q[k][t] = (src && b < B.nblk) ? src[(size_t)b * st] : 0.;
                }
            }
#pragma unroll
            for (int k = 0; k < RB; ++k)
#pragma unroll
                for (int t = 0; t < BK; ++t)
                    if (b0 + lane + 64 * t < B.nblk) v[k] += q[k][t];
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int e = e0 + k;
            double w = v[k];
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) w += __shfl_xor(w, off);
            if (lane == 0 && e < ntot) {
                if (e < nmat) zs[(e / nG) * NGMAX + e % nG] = w;
                else gs[e - nmat] = w;
            }
        }
    }
    __syncthreads();
    double *Ct = B.FT;  // NGMAX x NGMAX lower, diagonal 1/C_jj
    if (factor) {
        // row `lane` of T
        double a[NGT];
#pragma unroll
        for (int c = 0; c < NGT; ++c) {
            double v = 0.;
            if (lane < nG && c <= lane) v = B.Gd[lane * NGMAX + c] - zs[lane * NGMAX + c];
            else if (lane < NGT && lane >= nG && c == lane) v = 1.;
            a[c] = v;
        }
        // rows / columns >= nG are identity padding: their pivots change
        // nothing, so the chain stops at nG (their 1 / C_jj is 1)
        double rsl = lane >= nG ? 1. : 0.;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < NGT; ++j) {
            if (j < nG) {  // (wave-uniform)
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
                for (int c = j + 1; c < NGT; ++c) a[c] = fma(-l, wave_rdlane(l, c), a[c]);
            }
        }
        if (bad && lane == 0) atomicOr(fail, 1);
        if (lane < NGT)
#pragma unroll
            for (int c = 0; c < NGT; ++c) Ct[lane * NGMAX + c] = c == lane ? rsl : (c < lane ? a[c] : 0.);
        __syncthreads();
    }
    // y_G = Ct^-1 (r_G - gs), x_G = Ct^-T y_G: serial in one lane (nG <= 16)
    if (lane == 0) {
        double v[NGT];
        for (int q = 0; q < nG; ++q) {
            double s = r[nb + q] - gs[q];
            for (int c = 0; c < q; ++c) s = fma(-Ct[q * NGMAX + c], v[c], s);
            v[q] = s * Ct[q * NGMAX + q];
            y[nb + q] = v[q];
        }
        if (x) {
            for (int q = nG - 1; q >= 0; --q) {
                double s = v[q];
                for (int c = q + 1; c < nG; ++c) s = fma(-Ct[c * NGMAX + q], v[c], s);
                v[q] = s * Ct[q * NGMAX + q];
                x[nb + q] = v[q];
                if (xs) xs[B.row_param[nb + q]] = v[q];
            }
        }
    }
}

// Damped solve straight from the normal equations when there is no arrow
// (nG == 0): S_b = Acc_b + lam D_b^2 with k_schur_init's rules (an exactly
// zero diagonal at lam == 0 becomes 1 with a zero right-hand side: the
// component solves to 0), augmented Cholesky, back substitution from the
// register rows, scatter to parameter order, and ||D xs||^2 plus the fail
// flag reduced by the last block into scalar[dn_slot] / scalar[fail_slot]
// (the flag is cleared).  One launch replaces k_schur_init, k_bd_factor,
// k_bd_back, k_sumsq and k_reduce_multi.  Workgroups [nb, nb + spec.nrows)
// reduce the rows of the Jacobian epilogue's deferred reduction (Plan::
// red_defer_ok; k_reduce_multi's arithmetic, reduce_row_block) -- the C2
// iteration's separate k_reduce_multi launch.
template <int PC>
__global__ void __launch_bounds__(256) k_bd_direct(DevProblem P, BdDev B,
                                                   const double *__restrict__ Acc,
                                                   const double *__restrict__ g,
                                                   const double *__restrict__ diag, double lam,
                                                   double *xR, double *xs, int *fail,
                                                   double *scalar, int dn_slot, int fail_slot,
                                                   int nb, const double *__restrict__ partial,
                                                   const RedSpec spec) {
    __shared__ double wpart[4];
    __shared__ double red[256];
    __shared__ int last;
    if ((int)blockIdx.x >= nb) {
        const RedRow rw = spec.row[blockIdx.x - nb];
        const double v = reduce_row_block<false>(partial, rw, red);
        if (threadIdx.x == 0) scalar[rw.slot] = v;
        return;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int b = blockIdx.x * 4 + wv;
    double dn = 0.;
    if (b < B.nblk) {
        const int cf = B.cf[b], r0 = B.roff[b], pc = B.pc[b];
        const int v0 = P.cf_var_off[cf] + 1;
        const double *A = &Acc[(size_t)cf * PCMAX * PCMAX];
        int pk = -1;
        double dk = 0.;
        if (lane < pc) {
            pk = P.cf_var_param[v0 + lane];
            dk = diag[pk];
        }
        double a[PC];
#pragma unroll
        for (int c = 0; c < PC; ++c) {
            double v = 0.;
            if (lane < pc) {
                if (c <= lane) {
                    v = A[lane * PCMAX + c];
                    if (c == lane) {
                        v += lam * (dk * dk);
                        if (v == 0.) v = 1.;
                    }
                }
            } else if (lane < PC) {
                v = c == lane ? 1. : 0.;
            } else if (lane == BD_R && c < pc) {
                v = (A[c * PCMAX + c] == 0. && lam == 0.) ? 0. : g[P.cf_var_param[v0 + c]];
            }
            a[c] = v;
        }
        double rsl = 0.;
        bool bad = false;
        bd_chol_aug<PC>(a, rsl, bad);
        if (bad && lane == 0) atomicOr(fail, 1);
        double *FC = B.FC + (size_t)b * PC * PC;  // rows for the Newton forward solve
        if (lane < PC) {
#pragma unroll
            for (int c = 0; c < PC; ++c) FC[lane * PC + c] = (c == lane) ? rsl : (c < lane ? a[c] : 0.);
        }
        double acc = 0.;
#pragma unroll
        for (int j = 0; j < PC; ++j) {
            const double y = wave_rdlane(a[j], BD_R);
            if (lane == j) acc = y;
        }
#pragma unroll
        for (int i = PC - 1; i >= 0; --i) {
            const double xi = wave_rdlane(acc, i) * wave_rdlane(rsl, i);
            if (lane == i) acc = xi;
#pragma unroll
            for (int j = 0; j < i; ++j) {
                const double cij = wave_rdlane(a[j], i);
                if (lane == j) acc = fma(-cij, xi, acc);
            }
        }
        if (lane < pc) {
            xR[r0 + lane] = acc;
            xs[pk] = acc;
            const double t = dk * acc;
            dn = t * t;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) dn += __shfl_xor(dn, off);
    }
    if (lane == 0) wpart[wv] = dn;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double v = (wpart[0] + wpart[1]) + (wpart[2] + wpart[3]);
        __hip_atomic_store(&B.part[blockIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __threadfence();
        last = atomicAdd(B.ticket, 1u) == (unsigned)nb - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    double s = 0.;
    for (int i = threadIdx.x; i < nb; i += blockDim.x)
        s += __hip_atomic_load(&B.part[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        scalar[dn_slot] = red[0];
        scalar[fail_slot] = (double)__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(B.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

void bd_direct(hipStream_t s, const DevProblem &P, const BdDev &D, const double *Acc,
               const double *g, const double *diag, double lam, double *xR, double *xs,
               int *fail, double *scalar, int dn_slot, int fail_slot, const RedSpec *red,
               const double *partial) {
    const int grid = (D.nblk + 3) / 4;
    const RedSpec rs = red ? *red : RedSpec{};
    const int nr = red ? red->nrows : 0;
    if (D.PC <= 8)
        k_bd_direct<8><<<grid + nr, 256, 0, s>>>(P, D, Acc, g, diag, lam, xR, xs, fail, scalar,
                                                 dn_slot, fail_slot, grid, partial, rs);
    else
        k_bd_direct<PCMAX><<<grid + nr, 256, 0, s>>>(P, D, Acc, g, diag, lam, xR, xs, fail,
                                                     scalar, dn_slot, fail_slot, grid, partial,
                                                     rs);
}

static void bd_root(hipStream_t s, const BdDev &D, const double *r, double *y, double *x,
                    double *xs, int factor, int *fail) {
    if (D.nG <= 16)
        k_bd_root<16><<<1, 64, 0, s>>>(D, r, y, x, xs, factor, fail);
    else if (D.nG <= 32)
        k_bd_root<32><<<1, 64, 0, s>>>(D, r, y, x, xs, factor, fail);
    else
        k_bd_root<NGMAX><<<1, 64, 0, s>>>(D, r, y, x, xs, factor, fail);
}

template <int PC>
static void bd_factor_k(hipStream_t s, const BdDev &D, int *fail, const double *r, double *y,
                        double *x, double *xs) {
    const int g = (D.nblk + 3) / 4;
    if (D.nG == 0) {
        // factor + forward, then back
        k_bd_factor<PC><<<g, 256, 0, s>>>(D, r, y, fail);
        if (x) k_bd_back<PC><<<g, 256, 0, s>>>(D, y, x, xs);
        return;
    }
    k_bd_factor<PC><<<g, 256, 0, s>>>(D, r, y, fail);
    bd_root(s, D, r, y, x, xs, 1, fail);
    if (x) k_bd_back<PC><<<g, 256, 0, s>>>(D, y, x, xs);
}

void bd_factor_solve(hipStream_t s, const BdDev &D, int *fail, const double *r, double *y,
                     double *x, double *xs) {
    if (D.PC <= 8)
        bd_factor_k<8>(s, D, fail, r, y, x, xs);
    else
        bd_factor_k<PCMAX>(s, D, fail, r, y, x, xs);
}

void bd_forward(hipStream_t s, const BdDev &D, const double *w, double *y) {
    const int g = (D.nblk + 3) / 4;
    if (D.PC <= 8)
        k_bd_fwd<8><<<g, 256, 0, s>>>(D, w, y);
    else
        k_bd_fwd<PCMAX><<<g, 256, 0, s>>>(D, w, y);
    if (D.nG > 0) bd_root(s, D, w, y, nullptr, nullptr, 0, nullptr);
}

}  // namespace mmba
