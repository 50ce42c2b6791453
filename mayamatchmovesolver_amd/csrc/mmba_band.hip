// mmba_band.hip -- Cholesky factorisation and triangular solves of the reduced
// system in band + arrow layout (CDNA4 / gfx950, fp64).
//
// For frame-ordered camera-frame parameters the reduced system
//   S = [ B   Gᵀ ]   B: nb x nb banded (half bandwidth w: a bundle couples the
//       [ G   D  ]      camera-frames of the frames it is tracked in),
//                    G: nG x nb dense arrow rows (lens, static camera attrs),
// factors as L = [Lb 0; Ga Ld] with no fill outside the band and the arrow.
// The factorisation is a chain: column j needs every update of columns < j,
// so it runs as ONE workgroup that walks 16-column blocks through an LDS
// window of BWR band rows (right-looking):
//   A. wave 0 factors and inverts the 16x16 diagonal block in registers
//      (lane = row, v_readlane broadcasts); meanwhile waves 1-3 move the rows
//      the next block needs into the window and the finished rows out,
//   B. the <= w panel rows below and the arrow rows: P = P Dinv^T,
//   C. trailing update of the w x w window and the arrow (rank 16).
// One launch replaces the ~2 NT launches of the tiled path; every LDS access
// after the initial load is on-chip.  The solves use the stored block
// inverses so each 16-row block costs two short reductions.
#include "mmba_kernels.h"

namespace mmba {

constexpr int BW1 = WBAND_MAX + 1;
constexpr int BMASK = BWR - 1;

// Broadcast lane l's double to the whole wave (v_readlane: l is wave-uniform).
__device__ __forceinline__ double rdlane(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// 1/sqrt(d): v_rsq_f64 plus two Newton steps (full fp64 precision).
__device__ __forceinline__ double rsq_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

// Factor a 16x16 SPD block held one row per lane (lane r = row r; lanes
// 16..63 mirror 0..15) and invert the factor: on return a[c], c <= r, is row
// r of L and x[] is column r of L^-1 (upper entries of a[] are scratch).
// Rows >= nd must be identity padding.  Branch-free: every lane runs every
// update, broadcasts are v_readlane of wave-uniform lanes, 1/L_jj comes from
// the rsq of the pivot.  Returns non-zero if a pivot was replaced.
template <int NB>
__device__ __forceinline__ int potrf_inv(double (&a)[NB], double (&x)[NB]) {
    const int r = threadIdx.x & (NB - 1);
    int badl = 0;
    double y[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) {
        double d = rdlane(a[j], j);
        if (!(d > 0.) || !isfinite(d)) {
            badl = 1;
            d = 1.;
            if (r == j) a[j] = 1.;
        }
        y[j] = rsq_nr(d);
        const double lj = a[j] * y[j];  // lane j: sqrt(d); lanes > j: L[r][j]
        a[j] = lj;
#pragma unroll
        for (int c = j + 1; c < NB; ++c) a[c] = fma(-lj, rdlane(lj, c), a[c]);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        double s = (i == r) ? 1. : 0.;
#pragma unroll
        for (int t = 0; t < i; ++t) s = fma(-rdlane(a[t], i), x[t], s);
        x[i] = s * y[i];
    }
    return badl;
}

template <int NB>
__global__ void __launch_bounds__(256) k_band_potrf(SView V, int nG, double *Dinv, double *Gdinv,
                                                    int *fail, long long *probe) {
    // probe (diagnostic builds of the bench only, MMBA_PROBE=1): thread 0
    // accumulates s_memtime cycles per phase; never read by the solver.
    long long pt[4] = {0, 0, 0, 0}, tprev = probe ? (long long)clock64() : 0;
    auto stamp = [&](int ph) {
        if (probe && threadIdx.x == 0) {
            const long long t = (long long)clock64();
            pt[ph] += t - tprev;
            tprev = t;
        }
    };
    __shared__ double win[BWR][BW1];
    __shared__ double gwin[NGMAX][BWR];
    __shared__ double sX[NB][NB + 1];
    __shared__ double sP[WBAND_MAX][NB + 1];
    __shared__ double sPG[NGMAX][NB + 1];
    __shared__ double sGd[NGMAX][NGMAX + 1];
    __shared__ int bad;
    const int tid = threadIdx.x;
    const int w = V.w, nb = V.nb, W1 = w + 1;
    if (tid == 0) bad = 0;
    for (int e = tid; e < NGMAX * NGMAX; e += blockDim.x) {
        const int q = e / NGMAX, q2 = e % NGMAX;
        sGd[q][q2] = (q < nG && q2 <= q) ? V.Gd[q * NGMAX + q2] : 0.;
    }
    // rows [r0, r1) enter the window; t0/nt: the participating threads
    auto load_rows = [&](int r0, int r1, int t0, int nt) {
        for (int e = t0; e < (r1 - r0) * W1; e += nt) {
            const int row = r0 + e / W1, k = e % W1;
            win[row & BMASK][k] = (row - w + k >= 0) ? V.Bd[(size_t)row * W1 + k] : 0.;
        }
        for (int e = t0; e < nG * (r1 - r0); e += nt) {
            const int q = e / (r1 - r0), row = r0 + e % (r1 - r0);
            gwin[q][row & BMASK] = V.Ga[(size_t)q * nb + row];
        }
    };
    // rows [r0, r1) are final: window -> HBM
    auto store_rows = [&](int r0, int r1, int t0, int nt) {
        for (int e = t0; e < (r1 - r0) * W1; e += nt) {
            const int row = r0 + e / W1, k = e % W1;
            V.Bd[(size_t)row * W1 + k] = win[row & BMASK][k];
        }
        for (int e = t0; e < nG * (r1 - r0); e += nt) {
            const int q = e / (r1 - r0), row = r0 + e % (r1 - r0);
            V.Ga[(size_t)q * nb + row] = gwin[q][row & BMASK];
        }
    };
    int loaded = min(nb, NB + w);
    load_rows(0, loaded, tid, blockDim.x);
    __syncthreads();
    for (int j0 = 0, b = 0; j0 < nb; j0 += NB, ++b) {
        const int nd = min(NB, nb - j0);
        // A. wave 0: diagonal block factor + inverse (the serial chain);
        //    waves 1-3: rows of the next block enter, the previous block leaves.
        if (tid < 64) {
            const int r = tid & (NB - 1);
            double a[NB], x[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                a[c] = 0.;
                if (c <= r && r < nd && r - c <= w) a[c] = win[(j0 + r) & BMASK][c - r + w];
            }
            if (r >= nd) a[r] = 1.;
            const int badl = potrf_inv<NB>(a, x);
            if (tid < NB) {
#pragma unroll
                for (int c = 0; c < NB; ++c) {
                    if (c <= r && r < nd && r - c <= w) win[(j0 + r) & BMASK][c - r + w] = a[c];
                    sX[c][r] = x[c];
                }
            }
            if (tid == 0 && badl) bad = 1;
        } else {
            const int want = min(nb, j0 + 2 * NB + w);
            if (want > loaded) load_rows(loaded, want, tid - 64, blockDim.x - 64);
            if (j0 > 0) store_rows(j0 - NB, j0, tid - 64, blockDim.x - 64);
        }
        loaded = max(loaded, min(nb, j0 + 2 * NB + w));
        __syncthreads();
        stamp(0);
        // B. panel rows [j0+NB, pend) and arrow rows: P <- P Dinv^T
        const int pend = min(nb, j0 + NB + w);
        const int npan = max(0, pend - (j0 + NB));
        for (int e = tid; e < npan * NB; e += blockDim.x) {
            const int li = e / NB, c = e % NB, i = j0 + NB + li;
            const double *wr = &win[i & BMASK][0];
            double pv[NB];
#pragma unroll
            for (int t = 0; t < NB; ++t) {
                const int k = j0 + t - i + w;  // band slot of column j0+t
                pv[t] = (k >= 0) ? wr[k] : 0.;
            }
            double s = 0.;
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(pv[t], sX[c][t], s);  // sX upper = 0
            sP[li][c] = s;
        }
        for (int e = tid; e < nG * NB; e += blockDim.x) {
            const int q = e / NB, c = e % NB;
            double s = 0.;
#pragma unroll
            for (int t = 0; t < NB; ++t)
                s = fma((t < nd) ? gwin[q][(j0 + t) & BMASK] : 0., sX[c][t], s);
            sPG[q][c] = s;
        }
        __syncthreads();
        stamp(1);
        // C. trailing update (rank NB), panel and arrow columns written back
        for (int e = tid; e < npan * W1; e += blockDim.x) {
            const int li = e / W1, kk = e % W1;
            const int i = j0 + NB + li, k = i - kk;
            if (k < j0 + NB) continue;
            const int lk = k - j0 - NB;
            double s = win[i & BMASK][w - kk];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sP[li][t], sP[lk][t], s);
            win[i & BMASK][w - kk] = s;
        }
        for (int e = tid; e < npan * NB; e += blockDim.x) {
            const int li = e / NB, c = e % NB, i = j0 + NB + li, col = j0 + c;
            if (i - col <= w) win[i & BMASK][col - i + w] = sP[li][c];
        }
        for (int e = tid; e < nG * npan; e += blockDim.x) {
            const int q = e / npan, li = e % npan, i = j0 + NB + li;
            double s = gwin[q][i & BMASK];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sPG[q][t], sP[li][t], s);
            gwin[q][i & BMASK] = s;
        }
        for (int e = tid; e < nG * nG; e += blockDim.x) {
            const int q = e / nG, q2 = e % nG;
            if (q2 > q) continue;
            double s = sGd[q][q2];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sPG[q][t], sPG[q2][t], s);
            sGd[q][q2] = s;
        }
        for (int e = tid; e < nG * nd; e += blockDim.x) {
            const int q = e / nd, c = e % nd;
            gwin[q][(j0 + c) & BMASK] = sPG[q][c];
        }
        for (int e = tid; e < NB * NB; e += blockDim.x)
            Dinv[(size_t)b * NB * NB + e] = sX[e / NB][e % NB];
        __syncthreads();
        stamp(2);
    }
    {
        const int jl = ((nb - 1) / NB) * NB;
        if (nb > 0) store_rows(jl, nb, tid, blockDim.x);
    }
    // arrow corner: Ld Ld^T = D - Ga Ga^T (already accumulated in sGd)
    if (nG > 0) {
        if (tid < 64) {
            const int r = tid & (BNB - 1);
            double a[BNB], x[BNB];
#pragma unroll
            for (int c = 0; c < BNB; ++c) a[c] = (c <= r && r < nG) ? sGd[r][c] : 0.;
            if (r >= nG) a[r] = 1.;
            const int badl = potrf_inv<BNB>(a, x);
            if (tid < BNB) {
#pragma unroll
                for (int c = 0; c < BNB; ++c) {
                    V.Gd[r * NGMAX + c] = (c <= r) ? a[c] : 0.;
                    Gdinv[c * NGMAX + r] = x[c];
                }
            }
            if (tid == 0 && badl) bad = 1;
        }
    }
    __syncthreads();
    stamp(3);
    if (tid == 0 && bad) atomicOr(fail, 1);
    if (probe && tid == 0)
        for (int k = 0; k < 4; ++k) atomicAdd((unsigned long long *)&probe[k], (unsigned long long)pt[k]);
}

// Sum over the 16 lanes of a lane group (rows of a block are 16-lane groups).
__device__ __forceinline__ double sum16(double v) {
    v += __shfl_xor(v, 8, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 1, 16);
    return v;
}

// L y = r.  Thread (i = tid/16, l = tid%16): row i of the current block.
template <int NB>
__global__ void __launch_bounds__(256) k_band_fwd(SView V, int nG, const double *__restrict__ Dinv,
                                                  const double *__restrict__ Gdinv,
                                                  const double *__restrict__ r, double *y) {
    __shared__ double ywin[BWR];
    __shared__ double t[NB];
    __shared__ double sumG[NGMAX];
    __shared__ double tg[NGMAX];
    const int tid = threadIdx.x, i = tid >> 4, l = tid & 15;
    const int w = V.w, nb = V.nb, W1 = w + 1;
    if (tid < NGMAX) sumG[tid] = 0.;
    __syncthreads();
    for (int j0 = 0, b = 0; j0 < nb; j0 += NB, ++b) {
        const int nd = min(NB, nb - j0);
        const int row = j0 + i;
        double s = 0.;
        if (i < nd) {
            // columns k in [max(0, row - w), j0): kk = j0 - 1 - k < w - i
            for (int kk = l; kk < w - i; kk += 16) {
                const int k = j0 - 1 - kk;
                if (k < 0) break;
                s += V.Bd[(size_t)row * W1 + (k - row + w)] * ywin[k & BMASK];
            }
        }
        s = sum16(s);
        if (l == 0 && i < nd) t[i] = r[row] - s;
        __syncthreads();
        double s2 = (i < nd && l <= i) ? Dinv[(size_t)b * NB * NB + i * NB + l] * t[l] : 0.;
        s2 = sum16(s2);
        if (l == 0 && i < nd) {
            ywin[row & BMASK] = s2;
            y[row] = s2;
        }
        __syncthreads();
        if (nG > 0) {
            // arrow: sumG[q] += sum_c Ga[q][j0+c] y_{j0+c}, q = i, c = l
            double p = (i < nG && l < nd) ? V.Ga[(size_t)i * nb + j0 + l] * ywin[(j0 + l) & BMASK] : 0.;
            p = sum16(p);
            if (l == 0 && i < nG) sumG[i] += p;
        }
    }
    __syncthreads();
    if (nG > 0) {
        if (tid < nG) tg[tid] = r[nb + tid] - sumG[tid];
        __syncthreads();
        if (tid < nG) {
            double s = 0.;
            for (int q2 = 0; q2 <= tid; ++q2) s += Gdinv[tid * NGMAX + q2] * tg[q2];
            y[nb + tid] = s;
        }
    }
}

// L^T x = y.
template <int NB>
__global__ void __launch_bounds__(256) k_band_bwd(SView V, int nG, const double *__restrict__ Dinv,
                                                  const double *__restrict__ Gdinv,
                                                  const double *__restrict__ y, double *x) {
    __shared__ double xwin[BWR];
    __shared__ double t[NB];
    __shared__ double xG[NGMAX];
    const int tid = threadIdx.x, i = tid >> 4, l = tid & 15;
    const int w = V.w, nb = V.nb, W1 = w + 1;
    if (tid < NGMAX) {
        double s = 0.;
        if (tid < nG)
            for (int q2 = tid; q2 < nG; ++q2) s += Gdinv[q2 * NGMAX + tid] * y[nb + q2];
        xG[tid] = s;
        if (tid < nG) x[nb + tid] = s;
    }
    __syncthreads();
    const int nblkb = (nb + NB - 1) / NB;
    for (int b = nblkb - 1; b >= 0; --b) {
        const int j0 = b * NB;
        const int nd = min(NB, nb - j0);
        const int col = j0 + i;
        double s = 0.;
        if (i < nd) {
            // rows k in [j0+NB, min(nb, col+w+1))
            for (int k = j0 + NB + l; k <= col + w && k < nb; k += 16)
                s += V.Bd[(size_t)k * W1 + (col - k + w)] * xwin[k & BMASK];
            if (l < nG) s += V.Ga[(size_t)l * nb + col] * xG[l];
        }
        s = sum16(s);
        if (l == 0 && i < nd) t[i] = y[col] - s;
        __syncthreads();
        double s2 = (i < nd && l >= i && l < nd) ? Dinv[(size_t)b * NB * NB + l * NB + i] * t[l] : 0.;
        s2 = sum16(s2);
        if (l == 0 && i < nd) {
            xwin[col & BMASK] = s2;
            x[col] = s2;
        }
        __syncthreads();
    }
}

void launch_band_potrf(hipStream_t s, const SView &V, int nG, double *Dinv, double *Gdinv,
                       int *fail, long long *probe, int nbk) {
    if (nbk == 8)
        k_band_potrf<8><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, fail, probe);
    else
        k_band_potrf<16><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, fail, probe);
}
void launch_band_fwd(hipStream_t s, const SView &V, int nG, const double *Dinv,
                     const double *Gdinv, const double *r, double *y, int nbk) {
    if (nbk == 8)
        k_band_fwd<8><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, r, y);
    else
        k_band_fwd<16><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, r, y);
}
void launch_band_bwd(hipStream_t s, const SView &V, int nG, const double *Dinv,
                     const double *Gdinv, const double *y, double *x, int nbk) {
    if (nbk == 8)
        k_band_bwd<8><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, y, x);
    else
        k_band_bwd<16><<<1, 256, 0, s>>>(V, nG, Dinv, Gdinv, y, x);
}

}  // namespace mmba
