// mmba_band.hip -- Cholesky factorisation and triangular solves of the reduced
// system in band + arrow layout (CDNA4 / gfx950, fp64).
//
// For frame-ordered camera-frame parameters the reduced system
//   S = [ B   Gᵀ ]   B: nb x nb banded (half bandwidth w: a bundle couples the
//       [ G   D  ]      camera-frames of the frames it is tracked in),
//                    G: nG x nb dense arrow rows (lens, static camera attrs),
// factors with no fill outside the band and the arrow.  A band factorisation
// is a chain (column j needs every update of columns < j), so the rows are
// split into P partitions (nested dissection on the frame axis):
//
//   partition p = interior rows I_p | separator rows S_p (its last w rows)
//   I_p couples only to S_{p-1}, S_p and G, never to another interior.
//
// Stage 1 (one workgroup per partition, concurrently): factor B[I_p, I_p];
// the separator and global rows that touch I_p are the partition's "arrow"
// A_p (<= 2w + nG rows), reduced to Y_p = A_p L_p^-T, and Z_p = Y_p Y_p^T is
// the partition's Schur term.  Stage 2: the separator system
// T = S[seps + G] - sum_p Z_p (band 2w-1 + arrow) is assembled and factored
// by the same kernel with P = 1 ("corner" mode: the global rows are factored
// at the end).  With P = 1 stage 1 alone is the whole factorisation.
//
// Inside one workgroup the band rows stream through an LDS window of WR rows
// in NB-column blocks (right-looking):
//   A. wave 0 factors and inverts the NB x NB diagonal block in registers
//      (lane = row, v_readlane broadcasts); waves 1-3 move the rows the next
//      block needs into the window and the finished rows out,
//   B. panel rows below and arrow rows: P <- P Dinv^T,
//   C. trailing update of the window, the arrow rows and Z (rank NB).
// The solves use the stored NB x NB block inverses: two short reductions per
// block.
#include <cstdlib>

#include "mmba_kernels.h"

namespace mmba {

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

// Row q of a packed lower triangle holding entry e (q(q+1)/2 <= e).
__device__ __forceinline__ int tri_row(int e) {
    int q = (int)((sqrtf(8.f * (float)e + 1.f) - 1.f) * 0.5f);
    if ((q + 1) * (q + 2) / 2 <= e) ++q;
    if (q * (q + 1) / 2 > e) --q;
    return q;
}

// Factor an NB x NB SPD block held one row per lane (lane r = row r; lanes
// >= NB mirror) and invert the factor: on return a[c], c <= r, is row r of L
// and x[] is column r of L^-1 (upper entries of a[] are scratch).  Padding
// rows must be identity.  Branch-free: every lane runs every update,
// broadcasts are v_readlane of wave-uniform lanes, 1/L_jj is the rsq of the
// pivot.  Returns non-zero if a pivot was replaced.
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

// Corner factor of the arrow, one wave: Ld (lower) and Ld^-1 of the packed
// lower nc x nc matrix sZ (na rows used, identity padding), NC a power of 2
// (64 for arrows wider than 32: NGMAX = 48 is not one).
template <int NC>
__device__ __forceinline__ int band_corner(const double *sZ, int na, double *Gd, double *Gdinv) {
    const int tid = threadIdx.x, r = tid & (NC - 1);
    double a[NC], x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) a[c] = (c <= r && r < na) ? sZ[r * (r + 1) / 2 + c] : 0.;
    if (r >= na) a[r] = 1.;
    const int badl = potrf_inv<NC>(a, x);
    if (tid < NC && r < NGMAX) {  // (NC = 64 > NGMAX: the padding rows stay out)
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            if (c >= NGMAX) break;
            Gd[r * NGMAX + c] = (c <= r) ? a[c] : 0.;
            Gdinv[c * NGMAX + r] = x[c];
        }
    }
    return badl;
}

// ---------------------------------------------------------------------------
// Stage-1 / corner factorisation, one workgroup per partition.  CORNER: the
// arrow rows are the nG global rows, Z starts from Gd and is factored at the
// end into Gd / Gdinv.  Otherwise -Z_p (packed lower, na rows) goes to zpool.
// ---------------------------------------------------------------------------
template <int NB, int WR, int WMAX, int NAMAX, bool CORNER>
__global__ void __launch_bounds__(256)
    k_band_factor(double *Bd, int w, const BandPart *__restrict__ parts, double *apool,
                  double *zpool, double *Dinv, double *Gd, double *Gdinv, int *fail,
                  long long *probe) {
    constexpr int WM = WR - 1;
    __shared__ double win[WR][WMAX + 1];
    __shared__ double gwin[NAMAX][WR];
    __shared__ double sX[NB][NB + 1];
    __shared__ double sP[WMAX][NB + 1];
    __shared__ double sPG[NAMAX][NB + 1];
    __shared__ double sZ[NAMAX * (NAMAX + 1) / 2];
    __shared__ int bad;
    // probe (diagnostic, MMBA_PATH_PROBE = 1): thread 0 of workgroup 0 accumulates
    // s_memtime cycles per phase; never read by the solver.
    const bool prb = probe && blockIdx.x == 0 && threadIdx.x == 0;
    long long pt[4] = {0, 0, 0, 0}, tprev = prb ? (long long)clock64() : 0;
    auto stamp = [&](int ph) {
        if (prb) {
            const long long t = (long long)clock64();
            pt[ph] += t - tprev;
            tprev = t;
        }
    };
    const BandPart pd = parts[blockIdx.x];
    const int tid = threadIdx.x;
    const int r0 = pd.r0, r1 = pd.r1, na = pd.na, W1 = w + 1;
    const int ast = r1 - r0;
    const int nz = na * (na + 1) / 2;
    double *A = apool + pd.aoff;
    if (tid == 0) bad = 0;
    for (int e = tid; e < nz; e += blockDim.x) {
        double v = 0.;
        if (CORNER) {
            const int q = tri_row(e);
            v = Gd[q * NGMAX + (e - q * (q + 1) / 2)];
        }
        sZ[e] = v;
    }
    // rows [a, b) enter the window (band entries left of r0 belong to the
    // arrow of this partition and are dropped); t0/nt: participating threads
    auto load_rows = [&](int a, int b, int t0, int nt) {
        for (int e = t0; e < (b - a) * W1; e += nt) {
            const int row = a + e / W1, k = e % W1;
            win[row & WM][k] = (row - w + k >= r0) ? Bd[(size_t)row * W1 + k] : 0.;
        }
        for (int e = t0; e < na * (b - a); e += nt) {
            const int q = e / (b - a), row = a + e % (b - a);
            gwin[q][row & WM] = A[(size_t)q * ast + (row - r0)];
        }
    };
    auto store_rows = [&](int a, int b, int t0, int nt) {
        for (int e = t0; e < (b - a) * W1; e += nt) {
            const int row = a + e / W1, k = e % W1;
            Bd[(size_t)row * W1 + k] = win[row & WM][k];
        }
        for (int e = t0; e < na * (b - a); e += nt) {
            const int q = e / (b - a), row = a + e % (b - a);
            A[(size_t)q * ast + (row - r0)] = gwin[q][row & WM];
        }
    };
    int loaded = min(r1, r0 + NB + w);
    load_rows(r0, loaded, tid, blockDim.x);
    __syncthreads();
    for (int j0 = r0, b = pd.doff; j0 < r1; j0 += NB, ++b) {
        const int nd = min(NB, r1 - j0);
        // A. diagonal block (wave 0) || window traffic (waves 1-3)
        if (tid < 64) {
            const int r = tid & (NB - 1);
            double a[NB], x[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
                a[c] = 0.;
                if (c <= r && r < nd && r - c <= w) a[c] = win[(j0 + r) & WM][c - r + w];
            }
            if (r >= nd) a[r] = 1.;
            const int badl = potrf_inv<NB>(a, x);
            if (tid < NB) {
#pragma unroll
                for (int c = 0; c < NB; ++c) {
                    if (c <= r && r < nd && r - c <= w) win[(j0 + r) & WM][c - r + w] = a[c];
                    sX[c][r] = x[c];
                }
            }
            if (tid == 0 && badl) bad = 1;
        } else {
            const int want = min(r1, j0 + 2 * NB + w);
            if (want > loaded) load_rows(loaded, want, tid - 64, blockDim.x - 64);
            if (j0 > r0) store_rows(j0 - NB, j0, tid - 64, blockDim.x - 64);
        }
        loaded = max(loaded, min(r1, j0 + 2 * NB + w));
        __syncthreads();
        stamp(0);
        // B. panel rows [j0+NB, pend) and arrow rows: P <- P Dinv^T
        const int pend = min(r1, j0 + NB + w);
        const int npan = max(0, pend - (j0 + NB));
        for (int e = tid; e < npan * NB; e += blockDim.x) {
            const int li = e / NB, c = e % NB, i = j0 + NB + li;
            const double *wr = &win[i & WM][0];
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
        for (int e = tid; e < na * NB; e += blockDim.x) {
            const int q = e / NB, c = e % NB;
            double s = 0.;
#pragma unroll
            for (int t = 0; t < NB; ++t)
                s = fma((t < nd) ? gwin[q][(j0 + t) & WM] : 0., sX[c][t], s);
            sPG[q][c] = s;
        }
        __syncthreads();
        stamp(1);
        // C. trailing update (rank NB), panel / arrow columns written back
        for (int e = tid; e < npan * W1; e += blockDim.x) {
            const int li = e / W1, kk = e % W1;
            const int i = j0 + NB + li, k = i - kk;
            if (k < j0 + NB) continue;
            const int lk = k - j0 - NB;
            double s = win[i & WM][w - kk];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sP[li][t], sP[lk][t], s);
            win[i & WM][w - kk] = s;
        }
        for (int e = tid; e < npan * NB; e += blockDim.x) {
            const int li = e / NB, c = e % NB, i = j0 + NB + li, col = j0 + c;
            if (i - col <= w) win[i & WM][col - i + w] = sP[li][c];
        }
        for (int e = tid; e < na * npan; e += blockDim.x) {
            const int q = e / npan, li = e % npan, i = j0 + NB + li;
            double s = gwin[q][i & WM];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sPG[q][t], sP[li][t], s);
            gwin[q][i & WM] = s;
        }
        for (int e = tid; e < nz; e += blockDim.x) {
            const int q = tri_row(e), q2 = e - q * (q + 1) / 2;
            double s = sZ[e];
#pragma unroll
            for (int t = 0; t < NB; ++t) s = fma(-sPG[q][t], sPG[q2][t], s);
            sZ[e] = s;
        }
        for (int e = tid; e < na * nd; e += blockDim.x) {
            const int q = e / nd, c = e % nd;
            gwin[q][(j0 + c) & WM] = sPG[q][c];
        }
        for (int e = tid; e < NB * NB; e += blockDim.x)
            Dinv[(size_t)b * NB * NB + e] = sX[e / NB][e % NB];
        __syncthreads();
        stamp(2);
    }
    if (r1 > r0) {
        const int jl = r0 + ((r1 - r0 - 1) / NB) * NB;
        store_rows(jl, r1, tid, blockDim.x);
    }
    if (CORNER) {
        // Ld Ld^T = D - Y Y^T (accumulated in sZ), na = nG <= NGMAX
        if (na > 0 && tid < 64) {
            // (NC a power of two: lanes r = tid & (NC - 1))
            const int badl = na <= 16   ? band_corner<16>(sZ, na, Gd, Gdinv)
                             : na <= 32 ? band_corner<32>(sZ, na, Gd, Gdinv)
                                        : band_corner<64>(sZ, na, Gd, Gdinv);
            if (tid == 0 && badl) bad = 1;
        }
    } else {
        for (int e = tid; e < nz; e += blockDim.x) zpool[pd.zoff + e] = sZ[e];
    }
    __syncthreads();
    stamp(3);
    if (tid == 0 && bad) atomicOr(fail, 1);
    if (prb)
        for (int k = 0; k < 4; ++k) atomicAdd((unsigned long long *)&probe[k], (unsigned long long)pt[k]);
}

// Sum over the 16 lanes of a lane group.
__device__ __forceinline__ double sum16(double v) {
    v += __shfl_xor(v, 8, 16);
    v += __shfl_xor(v, 4, 16);
    v += __shfl_xor(v, 2, 16);
    v += __shfl_xor(v, 1, 16);
    return v;
}

// ---------------------------------------------------------------------------
// Forward solve of one partition: y_I = L_I^-1 r_I and the arrow sums
// c_a = sum_c Y[a][c] y_c.  CORNER: y_G = Ld^-1 (r_G - c) into y[nb + q];
// otherwise c goes to cpool.  Thread (i = tid/16, l = tid%16): row i of the
// current block.  r and y are in reduced-system order (length nb + nG).
// ---------------------------------------------------------------------------
template <int NB, int WR, bool CORNER>
__global__ void __launch_bounds__(256)
    k_band_fwd(const double *__restrict__ Bd, int w, int nb, const BandPart *__restrict__ parts,
               const double *__restrict__ apool, const double *__restrict__ Dinv,
               const double *__restrict__ Gdinv, double *cpool, const double *__restrict__ r,
               double *y) {
    constexpr int WM = WR - 1;
    __shared__ double ywin[WR];
    __shared__ double t[NB];
    __shared__ double csum[2 * WBAND_PART + NGMAX];
    __shared__ double tg[NGMAX];
    const BandPart pd = parts[blockIdx.x];
    const int tid = threadIdx.x, i = tid >> 4, l = tid & 15;
    const int r0 = pd.r0, r1 = pd.r1, na = pd.na, W1 = w + 1, ast = r1 - r0;
    const double *A = apool + pd.aoff;
    for (int a = tid; a < na; a += blockDim.x) csum[a] = 0.;
    __syncthreads();
    for (int j0 = r0, b = pd.doff; j0 < r1; j0 += NB, ++b) {
        const int nd = min(NB, r1 - j0);
        const int row = j0 + i;
        double s = 0.;
        if (i < nd) {
            // columns k in [max(r0, row - w), j0): kk = j0 - 1 - k < w - i
            for (int kk = l; kk < w - i; kk += 16) {
                const int k = j0 - 1 - kk;
                if (k < r0) break;
                s += Bd[(size_t)row * W1 + (k - row + w)] * ywin[k & WM];
            }
        }
        s = sum16(s);
        if (l == 0 && i < nd) t[i] = r[row] - s;
        __syncthreads();
        double s2 = (i < nd && l <= i) ? Dinv[(size_t)b * NB * NB + i * NB + l] * t[l] : 0.;
        s2 = sum16(s2);
        if (l == 0 && i < nd) {
            ywin[row & WM] = s2;
            y[row] = s2;
        }
        __syncthreads();
        // arrow sums: lane group i takes arrow rows i, i+16, ...; lane l = column
        for (int a = i; a < na; a += 16) {
            double p = (l < nd) ? A[(size_t)a * ast + (j0 - r0 + l)] * ywin[(j0 + l) & WM] : 0.;
            p = sum16(p);
            if (l == 0) csum[a] += p;
        }
    }
    __syncthreads();
    if (CORNER) {
        if (tid < na) tg[tid] = r[nb + tid] - csum[tid];
        __syncthreads();
        if (tid < na) {
            double s = 0.;
            for (int q2 = 0; q2 <= tid; ++q2) s += Gdinv[tid * NGMAX + q2] * tg[q2];
            y[nb + tid] = s;
        }
    } else {
        for (int a = tid; a < na; a += blockDim.x) cpool[pd.coff + a] = csum[a];
    }
}

// ---------------------------------------------------------------------------
// Backward solve of one partition: x_I = L_I^-T (y_I - Y^T x_A).  CORNER: x_A
// = x_G = Ld^-T y_G (also written to x[nb + q]); otherwise x_A is read from x
// at the separator / global positions (filled by the separator solve first).
// ---------------------------------------------------------------------------
template <int NB, int WR, bool CORNER>
__global__ void __launch_bounds__(256)
    k_band_bwd(const double *__restrict__ Bd, int w, int nb, const BandPart *__restrict__ parts,
               const double *__restrict__ apool, const double *__restrict__ Dinv,
               const double *__restrict__ Gdinv, const double *__restrict__ y, double *x) {
    constexpr int WM = WR - 1;
    __shared__ double xwin[WR];
    __shared__ double t[NB];
    __shared__ double xA[2 * WBAND_PART + NGMAX];
    const BandPart pd = parts[blockIdx.x];
    const int tid = threadIdx.x, i = tid >> 4, l = tid & 15;
    const int r0 = pd.r0, r1 = pd.r1, na = pd.na, W1 = w + 1, ast = r1 - r0;
    const double *A = apool + pd.aoff;
    if (CORNER) {
        if (tid < na) {
            double s = 0.;
            for (int q2 = tid; q2 < na; ++q2) s += Gdinv[q2 * NGMAX + tid] * y[nb + q2];
            xA[tid] = s;
            x[nb + tid] = s;
        }
    } else {
        for (int a = tid; a < na; a += blockDim.x) {
            int src;
            if (a < pd.nprev)
                src = pd.sprev + a;
            else if (a < pd.nprev + pd.nnext)
                src = pd.snext + (a - pd.nprev);
            else
                src = nb + (a - pd.nprev - pd.nnext);
            xA[a] = x[src];
        }
    }
    __syncthreads();
    const int nblk = (r1 - r0 + NB - 1) / NB;
    for (int bb = nblk - 1; bb >= 0; --bb) {
        const int j0 = r0 + bb * NB, b = pd.doff + bb;
        const int nd = min(NB, r1 - j0);
        const int col = j0 + i;
        double s = 0.;
        if (i < nd) {
            for (int k = j0 + NB + l; k <= col + w && k < r1; k += 16)
                s += Bd[(size_t)k * W1 + (col - k + w)] * xwin[k & WM];
            for (int a = l; a < na; a += 16) s += A[(size_t)a * ast + (col - r0)] * xA[a];
        }
        s = sum16(s);
        if (l == 0 && i < nd) t[i] = y[col] - s;
        __syncthreads();
        double s2 =
            (i < nd && l >= i && l < nd) ? Dinv[(size_t)b * NB * NB + l * NB + i] * t[l] : 0.;
        s2 = sum16(s2);
        if (l == 0 && i < nd) {
            xwin[col & WM] = s2;
            x[col] = s2;
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Partition plumbing (P > 1).
// ---------------------------------------------------------------------------
// Arrow rows of every partition from the band / global rows; thread per
// (arrow row, interior column), blockIdx.y = partition.
__global__ void k_band_extract(const double *__restrict__ Bd, int w,
                               const double *__restrict__ Ga, int nb,
                               const BandPart *__restrict__ parts, int P, double *apool) {
    const int p = blockIdx.y;
    if (p >= P) return;
    const BandPart pd = parts[p];
    const int ast = pd.r1 - pd.r0;
    const int W1 = w + 1;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < pd.na * ast;
         e += gridDim.x * blockDim.x) {
        const int a = e / ast, c = pd.r0 + e % ast;
        double v = 0.;
        if (a < pd.nprev) {
            const int k = pd.sprev + a;  // k < c: S[c][k] lives in row c
            if (c - k <= w) v = Bd[(size_t)c * W1 + (k - c + w)];
        } else if (a < pd.nprev + pd.nnext) {
            const int k = pd.snext + (a - pd.nprev);  // k > c: S[k][c] in row k
            if (k - c <= w) v = Bd[(size_t)k * W1 + (c - k + w)];
        } else {
            v = Ga[(size_t)(a - pd.nprev - pd.nnext) * nb + c];
        }
        apool[pd.aoff + e] = v;
    }
}

// zpool entry (a, b) of partition pd: -Z_p[a][b] (packed lower triangle).
__device__ __forceinline__ double zget(const double *zp, const BandPart &pd, int a, int b) {
    if (a < b) {
        const int t = a;
        a = b;
        b = t;
    }
    return zp[pd.zoff + a * (a + 1) / 2 + b];
}

// Separator system T = S[seps + G] - sum_p Z_p (zpool holds -Z_p, the
// partitions' Schur updates, so they are added).  Separator s (band rows
// [parts[s].snext, +w)) -> T rows [s*w, (s+1)*w); half bandwidth wT = 2w-1.
// Partition p has prev separator p-1 (arrow rows 0..w-1) and next separator
// p (arrow rows nprev..nprev+w-1).  Thread per T entry, fixed summation order.
// Sharded: only the partitions [plo, phi) of this shard (and the separator
// rows they own) contribute; the shards' partial T are then summed.
__global__ void k_band_tassemble(const double *__restrict__ Bd, int w,
                                 const double *__restrict__ Ga, const double *__restrict__ Gd,
                                 int nb, int nG, const BandPart *__restrict__ parts, int P,
                                 int plo, int phi, const double *__restrict__ zpool, double *TBd,
                                 double *TGa, double *TGd) {
    auto loc = [&](int p) { return p >= plo && p < phi; };
    const int nsep = P - 1, nbT = nsep * w, wT = 2 * w - 1, W1T = wT + 1, W1 = w + 1;
    const int nband = nbT * W1T, narrow = nG * nbT, ncorner = NGMAX * NGMAX;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nband) {
        const int R = e / W1T, k = e % W1T, C = R - wT + k;
        double v = 0.;
        if (C >= 0) {
            const int sR = R / w, uR = R % w, sC = C / w, uC = C % w;
            const BandPart &pa = parts[sR];
            const int gR = pa.snext + uR, gC = parts[sC].snext + uC;
            if (loc(sR) && gR - gC <= w) v = Bd[(size_t)gR * W1 + (gC - gR + w)];
            if (sR == sC) {
                const BandPart &pb = parts[sR + 1];
                if (loc(sR)) v += zget(zpool, pa, pa.nprev + uR, pa.nprev + uC);
                if (loc(sR + 1)) v += zget(zpool, pb, uR, uC);
            } else if (sR == sC + 1) {  // partition sR: prev = sC, next = sR
                if (loc(sR)) v += zget(zpool, pa, pa.nprev + uR, uC);
            }  // sR == sC + 2 lies inside the T band but is structurally zero
        }
        TBd[e] = v;
    } else if (e < nband + narrow) {
        const int q = (e - nband) / nbT, C = (e - nband) % nbT;
        const int sC = C / w, uC = C % w;
        const BandPart &pa = parts[sC], &pb = parts[sC + 1];
        double v = 0.;
        if (loc(sC)) {
            v = Ga[(size_t)q * nb + pa.snext + uC];
            v += zget(zpool, pa, pa.nprev + pa.nnext + q, pa.nprev + uC);
        }
        if (loc(sC + 1)) v += zget(zpool, pb, pb.nprev + pb.nnext + q, uC);
        TGa[(size_t)q * nbT + C] = v;
    } else if (e < nband + narrow + ncorner) {
        const int q = (e - nband - narrow) / NGMAX, q2 = (e - nband - narrow) % NGMAX;
        double v = 0.;
        if (q < nG && q2 <= q) {
            v = Gd[q * NGMAX + q2];  // this shard's partial global block
            for (int p = plo; p < phi; ++p) {
                const BandPart &pd = parts[p];
                v += zget(zpool, pd, pd.nprev + pd.nnext + q, pd.nprev + pd.nnext + q2);
            }
        }
        TGd[q * NGMAX + q2] = v;
    }
}

// Separator right-hand side: rT = r[seps + G] - sum_p c_p.
__global__ void k_band_trhs(const double *__restrict__ r, int w, int nb, int nG,
                            const BandPart *__restrict__ parts, int P, int plo, int phi,
                            const double *__restrict__ cpool, double *rT) {
    const int nbT = (P - 1) * w;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    auto loc = [&](int p) { return p >= plo && p < phi; };
    if (e < nbT) {
        const int s = e / w, u = e % w;
        const BandPart &pa = parts[s], &pb = parts[s + 1];
        double v = 0.;
        if (loc(s)) v = r[pa.snext + u] - cpool[pa.coff + pa.nprev + u];
        if (loc(s + 1)) v -= cpool[pb.coff + u];
        rT[e] = v;
    } else if (e < nbT + nG) {
        const int q = e - nbT;
        double v = r[nb + q];  // this shard's partial global rows
        for (int p = plo; p < phi; ++p)
            v -= cpool[parts[p].coff + parts[p].nprev + parts[p].nnext + q];
        rT[e] = v;
    }
}

// T-order vector -> reduced-system order (separator rows and globals).
__global__ void k_band_tscatter(const double *__restrict__ vT, int w, int nb, int nG,
                                const BandPart *__restrict__ parts, int P, double *v) {
    const int nbT = (P - 1) * w;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nbT)
        v[parts[e / w].snext + e % w] = vT[e];
    else if (e < nbT + nG)
        v[nb + (e - nbT)] = vT[e];
}

// ---------------------------------------------------------------------------
// Separator form of the sharded solve (BandSolver::pcr_int): the shard's one
// partition has its interior eliminated by parallel cyclic reduction, XA =
// S_II^-1 A^T (column-major, ast rows) and yI = S_II^-1 r_I come from
// pcr_rhs_mc.  A (apool, row-major na x ast) is non-zero only on the first
// and last w interior columns, so every product below runs over those.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int sep_col(int t, int ast, int w) {
    // t-th column of A's non-zero range: [0, min(w, ast)) then [max(w, ast - w), ast)
    const int n0 = min(w, ast);
    return t < n0 ? t : max(w, ast - w) + (t - n0);
}
__device__ __forceinline__ int sep_ncols(int ast, int w) {
    return min(w, ast) + (ast - max(w, ast - w));
}

// zpool: -Z_p = -(A XA) (packed lower), the partition's Schur update of T
__global__ void k_sep_z(const BandPart *__restrict__ part, int w, const double *__restrict__ apool,
                        const double *__restrict__ XA, double *zpool) {
    const BandPart pd = *part;
    const int na = pd.na, ast = pd.r1 - pd.r0, nc = sep_ncols(ast, w);
    const double *A = apool + pd.aoff;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= na * (na + 1) / 2) return;
    int a = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
    while ((a + 1) * (a + 2) / 2 <= e) ++a;
    while (a * (a + 1) / 2 > e) --a;
    const int b = e - a * (a + 1) / 2;
    double acc = 0.;
    for (int t = 0; t < nc; ++t) {
        const int c = sep_col(t, ast, w);
        acc = fma(A[(size_t)a * ast + c], XA[(size_t)b * ast + c], acc);
    }
    zpool[pd.zoff + e] = -acc;
}

// cpool: c_p = A yI (what the partition takes from the separators' rhs)
__global__ void k_sep_c(const BandPart *__restrict__ part, int w, const double *__restrict__ apool,
                        const double *__restrict__ y, double *cpool) {
    const BandPart pd = *part;
    const int na = pd.na, ast = pd.r1 - pd.r0, nc = sep_ncols(ast, w);
    const double *A = apool + pd.aoff;
    const int a = blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= na) return;
    double acc = 0.;
    for (int t = 0; t < nc; ++t) {
        const int c = sep_col(t, ast, w);
        acc = fma(A[(size_t)a * ast + c], y[pd.r0 + c], acc);
    }
    cpool[pd.coff + a] = acc;
}

// x_I = yI - XA x_A, x_A = x at the partition's separator rows (solved first)
__global__ void k_sep_back(const BandPart *__restrict__ part, const double *__restrict__ XA,
                           const double *__restrict__ y, double *x) {
    __shared__ double xA[2 * WBAND_PART];
    const BandPart pd = *part;
    const int na = pd.na, ast = pd.r1 - pd.r0;
    for (int a = threadIdx.x; a < na; a += blockDim.x)
        xA[a] = x[a < pd.nprev ? pd.sprev + a : pd.snext + (a - pd.nprev)];
    __syncthreads();
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= ast) return;
    double acc = y[pd.r0 + r];
    for (int a = 0; a < na; ++a) acc = fma(-XA[(size_t)a * ast + r], xA[a], acc);
    x[pd.r0 + r] = acc;
}

// ---------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------
static inline int nblk_(long n, int bs) { return (int)((n + bs - 1) / bs); }

void band_factor(hipStream_t s, const BandSolver &B, int *fail, long long *probe) {
    if (B.use_bcr) {
        bcr_factor(s, B, fail, probe);
        return;
    }
    if (B.P == 1) {
        if (B.w <= WBAND_PART)
            k_band_factor<8, 64, WBAND_PART, NGMAX, true><<<1, 256, 0, s>>>(
                B.Bd, B.w, B.d_parts, B.Ga, nullptr, B.Dinv, B.Gd, B.Gdinv, fail, probe);
        else
            k_band_factor<8, 128, WBAND_MAX, NGMAX, true><<<1, 256, 0, s>>>(
                B.Bd, B.w, B.d_parts, B.Ga, nullptr, B.Dinv, B.Gd, B.Gdinv, fail, probe);
        return;
    }
    const int nbT = (B.P - 1) * B.w;
    const int nloc = B.p_hi - B.p_lo;
    {
        dim3 grid(nblk_(B.max_arrow, 256), nloc);
        k_band_extract<<<grid, 256, 0, s>>>(B.Bd, B.w, B.Ga, B.nb, B.d_parts + B.p_lo, nloc,
                                            B.apool);
    }
    if (B.pcr_int && !B.df_off) {  // (a timed-out wait: the band chains)
        // the interior's reduction (its logs), then XA = S_II^-1 A^T and -A XA
        const BandPart &hp = B.hpart;
        const int ast = hp.r1 - hp.r0;
        pcr_solve(s, B.ipcr, B.izero, B.ix, nullptr, fail);
        pcr_rhs_mc(s, B.ipcr, B.apool + hp.aoff, ast, hp.na, B.XA, ast, fail);
        k_sep_z<<<nblk_((long)hp.na * (hp.na + 1) / 2, 256), 256, 0, s>>>(
            B.d_parts + B.p_lo, B.w, B.apool, B.XA, B.zpool);
    } else {
        k_band_factor<8, 64, WBAND_PART, 2 * WBAND_PART + NGPART, false><<<nloc, 256, 0, s>>>(
            B.Bd, B.w, B.d_parts + B.p_lo, B.apool, B.zpool, B.Dinv, nullptr, nullptr, fail, probe);
    }
    {
        const int n = nbT * (2 * B.w) + B.nG * nbT + NGMAX * NGMAX;
        k_band_tassemble<<<nblk_(n, 256), 256, 0, s>>>(B.Bd, B.w, B.Ga, B.Gd, B.nb, B.nG,
                                                       B.d_parts, B.P, B.p_lo, B.p_hi, B.zpool,
                                                       B.TBd, B.TGa, B.TGd);
    }
    if (B.comm) B.comm->allreduce(B.TBd, B.tcount, ReduceOp::Sum, s);
    k_band_factor<8, 128, WBAND_MAX, NGMAX, true><<<1, 256, 0, s>>>(
        B.TBd, 2 * B.w - 1, B.d_tpart, B.TGa, nullptr, B.TDinv, B.TGd, B.TGdinv, fail, nullptr);
}

void band_factor_forward(hipStream_t s, const BandSolver &B, int *fail, long long *probe,
                         const double *r, double *y) {
    if (B.use_bcr) {
        bcr_factor(s, B, fail, probe, r, y);
        return;
    }
    band_factor(s, B, fail, probe);
    band_forward(s, B, r, y);
}

void band_forward(hipStream_t s, const BandSolver &B, const double *r, double *y) {
    if (B.use_bcr) {
        bcr_forward(s, B, r, y);
        return;
    }
    if (B.P == 1) {
        if (B.w <= WBAND_PART)
            k_band_fwd<8, 64, true><<<1, 256, 0, s>>>(B.Bd, B.w, B.nb, B.d_parts, B.Ga, B.Dinv,
                                                       B.Gdinv, nullptr, r, y);
        else
            k_band_fwd<8, 128, true><<<1, 256, 0, s>>>(B.Bd, B.w, B.nb, B.d_parts, B.Ga, B.Dinv,
                                                        B.Gdinv, nullptr, r, y);
        return;
    }
    const int nbT = (B.P - 1) * B.w;
    const int nloc = B.p_hi - B.p_lo;
    if (B.pcr_int && !B.df_off) {  // y_I = S_II^-1 r_I, c = A y_I
        const BandPart &hp = B.hpart;
        const int ast = hp.r1 - hp.r0;
        pcr_rhs_mc(s, B.ipcr, r + hp.r0, ast, 1, y + hp.r0, ast, B.fail);
        k_sep_c<<<1, 64, 0, s>>>(B.d_parts + B.p_lo, B.w, B.apool, y, B.cpool);
    } else {
        k_band_fwd<8, 64, false><<<nloc, 256, 0, s>>>(B.Bd, B.w, B.nb, B.d_parts + B.p_lo,
                                                       B.apool, B.Dinv, nullptr, B.cpool, r, y);
    }
    k_band_trhs<<<nblk_(nbT + B.nG, 256), 256, 0, s>>>(r, B.w, B.nb, B.nG, B.d_parts, B.P,
                                                       B.p_lo, B.p_hi, B.cpool, B.rT);
    if (B.comm) B.comm->allreduce(B.rT, nbT + B.nG, ReduceOp::Sum, s);
    k_band_fwd<8, 128, true><<<1, 256, 0, s>>>(B.TBd, 2 * B.w - 1, nbT, B.d_tpart, B.TGa,
                                                B.TDinv, B.TGdinv, nullptr, B.rT, B.yT);
    k_band_tscatter<<<nblk_(nbT + B.nG, 256), 256, 0, s>>>(B.yT, B.w, B.nb, B.nG, B.d_parts,
                                                           B.P, y);
}

void band_backward(hipStream_t s, const BandSolver &B, const double *y, double *x) {
    if (B.use_bcr) {
        bcr_backward(s, B, y, x);
        return;
    }
    if (B.P == 1) {
        if (B.w <= WBAND_PART)
            k_band_bwd<8, 64, true><<<1, 256, 0, s>>>(B.Bd, B.w, B.nb, B.d_parts, B.Ga, B.Dinv,
                                                       B.Gdinv, y, x);
        else
            k_band_bwd<8, 128, true><<<1, 256, 0, s>>>(B.Bd, B.w, B.nb, B.d_parts, B.Ga, B.Dinv,
                                                        B.Gdinv, y, x);
        return;
    }
    const int nbT = (B.P - 1) * B.w;
    // the separator system first (its right-hand side is the yT band_forward
    // left for this y), then every partition
    k_band_bwd<8, 128, true><<<1, 256, 0, s>>>(B.TBd, 2 * B.w - 1, nbT, B.d_tpart, B.TGa,
                                                B.TDinv, B.TGdinv, B.yT, B.xT);
    k_band_tscatter<<<nblk_(nbT + B.nG, 256), 256, 0, s>>>(B.xT, B.w, B.nb, B.nG, B.d_parts,
                                                           B.P, x);
    if (B.pcr_int && !B.df_off) {  // (a timed-out wait: the band chains)
        const int ast = B.hpart.r1 - B.hpart.r0;
        k_sep_back<<<nblk_(ast, 256), 256, 0, s>>>(B.d_parts + B.p_lo, B.XA, y, x);
        return;
    }
    k_band_bwd<8, 64, false><<<B.p_hi - B.p_lo, 256, 0, s>>>(
        B.Bd, B.w, B.nb, B.d_parts + B.p_lo, B.apool, B.Dinv, nullptr, y, x);
}

}  // namespace mmba
