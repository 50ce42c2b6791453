// mmba_bcr.hip -- block cyclic reduction (BCR) Cholesky of the reduced
// camera system for CDNA4 (gfx950), fp64.
//
// The band + arrow system of mmba_band.hip (half bandwidth w <= 32, nG <= 16
// dense arrow rows) is viewed as block tridiagonal with K x K blocks, K = the
// smallest multiple of 8 >= w, plus the arrow:
//
//   block b: diagonal D_b, coupling L_b = S[b, b-1] (K x K), arrow G_b (nG x K).
//
// A sequential band Cholesky is a chain of nb columns.  BCR factors the same
// matrix in the odd-even (nested-dissection) order: at level l (stride s =
// 2^l) every odd active block o is eliminated at once,
//
//   C_o C_o^T = D_o,  U_o = C_o^-1 L_o,  V_o = C_o^-1 L_{o+s}^T,  Y_o = C_o^-1 G_o^T,
//   D_{o-s} -= U_o^T U_o,  D_{o+s} -= V_o^T V_o,  L'_{o+s} = -V_o^T U_o,
//   G_{o-s} -= Y_o^T U_o,  G_{o+s} -= Y_o^T V_o,  D_G -= Y_o^T Y_o,
//
// which is exactly the Cholesky factor of the permuted matrix (its column o
// holds C_o, U_o^T, V_o^T, Y_o^T), so ||L^-1 r|| and the solution are those of
// any Cholesky of S.  The chain shrinks from nb columns to log2(nb / K) levels
// of K columns each; C4 (nb = 2,994, w = 23): 125 blocks of 24, 7 levels.
//
// One launch per level.  Workgroup per even active block e ("even owner"):
// waves 0 / 1 factor the two odd neighbours o1 = e - s / o2 = e + s
// concurrently (lane = row, pivots and columns broadcast through LDS), every
// wave then forms the products with the explicit inverses C^-1, and the
// workgroup updates D_e, G_e and the new coupling of e in place.  o2 is owned
// by e (its C^-1, U, V, Y are stored for the solves and its Y^T Y for the
// corner); o1 is recomputed bit-identically by e and by its owner e - 2s, so a
// level needs no second launch.  L is double-buffered across levels (the new
// coupling of e + 2s is written while e still reads the old one).  The last
// active block and the arrow corner are factored densely by one workgroup.
//
// Solves: forward, one launch per level (workgroup per even block, both odd
// neighbours' y = C^-1 r by matrix-vector products, r_e updated in place in a
// work copy); backward, one launch per level (workgroup per odd block).
#include <algorithm>
#include <atomic>

#include "mmba_bcr_dev.h"
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

__device__ __forceinline__ double *bcr_blk(double *base, int b, int K) {
    return base + (size_t)b * K * K;
}

// Vector entry R of a reduced-order vector; block rows at or beyond nb are
// padding (value 0, never stored).
__device__ __forceinline__ double bcr_get(const double *v, int R, int nb) {
    return R < nb ? v[R] : 0.;
}
// bcr_get of a handed-off vector (sc1 load, see bcr_ld)
__device__ __forceinline__ double bcr_get_sc1(const double *v, int R, int nb) {
    return R < nb ? bcr_ld(v + R) : 0.;
}


// ---------------------------------------------------------------------------
// Band rows -> blocks.  Workgroup per block b.
// ---------------------------------------------------------------------------
template <int K>
__global__ void __launch_bounds__(256) k_bcr_load(BcrDev B, const double *r) {
    const int b = blockIdx.x;
    if (r) {  // fused forward solve: work copy of the right-hand side
        for (int i = threadIdx.x; i < K; i += blockDim.x)
            if (b * K + i < B.nb) B.rw[b * K + i] = r[b * K + i];
        if (b == 0)
            for (int q = threadIdx.x; q < B.nG; q += blockDim.x) B.rw[B.nb + q] = r[B.nb + q];
    }
    const int W1 = B.w + 1;
    double *D = bcr_blk(B.Dk, b, K), *L = bcr_blk(B.Lk0, b, K);
    for (int e = threadIdx.x; e < K * K; e += blockDim.x) {
        const int i = e / K, c = e % K;
        const int R = b * K + i;
        double dv = 0., lv = 0.;
        if (R < B.nb) {
            const int C = b * K + c;
            if (c <= i && R - C <= B.w) dv = B.Bd[(size_t)R * W1 + (C - R + B.w)];
            const int Cp = (b - 1) * K + c;  // previous block's column
            if (b > 0 && R - Cp <= B.w) lv = B.Bd[(size_t)R * W1 + (Cp - R + B.w)];
        } else if (i == c) {
            dv = 1.;  // padding rows: identity, uncoupled
        }
        D[e] = dv;
        L[e] = lv;
    }
    for (int e = threadIdx.x; e < B.nG * K; e += blockDim.x) {
        const int q = e / K, c = e % K, C = b * K + c;
        B.Gk[((size_t)b * B.nG + q) * K + c] = C < B.nb ? B.Ga[(size_t)q * B.nb + C] : 0.;
    }
}

// Cholesky + explicit inverse of one K x K block by ONE wave (no workgroup
// barriers): lane r < K holds row r in registers; the pivot is broadcast with
// v_readlane, column j through LDS.  The inverse is formed column-oriented
// (lane = column of the identity, axpy updates: K short dependent steps).
// M: lower, row stride KS -> C.  Ci: C^-1, lower.  col: 64 doubles, idg: K.
template <int K, int KS>
__device__ __forceinline__ void bcr_chol_inv_wave(double *M, double *Ci, double *col, int &bad) {
    const int lane = threadIdx.x & 63;
    double a[K], rsv[K];
#pragma unroll
    for (int c = 0; c < K; ++c) a[c] = (lane < K && c <= lane) ? M[lane * KS + c] : 0.;
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const long long dv = __double_as_longlong(a[j]);
        const int lo = __builtin_amdgcn_readlane((int)(dv & 0xffffffffll), j);
        const int hi = __builtin_amdgcn_readlane((int)(dv >> 32), j);
        double d = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
        if (!(d > 0.) || !isfinite(d)) {
            bad = 1;
            d = 1.;
        }
        const double rs = bcr_rsq(d);
        rsv[j] = rs;  // wave-uniform: 1 / C_jj
        const double l = (lane > j) ? a[j] * rs : 0.;
        a[j] = (lane == j) ? d * rs : (lane > j ? l : a[j]);
        if (lane < K) col[lane] = l;
        wave_lds_sync();
        // rank-1 update of this lane's row; entries right of the diagonal
        // (c > lane) are dead and updated unconditionally (no exec masking)
#pragma unroll
        for (int c = j + 1; c < K; ++c) a[c] = fma(-l, col[c], a[c]);
        wave_lds_sync();
    }
    if (lane < K)
#pragma unroll
        for (int c = 0; c < K; ++c) M[lane * KS + c] = (c <= lane) ? a[c] : 0.;
    wave_lds_sync();
    // inverse, column-oriented: lane = column cc of the identity
    if (lane < K) {
        const int cc = lane;
        double x[K];
#pragma unroll
        for (int i = 0; i < K; ++i) x[i] = (i == cc) ? 1. : 0.;
#pragma unroll
        for (int t = 0; t < K; ++t) {
            x[t] *= rsv[t];  // zero above the diagonal stays zero
#pragma unroll
            for (int i = t + 1; i < K; ++i) x[i] = fma(-M[i * KS + t], x[t], x[i]);
            wave_lds_sync();  // keeps the column loads of step t from being hoisted
        }
#pragma unroll
        for (int i = 0; i < K; ++i) Ci[i * KS + cc] = x[i];
    }
}

// Cholesky of one K x K block by ONE wave (as bcr_chol_inv_wave, without the
// inverse): M (lower, row stride KS) -> C, rs[j] = 1 / C_jj.
template <int K, int KS>
__device__ __forceinline__ void bcr_chol_wave(double *M, double *rs_out, double *col, int &bad) {
    const int lane = threadIdx.x & 63;
    double a[K];
#pragma unroll
    for (int c = 0; c < K; ++c) a[c] = (lane < K && c <= lane) ? M[lane * KS + c] : 0.;
    // Look-ahead: the next pivot only needs column j + 1, whose multiplier
    // l_(j+1) is lane j + 1's own l (broadcast by v_readlane, no LDS), so
    // column j + 1 is updated and the next pivot and its reciprocal root are
    // formed before the LDS round trip of the remaining columns -- the
    // pivot chain overlaps the bulk update.  Same operations and operands as
    // the plain loop (a[j+1] = fma(-l, col[j+1], a[j+1]) with col[j+1] = l_(j+1)).
    double d = bcr_rdlane(a[0], 0);
    bool dbad = !(d > 0.) || !isfinite(d);
    if (dbad) d = 1.;
    double rs = bcr_rsq(d);
#pragma unroll
    for (int j = 0; j < K; ++j) {
        if (dbad) bad = 1;
        const double l = (lane > j) ? a[j] * rs : 0.;
        a[j] = (lane == j) ? d * rs : (lane > j ? l : a[j]);
        if (lane < K) col[lane] = l;
        if (lane == 0) rs_out[j] = rs;
        if (j + 1 < K) {
            const double lj1 = bcr_rdlane(l, j + 1);
            a[j + 1] = fma(-l, lj1, a[j + 1]);
            d = bcr_rdlane(a[j + 1], j + 1);
            dbad = !(d > 0.) || !isfinite(d);
            if (dbad) d = 1.;
            rs = bcr_rsq(d);
        }
        wave_lds_sync();
#pragma unroll
        for (int c = j + 2; c < K; ++c) a[c] = fma(-l, col[c], a[c]);
        wave_lds_sync();
    }
    if (lane < K)
#pragma unroll
        for (int c = 0; c < K; ++c) M[lane * KS + c] = (c <= lane) ? a[c] : 0.;
}

// Augmented Cholesky by ONE wave: lanes 0..K-1 hold the rows of the K x K
// block (lower part of a), lanes K..63 hold right-hand-side columns b
// (a = b^T, all K entries).  Factoring [D, B; B^T, *] leaves C in the block
// rows and (C^-1 b)^T in every right-hand-side lane: the forward
// substitutions ride on the pivot chain (same operations as bcr_trsv_col:
// x_j *= 1 / C_jj, x_c -= C_cj x_j).  The caller loads a[] and stores it
// back (so two waves can factor the same block without an LDS race).
template <int K>
__device__ __forceinline__ void bcr_chol_aug_wave(double (&a)[K], double *rs_out, double *col,
                                                  int &bad) {
    const int lane = threadIdx.x & 63;
    // per-step bookkeeping stays in one register each: lane j keeps 1 / C_jj
    // (stored once after the chain), the pivot checks fold into one flag
    double rsl = 0.;
    double d = bcr_rdlane(a[0], 0);
    double rs = bcr_rsq(d);  // bad pivots: checked once after the chain (bcr_chol_aug_blk)
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const double l = (lane > j) ? a[j] * rs : 0.;
        a[j] = (lane == j) ? d * rs : (lane > j ? l : a[j]);
        if (lane == j) rsl = rs;
        if (lane < K) col[lane] = l;
        // column j is published before the pivot look-ahead, so its LDS
        // reads are in flight while the next reciprocal root is formed
        wave_lds_sync();
        double cv[K];
#pragma unroll
        for (int c = j + 2; c < K; ++c) cv[c] = col[c];
        if (j + 1 < K) {
            const double lj1 = bcr_rdlane(l, j + 1);
            a[j + 1] = fma(-l, lj1, a[j + 1]);
            d = bcr_rdlane(a[j + 1], j + 1);
            rs = bcr_rsq(d);
        }
#pragma unroll
        for (int c = j + 2; c < K; ++c) a[c] = fma(-l, cv[c], a[c]);
        wave_lds_sync();
    }
    const bool anybad = lane < K && !(rsl > 0. && rsl < __builtin_inf());
    if (__builtin_amdgcn_ballot_w64(anybad) != 0) bad = 1;
    if (rs_out && lane < K) rs_out[lane] = rsl;
}

// In-place forward substitution X <- C^-1 X for the column this lane owns
// (x points at its first entry, stride xs between rows); column-oriented
// (axpy) steps so the K dependent steps are short.
template <int K, int KS>
__device__ __forceinline__ void bcr_trsv_col(const double *C, const double *rs, double *x0,
                                             int xs) {
    double x[K];
#pragma unroll
    for (int i = 0; i < K; ++i) x[i] = x0[i * xs];
#pragma unroll
    for (int t = 0; t < K; ++t) {
        x[t] *= rs[t];
#pragma unroll
        for (int i = t + 1; i < K; ++i) x[i] = fma(-C[i * KS + t], x[t], x[i]);
        wave_lds_sync();  // keeps the column loads of step t from being hoisted
    }
#pragma unroll
    for (int i = 0; i < K; ++i) x0[i * xs] = x[i];
}

typedef double bcr_d4 __attribute__((ext_vector_type(4)));

// Updates of the even block with fp64 MFMA (v_mfma_f64_16x16x4_f64): wave w
// owns the 16 x 16 output tile (w >> 1, w & 1) of the (padded 32 x 32)
// K x K results
//   D_e -= V1^T V1 + U2^T U2   (lower tiles),   L'_e = -V1^T U1,
// summing u in K / 4 steps of 4.  A operand lane l: A[l & 15][l >> 4] =
// X[u0 + (l >> 4)][row], B operand B[l >> 4][l & 15] = Y[u0 + (l >> 4)][col];
// result lane l, register r: row (l >> 4) + 4 r, column l & 15.
template <int K, int KS>
__device__ __forceinline__ void bcr_updates_mfma(const double *U1, const double *V1,
                                                 const double *U2, const double *sDe, double *De,
                                                 double *Lo, bool h1, int wv, int lane) {
    const int ti = wv >> 1, tc = wv & 1;
    const int i = ti * 16 + (lane & 15), c = tc * 16 + (lane & 15), k4 = lane >> 4;
    const bool dtile = tc <= ti;
    bcr_d4 dacc = {0., 0., 0., 0.}, lacc = {0., 0., 0., 0.};
#pragma unroll
    for (int u0 = 0; u0 < K; u0 += 4) {
        const int u = u0 + k4;
        const double v1i = i < K ? V1[u * KS + i] : 0.;
        if (dtile) {
            const double v1c = c < K ? V1[u * KS + c] : 0.;
            const double u2i = i < K ? U2[u * KS + i] : 0.;
            const double u2c = c < K ? U2[u * KS + c] : 0.;
            dacc = __builtin_amdgcn_mfma_f64_16x16x4f64(v1i, v1c, dacc, 0, 0, 0);
            dacc = __builtin_amdgcn_mfma_f64_16x16x4f64(u2i, u2c, dacc, 0, 0, 0);
        }
        if (h1) {
            const double u1c = c < K ? U1[u * KS + c] : 0.;
            lacc = __builtin_amdgcn_mfma_f64_16x16x4f64(v1i, u1c, lacc, 0, 0, 0);
        }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int row = ti * 16 + k4 + 4 * r, col = tc * 16 + (lane & 15);
        if (row < K && col < K) {
            if (dtile && col <= row) bcr_st(&De[row * K + col], sDe[row * KS + col] - dacc[r]);
            if (h1) bcr_st(&Lo[row * K + col], -lacc[r]);
        }
    }
}

// Entry (i, c) of block b of D and of the coupling L = S[b, b-1], read from
// the band layout (k_bcr_load's job; padding rows: identity, uncoupled).
template <int K>
__device__ __forceinline__ void bcr_band_dl(const BcrDev &B, int b, int q, double &dv,
                                            double &lv) {
    const int i = q / K, c = q % K, R = b * K + i, W1 = B.w + 1;
    dv = 0.;
    lv = 0.;
    if (R < B.nb) {
        const int C = b * K + c;
        if (c <= i && R - C <= B.w) dv = B.Bd[(size_t)R * W1 + (C - R + B.w)];
        const int Cp = (b - 1) * K + c;
        if (b > 0 && R - Cp <= B.w) lv = B.Bd[(size_t)R * W1 + (Cp - R + B.w)];
    } else if (i == c) {
        dv = 1.;
    }
}

// ---------------------------------------------------------------------------
// One elimination level, one item: the even block e = t s (t even) and its
// odd neighbours.  band: level 0 of the dataflow factor, operands staged
// straight from the band layout and the right-hand side rsrc (no load pass).
// ---------------------------------------------------------------------------
// GX: arrow capacity (NGLANE: the arrow rides in spare lanes of the augmented
// pivot chains; NGMAX: wider arrows, the separate triangular solves)
template <int K, int CH, bool MF, int GX = NGLANE>  // CH: pivot chain variant (BcrDev::regchol); MF: MFMA updates
__device__ __forceinline__ void bcr_level_item(const BcrDev &B, int s, int nact, int ping,
                                               const int t, int *fail, long long *probe,
                                               double *y, bool band, const double *rsrc,
                                               int *pub = nullptr, unsigned pub_epoch = 0) {
    constexpr int KS = K + 2;     // even row stride: 16-B aligned rows
    constexpr int CG = K / 4;     // columns per update task
    constexpr int GS = GX;        // row stride of the K x nG arrays
    __shared__ double sD[2][K * KS];   // D_o1, D_o2 -> C_o1, C_o2
    // right-hand sides, solved in place: Lo1 -> U1, Le^T -> V1, Lo2 -> U2, Ln^T -> V2
    __shared__ double sB[4][K * KS];
    __shared__ double sGT[2][K * GS];  // G_o^T -> Y_o
    __shared__ double sR[3][K];        // r_o1 -> y1, r_o2 -> y2, r_e (fused forward solve)
    __shared__ double sRs[2][K];       // 1 / C_jj
    __shared__ double col[4][64 * (MMBA_BCR_PW > 8 ? MMBA_BCR_PW : 8)];  // pivot column (LDS chain) / panel image (blocked chain)
    __shared__ double sDe[K * KS], sGe[GX * K];
    __shared__ double sZero[2];
    __shared__ int bad_s;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int e = t * s;
    const bool h1 = t >= 2;                 // o1 = e - s exists (and so does its prev e - 2s)
    const bool h2 = t + 1 < nact;           // o2 = e + s
    const bool hn = t + 2 < nact;           // e + 2s (o2's next)
    const int o1 = e - s, o2 = e + s, en = e + 2 * s;
    const int nG = B.nG;
    const bool fwd = y != nullptr;
    const double *Lin = ping ? B.Lk1 : B.Lk0;
    double *Lout = ping ? B.Lk0 : B.Lk1;
    if (tid == 0) bad_s = 0;
    if (tid == 1) sZero[0] = 0.;
    // probe (diagnostic, MMBA_PATH_PROBE = 1): thread 0 of workgroup 0 accumulates
    // wall-clock ticks (100 MHz) per phase; never read by the solver.
    const bool prb = probe && blockIdx.x == 0 && tid == 0;
    long long tprev = prb ? (long long)wall_clock64() : 0;
    auto stamp = [&](int ph) {
        if (prb) {
            const long long tn = (long long)wall_clock64();
            atomicAdd((unsigned long long *)&probe[ph], (unsigned long long)(tn - tprev));
            tprev = tn;
        }
    };
    // the right-hand-side rows first: their loads join the operand loads
    // below (one memory round trip for the whole stage)
    double rv = 0.;
    if (tid < 3 * K) {
        const int w = tid / K, i = tid % K;
        const int blk = w == 0 ? o1 : (w == 1 ? o2 : e);
        const bool hv = fwd && (w == 0 ? h1 : (w == 1 ? h2 : true));
        rv = hv ? (band ? bcr_get(rsrc, blk * K + i, B.nb) : bcr_get_sc1(B.rw, blk * K + i, B.nb))
                : 0.;
    }
    // stage every operand (zeros where a neighbour does not exist); fixed
    // trip count so every round's loads are issued before the first store
#pragma unroll
    for (int q0 = 0; q0 < K * K; q0 += 256) {
        const int q = q0 + tid;
        if (q >= K * K) break;
        const int i = q / K, c = q % K, x = i * KS + c, xt = c * KS + i;
        double d0 = 0., d1 = 0., b0 = 0., b1 = 0., b2 = 0., b3 = 0., de, dz;
        if (band) {
            if (h1) bcr_band_dl<K>(B, o1, q, d0, b0);
            bcr_band_dl<K>(B, e, q, de, b1);
            if (!h1) b1 = 0.;
            if (h2) bcr_band_dl<K>(B, o2, q, d1, b2);
            if (hn) bcr_band_dl<K>(B, en, q, dz, b3);
        } else {
            // lower part only (the upper part of a stored block is never written)
            // (stored by the previous level's items of this launch: sc1 loads)
            if (h1 && c <= i) d0 = bcr_ld(bcr_blk(B.Dk, o1, K) + q);
            if (h2 && c <= i) d1 = bcr_ld(bcr_blk(B.Dk, o2, K) + q);
            if (h1) b0 = bcr_ld(bcr_blk((double *)Lin, o1, K) + q);
            if (h1) b1 = bcr_ld(bcr_blk((double *)Lin, e, K) + q);
            if (h2) b2 = bcr_ld(bcr_blk((double *)Lin, o2, K) + q);
            if (hn) b3 = bcr_ld(bcr_blk((double *)Lin, en, K) + q);
            de = bcr_ld(bcr_blk(B.Dk, e, K) + q);
        }
        sD[0][x] = d0;
        sD[1][x] = d1;
        sB[0][x] = b0;
        sB[1][xt] = b1;  // Le^T
        sB[2][x] = b2;
        sB[3][xt] = b3;  // Ln^T
        sDe[x] = de;
    }
    for (int q = tid; q < 2 * K * GS; q += blockDim.x) {
        const int which = q / (K * GS), r = q % (K * GS), u = r / GS, qq = r % GS;
        const int o = which ? o2 : o1;
        const bool h = which ? h2 : h1;
        double g = 0.;
        if (h && qq < nG) {
            const int C = o * K + u;
            g = band ? (C < B.nb ? B.Ga[(size_t)qq * B.nb + C] : 0.)
                     : bcr_ld(&B.Gk[((size_t)o * nG + qq) * K + u]);
        }
        sGT[which][r] = g;
    }
    for (int q = tid; q < nG * K; q += blockDim.x) {
        const int C = e * K + q % K;
        sGe[q] = band ? (C < B.nb ? B.Ga[(size_t)(q / K) * B.nb + C] : 0.)
                      : bcr_ld(&B.Gk[(size_t)e * nG * K + q]);
    }
    if (tid < 3 * K) sR[tid / K][tid % K] = rv;
    __syncthreads();
    stamp(0);
    int bad = 0;
    if constexpr (2 * K + GX <= 64) {
        // A+B. Cholesky of the two odd neighbours with their triangular
        // solves fused into the pivot chain (bcr_chol_aug_wave): wave w
        // factors neighbour w & 1; waves 0/1 carry U (and y) in lanes K..,
        // waves 2/3 carry V and Y^T.  Both waves of a neighbour form the
        // same C bit for bit; waves 0/1 store it.
        const int w = wv & 1, half = wv >> 1;
        const bool act = w == 0 ? h1 : h2;
        double *xp = nullptr;
        int xs = 0;
        if (lane >= K && lane < 2 * K) {
            xp = &sB[2 * w + half][lane - K];
            xs = KS;
        } else if (lane >= 2 * K) {
            if (half == 0 && lane == 2 * K && fwd) {
                xp = &sR[w][0];
                xs = 1;
            } else if (half == 1 && lane - 2 * K < nG) {
                xp = &sGT[w][lane - 2 * K];
                xs = GS;
            }
        }
        // one LDS source per lane (rows: D_o with its upper part zeroed by
        // the stage; lanes without an operand read a zero), no per-entry masks
        const double *src = sZero;
        int st = 0;
        if (lane < K) {
            src = &sD[w][lane * KS];
            st = 1;
        } else if (xp) {
            src = xp;
            st = xs;
        }
        double a[K];
#pragma unroll
        for (int c = 0; c < K; ++c) a[c] = src[c * st];
        __syncthreads();  // every wave holds its operands: stores below may overwrite them
        stamp(1);
        if (act) {
            if constexpr (CH == 2)
                bcr_chol_aug_blk<K, MMBA_BCR_PW>(a, half == 0 ? sRs[w] : nullptr, col[wv], bad);
            else
                bcr_chol_aug_wave<K>(a, half == 0 ? sRs[w] : nullptr, col[wv], bad);
        }
        stamp(2);
        if (act) {
            // one LDS destination per lane: C (rows of the half-0 wave; its
            // dead upper entries are stored too, every reader of FC masks
            // them), the solved right-hand sides; other lanes write their own
            // slot of the chain scratch
            double *dst = &col[wv][lane * 8];
            int dt = 0;
            if (lane < K) {
                if (half == 0) {
                    dst = &sD[w][lane * KS];
                    dt = 1;
                }
            } else if (xp) {
                dst = xp;
                dt = xs;
            }
#pragma unroll
            for (int c = 0; c < K; ++c) dst[c * dt] = a[c];
        }
        if (bad) atomicOr(&bad_s, 1);
        __syncthreads();
        stamp(3);
    } else {
    // A. Cholesky of the two odd neighbours, one wave each
    if (wv == 0 && h1) bcr_chol_wave<K, KS>(sD[0], sRs[0], col[0], bad);
    if (wv == 1 && h2) bcr_chol_wave<K, KS>(sD[1], sRs[1], col[1], bad);
    if (bad) atomicOr(&bad_s, 1);
    __syncthreads();
    stamp(1);
    // B. triangular solves, lane = right-hand-side column: wave 0 U1 | V1,
    // wave 1 U2 | V2, wave 2 Y1 | y1, wave 3 Y2 | y2 (C^-1 never formed)
    {
        const int w = wv & 1;  // which neighbour
        if (w == 0 ? h1 : h2) {
            if (wv < 2) {
                if (lane < 2 * K) {
                    const int m = 2 * w + lane / K, c = lane % K;
                    bcr_trsv_col<K, KS>(sD[w], sRs[w], &sB[m][c], KS);
                }
            } else if (lane < nG) {
                bcr_trsv_col<K, KS>(sD[w], sRs[w], &sGT[w][lane], GS);
            } else if (lane == 32 && fwd) {
                bcr_trsv_col<K, KS>(sD[w], sRs[w], &sR[w][0], 1);
            }
        }
    }
    __syncthreads();
    stamp(2);
    stamp(3);
    }
    // C. updates of the even block: D_e -= V1^T V1 + U2^T U2 (lower), new
    // coupling -V1^T U1, G_e -= Y1^T V1 + Y2^T U2; stored factor columns of o2
    const double *U1 = sB[0], *V1 = sB[1], *U2 = sB[2], *V2 = sB[3];
    const double *Y1 = sGT[0], *Y2 = sGT[1];
    double *De = bcr_blk(B.Dk, e, K);
    if constexpr (MF && K <= 32) {
        bcr_updates_mfma<K, KS>(U1, V1, U2, sDe, De, bcr_blk(Lout, e, K), h1, wv, lane);
        stamp(4);
    } else
    for (int q = tid; q < 2 * 4 * K; q += blockDim.x) {
        const int m = q / (4 * K), r = q % (4 * K), i = r / 4, c0 = (r % 4) * CG;
        if (m == 0) {
            if (c0 > i) continue;
            double acc[CG];
#pragma unroll
            for (int c = 0; c < CG; ++c) acc[c] = 0.;
#pragma unroll 2
            for (int u = 0; u < K; ++u) {
                const double v = V1[u * KS + i], w2 = U2[u * KS + i];
#pragma unroll
                for (int c = 0; c < CG; ++c)
                    acc[c] = fma(v, V1[u * KS + c0 + c], fma(w2, U2[u * KS + c0 + c], acc[c]));
            }
#pragma unroll
            for (int c = 0; c < CG; ++c)
                if (c0 + c <= i) bcr_st(&De[i * K + c0 + c], sDe[i * KS + c0 + c] - acc[c]);
        } else if (h1) {
            double acc[CG];
#pragma unroll
            for (int c = 0; c < CG; ++c) acc[c] = 0.;
#pragma unroll 2
            for (int u = 0; u < K; ++u) {
                const double v = V1[u * KS + i];
#pragma unroll
                for (int c = 0; c < CG; ++c) acc[c] = fma(v, U1[u * KS + c0 + c], acc[c]);
            }
#pragma unroll
            for (int c = 0; c < CG; ++c) bcr_st(&bcr_blk(Lout, e, K)[i * K + c0 + c], -acc[c]);
        }
    }
    if (fwd) {  // r_e -= V1^T y1 + U2^T y2; the owner of o2 stores y2 and Y2^T y2
        const int ft = (tid + 256 - ((8 * K) & 255)) & 255;  // threads idle in the loop above first
        if (ft < K) {
            double acc0 = 0., acc1 = 0.;
#pragma unroll
            for (int u = 0; u < K; ++u) {
                acc0 = fma(V1[u * KS + ft], sR[0][u], acc0);
                acc1 = fma(U2[u * KS + ft], sR[1][u], acc1);
            }
            const int R = e * K + ft;
            if (R < B.nb) bcr_st(&B.rw[R], sR[2][ft] - (acc0 + acc1));
        } else if (h2 && ft >= 32 && ft < 32 + K) {
            const int i = ft - 32, R = o2 * K + i;
            if (R < B.nb) y[R] = sR[1][i];
        } else if (h2 && ft >= 64 && ft < 64 + nG) {
            const int q = ft - 64;
            double acc = 0.;
            for (int u = 0; u < K; ++u) acc = fma(Y2[u * GS + q], sR[1][u], acc);
            bcr_st(&B.gpart[(size_t)o2 * nG + q], acc);
        }
    }
    if (pub && nG == 0) {
        // dataflow factor without an arrow: the next level reads only D_e,
        // the new coupling and r_e, all stored above -- release them now;
        // the factor columns of o2 below are read by later launches only
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            __hip_atomic_store((bcr_gu32 *)pub, pub_epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int q = tid; q < nG * 4; q += blockDim.x) {
        const int qq = q / 4, c0 = (q % 4) * CG;
        double acc[CG];
#pragma unroll
        for (int c = 0; c < CG; ++c) acc[c] = 0.;
#pragma unroll 2
        for (int u = 0; u < K; ++u) {
            const double y1 = Y1[u * GS + qq], y2 = Y2[u * GS + qq];
#pragma unroll
            for (int c = 0; c < CG; ++c)
                acc[c] = fma(y1, V1[u * KS + c0 + c], fma(y2, U2[u * KS + c0 + c], acc[c]));
        }
#pragma unroll
        for (int c = 0; c < CG; ++c)
            bcr_st(&B.Gk[((size_t)e * nG + qq) * K + c0 + c], sGe[qq * K + c0 + c] - acc[c]);
    }
    if (h2) {
        // factor column of o2 for the solves: C with its diagonal replaced by
        // 1 / C_jj, U2, V2 (K x K), Y2 (K x nG), and the corner term Y2^T Y2
        for (int q = tid; q < K * K; q += blockDim.x) {
            const int i = q / K, c = q % K;
            bcr_blk(B.FC, o2, K)[q] = (c == i) ? sRs[1][i] : sD[1][i * KS + c];
            bcr_blk(B.FU, o2, K)[q] = U2[i * KS + c];
            bcr_blk(B.FV, o2, K)[q] = V2[i * KS + c];
        }
        for (int q = tid; q < K * nG; q += blockDim.x) {
            const int i = q / nG, qq = q % nG;
            B.FY[(size_t)o2 * K * nG + q] = Y2[i * GS + qq];
        }
        for (int q = tid; q < nG * nG; q += blockDim.x) {
            const int a = q / nG, c = q % nG;
            double acc = 0.;
            for (int u = 0; u < K; ++u) acc = fma(Y2[u * GS + a], Y2[u * GS + c], acc);
            bcr_st(&B.Zc[(size_t)o2 * nG * nG + q], acc);
        }
    }
    stamp(5);
    if (tid == 0 && bad_s) atomicOr(fail, 1);  // bad_s settled at the solve barrier
}

// One elimination level.  blockIdx.x = even index / 2 (t = 2 blockIdx.x).
template <int K, int CH, bool MF, int GX = NGLANE>
__global__ void __launch_bounds__(256) k_bcr_level(BcrDev B, int s, int nact, int ping,
                                                   int *fail, long long *probe, double *y) {
    bcr_level_item<K, CH, MF, GX>(B, s, nact, ping, 2 * blockIdx.x, fail, probe, y, false,
                                  nullptr);
}

// ---------------------------------------------------------------------------
// Root: block 0 and the arrow corner, dense, one wave.  N = K + nG rounded up
// to 8 (identity padding).  T = [D_0, G_0^T; G_0, Gd - sum_o Y_o^T Y_o] =
// Ct Ct^T, FT = Ct^-1 (lower, N x N).
// ---------------------------------------------------------------------------
// ONE wave (lanes 0..63 of the workgroup; no workgroup barrier inside).
// rg: the arrow rows of the right-hand side (nG entries).
template <int N>
__device__ __forceinline__ void bcr_root_wave(const BcrDev &B, int *fail, double *y,
                                              const double *rg) {
    constexpr int NS = N + 2;
    __shared__ double T[N * NS], Ti[N * NS], col[64];
    __shared__ double zsum[NGMAX * NGMAX], gsum[NGMAX];
    const int lane = threadIdx.x & 63;
    const int K = B.K, nG = B.nG, n0 = K + nG;
    const double *D0 = B.Dk;
    // sum_o Y_o^T Y_o and sum_o gpart_o over the eliminated blocks: lanes
    // stride over o, then a fixed xor-shuffle tree (a serial loop over the
    // blocks was a chain of nblk dependent loads: 78 us at nblk = 360)
    for (int e = 0; e < nG * nG + (y ? nG : 0); ++e) {
        double v = 0.;
        if (e < nG * nG) {
            for (int o = 1 + lane; o < B.nblk; o += 64) v += bcr_ld(&B.Zc[(size_t)o * nG * nG + e]);
        } else {
            const int q = e - nG * nG;
            for (int o = 1 + lane; o < B.nblk; o += 64) v += bcr_ld(&B.gpart[(size_t)o * nG + q]);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        if (lane == 0) {
            if (e < nG * nG)
                zsum[e] = v;
            else
                gsum[e - nG * nG] = v;
        }
    }
    wave_lds_sync();
    // every load of the fill is issued before the first LDS store (a loop of
    // load -> store rounds cost one memory round trip per round)
    constexpr int TR = (N * N + 63) / 64;
    double tv[TR];
#pragma unroll
    for (int t = 0; t < TR; ++t) {
        const int q = lane + 64 * t;
        const int i = q / N, c = q % N;
        double v = 0.;
        if (q >= N * N) {
        } else if (i < K && c < K) {
            v = c <= i ? bcr_ld(&D0[i * K + c]) : 0.;
        } else if (i >= K && i < n0 && c < K) {
            v = bcr_ld(&B.Gk[(i - K) * K + c]);  // block 0 arrow
        } else if (i >= K && i < n0 && c >= K && c <= i) {
            const int a = i - K, b = c - K;
            v = B.Gd[a * NGMAX + b] - zsum[a * nG + b];
        } else if (i == c) {
            v = 1.;  // padding beyond n0
        }
        tv[t] = v;
    }
#pragma unroll
    for (int t = 0; t < TR; ++t) {
        const int q = lane + 64 * t;
        if (q < N * N) T[(q / N) * NS + q % N] = tv[t];
    }
    wave_lds_sync();
    int bad = 0;
    if constexpr (2 * N <= 64) {
        // augmented chain: identity columns in lanes N..2N-1 come out as the
        // columns of Ct^-1 (the same operations as the column-oriented
        // inverse of bcr_chol_inv_wave, riding on the one pivot chain)
        double a[N];
        const int cc = lane - N;
#pragma unroll
        for (int c = 0; c < N; ++c)
            a[c] = lane < N ? (c <= lane ? T[lane * NS + c] : 0.) : (c == cc ? 1. : 0.);
        bcr_chol_aug_wave<N>(a, nullptr, col, bad);
        if (lane >= N && lane < 2 * N)
#pragma unroll
            for (int i = 0; i < N; ++i) Ti[i * NS + cc] = a[i];
    } else {
        bcr_chol_inv_wave<N, NS>(T, Ti, col, bad);
    }
    wave_lds_sync();
    for (int q = lane; q < N * N; q += 64) B.FT[q] = Ti[(q / N) * NS + q % N];
    if (bad && lane == 0) atomicOr(fail, 1);
    if (y) {  // fused forward root: y_T = FT [r_0; r_G - sum_o gpart_o]
        const int nb = B.nb;
        if (lane < K) col[lane] = bcr_get_sc1(B.rw, lane, nb);
        if (lane >= K && lane < n0) {
            const int q = lane - K;
            col[lane] = rg[q] - gsum[q];
        }
        wave_lds_sync();
        if (lane < n0) {
            double acc = 0.;
            for (int u = 0; u <= lane; ++u) acc = fma(Ti[lane * NS + u], col[u], acc);
            if (lane < K) {
                if (lane < nb) y[lane] = acc;
            } else {
                y[nb + lane - K] = acc;
            }
        }
    }
}

template <int N>
__global__ void __launch_bounds__(64) k_bcr_root(BcrDev B, int *fail, double *y) {
    bcr_root_wave<N>(B, fail, y, B.rw + B.nb);
}

// ---------------------------------------------------------------------------
// Solves.  Vectors are in reduced-system order (nb band rows, then nG global
// rows); block rows at or beyond nb are padding (value 0, never stored).
// ---------------------------------------------------------------------------

// Forward level: workgroup (64 lanes) per even block e; lanes 0..K-1 handle
// o1 = e - s, lanes 32..32+K-1 handle o2 = e + s.  y_o = C_o^-1 r_o by
// substitution (row i of C in lane i's registers, y_t broadcast by
// v_readlane); every factor entry is loaded at entry, so the only dependent
// global load is r itself.
template <int K>
__global__ void __launch_bounds__(64) k_bcr_fwd(BcrDev B, int s, int nact, double *rw,
                                                double *y) {
    __shared__ double sy[2][K], sp[2][K];
    const int lane = threadIdx.x, h = lane >> 5, i = lane & 31;
    const int t = 2 * blockIdx.x, e = t * s;
    const bool h1 = t >= 2, h2 = t + 1 < nact;
    const int o = h ? e + s : e - s;
    const bool act = (h ? h2 : h1) && i < K;
    const int nb = B.nb, nG = B.nG;
    double cr[K], cv[K];  // row i of C_o (diagonal 1/C_ii); column i of V_o1 / U_o2
    double r = 0.;
    if (act) {
        const double *Cf = bcr_blk(B.FC, o, K);
        const double *Vc = bcr_blk(h ? B.FU : B.FV, o, K);
#pragma unroll
        for (int u = 0; u < K; ++u) {
            cr[u] = u <= i ? Cf[i * K + u] : 0.;
            cv[u] = Vc[u * K + i];
        }
        r = bcr_get(rw, o * K + i, nb);
    } else {
#pragma unroll
        for (int u = 0; u < K; ++u) cr[u] = cv[u] = 0.;
    }
#pragma unroll
    for (int u = 0; u < K; ++u) {
        if (i == u) r *= cr[u];
        const double y0 = bcr_rdlane(r, u), y1 = bcr_rdlane(r, 32 + u);
        if (i > u) r = fma(-cr[u], h ? y1 : y0, r);
    }
    if (i < K) sy[h][i] = act ? r : 0.;
    __syncthreads();
    if (i < K) {
        double acc = 0.;
#pragma unroll
        for (int u = 0; u < K; ++u) acc = fma(cv[u], sy[h][u], acc);
        sp[h][i] = acc;
    }
    __syncthreads();
    if (lane < K) {  // r_e -= V1^T y1 + U2^T y2
        const int R = e * K + lane;
        if (R < nb) rw[R] -= sp[0][lane] + sp[1][lane];
    }
    if (h2) {  // owner of o2: y and the arrow partial Y2^T y2
        if (h == 1 && i < K && (e + s) * K + i < nb) y[(e + s) * K + i] = r;
        for (int q = lane; q < nG; q += 64) {
            const double *Y2 = B.FY + (size_t)(e + s) * K * nG;
            double acc = 0.;
            for (int u = 0; u < K; ++u) acc = fma(Y2[u * nG + q], sy[1][u], acc);
            B.gpart[(size_t)(e + s) * nG + q] = acc;
        }
    }
}

// Forward root: y_T = FT [r_0; r_G - sum_o gpart_o].
template <int K>
__global__ void __launch_bounds__(64) k_bcr_fwd_root(BcrDev B, const double *rw, double *y) {
    const int N = B.NR;
    __shared__ double v[K + NGMAX];
    const int lane = threadIdx.x, nb = B.nb, nG = B.nG;
    if (lane < K) v[lane] = bcr_get(rw, lane, nb);
    if (lane < NGMAX) v[K + lane] = 0.;
    for (int q = 0; q < nG; ++q) {  // lanes stride over the blocks (see k_bcr_root)
        double gs = 0.;
        for (int o = 1 + lane; o < B.nblk; o += 64) gs += B.gpart[(size_t)o * nG + q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) gs += __shfl_xor(gs, off);
        if (lane == 0) v[K + q] = rw[nb + q] - gs;
    }
    __syncthreads();
    if (lane < K + nG) {
        double acc = 0.;
        for (int u = 0; u <= lane; ++u) acc = fma(B.FT[lane * N + u], v[u], acc);
        if (lane < K) {
            if (lane < nb) y[lane] = acc;
        } else {
            y[nb + lane - K] = acc;
        }
    }
}

// Backward root: x_T = FT^T y_T.
template <int K>
__global__ void __launch_bounds__(64) k_bcr_bwd_root(BcrDev B, const double *y, double *x) {
    const int N = B.NR;
    __shared__ double v[K + NGMAX];
    const int lane = threadIdx.x, nb = B.nb, nG = B.nG;
    if (lane < K) v[lane] = bcr_get(y, lane, nb);
    if (lane < NGMAX) v[K + lane] = lane < nG ? y[nb + lane] : 0.;
    __syncthreads();
    if (lane < K + nG) {
        double acc = 0.;
        for (int u = lane; u < K + nG; ++u) acc = fma(B.FT[u * N + lane], v[u], acc);
        if (lane < K) {
            if (lane < nb) x[lane] = acc;
        } else {
            x[nb + lane - K] = acc;
        }
    }
}

// Backward level: workgroup per odd block o (t = 2 blockIdx.x + 1):
// x_o = C_o^-T (y_o - U_o x_{o-s} - V_o x_{o+s} - Y_o x_G), the last step by
// back substitution (column i of C in lane i's registers).  Factor entries
// are loaded at entry, before the (dependent) x loads.
template <int K>
__global__ void __launch_bounds__(64) k_bcr_bwd(BcrDev B, int s, int nact, const double *y,
                                                double *x) {
    __shared__ double xg[NGMAX], xp[K], xn[K];
    const int lane = threadIdx.x;
    const int t = 2 * blockIdx.x + 1, o = t * s;
    const bool hn = t + 1 < nact;
    const int nb = B.nb, nG = B.nG;
    double ur[K], vr[K], cc[K];  // row lane of U_o, V_o; column lane of C_o (diag 1/C_ii)
    double yo = 0.;
    if (lane < K) {
        const double *U = bcr_blk(B.FU, o, K), *V = bcr_blk(B.FV, o, K);
        const double *Cf = bcr_blk(B.FC, o, K);
#pragma unroll
        for (int u = 0; u < K; ++u) {
            ur[u] = U[lane * K + u];
            vr[u] = hn ? V[lane * K + u] : 0.;
            cc[u] = u >= lane ? Cf[u * K + lane] : 0.;
        }
        yo = bcr_get(y, o * K + lane, nb);
        xp[lane] = bcr_get(x, (o - s) * K + lane, nb);
        xn[lane] = hn ? bcr_get(x, (o + s) * K + lane, nb) : 0.;
    } else {
#pragma unroll
        for (int u = 0; u < K; ++u) ur[u] = vr[u] = cc[u] = 0.;
    }
    if (lane < nG) xg[lane] = x[nb + lane];
    __syncthreads();
    double v = 0.;
    if (lane < K) {
        const double *Y = B.FY + (size_t)o * K * nG;
        v = yo;
#pragma unroll
        for (int u = 0; u < K; ++u) v = fma(-ur[u], xp[u], fma(-vr[u], xn[u], v));
        for (int q = 0; q < nG; ++q) v = fma(-Y[lane * nG + q], xg[q], v);
    }
#pragma unroll
    for (int u = K - 1; u >= 0; --u) {
        if (lane == u) v *= cc[u];
        const double xu = bcr_rdlane(v, u);
        if (lane < u) v = fma(-cc[u], xu, v);
    }
    if (lane < K) {
        const int R = o * K + lane;
        if (R < nb) x[R] = v;
    }
}

// ---------------------------------------------------------------------------
// Backward solve in ONE launch (dataflow): the root and every level's blocks
// are items of a list in dependency order (root, coarsest level, ...,
// level 0; B.ord), dealt round robin to G <= 256 one-wave workgroups (all
// resident, so a wait always ends).  Block o = t 2^l (t odd) needs x of o - s
// and o + s (s = 2^l, both finished earlier in the list) and of the root
// when there is an arrow.  Hand-off per MI355X guide G16 (R1): x rows are
// stored write-through (agent-scope relaxed atomic stores), the storing
// wave drains (vmcnt 0) and one lane stores the block's flag = epoch; a
// consumer polls the producers' flags relaxed (s_sleep), then loads x with
// sc1 loads (bcr_ld; no agent-scope acquire).  Factor rows and y (written by earlier
// launches) are loaded before the wait.  Every spin is bounded: a timeout
// sets bit 1 of *fail (the solve then counts as failed) instead of hanging.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void bcr_put(double *x, int R, double v) {
    __hip_atomic_store((bcr_gu64 *)(x + R), (unsigned long long)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void bcr_publish(int *flags, int o, unsigned epoch, int lane) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0)
        __hip_atomic_store((bcr_gu32 *)(flags + o), epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// true when flags[a] (and flags[b], b >= 0) == epoch; false after the bound
__device__ __forceinline__ bool bcr_wait(const int *flags, int a, int b, unsigned epoch) {
    for (unsigned spins = 0;; ++spins) {
        unsigned fa = __hip_atomic_load((bcr_gu32 *)(flags + a), __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_AGENT);
        unsigned fb = b >= 0 ? __hip_atomic_load((bcr_gu32 *)(flags + b), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : epoch;
        fa = __builtin_amdgcn_readfirstlane(fa);
        fb = __builtin_amdgcn_readfirstlane(fb);
        if (fa == epoch && fb == epoch) break;
        if (spins > (1u << 22)) return false;
        __builtin_amdgcn_s_sleep(2);
    }
    // no agent-scope acquire: every x row is stored and loaded sc1 (bcr_ld);
    // the workgroup fence keeps the compiler from moving loads above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return true;
}

// Item tickets (both dataflow launches): every workgroup draws its first item
// from the launch's counter, and the next one as it starts an item, so
// tickets are handed out in dependency order and every item waited on has
// been drawn by a running workgroup -- forward progress holds with any number
// of resident workgroups (other streams on the device, fewer CUs).  A
// workgroup draws 1 + (items it runs) tickets, so one launch draws exactly
// G + items: the host advances tbase by that (counters wrap modulo 2^32).
__device__ __forceinline__ unsigned bcr_ticket(unsigned *ctr) {
    return __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int K>
__global__ void __launch_bounds__(64) k_bcr_bwd_all(BcrDev B, const double *y, double *x,
                                                    unsigned epoch, int *fail, unsigned tbase) {
    __shared__ double xg[NGMAX], xp[K], xn[K], v0[K + NGMAX];
    const int lane = threadIdx.x;
    const int nb = B.nb, nG = B.nG, nblk = B.nblk;
    int k = (int)(__builtin_amdgcn_readfirstlane(lane == 0 ? bcr_ticket(B.tick + 1) : 0u) - tbase);
    for (; k < nblk;) {
        const int o = B.ord[k];
        // the next item's ticket, drawn as this one starts (one lane; the
        // value is wave-uniform after readfirstlane)
        unsigned nxt = lane == 0 ? bcr_ticket(B.tick + 1) : 0u;
        if (o == 0) {  // root: x_T = FT^T y_T (k_bcr_bwd_root)
            const int N = B.NR;
            if (lane < K) v0[lane] = bcr_get(y, lane, nb);
            if (lane < NGMAX) v0[K + lane] = lane < nG ? y[nb + lane] : 0.;
            __syncthreads();
            if (lane < K + nG) {
                // FT column loads issued together, then the same ascending sum
                double ft[K + NGMAX];
#pragma unroll
                for (int u = 0; u < K + NGMAX; ++u)
                    ft[u] = (u >= lane && u < K + nG) ? B.FT[u * N + lane] : 0.;
                double acc = 0.;
#pragma unroll
                for (int u = 0; u < K + NGMAX; ++u)
                    if (u >= lane && u < K + nG) acc = fma(ft[u], v0[u], acc);
                const int R = lane < K ? lane : nb + lane - K;
                if (lane >= K || lane < nb) {
                    bcr_put(x, R, acc);
                    if (B.xs && B.row_param[R] >= 0) B.xs[B.row_param[R]] = acc;
                }
            }
            bcr_publish(B.flags, 0, epoch, lane);
            __syncthreads();
            k = (int)(__builtin_amdgcn_readfirstlane(nxt) - tbase);
            continue;
        }
        const int s = 1 << __builtin_ctz(o);
        const bool hn = o + s < nblk;
        // factor rows and y_o first (written by earlier launches)
        double ur[K], vr[K], cc[K];  // row lane of U_o, V_o; column lane of C_o (diag 1/C_ii)
        double yo = 0.;
        if (lane < K) {
            const double *U = bcr_blk(B.FU, o, K), *V = bcr_blk(B.FV, o, K);
            const double *Cf = bcr_blk(B.FC, o, K);
#pragma unroll
            for (int u = 0; u < K; ++u) {
                ur[u] = U[lane * K + u];
                vr[u] = hn ? V[lane * K + u] : 0.;
                cc[u] = u >= lane ? Cf[u * K + lane] : 0.;
            }
            yo = bcr_get(y, o * K + lane, nb);
        } else {
#pragma unroll
            for (int u = 0; u < K; ++u) ur[u] = vr[u] = cc[u] = 0.;
        }
        // producers: o - s, o + s (if any), the root (arrow rows)
        bool ok = bcr_wait(B.flags, o - s, hn ? o + s : -1, epoch);
        if (ok && nG > 0 && o - s != 0) ok = bcr_wait(B.flags, 0, -1, epoch);
        if (!ok) {
            if (lane == 0) atomicOr(fail, 2);
            k = (int)(__builtin_amdgcn_readfirstlane(nxt) - tbase);
            continue;
        }
        if (lane < K) {  // x rows of this launch's producers: sc1 loads (bcr_ld)
            xp[lane] = bcr_get_sc1(x, (o - s) * K + lane, nb);
            xn[lane] = hn ? bcr_get_sc1(x, (o + s) * K + lane, nb) : 0.;
        }
        if (lane < nG) xg[lane] = bcr_ld(x + nb + lane);
        __syncthreads();
        double v = 0.;
        if (lane < K) {
            const double *Y = B.FY + (size_t)o * K * nG;
            v = yo;
#pragma unroll
            for (int u = 0; u < K; ++u) v = fma(-ur[u], xp[u], fma(-vr[u], xn[u], v));
            for (int q = 0; q < nG; ++q) v = fma(-Y[lane * nG + q], xg[q], v);
        }
#pragma unroll
        for (int u = K - 1; u >= 0; --u) {
            if (lane == u) v *= cc[u];
            const double xu = bcr_rdlane(v, u);
            if (lane < u) v = fma(-cc[u], xu, v);
        }
        if (lane < K) {
            const int R = o * K + lane;
            if (R < nb) {
                bcr_put(x, R, v);
                if (B.xs && B.row_param[R] >= 0) B.xs[B.row_param[R]] = v;  // k_scatter_xR
            }
        }
        bcr_publish(B.flags, o, epoch, lane);
        __syncthreads();
        k = (int)(__builtin_amdgcn_readfirstlane(nxt) - tbase);
    }
}

// ---------------------------------------------------------------------------
// Factorisation in ONE launch (dataflow; MMBA_PATH_BCR_DATAFLOW = 0: per-level launches).
// Items: the levels' even blocks in level order (level l has g_l = ceil(nact_l
// / 2) items), then the root; dealt round robin to G = min(g_0, 256)
// workgroups, all resident (one 256-thread workgroup per CU fits), each
// taking its items in increasing order, so every wait ends.  Item k of level
// l (e = 2k s) reads blocks e - s, e, e + s, e + 2s, which are the even blocks
// of items 2k-1 .. 2k+2 of level l-1; it waits for exactly those (the same
// items are the only earlier readers of the coupling buffer it overwrites,
// Lin of level l-1).  Level 0 stages its operands from the band layout (no
// k_bcr_load pass); the root waits for every item (the arrow sums).
// Hand-off per MI355X guide G16 R1: every value read by another item is
// stored write-through (bcr_st), each storing wave drains (vmcnt 0), the
// workgroup barrier, one lane stores the item's flag = epoch; the consumer's
// wave 0 polls its producers' flags relaxed (sc1), and the barrier releases
// the other waves to load; every handed-off value is loaded sc1 (bcr_ld), so
// no agent-scope acquire is taken (MI355X guide, valid forms, first row).  Every spin is
// bounded (timeout: bit 1 of *fail, the solve counts as failed).  Without
// an arrow (nG = 0) the item publishes as soon as D_e, the new coupling and
// r_e are stored, before its factor-column stores (read by later launches).
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool bcr_wait_items(const int *flags, int lo, int hi,
                                               unsigned epoch) {
    // flags[lo .. hi) == epoch (hi - lo <= 64 per pass; wave-uniform result)
    const int lane = threadIdx.x & 63;
    for (int b = lo; b < hi; b += 64) {
        const int i = b + lane;
        for (unsigned spins = 0;; ++spins) {
            bool ok = true;
            if (i < hi)
                ok = __hip_atomic_load((bcr_gu32 *)(flags + i), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT) == epoch;
            if (__builtin_amdgcn_ballot_w64(!ok) == 0) break;
            if (spins > (1u << 22)) return false;
            __builtin_amdgcn_s_sleep(2);
        }
    }
    // no agent-scope acquire: every handed-off value is stored (bcr_st) and
    // loaded (bcr_ld) sc1; the workgroup fence keeps the compiler from moving
    // those loads above the poll
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return true;
}

template <int K, int N>
__global__ void __launch_bounds__(256) k_bcr_factor_df(BcrDev B, int *fail, const double *r,
                                                       double *y, unsigned epoch,
                                                       long long *trace, unsigned tbase) {
    // trace (diagnostic, MMBA_PATH_PROBE = 1): per item the 100 MHz wall clock at
    // entry, after the wait, after the item, after the flag store
    __shared__ int ok_s, it_s;
    const int tid = threadIdx.x;
    int base = 0, pbase = 0, pg = 0, s = 1, nact = B.nblk, lvl = 0;
    if (tid == 0) it_s = (int)(bcr_ticket(B.tick) - tbase);  // items in ticket order
    __syncthreads();
    for (int it = it_s;;) {
        while (nact > 1 && it >= base + (nact + 1) / 2) {
            pbase = base;
            pg = (nact + 1) / 2;
            base += pg;
            s *= 2;
            nact = pg;
            ++lvl;
        }
        if (nact <= 1) {  // the root: item index base, after every level item
            if (it == base && tid < 64) {
                if (trace && tid == 0) trace[4 * it] = (long long)wall_clock64();
                if (bcr_wait_items(B.fflags, 0, base, epoch)) {
                    if (trace && tid == 0) trace[4 * it + 1] = (long long)wall_clock64();
                    bcr_root_wave<N>(B, fail, y, y ? r + B.nb : nullptr);
                    if (trace && tid == 0) trace[4 * it + 2] = trace[4 * it + 3] =
                        (long long)wall_clock64();
                } else if (tid == 0) {
                    atomicOr(fail, 2);
                }
            }
            return;
        }
        const int k = it - base;
        unsigned nxt = 0;  // the next item's ticket, drawn as this one starts
        if (tid == 0) nxt = bcr_ticket(B.tick);
        if (trace && tid == 0) trace[4 * it] = (long long)wall_clock64();
        __syncthreads();  // the previous item's LDS reads are done
        if (lvl > 0) {
            if (tid < 64) {
                const int lo = max(2 * k - 1, 0), hi = min(2 * k + 3, pg);
                const bool ok = bcr_wait_items(B.fflags, pbase + lo, pbase + hi, epoch);
                if (tid == 0) ok_s = ok;
            }
            __syncthreads();
            if (!ok_s) {
                if (tid == 0) {
                    atomicOr(fail, 2);
                    it_s = (int)(nxt - tbase);
                }
                __syncthreads();
                it = it_s;
                continue;  // no flag: the items that need this one time out too
            }
        }
        if (trace && tid == 0) trace[4 * it + 1] = (long long)wall_clock64();
        bcr_level_item<K, 2, true>(B, s, nact, lvl & 1, 2 * k, fail, trace ? trace - 8 : nullptr, y,
                                   lvl == 0, r, B.fflags + it, epoch);
        if (trace && tid == 0) trace[4 * it + 2] = (long long)wall_clock64();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_store((bcr_gu32 *)(B.fflags + it), epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            if (trace) trace[4 * it + 3] = (long long)wall_clock64();
            it_s = (int)(nxt - tbase);
        }
        __syncthreads();
        it = it_s;
    }
}

static std::atomic<unsigned> g_bcr_epoch{0};


static unsigned bcr_next_epoch() {
    unsigned ep = ++g_bcr_epoch;
    if (ep == 0) ep = ++g_bcr_epoch;  // flags start at 0: never use epoch 0
    return ep;
}

// ---------------------------------------------------------------------------
// Host side.
// ---------------------------------------------------------------------------
// Factorisation; with r != nullptr the forward solve y = L^-1 r runs inside
// the same launches (r is copied to the work vector by the load kernel).
template <int K>
static void bcr_factor_k(hipStream_t s, const BandSolver &B, int *fail, long long *probe,
                         const double *r, double *y) {
    const BcrDev &D = B.bcr;
    double *yy = r ? y : nullptr;
    const bool wide = D.nG > NGLANE;  // arrows wider than NGLANE: per-level launches
    if (D.fflags && D.tick && !B.df_off && D.nblk >= 2 && D.regchol == 2 && D.mfma_upd && !wide) {
        const unsigned ep = bcr_next_epoch();
        // level items (the root is item `items`); G workgroups need not all
        // be resident (tickets), so the grid is the level-0 width (<= 256)
        int items = 0;
        for (int nact = D.nblk; nact > 1; nact = (nact + 1) / 2) items += (nact + 1) / 2;
        const int G = std::min((D.nblk + 1) / 2, B.df_grid);
        const unsigned tb = B.tick_f;
        B.tick_f += (unsigned)(G + items);
        long long *tr = probe ? probe + 8 : nullptr;
        switch (D.NR - K) {
            case 0: k_bcr_factor_df<K, K><<<G, 256, 0, s>>>(D, fail, r, yy, ep, tr, tb); break;
            case 8: k_bcr_factor_df<K, K + 8><<<G, 256, 0, s>>>(D, fail, r, yy, ep, tr, tb); break;
            default:
                k_bcr_factor_df<K, K + 16><<<G, 256, 0, s>>>(D, fail, r, yy, ep, tr, tb);
                break;
        }
        return;
    }
    k_bcr_load<K><<<D.nblk, 256, 0, s>>>(D, r);
    int ping = 0;
    for (int st = 1, nact = D.nblk; nact > 1; st *= 2, nact = (nact + 1) / 2) {
        const int g = (nact + 1) / 2;
        if (wide) {
            k_bcr_level<K, 2, true, NGMAX><<<g, 256, 0, s>>>(D, st, nact, ping, fail, probe, yy);
        } else if (D.regchol == 2) {
            if (D.mfma_upd)
                k_bcr_level<K, 2, true><<<g, 256, 0, s>>>(D, st, nact, ping, fail, probe, yy);
            else
                k_bcr_level<K, 2, false><<<g, 256, 0, s>>>(D, st, nact, ping, fail, probe, yy);
        } else {
            if (D.mfma_upd)
                k_bcr_level<K, 0, true><<<g, 256, 0, s>>>(D, st, nact, ping, fail, probe, yy);
            else
                k_bcr_level<K, 0, false><<<g, 256, 0, s>>>(D, st, nact, ping, fail, probe, yy);
        }
        ping ^= 1;
    }
    switch (D.NR) {
        case 8: k_bcr_root<8><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 16: k_bcr_root<16><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 24: k_bcr_root<24><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 32: k_bcr_root<32><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 40: k_bcr_root<40><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 48: k_bcr_root<48><<<1, 64, 0, s>>>(D, fail, yy); break;
        case 56: k_bcr_root<56><<<1, 64, 0, s>>>(D, fail, yy); break;
        default: k_bcr_root<64><<<1, 64, 0, s>>>(D, fail, yy); break;
    }
}

template <int K>
static void bcr_forward_k(hipStream_t s, const BandSolver &B, const double *r, double *y) {
    const BcrDev &D = B.bcr;
    MMBA_HIP(hipMemcpyAsync(D.rw, r, sizeof(double) * (size_t)(D.nb + D.nG),
                                  hipMemcpyDeviceToDevice, s));
    for (int st = 1, nact = D.nblk; nact > 1; st *= 2, nact = (nact + 1) / 2)
        k_bcr_fwd<K><<<(nact + 1) / 2, 64, 0, s>>>(D, st, nact, D.rw, y);
    k_bcr_fwd_root<K><<<1, 64, 0, s>>>(D, D.rw, y);
}

template <int K>
static void bcr_backward_k(hipStream_t s, const BandSolver &B, const double *y, double *x) {
    const BcrDev &D = B.bcr;
    if (D.flags && D.fail && D.tick && !B.df_off) {  // one dataflow launch
        const unsigned ep = bcr_next_epoch();
        const int G = std::min(D.nblk, B.df_grid);
        const unsigned tb = B.tick_b;
        B.tick_b += (unsigned)(G + D.nblk);
        k_bcr_bwd_all<K><<<G, 64, 0, s>>>(D, y, x, ep, D.fail, tb);
        return;
    }
    k_bcr_bwd_root<K><<<1, 64, 0, s>>>(D, y, x);
    std::vector<std::pair<int, int>> lv;  // (stride, nact) per level, coarse to fine
    for (int st = 1, nact = D.nblk; nact > 1; st *= 2, nact = (nact + 1) / 2) lv.push_back({st, nact});
    for (int l = (int)lv.size() - 1; l >= 0; --l)
        k_bcr_bwd<K><<<lv[l].second / 2, 64, 0, s>>>(D, lv[l].first, lv[l].second, y, x);
}

void bcr_factor(hipStream_t s, const BandSolver &B, int *fail, long long *probe,
                const double *r, double *y) {
    switch (B.bcr.K) {
        case 8: bcr_factor_k<8>(s, B, fail, probe, r, y); break;
        case 16: bcr_factor_k<16>(s, B, fail, probe, r, y); break;
        case 24: bcr_factor_k<24>(s, B, fail, probe, r, y); break;
        default: bcr_factor_k<32>(s, B, fail, probe, r, y); break;
    }
}

void bcr_forward(hipStream_t s, const BandSolver &B, const double *r, double *y) {
    switch (B.bcr.K) {
        case 8: bcr_forward_k<8>(s, B, r, y); break;
        case 16: bcr_forward_k<16>(s, B, r, y); break;
        case 24: bcr_forward_k<24>(s, B, r, y); break;
        default: bcr_forward_k<32>(s, B, r, y); break;
    }
}

void bcr_backward(hipStream_t s, const BandSolver &B, const double *y, double *x) {
    switch (B.bcr.K) {
        case 8: bcr_backward_k<8>(s, B, y, x); break;
        case 16: bcr_backward_k<16>(s, B, y, x); break;
        case 24: bcr_backward_k<24>(s, B, y, x); break;
        default: bcr_backward_k<32>(s, B, y, x); break;
    }
}

}  // namespace mmba
