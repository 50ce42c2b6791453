// mmba_gemm.hip -- hand-written fp64 MFMA GEMM / SYRK for the dense reduced
// camera system (CDNA4 / gfx950).
//
//   C = beta C + alpha A B^T      A: M x Kd, B: N x Kd, C: M x N, column-major
//
// with TRI (SYRK, A == B, M == N): only the lower triangle of C is formed
// (tiles (ti, tj) with ti >= tj, and i >= j inside the diagonal tiles).
//
// Workgroup tile 128 x 128, four waves in a 2 x 2 grid, each wave 64 x 64 =
// 4 x 4 tiles of v_mfma_f64_16x16x4_f64 (16 accumulators of 4 doubles), two
// workgroups per CU (196 VGPRs: two waves per SIMD; 74 KB of LDS each --
// measured 32.4 TF/s on C3 against 25.3 at one workgroup per CU and 29.9
// with 256 x 128 tiles of eight waves).  The
// K dimension is staged through LDS 16 columns at a time, double buffered:
// the global loads of stage k + 1 are issued into registers before the
// MFMAs of stage k and written to the other buffer after them, so each
// stage costs one barrier.  LDS rows (one per k) are 16 doubles longer than
// the panel (32 mod 64 banks), so the four 16-lane groups of a fragment
// read fall on two bank halves -- the minimum of two LDS cycles for a
// 64-lane 8-byte read.  Fragment layouts (MI355X guide, f64 MFMA): A/B operand
// lane l holds row (l & 15) of k = l >> 4; result lane l, register r holds
// row (l >> 4) + 4 r, column l & 15.
//
// A and C may be the same array when every workgroup's rows of A are its own
// rows of C (the in-place panel solve, N <= 128).  Used by mmba_dense.hip for
// the panel solves, the in-block updates and the
// rank-512 trailing updates of the dense blocked Cholesky.
#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

typedef double gm_d4 __attribute__((ext_vector_type(4)));

constexpr int GM_TM = 128;  // workgroup tile: rows of A (C rows); TN (C columns): 128 or 64
constexpr int GM_KT = 16;   // K columns per LDS stage
constexpr int GM_LA = GM_TM + 16;  // LDS row stride of A (32 mod 64 banks)

// Stage loader for an R-row panel: thread t loads R * KT / NT consecutive
// rows of one column (16-B vector loads when the rows are in range).
template <int R, int NT>
__device__ __forceinline__ void gm_load(const double *X, int ld, int rows, int i0,
                                        int k0, int t, double (&v)[R * GM_KT / NT]) {
    constexpr int PER = R * GM_KT / NT, TPK = R / PER;  // rows per thread, threads per column
    const int k = t / TPK, r0 = (t % TPK) * PER;
    const double *p = X + (size_t)(k0 + k) * ld + i0 + r0;
    if (i0 + r0 + PER <= rows) {
        const double2 *q = reinterpret_cast<const double2 *>(p);
#pragma unroll
        for (int u = 0; u < PER / 2; ++u) {
            const double2 w = q[u];
            v[2 * u] = w.x;
            v[2 * u + 1] = w.y;
        }
    } else {
#pragma unroll
        for (int u = 0; u < PER; ++u) v[u] = (i0 + r0 + u < rows) ? p[u] : 0.;
    }
}

template <int R, int LS, int NT>
__device__ __forceinline__ void gm_store_lds(double *S, int t, const double (&v)[R * GM_KT / NT]) {
    constexpr int PER = R * GM_KT / NT, TPK = R / PER;
    const int k = t / TPK, r0 = (t % TPK) * PER;
    double2 *q = reinterpret_cast<double2 *>(&S[k * LS + r0]);
#pragma unroll
    for (int u = 0; u < PER / 2; ++u) q[u] = make_double2(v[2 * u], v[2 * u + 1]);
}

template <bool TRI, int TN>
__global__ void __launch_bounds__(128 * (TN / 64), 2) k_dgemm_nt(int M, int N, int Kd,
                                                       const double *A, int lda,
                                                       const double *__restrict__ B, int ldb,
                                                       double *C, int ldc,
                                                       double alpha, double beta) {
    static_assert(!TRI || TN == GM_TM, "the triangular tile list assumes square tiles");
    constexpr int NT = 128 * (TN / 64), LB = TN + 16;
    __shared__ double As[2][GM_KT * GM_LA], Bs[2][GM_KT * LB];
    constexpr int PA = GM_TM * GM_KT / NT, PB = TN * GM_KT / NT;
    // tiles: TRI lists the lower-triangle tiles row by row, b = ti (ti + 1)
    // / 2 + tj (tj <= ti).  XCD-aware order: workgroups are dealt round
    // robin to the 8 XCDs, so workgroup w takes tile (w % 8) ceil(G / 8) +
    // w / 8 -- each XCD sweeps a contiguous run of tiles (mostly one tile
    // row: its A panel stays in that XCD's L2 while the B panels stream).
    // The grid is 8 ceil(G / 8) workgroups, G = number of tiles.
    const int nti = (M + GM_TM - 1) / GM_TM, ntj = (N + TN - 1) / TN;
    const int G = TRI ? nti * (nti + 1) / 2 : nti * ntj;
    const int w = blockIdx.x, per = (G + 7) / 8;
    const int lin = (w % 8) * per + w / 8;
    if (lin >= G) return;
    int ti, tj;
    if (TRI) {
        ti = (int)((sqrt(8.0 * lin + 1.0) - 1.0) * 0.5);
        while ((ti + 1) * (ti + 2) / 2 <= lin) ++ti;
        while (ti * (ti + 1) / 2 > lin) --ti;
        tj = lin - ti * (ti + 1) / 2;
    } else {  // consecutive tiles share the B panel (tj), A panels stream
        ti = lin % nti;
        tj = lin / nti;
    }
    const int i0 = ti * GM_TM, j0 = tj * TN;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int wi = (wv % (GM_TM / 64)) * 64, wj = (wv / (GM_TM / 64)) * 64;
    gm_d4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = gm_d4{0., 0., 0., 0.};
    double va[PA], vb[PB];
    gm_load<GM_TM, NT>(A, lda, M, i0, 0, t, va);
    gm_load<TN, NT>(B, ldb, N, j0, 0, t, vb);
    gm_store_lds<GM_TM, GM_LA, NT>(As[0], t, va);
    gm_store_lds<TN, LB, NT>(Bs[0], t, vb);
    __syncthreads();
    const int nst = Kd / GM_KT;
    for (int st = 0; st < nst; ++st) {
        const int cur = st & 1;
        const bool more = st + 1 < nst;
        if (more) {  // next stage's loads in flight during this stage's MFMAs
            gm_load<GM_TM, NT>(A, lda, M, i0, (st + 1) * GM_KT, t, va);
            gm_load<TN, NT>(B, ldb, N, j0, (st + 1) * GM_KT, t, vb);
        }
        const double *as = As[cur], *bs = Bs[cur];
#pragma unroll
        for (int k4 = 0; k4 < GM_KT; k4 += 4) {
            const int kk = k4 + (lane >> 4), li = lane & 15;
            double fa[4], fb[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                fa[u] = as[kk * GM_LA + li + wi + 16 * u];
                fb[u] = bs[kk * LB + li + wj + 16 * u];
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
        if (more) {
            gm_store_lds<GM_TM, GM_LA, NT>(As[cur ^ 1], t, va);
            gm_store_lds<TN, LB, NT>(Bs[cur ^ 1], t, vb);
        }
        __syncthreads();
    }
    // epilogue, 32 columns at a time through LDS (the stage buffers are
    // free after the last barrier): the waves holding those columns write
    // their accumulators column-major, then every thread updates 16
    // consecutive rows of one column -- whole 128-row columns of C are read
    // and written with 16-B accesses (the MFMA result layout would touch 16
    // columns x 32 B per store)
    constexpr int CS = GM_TM + 2;  // LDS column stride (doubles)
    static_assert(32 * CS <= 2 * GM_KT * GM_LA, "epilogue staging must fit the A buffers");
    double *cst = &As[0][0];
#pragma unroll
    for (int cb = 0; cb < TN / 32; ++cb) {
        if (wj == (cb / 2) * 64) {
#pragma unroll
            for (int bb = 0; bb < 2; ++bb) {
                const int b = (cb % 2) * 2 + bb;
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        cst[(16 * bb + (lane & 15)) * CS + wi + 16 * a + (lane >> 4) + 4 * r] =
                            acc[a][b][r];
            }
        }
        __syncthreads();
        {
            // 256 threads: a column each 8; 128 threads: two passes
#pragma unroll
            for (int t2 = t; t2 < 256; t2 += NT) {
            const int c = t2 >> 3, r0 = (t2 & 7) * 16;
            const int j = j0 + 32 * cb + c;
            if (j < N) {
                double *col = &C[(size_t)j * ldc + i0 + r0];
                const double *src = &cst[c * CS + r0];
                const int i = i0 + r0;
                const bool full = i + 16 <= M && (!TRI || i >= j) &&
                                  ((reinterpret_cast<size_t>(col) & 15) == 0);
                if (full) {
                    double2 *q = reinterpret_cast<double2 *>(col);
#pragma unroll
                    for (int u = 0; u < 8; ++u) {
                        double2 cv = make_double2(0., 0.);
                        if (beta != 0.) cv = q[u];
                        const double v0 = alpha * src[2 * u], v1 = alpha * src[2 * u + 1];
                        q[u] = beta == 0. ? make_double2(v0, v1)
                                          : make_double2(fma(beta, cv.x, v0), fma(beta, cv.y, v1));
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < 16; ++u) {
                        if (i + u < M && (!TRI || i + u >= j)) {
                            const double v = alpha * src[u];
                            col[u] = beta == 0. ? v : fma(beta, col[u], v);
                        }
                    }
                }
            }
            }
        }
        __syncthreads();
    }
}

// C = beta C + alpha A B^T (M x N, K a multiple of 16); tri: lower triangle
// only (A == B, M == N).
void launch_dgemm_nt(hipStream_t s, bool tri, int M, int N, int Kd, const double *A, int lda,
                     const double *B, int ldb, double *C, int ldc, double alpha, double beta) {
    if (M <= 0 || N <= 0 || Kd <= 0) return;
    if (Kd % GM_KT) throw Invalid{"dgemm_nt: K must be a multiple of 16"};
    if (tri && M != N) throw Invalid{"dgemm_nt: triangular update needs M == N"};
    const int ti = (M + GM_TM - 1) / GM_TM;
    if (!tri && N <= 64) {  // panel solves (N = 64): 128 x 64 tiles, two waves
        const int grid = 8 * ((ti + 7) / 8);
        k_dgemm_nt<false, 64><<<grid, 128, 0, s>>>(M, N, Kd, A, lda, B, ldb, C, ldc, alpha, beta);
        return;
    }
    const int tj = (N + 127) / 128;
    const int G = tri ? ti * (ti + 1) / 2 : ti * tj;
    const int grid = 8 * ((G + 7) / 8);
    if (tri)
        k_dgemm_nt<true, 128><<<grid, 256, 0, s>>>(M, N, Kd, A, lda, B, ldb, C, ldc, alpha, beta);
    else
        k_dgemm_nt<false, 128><<<grid, 256, 0, s>>>(M, N, Kd, A, lda, B, ldb, C, ldc, alpha, beta);
}

}  // namespace mmba
