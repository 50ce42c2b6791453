// mmba_chol.hip -- tiled Cholesky of the reduced (camera-frame + global)
// Schur complement and the triangular solves on it (CDNA4 / gfx950, fp64).
//
// S is stored as 64x64 row-major tiles of its lower triangle; slot[I*NT+J]
// (I >= J) names the tile or is -1 for a structurally zero tile.  The
// factorisation is right-looking over tile panels:
//   k_chol_panel   block 0:   L_kk = chol(S_kk), Linv_kk = L_kk^-1
//                  block b>0: L_Ik = S_Ik L_kk^-T for the panel's rows I
//   k_chol_update  S_IJ -= L_Ik L_Jk^T (fp64 MFMA 16x16x4, one block per pair)
// The diagonal factorisation is blocked by 16 columns in LDS (a register
// 16x16 factor in wave 0, a row-parallel triangular solve and a 256-thread
// trailing update) so the serial chain per panel is 4 short steps rather than
// 64 column steps; every panel block factors S_kk redundantly instead of
// waiting on block 0.
#include "mmba_kernels.h"

namespace mmba {

constexpr int LDP = TILE + 1;  // padded LDS row: conflict-free column walks
constexpr int NB = 16;         // inner blocking of the 64-wide tiles

// Blocked right-looking Cholesky of the 64x64 tile in A (lower part used).
// A non-positive or non-finite pivot is replaced by 1 and reported in *bad.
__device__ void blk_potrf(double (*A)[LDP], int *bad) {
    const int tid = threadIdx.x;
    for (int jb = 0; jb < TILE; jb += NB) {
        if (tid < 64) {
            const int r = tid & (NB - 1);
            double a[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) a[c] = A[jb + r][jb + c];
            int badl = 0;
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                double d = __shfl(a[j], j, 64);
                if (!(d > 0.) || !isfinite(d)) {
                    badl = 1;
                    d = 1.;
                }
                d = sqrt(d);
                if (r == j) a[j] = d;
                else if (r > j) a[j] = a[j] / d;
#pragma unroll
                for (int c = j + 1; c < NB; ++c) {
                    const double lcj = __shfl(a[j], c, 64);
                    if (r >= c) a[c] -= a[j] * lcj;
                }
            }
            if (tid < NB) {
#pragma unroll
                for (int c = 0; c < NB; ++c)
                    if (c <= r) A[jb + r][jb + c] = a[c];
            }
            if (tid == 0 && badl) *bad = 1;
        }
        __syncthreads();
        const int m = TILE - jb - NB;
        if (m == 0) break;
        // rows below the diagonal block: x L_dd^T = a  (one thread per row)
        if (tid < m) {
            const int r = jb + NB + tid;
            double x[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) x[c] = A[r][jb + c];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
#pragma unroll
                for (int t = 0; t < c; ++t) x[c] -= x[t] * A[jb + c][jb + t];
                x[c] = x[c] / A[jb + c][jb + c];
            }
#pragma unroll
            for (int c = 0; c < NB; ++c) A[r][jb + c] = x[c];
        }
        __syncthreads();
        // trailing update of the lower triangle, rank NB
        for (int e = tid; e < m * m; e += blockDim.x) {
            const int r = jb + NB + e / m, c = jb + NB + e % m;
            if (c > r) continue;
            double s = A[r][c];
#pragma unroll
            for (int t = 0; t < NB; ++t) s -= A[r][jb + t] * A[c][jb + t];
            A[r][c] = s;
        }
        __syncthreads();
    }
}

// Solve X L^T = B in place (B: 64 rows in LDS, L lower 64x64 in LDS),
// blocked by NB columns.
__device__ void blk_trsm_rt(double (*L)[LDP], double (*B)[LDP]) {
    const int tid = threadIdx.x;
    for (int jb = 0; jb < TILE; jb += NB) {
        if (tid < TILE) {
            double x[NB];
#pragma unroll
            for (int c = 0; c < NB; ++c) x[c] = B[tid][jb + c];
#pragma unroll
            for (int c = 0; c < NB; ++c) {
#pragma unroll
                for (int t = 0; t < c; ++t) x[c] -= x[t] * L[jb + c][jb + t];
                x[c] = x[c] / L[jb + c][jb + c];
            }
#pragma unroll
            for (int c = 0; c < NB; ++c) B[tid][jb + c] = x[c];
        }
        __syncthreads();
        const int m = TILE - jb - NB;
        if (m == 0) break;
        for (int e = tid; e < TILE * m; e += blockDim.x) {
            const int r = e / m, c = jb + NB + e % m;
            double s = B[r][c];
#pragma unroll
            for (int t = 0; t < NB; ++t) s -= B[r][jb + t] * L[c][jb + t];
            B[r][c] = s;
        }
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_chol_panel(double *S, const int *__restrict__ slot,
                                                    int NT, int k,
                                                    const int *__restrict__ rows,
                                                    double *Linv, int *fail) {
    __shared__ double A[TILE][LDP];
    __shared__ double B[TILE][LDP];
    __shared__ int bad;
    const int tid = threadIdx.x;
    if (tid == 0) bad = 0;
    double *D = &S[(size_t)slot[k * NT + k] * TILE * TILE];
    double *Bg = nullptr;
    if (blockIdx.x > 0) Bg = &S[(size_t)slot[rows[blockIdx.x - 1] * NT + k] * TILE * TILE];
    for (int t = tid; t < TILE * TILE; t += blockDim.x) {
        const int r = t / TILE, c = t % TILE;
        A[r][c] = D[t];
        B[r][c] = Bg ? Bg[t] : (r == c ? 1. : 0.);
    }
    __syncthreads();
    blk_potrf(A, &bad);
    blk_trsm_rt(A, B);  // block 0: B = L^-T (upper); others: L_Ik
    if (blockIdx.x == 0) {
        if (tid == 0 && bad) atomicOr(fail, 1);
        double *Li = &Linv[(size_t)k * TILE * TILE];
        for (int t = tid; t < TILE * TILE; t += blockDim.x) {
            const int r = t / TILE, c = t % TILE;
            D[t] = (c <= r) ? A[r][c] : 0.;
            Li[t] = (c <= r) ? B[c][r] : 0.;
        }
        return;
    }
    for (int t = tid; t < TILE * TILE; t += blockDim.x) Bg[t] = B[t / TILE][t % TILE];
}

typedef double dbl4 __attribute__((ext_vector_type(4)));

// Trailing update S_IJ -= L_Ik L_Jk^T for the listed (I, J) pairs of panel k,
// fp64 MFMA 16x16x4: 4 waves, each owns a 16x64 row strip (4 MFMA tiles).
__global__ void __launch_bounds__(256) k_chol_update(double *S, const int *__restrict__ slot,
                                                     int NT, int k,
                                                     const int2 *__restrict__ pairs) {
    __shared__ double A[TILE][LDP];
    __shared__ double B[TILE][LDP];
    const int2 pr = pairs[blockIdx.x];
    const int I = pr.x, Jt = pr.y;
    const double *Lik = &S[(size_t)slot[I * NT + k] * TILE * TILE];
    const double *Ljk = &S[(size_t)slot[Jt * NT + k] * TILE * TILE];
    for (int t = threadIdx.x; t < TILE * TILE; t += blockDim.x) {
        A[t / TILE][t % TILE] = Lik[t];
        B[t / TILE][t % TILE] = Ljk[t];
    }
    __syncthreads();
    const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
    const int li = lane & 15, lk = lane >> 4;
    dbl4 acc[4];
    for (int tj = 0; tj < 4; ++tj) acc[tj] = (dbl4){0., 0., 0., 0.};
    const int ti = wave;
    for (int ks = 0; ks < TILE / 4; ++ks) {
        const double a = A[ti * 16 + li][ks * 4 + lk];
#pragma unroll
        for (int tj = 0; tj < 4; ++tj) {
            const double bv = B[tj * 16 + li][ks * 4 + lk];
            acc[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, bv, acc[tj], 0, 0, 0);
        }
    }
    double *C = &S[(size_t)slot[I * NT + Jt] * TILE * TILE];
#pragma unroll
    for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = ti * 16 + lk + 4 * r;
            const int col = tj * 16 + li;
            C[row * TILE + col] -= acc[tj][r];
        }
}

// Forward substitution L y = r, panel k: y_k = Linv_kk r_k, r_I -= L_Ik y_k.
__global__ void __launch_bounds__(64) k_trsv_fwd(const double *__restrict__ S, const int *__restrict__ slot, int NT,
                           int k, const int *__restrict__ rows, const double *__restrict__ Linv,
                           double *r, double *y) {
    __shared__ double yk[TILE];
    const double *Li = &Linv[(size_t)k * TILE * TILE];
    for (int row = threadIdx.x; row < TILE; row += blockDim.x) {
        double s = 0.;
        for (int t = 0; t <= row; ++t) s += Li[row * TILE + t] * r[k * TILE + t];
        yk[row] = s;
    }
    __syncthreads();
    if (blockIdx.x == 0) {
        for (int row = threadIdx.x; row < TILE; row += blockDim.x) y[k * TILE + row] = yk[row];
        return;
    }
    const int I = rows[blockIdx.x - 1];
    const double *L = &S[(size_t)slot[I * NT + k] * TILE * TILE];
    for (int row = threadIdx.x; row < TILE; row += blockDim.x) {
        double s = 0.;
        for (int c = 0; c < TILE; ++c) s += L[row * TILE + c] * yk[c];
        r[I * TILE + row] -= s;
    }
}

// Back substitution L^T x = y, panel k (descending): x_k = Linv_kk^T y_k,
// y_J -= L_kJ^T x_k for every J < k with L_kJ structurally non-zero.
__global__ void __launch_bounds__(64) k_trsv_bwd(const double *__restrict__ S, const int *__restrict__ slot, int NT,
                           int k, const int *__restrict__ cols, const double *__restrict__ Linv,
                           double *y, double *x) {
    __shared__ double xk[TILE];
    const double *Li = &Linv[(size_t)k * TILE * TILE];
    for (int row = threadIdx.x; row < TILE; row += blockDim.x) {
        double s = 0.;
        for (int t = row; t < TILE; ++t) s += Li[t * TILE + row] * y[k * TILE + t];
        xk[row] = s;
    }
    __syncthreads();
    if (blockIdx.x == 0) {
        for (int row = threadIdx.x; row < TILE; row += blockDim.x) x[k * TILE + row] = xk[row];
        return;
    }
    const int Jt = cols[blockIdx.x - 1];
    const double *L = &S[(size_t)slot[k * NT + Jt] * TILE * TILE];
    for (int c = threadIdx.x; c < TILE; c += blockDim.x) {
        double s = 0.;
        for (int rr = 0; rr < TILE; ++rr) s += L[rr * TILE + c] * xk[rr];
        y[Jt * TILE + c] -= s;
    }
}

// Whole forward substitution in one block (narrow structures: few rows per
// panel).  256 threads = 64 rows x 4 column quarters; quarter partial sums
// are combined with lane shuffles inside the wave.  r is updated in place;
// the block's own global writes are visible to it after a barrier.
__global__ void __launch_bounds__(256) k_trsv_fwd_all(const double *__restrict__ S,
                                                      const int *__restrict__ slot, int NT,
                                                      const int *__restrict__ rows_off,
                                                      const int *__restrict__ rows,
                                                      const double *__restrict__ Linv, double *r,
                                                      double *y) {
    __shared__ double yk[TILE];
    const int tid = threadIdx.x, row = tid >> 2, q = tid & 3;
    for (int k = 0; k < NT; ++k) {
        const double *Li = &Linv[(size_t)k * TILE * TILE + row * TILE];
        const double *rk = &r[k * TILE];
        double s = 0.;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int c = q * 16 + t;
            s += Li[c] * rk[c];  // Linv is stored with zeros above the diagonal
        }
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        if (q == 0) {
            yk[row] = s;
            y[k * TILE + row] = s;
        }
        __syncthreads();
        for (int e = rows_off[k]; e < rows_off[k + 1]; ++e) {
            const int I = rows[e];
            const double *L = &S[(size_t)slot[I * NT + k] * TILE * TILE + row * TILE];
            double u = 0.;
#pragma unroll
            for (int t = 0; t < 16; ++t) u += L[q * 16 + t] * yk[q * 16 + t];
            u += __shfl_xor(u, 1, 64);
            u += __shfl_xor(u, 2, 64);
            if (q == 0) r[I * TILE + row] -= u;
        }
        __syncthreads();
    }
}

// Whole back substitution in one block (narrow structures).  Thread
// (col = tid & 63, quarter = tid >> 6) reads Linv / L_kJ column-coalesced;
// quarters are combined through LDS.
__global__ void __launch_bounds__(256) k_trsv_bwd_all(const double *__restrict__ S,
                                                      const int *__restrict__ slot, int NT,
                                                      const int *__restrict__ cols_off,
                                                      const int *__restrict__ cols,
                                                      const double *__restrict__ Linv, double *y,
                                                      double *x) {
    __shared__ double part[4][TILE];
    __shared__ double xk[TILE];
    const int tid = threadIdx.x, col = tid & 63, q = tid >> 6;
    for (int k = NT - 1; k >= 0; --k) {
        const double *Li = &Linv[(size_t)k * TILE * TILE];
        const double *yk = &y[k * TILE];
        double s = 0.;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int rr = q * 16 + t;
            s += Li[rr * TILE + col] * yk[rr];  // zeros above the diagonal
        }
        part[q][col] = s;
        __syncthreads();
        if (q == 0) {
            const double v = part[0][col] + part[1][col] + part[2][col] + part[3][col];
            xk[col] = v;
            x[k * TILE + col] = v;
        }
        __syncthreads();
        for (int e = cols_off[k]; e < cols_off[k + 1]; ++e) {
            const int Jt = cols[e];
            const double *L = &S[(size_t)slot[k * NT + Jt] * TILE * TILE];
            double u = 0.;
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const int rr = q * 16 + t;
                u += L[rr * TILE + col] * xk[rr];
            }
            part[q][col] = u;
            __syncthreads();
            if (q == 0) y[Jt * TILE + col] -= part[0][col] + part[1][col] + part[2][col] + part[3][col];
            __syncthreads();
        }
    }
}

void launch_chol_panel(hipStream_t s, double *S, const int *slot, int NT, int k, const int *rows,
                       int nrows, double *Linv, int *fail) {
    k_chol_panel<<<1 + nrows, 256, 0, s>>>(S, slot, NT, k, rows, Linv, fail);
}
void launch_chol_update(hipStream_t s, double *S, const int *slot, int NT, int k,
                        const int2 *pairs, int npairs) {
    if (npairs == 0) return;
    k_chol_update<<<npairs, 256, 0, s>>>(S, slot, NT, k, pairs);
}
void launch_trsv_fwd(hipStream_t s, const double *S, const int *slot, int NT, int k,
                     const int *rows, int nrows, const double *Linv, double *r, double *y) {
    k_trsv_fwd<<<1 + nrows, 64, 0, s>>>(S, slot, NT, k, rows, Linv, r, y);
}
void launch_trsv_bwd(hipStream_t s, const double *S, const int *slot, int NT, int k,
                     const int *cols, int ncols, const double *Linv, double *y, double *x) {
    k_trsv_bwd<<<1 + ncols, 64, 0, s>>>(S, slot, NT, k, cols, Linv, y, x);
}
void launch_trsv_fwd_all(hipStream_t s, const double *S, const int *slot, int NT,
                         const int *rows_off, const int *rows, const double *Linv, double *r,
                         double *y) {
    k_trsv_fwd_all<<<1, 256, 0, s>>>(S, slot, NT, rows_off, rows, Linv, r, y);
}
void launch_trsv_bwd_all(hipStream_t s, const double *S, const int *slot, int NT,
                         const int *cols_off, const int *cols, const double *Linv, double *y,
                         double *x) {
    k_trsv_bwd_all<<<1, 256, 0, s>>>(S, slot, NT, cols_off, cols, Linv, y, x);
}

}  // namespace mmba
