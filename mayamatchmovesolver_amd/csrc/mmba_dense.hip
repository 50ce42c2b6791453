// mmba_dense.hip -- dense reduced camera system (CDNA4 / gfx950, fp64).
//
// When the bundles tie most camera-frames together (C3: every bundle is
// tracked by five cameras over windows spread across the whole shot) the
// reduced system S has almost no zero tiles and its Cholesky factor is
// dense.  S is then held as one column-major lower triangle A (n = nRpad
// columns, ld = n + 64 rows) and factored right-looking in 64-column panels
// grouped into 512-column blocks:
//
//   panel k:  L_kk = chol(A_kk), Linv_kk = L_kk^-1     k_dense_potf64 (two waves)
//             L_ik = A_ik Linv_kk^T                    k_dgemm_nt (fp64 MFMA)
//             in-block trailing columns                 k_dgemm_nt<TRI> / k_dgemm_nt
//   block:    A_22 -= L_21 L_21^T (rank 512)            k_dgemm_nt<TRI> (fp64 MFMA)
//
// k_dgemm_nt is the hand-written fp64 MFMA GEMM/SYRK of mmba_gemm.hip (it
// replaced rocBLAS dgemm / dsyrk, which ran the same steps up to round 3).
//
// The right-hand side rides along as row n of A (A[n, j] = r_j): the panel
// GEMMs and trailing updates that produce L also produce row n of the
// factor of [S r; r^T .], which is y = L^-1 r -- the forward solve costs
// nothing extra.  The backward solve x = L^-T y (and a stand-alone forward
// solve for lmpar's Newton term) walk the 64-row blocks with one launch per
// block (k_dense_fwd_step / k_dense_bwd_step: the diagonal block through the
// stored Linv_kk, computed by every workgroup, then the workgroup's slice of
// the update of the rest).  The flops are those of a dense Cholesky, n^3/3,
// in fp64 MFMA GEMMs; the panel factorisation is the latency-bound part.

#include <algorithm>
#include <cstdlib>

#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

__device__ __forceinline__ double dn_rdlane(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double dn_rsq(double d) {  // 1/sqrt(d), full fp64
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

__device__ __forceinline__ void dn_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// In-place Cholesky of the 64 x 64 diagonal block at A (column-major, ld)
// and its inverse Linv (column-major 64 x 64, lower, ld 64), two waves in
// lockstep: wave 0 holds row r in lane r and runs the pivot chain (pivot by
// v_readlane, column j published through LDS), wave 1 holds column cc of the
// identity in lane cc and forms L^-1 e_cc with the same column as it is
// published (x_j *= 1 / L_jj, x_i -= L_ij x_j) -- one barrier per step
// instead of a second 64-step pass over the stored factor.  Double-buffered
// column: step j + 2 overwrites the buffer of step j only after both waves
// passed the barrier of step j + 1.  A non-positive or non-finite pivot sets
// *fail and is replaced by 1 (the factorisation continues; the LM treats the
// solve as failed).
__global__ void __launch_bounds__(128) k_dense_potf64(double *A, int ld, double *Linv,
                                                      int *fail) {
    __shared__ double col[2][64];
    __shared__ double rsv[64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    double a[64];
    if (wv == 0) {
#pragma unroll
        for (int c = 0; c < 64; ++c) a[c] = c <= lane ? A[(size_t)c * ld + lane] : 0.;
    } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) a[i] = (i == lane) ? 1. : 0.;
    }
    int bad = 0;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        double l = 0.;
        if (wv == 0) {
            double d = dn_rdlane(a[j], j);
            if (!(d > 0.) || !isfinite(d)) {
                bad = 1;
                d = 1.;
            }
            const double rs = dn_rsq(d);
            l = lane > j ? a[j] * rs : 0.;
            a[j] = lane == j ? d * rs : (lane > j ? l : a[j]);
            col[j & 1][lane] = l;
            if (lane == 0) rsv[j] = rs;
        }
        __syncthreads();
        if (wv == 0) {
#pragma unroll
            for (int c = j + 1; c < 64; ++c) a[c] = fma(-l, col[j & 1][c], a[c]);
        } else {
            a[j] *= rsv[j];  // zero above the diagonal stays zero
#pragma unroll
            for (int i = j + 1; i < 64; ++i) a[i] = fma(-col[j & 1][i], a[j], a[i]);
        }
    }
    if (wv == 0) {
#pragma unroll
        for (int c = 0; c < 64; ++c)
            if (c <= lane) A[(size_t)c * ld + lane] = a[c];
        if (bad && lane == 0) atomicOr(fail, 1);
    } else {
#pragma unroll
        for (int i = 0; i < 64; ++i) Linv[(size_t)lane * 64 + i] = a[i];  // column lane
    }
}

// A[n, j] = r[j] (the right-hand side as row n of the factored matrix) and
// y[j] = A[n, j] after the factorisation.
__global__ void k_dense_row_put(double *A, int ld, int n, const double *r) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) A[(size_t)j * ld + n] = r[j];
}
__global__ void k_dense_row_get(const double *A, int ld, int n, double *y) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) y[j] = A[(size_t)j * ld + n];
}

// Forward step of block k (rows k..k+63): y_k = Linv_kk t_k (every workgroup
// forms it in LDS, workgroup 0 stores it), then t_i -= L_i,k y_k for the
// rows i >= k + 64, one row per thread (grid-stride, coalesced column reads).
// t_k is only read here and the rows below only written: no race.
__global__ void __launch_bounds__(256) k_dense_fwd_step(const double *__restrict__ A, int ld,
                                                        int n, int k,
                                                        const double *__restrict__ Li,
                                                        double *t, double *y) {
    __shared__ double st[64], sy[64];
    const int tid = threadIdx.x;
    if (tid < 64) st[tid] = t[k + tid];
    __syncthreads();
    if (tid < 64) {
        // Linv is stored whole (zeros above the diagonal): a fixed 64-term
        // chain whose loads are all issued ahead (a data-dependent trip
        // count waited out one L2 round trip per term); the leading zero
        // terms leave the sum as it was
        double li[64];
#pragma unroll
        for (int c = 0; c < 64; ++c) li[c] = Li[(size_t)c * 64 + tid];
        double s = 0.;
#pragma unroll
        for (int c = 0; c < 64; ++c) s = fma(li[c], st[c], s);
        sy[tid] = s;
        if (blockIdx.x == 0) y[k + tid] = s;
    }
    __syncthreads();
    for (int i = k + 64 + blockIdx.x * blockDim.x + tid; i < n; i += gridDim.x * blockDim.x) {
        const double *col = A + (size_t)k * ld + i;
        double s0 = 0., s1 = 0.;
#pragma unroll 8
        for (int c = 0; c < 64; c += 2) {
            s0 = fma(col[(size_t)c * ld], sy[c], s0);
            s1 = fma(col[(size_t)(c + 1) * ld], sy[c + 1], s1);
        }
        t[i] -= s0 + s1;
    }
}

// Backward step of block k: x_k = Linv_kk^T t_k (every workgroup; workgroup 0
// stores it), then t_j -= L_k,j^T x_k for the columns j < k: eight lanes per
// column, lane u reading rows 8u..8u+7 of the column's 64 contiguous rows
// (a wave reads eight whole 512-B columns; ld and k are even), the eight
// partial sums combined by a fixed butterfly.  (One thread per column read
// 285 GB/s on C3: 27 us per step, 469 steps per solve.)
__global__ void __launch_bounds__(256) k_dense_bwd_step(const double *__restrict__ A, int ld,
                                                        int k, const double *__restrict__ Li,
                                                        double *t, double *x) {
    __shared__ double st[64], sx[64];
    const int tid = threadIdx.x;
    if (tid < 64) st[tid] = t[k + tid];
    __syncthreads();
    if (tid < 64) {
        // column tid of Linv, stored whole (zeros above the diagonal): all 64
        // loads issued ahead of the chain (as in k_dense_fwd_step)
        const double2 *lc = (const double2 *)(Li + (size_t)tid * 64);
        double2 li[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) li[i] = lc[i];
        double s = 0.;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            s = fma(li[i].x, st[2 * i], s);
            s = fma(li[i].y, st[2 * i + 1], s);
        }
        sx[tid] = s;
        if (blockIdx.x == 0) x[k + tid] = s;
    }
    __syncthreads();
    const int u = tid & 7;
    for (int j0 = blockIdx.x * 32; j0 < k; j0 += gridDim.x * 32) {
        const int j = j0 + (tid >> 3);
        double s = 0.;
        if (j < k) {
            const double2 *col = (const double2 *)(A + (size_t)j * ld + k + 8 * u);
            double2 v[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = col[c];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                s = fma(v[c].x, sx[8 * u + 2 * c], s);
                s = fma(v[c].y, sx[8 * u + 2 * c + 1], s);
            }
        }
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        if (j < k && u == 0) t[j] -= s;
    }
}

void DenseSolver::init(hipStream_t) {}

// Panels of the block of columns [k0, k0 + nb); rows below the diagonal run
// to `end` (exclusive; includes the right-hand-side row).
void DenseSolver::block(hipStream_t s, double *A, int ld, int k0, int nb, int end, int *fail) {
    for (int p = k0; p < k0 + nb; p += 64) {
        double *App = A + (size_t)p * ld + p;
        double *Li = Linv + (size_t)(p / 64) * 64 * 64;
        k_dense_potf64<<<1, 128, 0, s>>>(App, ld, Li, fail);
        const int m = end - (p + 64);
        if (m <= 0) continue;
        double *Aip = App + 64;
        // L_ip = A_ip Linv^T, in place (each workgroup of k_dgemm_nt reads its
        // own 128 rows of A_ip in full before it writes them, and no other
        // workgroup reads them)
        launch_dgemm_nt(s, false, m, 64, 64, Aip, ld, Li, 64, Aip, ld, 1., 0.);
        // the rest of this block's columns [p + 64, k0 + nb)
        const int mb = k0 + nb - (p + 64);
        if (mb > 0) {
            double *Aqq = A + (size_t)(p + 64) * ld + (p + 64);
            const int mr = end - (k0 + nb);
            launch_dgemm_nt(s, true, mb, mb, 64, Aip, ld, Aip, ld, Aqq, ld, -1., 1.);
            launch_dgemm_nt(s, false, mr, mb, 64, Aip + mb, ld, Aip, ld, Aqq + mb, ld, -1., 1.);
        }
    }
}

void DenseSolver::setup(Plan &pl, int n) {
    this->n = n;
    ld = n + 64;
    A = pl.dalloc<double>((size_t)ld * (n + 1));  // column n: the unused A[n][n]
    Linv = pl.dalloc<double>((size_t)n * 64);
    ws = pl.dalloc<double>((size_t)(n + 64) * 64);
}

void DenseSolver::factor_forward(hipStream_t s, const double *r, double *y, int *fail) {
    k_dense_row_put<<<(n + 255) / 256, 256, 0, s>>>(A, ld, n, r);
    const int end = n + 1;  // rows 0..n-1 and the right-hand-side row n
    // block width of the trailing updates: 512 measured 229.6 ms per C3
    // factorisation with k_dgemm_nt (39.3 TF/s, 50 % of the fp64 MFMA peak)
    // against 251.6 ms at 256 -- half as many read-modify-write passes over
    // the trailing matrix
    constexpr int NB = 512;
    for (int k0 = 0; k0 < n; k0 += NB) {
        const int nb = std::min(NB, n - k0);
        block(s, A, ld, k0, nb, end, fail);
        const int m = end - (k0 + nb);
        if (k0 + nb >= n) break;
        // trailing update with the whole block, rhs row included (it also
        // updates the unused A[n][n])
        double *L21 = A + (size_t)k0 * ld + k0 + nb;
        double *S22 = A + (size_t)(k0 + nb) * ld + (k0 + nb);
        launch_dgemm_nt(s, true, m, m, nb, L21, ld, L21, ld, S22, ld, -1., 1.);
    }
    k_dense_row_get<<<(n + 255) / 256, 256, 0, s>>>(A, ld, n, y);
}

// y = L^-1 r: per 64-row block, y_k = Linv_kk t_k, then t_(k+1..) -= L_(k+1..),k y_k.
void DenseSolver::forward(hipStream_t s, const double *r, double *y) {
    double *t = ws;
    MMBA_HIP(hipMemcpyAsync(t, r, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    for (int k = 0; k < n; k += 64) {
        const int m = n - (k + 64);
        const int g = std::max(1, std::min((m + 255) / 256, 1024));
        k_dense_fwd_step<<<g, 256, 0, s>>>(A, ld, n, k, Linv + (size_t)(k / 64) * 64 * 64, t, y);
    }
}

// x = L^-T y: per 64-row block from the last, x_k = Linv_kk^T t_k, then
// t_(0..k) -= L_k,(0..k)^T x_k.
void DenseSolver::backward(hipStream_t s, const double *y, double *x) {
    double *t = ws;
    MMBA_HIP(hipMemcpyAsync(t, y, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    for (int k = n - 64; k >= 0; k -= 64) {
        const int g = std::max(1, std::min((k + 31) / 32, 512));
        k_dense_bwd_step<<<g, 256, 0, s>>>(A, ld, k, Linv + (size_t)(k / 64) * 64 * 64, t, x);
    }
}

}  // namespace mmba
