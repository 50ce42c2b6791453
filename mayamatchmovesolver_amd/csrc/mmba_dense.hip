// mmba_dense.hip -- dense reduced camera system (CDNA4 / gfx950, fp64).
//
// When the bundles tie most camera-frames together (C3: every bundle is
// tracked by five cameras over windows spread across the whole shot) the
// reduced system S has almost no zero tiles and its Cholesky factor is
// dense.  S is then held as one column-major lower triangle (ld = nRpad) and
// factored by a right-looking blocked Cholesky:
//
//   for each 64-column panel k:  L_kk = chol(S_kk)       k_dense_potf64 (one wave)
//                                L_ik = S_ik L_kk^-T      rocblas_dtrsm (MFMA)
//                                S_ii -= L_ik L_ik^T      rocblas_dsyrk (MFMA)
//
// grouped so the trailing updates run as large rank-256 SYRK/GEMM calls
// (the 64-column panels inside a 256-column block are factored with small
// trsm/syrk calls on the block only).  The flops are the n^3/3 of a dense
// Cholesky, in fp64 MFMA library GEMMs; the panel factorisation is a
// hand-written one-wave register kernel (the latency-bound part).
// Solves L y = r and L^T x = y are rocblas_dtrsv.
#include <rocblas/rocblas.h>

#include "mmba_kernels.h"
#include "mmba_plan.h"

namespace mmba {

__device__ __forceinline__ double dn_rdlane(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// In-place Cholesky of the 64 x 64 diagonal block at A (column-major, ld):
// lane r holds row r in registers, the pivot is broadcast with v_readlane and
// column j through LDS.  A non-positive or non-finite pivot sets *fail and is
// replaced by 1 (the factorisation continues; the LM treats the solve as
// failed).  Only the lower triangle is read and written.
__global__ void __launch_bounds__(64) k_dense_potf64(double *A, int ld, int *fail) {
    __shared__ double col[64];
    const int lane = threadIdx.x;
    double a[64];
#pragma unroll
    for (int c = 0; c < 64; ++c) a[c] = c <= lane ? A[(size_t)c * ld + lane] : 0.;
    int bad = 0;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
        double d = dn_rdlane(a[j], j);
        if (!(d > 0.) || !isfinite(d)) {
            bad = 1;
            d = 1.;
        }
        const double sd = sqrt(d);
        const double l = lane > j ? a[j] / sd : 0.;
        a[j] = lane == j ? sd : (lane > j ? l : a[j]);
        col[lane] = l;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int c = j + 1; c < 64; ++c) a[c] = fma(-l, col[c], a[c]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
#pragma unroll
    for (int c = 0; c < 64; ++c)
        if (c <= lane) A[(size_t)c * ld + lane] = a[c];
    if (bad && lane == 0) atomicOr(fail, 1);
}

#define MMBA_RB(call)                                                                    \
    do {                                                                                 \
        rocblas_status st_ = (call);                                                     \
        if (st_ != rocblas_status_success) {                                             \
            ::mmba::set_error(std::string(#call) + ": " + rocblas_status_to_string(st_)); \
            throw ::mmba::DeviceError();                                                 \
        }                                                                                \
    } while (0)

DenseSolver::~DenseSolver() {
    if (handle) (void)rocblas_destroy_handle((rocblas_handle)handle);
}

void DenseSolver::init(hipStream_t s) {
    if (!handle) {
        rocblas_handle h = nullptr;
        MMBA_RB(rocblas_create_handle(&h));
        handle = h;
    }
    MMBA_RB(rocblas_set_stream((rocblas_handle)handle, s));
    MMBA_RB(rocblas_set_pointer_mode((rocblas_handle)handle, rocblas_pointer_mode_host));
}

// Factor rows/columns [k0, k0 + nb) of the trailing matrix: 64-column panels,
// each followed by the trsm/syrk of the rows below it up to row `end`.
static void dense_block(rocblas_handle h, double *A, int ld, int k0, int nb, int end,
                        int *fail, hipStream_t s) {
    const double one = 1.0, mone = -1.0;
    for (int p = k0; p < k0 + nb; p += 64) {
        double *App = A + (size_t)p * ld + p;
        k_dense_potf64<<<1, 64, 0, s>>>(App, ld, fail);
        const int m = end - (p + 64);
        if (m <= 0) continue;
        double *Aip = App + 64;
        MMBA_RB(rocblas_dtrsm(h, rocblas_side_right, rocblas_fill_lower,
                              rocblas_operation_transpose, rocblas_diagonal_non_unit, m, 64,
                              &one, App, ld, Aip, ld));
        // update only the rest of this block's columns [p + 64, k0 + nb)
        const int mb = k0 + nb - (p + 64);
        if (mb > 0) {
            double *Aqq = A + (size_t)(p + 64) * ld + (p + 64);
            // S[p+64 .. end, p+64 .. k0+nb) -= L[p+64 .. end, p] L[p+64 .. k0+nb, p]^T
            MMBA_RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, mb, 64, &mone,
                                  Aip, ld, &one, Aqq, ld));
            const int mr = end - (k0 + nb);
            if (mr > 0)
                MMBA_RB(rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, mr,
                                      mb, 64, &mone, Aip + mb, ld, Aip, ld, &one, Aqq + mb,
                                      ld));
        }
    }
}

void DenseSolver::factor(hipStream_t s, double *A, int n, int ld, int *fail) {
    init(s);
    rocblas_handle h = (rocblas_handle)handle;
    const double one = 1.0, mone = -1.0;
    constexpr int NB = 256;
    for (int k0 = 0; k0 < n; k0 += NB) {
        const int nb = std::min(NB, n - k0);
        // panels of this block (their trsm covers every row below)
        dense_block(h, A, ld, k0, nb, n, fail, s);
        const int m = n - (k0 + nb);
        if (m <= 0) break;
        // trailing update with the whole block: S22 -= L21 L21^T (rank nb)
        double *L21 = A + (size_t)k0 * ld + k0 + nb;
        double *S22 = A + (size_t)(k0 + nb) * ld + (k0 + nb);
        MMBA_RB(rocblas_dsyrk(h, rocblas_fill_lower, rocblas_operation_none, m, nb, &mone, L21,
                              ld, &one, S22, ld));
    }
}

void DenseSolver::forward(hipStream_t s, const double *A, int n, int ld, const double *r,
                          double *y) {
    init(s);
    if (y != r) MMBA_HIP(hipMemcpyAsync(y, r, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    MMBA_RB(rocblas_dtrsv((rocblas_handle)handle, rocblas_fill_lower, rocblas_operation_none,
                          rocblas_diagonal_non_unit, n, A, ld, y, 1));
}

void DenseSolver::backward(hipStream_t s, const double *A, int n, int ld, const double *y,
                           double *x) {
    init(s);
    if (x != y) MMBA_HIP(hipMemcpyAsync(x, y, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    MMBA_RB(rocblas_dtrsv((rocblas_handle)handle, rocblas_fill_lower,
                          rocblas_operation_transpose, rocblas_diagonal_non_unit, n, A, ld, x,
                          1));
}

}  // namespace mmba
