// Microbenchmark (round 6): the one-pivot augmented Cholesky chain
// (bcr_chol_aug_blk<24, PW>) against the 2 x 2-pivot chain without square
// roots (bcr_ldl2_aug_blk<24, PW>) of mmba_bcr_dev.h: shader cycles per 24 x 24
// augmented factorisation (one wave, and four waves each running its own
// chain), and the accuracy of both on SPD blocks of rising condition number
// against C^-1 b computed on the host in long double.  Build (from this
// directory):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../mayamatchmovesolver_amd/csrc \
//     chain2.hip -o chain2
#include "mmba_bcr_dev.h"

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

using namespace mmba;
constexpr int K = 24, REPS = 64;

template <int V, int PW>
__device__ __forceinline__ void run_chain(double (&a)[K], double *pl, int &bad) {
    if constexpr (V == 0)
        bcr_chol_aug_blk<K, PW>(a, nullptr, pl, bad);
    else if constexpr (V == 1)
        bcr_ldl2_aug_blk<K, PW, 0>(a, pl, bad);
    else if constexpr (V == 2)
        bcr_ldl2_aug_blk<K, PW, 2>(a, pl, bad);
    else
        bcr_ldl1_aug_blk<K, PW>(a, pl, bad);
}

template <int V, int PW>
__global__ void __launch_bounds__(256) ktime(double *out, long long *cyc) {
    __shared__ double plw[4][2 * 64 * 12 + 64];
    double *pl = plw[threadIdx.x >> 6];
    const int lane = threadIdx.x & 63;
    double a0[K];
#pragma unroll
    for (int c = 0; c < K; ++c)
        a0[c] = lane < K ? (c == lane ? 30. : (c < lane ? 0.1 * ((lane * 7 + c * 3) % 11) / 11. : 0.))
                         : 0.01 * ((lane + c) % 13);
    double sink = 0.;
    int bad = 0;
    __syncthreads();
    long long t0 = clock64(), w0 = wall_clock64();
    for (int r = 0; r < REPS; ++r) {
        double a[K];
#pragma unroll
        for (int c = 0; c < K; ++c) a[c] = a0[c] + sink * 1e-300;
        run_chain<V, PW>(a, pl, bad);
        sink += a[K - 1] + a[3];
    }
    long long t1 = clock64(), w1 = wall_clock64();
    out[threadIdx.x] = sink + bad;
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / REPS;
        cyc[1] = (w1 - w0) * 10 / REPS;  // ns
    }
}

// one wave: lanes 0..K-1 rows of D (lower), lanes K..2K-1 columns of b
template <int V, int PW>
__global__ void kacc(const double *D, const double *B, double *X, int *badp) {
    __shared__ double pl[2 * 64 * 12 + 64];
    const int lane = threadIdx.x;
    double a[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
        if (lane < K)
            a[c] = c <= lane ? D[lane * K + c] : 0.;
        else if (lane < 2 * K)
            a[c] = B[(lane - K) * K + c];
        else
            a[c] = 0.;
    }
    int bad = 0;
    run_chain<V, PW>(a, pl, bad);
    if (lane >= K && lane < 2 * K)
#pragma unroll
        for (int c = 0; c < K; ++c) X[(lane - K) * K + c] = a[c];
    if (lane == 0) *badp = bad;
}

template <int V, int PW>
void timing(const char *nm, double *d, long long *c, int nw) {
    long long h[2];
    for (int w = 0; w < 3; ++w) ktime<V, PW><<<1, 64 * nw>>>(d, c);
    hipDeviceSynchronize();
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("  %-16s %7lld cycles %6lld ns per factorisation (%.1f cycles per pivot)\n", nm, h[0],
                h[1], h[0] / 24.);
}

template <int V, int PW>
double accuracy(const std::vector<double> &D, const std::vector<double> &B,
                const std::vector<long double> &Xr, double *dD, double *dB, double *dX, int *db,
                int &bad) {
    kacc<V, PW><<<1, 64>>>(dD, dB, dX, db);
    std::vector<double> X(K * K);
    hipMemcpy(X.data(), dX, K * K * 8, hipMemcpyDeviceToHost);
    hipMemcpy(&bad, db, 4, hipMemcpyDeviceToHost);
    long double num = 0, den = 0;
    for (int i = 0; i < K * K; ++i) {
        num = std::max(num, std::fabs((long double)X[i] - Xr[i]));
        den = std::max(den, std::fabs(Xr[i]));
    }
    return (double)(num / den);
}

int main() {
    double *d;
    long long *c;
    hipMalloc(&d, 256 * sizeof(double));
    hipMalloc(&c, 2 * sizeof(long long));
    for (int nw = 1; nw <= 4; nw *= 4) {
        std::printf("%d wave(s), each its own chain:\n", nw);
        timing<0, 6>("chol PW=6", d, c, nw);
        timing<2, 4>("ldl2p PW=4", d, c, nw);
        timing<3, 2>("ldl1 PW=2", d, c, nw);
        timing<3, 3>("ldl1 PW=3", d, c, nw);
        timing<3, 4>("ldl1 PW=4", d, c, nw);
        timing<3, 6>("ldl1 PW=6", d, c, nw);
        timing<3, 8>("ldl1 PW=8", d, c, nw);
    }
    // accuracy: D = Q diag(s) Q^T with singular values spread over 10^e
    double *dD, *dB, *dX;
    int *db;
    hipMalloc(&dD, K * K * 8);
    hipMalloc(&dB, K * K * 8);
    hipMalloc(&dX, K * K * 8);
    hipMalloc(&db, 4);
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    for (int e = 0; e <= 12; e += 3) {
        std::vector<long double> M(K * K), Q(K * K);
        for (auto &v : M) v = nd(rng);
        // Gram-Schmidt
        for (int j = 0; j < K; ++j) {
            for (int i = 0; i < K; ++i) Q[i * K + j] = M[i * K + j];
            for (int k = 0; k < j; ++k) {
                long double dot = 0;
                for (int i = 0; i < K; ++i) dot += Q[i * K + k] * Q[i * K + j];
                for (int i = 0; i < K; ++i) Q[i * K + j] -= dot * Q[i * K + k];
            }
            long double n = 0;
            for (int i = 0; i < K; ++i) n += Q[i * K + j] * Q[i * K + j];
            n = std::sqrt(n);
            for (int i = 0; i < K; ++i) Q[i * K + j] /= n;
        }
        std::vector<double> D(K * K), B(K * K);
        std::vector<long double> Dl(K * K);
        for (int i = 0; i < K; ++i)
            for (int j = 0; j < K; ++j) {
                long double s = 0;
                for (int k = 0; k < K; ++k) s += Q[i * K + k] * std::pow(10.0L, -(long double)e * k / (K - 1)) * Q[j * K + k];
                D[i * K + j] = (double)s;
            }
        for (int i = 0; i < K; ++i)
            for (int j = 0; j < K; ++j) Dl[i * K + j] = D[std::max(i, j) * K + std::min(i, j)];
        for (auto &v : B) v = nd(rng);
        // reference: Cholesky in long double, X row c = (C^-1 b_c)
        std::vector<long double> C(K * K, 0);
        for (int j = 0; j < K; ++j) {
            long double s = Dl[j * K + j];
            for (int k = 0; k < j; ++k) s -= C[j * K + k] * C[j * K + k];
            C[j * K + j] = std::sqrt(s);
            for (int i = j + 1; i < K; ++i) {
                long double t = Dl[i * K + j];
                for (int k = 0; k < j; ++k) t -= C[i * K + k] * C[j * K + k];
                C[i * K + j] = t / C[j * K + j];
            }
        }
        std::vector<long double> Xr(K * K);
        for (int col = 0; col < K; ++col)
            for (int i = 0; i < K; ++i) {
                long double t = B[col * K + i];
                for (int k = 0; k < i; ++k) t -= C[i * K + k] * Xr[col * K + k];
                Xr[col * K + i] = t / C[i * K + i];
            }
        hipMemcpy(dD, D.data(), K * K * 8, hipMemcpyHostToDevice);
        hipMemcpy(dB, B.data(), K * K * 8, hipMemcpyHostToDevice);
        int b0 = 0, b1 = 0;
        const double e0 = accuracy<0, 6>(D, B, Xr, dD, dB, dX, db, b0);
        const double e1 = accuracy<1, 6>(D, B, Xr, dD, dB, dX, db, b1);
        const double e2 = accuracy<2, 4>(D, B, Xr, dD, dB, dX, db, b1);
        const double e3 = accuracy<3, 4>(D, B, Xr, dD, dB, dX, db, b1);
        std::printf("cond 1e%-2d: max rel err chol %.2e (bad %d)  ldl2 PW6 %.2e  ldl2p PW4 %.2e ldl1 PW4 %.2e (bad %d)\n", e,
                    e0, b0, e1, e2, e3, b1);
    }
    return 0;
}
