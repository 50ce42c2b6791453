// Read-rate probe for the camera-frame normal equations' Jacobian pass (C2:
// 120 camera-frames x 1,664 observations, 7 camera columns): the same
// per-observation arithmetic (28 + 7 products of x / y rows) over
//   col   the plan's layout, row r of J at J[r * M + i] (stride M doubles)
//   colp  the same with the row stride padded to M + 64 + a 4 KiB multiple
//   aos   16 doubles per observation (jx[7] jy[7] fx fy), 128 B contiguous
//   sum   a plain streaming sum over the same bytes (the read floor)
// NS workgroups of 256 threads per camera-frame, partials to memory (no last-
// arriver sum: the probe times the observation loop).  Cold: a 512 MiB buffer
// is rewritten between launches (the infinity cache is 256 MiB).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int PC = 7, NCC = 28, NT = 35;

template <int LAYOUT>
__global__ void __launch_bounds__(256) k_read(const double *__restrict__ J, const double *__restrict__ f,
                                              size_t stride, int ncf, int per, int NS, double *out) {
    const int L = blockIdx.x;
    const int cf = L / NS, part = L % NS;
    const int o0 = cf * per, o1 = o0 + per;
    double acc[NT];
#pragma unroll
    for (int e = 0; e < NT; ++e) acc[e] = 0.;
    for (int i = o0 + 256 * part + threadIdx.x; i < o1; i += 256 * NS) {
        double jx[PC], jy[PC], fx, fy;
        if constexpr (LAYOUT == 0) {
#pragma unroll
            for (int a = 0; a < PC; ++a) {
                jx[a] = J[(2 * a) * stride + i];
                jy[a] = J[(2 * a + 1) * stride + i];
            }
            fx = f[2 * i];
            fy = f[2 * i + 1];
        } else {
            const double2 *r = reinterpret_cast<const double2 *>(J + (size_t)16 * i);
            double v[16];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const double2 t = r[q];
                v[2 * q] = t.x;
                v[2 * q + 1] = t.y;
            }
#pragma unroll
            for (int a = 0; a < PC; ++a) {
                jx[a] = v[a];
                jy[a] = v[7 + a];
            }
            fx = v[14];
            fy = v[15];
        }
        int e = 0;
#pragma unroll
        for (int a = 0; a < PC; ++a)
#pragma unroll
            for (int c = a; c < PC; ++c) acc[e++] += jx[a] * jx[c] + jy[a] * jy[c];
#pragma unroll
        for (int a = 0; a < PC; ++a) acc[NCC + a] += jx[a] * fx + jy[a] * fy;
    }
    double s = 0.;
#pragma unroll
    for (int e = 0; e < NT; ++e) s += acc[e] * (e + 1);
    out[(size_t)L * 256 + threadIdx.x] = s;
}

// the same loop with its operands behind a 1 KB by-value argument block (the
// library's kernels take DevProblem, 792 B, and NeEpi, 312 B, by value)
struct BigArg {
    double pad[128];
    const double *J, *f;
    size_t stride;
    int ncf, per, NS;
    double *out;
};
__global__ void __launch_bounds__(256) k_read_big(const BigArg a) {
    const int L = blockIdx.x;
    const int cf = L / a.NS, part = L % a.NS;
    const int o0 = cf * a.per, o1 = o0 + a.per;
    double acc[NT];
#pragma unroll
    for (int e = 0; e < NT; ++e) acc[e] = 0.;
    for (int i = o0 + 256 * part + threadIdx.x; i < o1; i += 256 * a.NS) {
        double jx[PC], jy[PC];
#pragma unroll
        for (int q = 0; q < PC; ++q) {
            jx[q] = a.J[(2 * q) * a.stride + i];
            jy[q] = a.J[(2 * q + 1) * a.stride + i];
        }
        const double fx = a.f[2 * i], fy = a.f[2 * i + 1];
        int e = 0;
#pragma unroll
        for (int q = 0; q < PC; ++q)
#pragma unroll
            for (int c = q; c < PC; ++c) acc[e++] += jx[q] * jx[c] + jy[q] * jy[c];
#pragma unroll
        for (int q = 0; q < PC; ++q) acc[NCC + q] += jx[q] * fx + jy[q] * fy;
    }
    double s = 0.;
#pragma unroll
    for (int e = 0; e < NT; ++e) s += acc[e] * (e + 1);
    a.out[(size_t)L * 256 + threadIdx.x] = s;
}

__global__ void k_sum(const double2 *__restrict__ a, size_t n2, double *out) {
    double s = 0.;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
        const double2 t = a[i];
        s += t.x + t.y;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the Jacobian pass's producer: every row of J (20 rows, stride M) written
__global__ void k_writeJ(double *J, size_t stride, size_t M, int rows) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= M) return;
    for (int r = 0; r < rows; ++r) J[r * stride + i] = (double)(i + r);
}

__global__ void k_flush(double *b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = (double)i;
}

int main() {
    const int ncf = 120, per = 1664;
    const size_t M = (size_t)ncf * per;
    const size_t strideP = ((M + 511) / 512) * 512 + 64;  // not a power-of-two multiple
    double *J, *f, *out, *flush;
    const size_t nflush = (size_t)64 << 20;  // 512 MiB
    CK(hipMalloc(&J, sizeof(double) * 16 * strideP));
    CK(hipMalloc(&f, sizeof(double) * 2 * M));
    CK(hipMalloc(&out, sizeof(double) * 256 * 8192));
    CK(hipMalloc(&flush, sizeof(double) * nflush));
    CK(hipMemset(J, 0, sizeof(double) * 16 * strideP));
    CK(hipMemset(f, 0, sizeof(double) * 2 * M));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = (double)M * 16 * 8;
    printf("M = %zu observations, %.1f MB read per launch\n", M, bytes / 1e6);
    // after a producer kernel that wrote J (20 rows): events between the two
    for (int NS : {1, 4, 16}) {
        double tsum = 0.;
        const int reps = 20;
        hipEvent_t em;
        CK(hipEventCreate(&em));
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(e0));
            k_writeJ<<<(M + 255) / 256, 256>>>(J, M, M, 16);
            CK(hipEventRecord(em));
            k_read<0><<<ncf * NS, 256>>>(J, f, M, ncf, per, NS, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms, mw;
            CK(hipEventElapsedTime(&ms, em, e1));
            CK(hipEventElapsedTime(&mw, e0, em));
            if (r >= 2) tsum += ms;
            if (r == reps + 1) printf("  (producer %.2f us)\n", 1e3 * mw);
        }
        printf("afterw col NS=%2d  %7.2f us  %6.2f TB/s\n", NS, 1e3 * tsum / reps, bytes / (1e3 * tsum / reps) / 1e6);
    }
    {  // by-value 1 KB argument block, warm, after the producer
        BigArg ba{};
        ba.J = J; ba.f = f; ba.stride = M; ba.ncf = ncf; ba.per = per; ba.NS = 4; ba.out = out;
        double tsum = 0., tsmall = 0.;
        const int reps = 20;
        hipEvent_t em;
        CK(hipEventCreate(&em));
        for (int r = 0; r < reps + 2; ++r) {
            k_writeJ<<<(M + 255) / 256, 256>>>(J, M, M, 16);
            CK(hipEventRecord(e0));
            k_read_big<<<ncf * 4, 256>>>(ba);
            CK(hipEventRecord(em));
            k_read<0><<<ncf * 4, 256>>>(J, f, M, ncf, per, 4, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float mb, ms;
            CK(hipEventElapsedTime(&mb, e0, em));
            CK(hipEventElapsedTime(&ms, em, e1));
            if (r >= 2) { tsum += mb; tsmall += ms; }
        }
        printf("bigarg NS=4  %7.2f us (small-argument kernel right after it: %7.2f us)\n",
               1e3 * tsum / reps, 1e3 * tsmall / reps);
    }
    for (int cold = 0; cold < 2; ++cold) {
        for (int lay = 0; lay < 4; ++lay) {
            for (int NS : {1, 4, 16}) {
                if (lay == 3 && NS != 4) continue;
                double tsum = 0.;
                const int reps = 20;
                for (int r = 0; r < reps + 2; ++r) {
                    if (cold) k_flush<<<4096, 256>>>(flush, nflush);
                    CK(hipEventRecord(e0));
                    if (lay == 0) k_read<0><<<ncf * NS, 256>>>(J, f, M, ncf, per, NS, out);
                    else if (lay == 1) k_read<0><<<ncf * NS, 256>>>(J, f, strideP, ncf, per, NS, out);
                    else if (lay == 2) k_read<1><<<ncf * NS, 256>>>(J, f, 0, ncf, per, NS, out);
                    else k_sum<<<2048, 256>>>(reinterpret_cast<const double2 *>(J), M * 8, out);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 2) tsum += ms;
                }
                const double us = 1e3 * tsum / reps;
                const char *nm[] = {"col", "colp", "aos", "sum"};
                printf("%s %-4s NS=%2d grid=%5d  %7.2f us  %6.2f TB/s\n", cold ? "cold" : "warm", nm[lay], NS,
                       lay == 3 ? 2048 : ncf * NS, us, bytes / us / 1e6);
            }
        }
    }
    return 0;
}
