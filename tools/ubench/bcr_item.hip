// Microbenchmark: one BCR elimination item (bcr_level_item<24, 2, true>) of
// mmba_bcr.hip repeated REPS times by one workgroup on synthetic SPD blocks:
// rep 0 runs with a cold instruction cache, the rest warm.  Wall clock
// (100 MHz) per rep.  Build like bcr_chain.hip.
#include "mmba_bcr.hip"

#include <cstdio>
#include <vector>

using namespace mmba;
constexpr int K = 24, NBLK = 8, REPS = 16;

template <int CH>
__global__ void __launch_bounds__(256) kitem(BcrDev B, int *fail, long long *t) {
    for (int r = 0; r < REPS; ++r) {
        __syncthreads();
        const long long t0 = wall_clock64();
        bcr_level_item<K, CH, true>(B, 2, NBLK, 0, 2, fail, r > 0 ? t + 64 : nullptr, B.rw + 4096,
                                   false, nullptr);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) t[r] = wall_clock64() - t0;
    }
}

// an unrelated code stream between launches (evicts the instruction cache)
__global__ void kother(double *x) {
    double v = x[threadIdx.x];
#pragma unroll
    for (int i = 0; i < 4000; ++i) v = v * 1.0000001 + (double)(i & 7);
    x[threadIdx.x] = v;
}

int main() {
    const size_t kk = (size_t)NBLK * K * K;
    std::vector<double> hD(kk, 0.), hL(kk, 0.);
    for (int b = 0; b < NBLK; ++b)
        for (int i = 0; i < K; ++i)
            for (int c = 0; c < K; ++c) {
                hD[(size_t)b * K * K + i * K + c] = (i == c) ? 40. : (c < i ? 0.3 * ((i + 2 * c) % 5) / 5. : 0.);
                hL[(size_t)b * K * K + i * K + c] = 0.2 * ((3 * i + c) % 7) / 7.;
            }
    BcrDev B;
    B.K = K;
    B.nb = NBLK * K;
    B.nG = 0;
    B.nblk = NBLK;
    B.w = 23;
    B.NR = K;
    double *buf[10];
    for (auto &p : buf) {
        hipMalloc(&p, kk * sizeof(double) + 8192 * sizeof(double));
        hipMemset(p, 0, kk * sizeof(double) + 8192 * sizeof(double));
    }
    B.Dk = buf[0];
    B.Lk0 = buf[1];
    B.Lk1 = buf[2];
    B.FC = buf[3];
    B.FU = buf[4];
    B.FV = buf[5];
    B.Gk = buf[6];
    B.FY = buf[7];
    B.Zc = buf[8];
    B.gpart = buf[8] + kk;
    B.rw = buf[9];
    int *fail;
    long long *t, h[REPS], ph[8];
    hipMalloc(&fail, sizeof(int));
    hipMalloc(&t, 128 * sizeof(long long));
    double *x;
    hipMalloc(&x, 256 * sizeof(double));
    hipMemset(x, 0, 256 * sizeof(double));
    for (int run = 0; run < 4; ++run) {
        hipMemcpy(B.Dk, hD.data(), kk * sizeof(double), hipMemcpyHostToDevice);
        hipMemcpy(B.Lk0, hL.data(), kk * sizeof(double), hipMemcpyHostToDevice);
        hipMemset(t, 0, 128 * sizeof(long long));
        kother<<<1024, 256>>>(x);
        if (run & 1)
            kitem<0><<<1, 256>>>(B, fail, t);
        else
            kitem<2><<<1, 256>>>(B, fail, t);
        hipDeviceSynchronize();
        hipMemcpy(h, t, sizeof(h), hipMemcpyDeviceToHost);
        std::printf("run %d (%s chain): item us per rep:", run, (run & 1) ? "LDS" : "blocked");
        for (int r = 0; r < REPS; ++r) std::printf(" %.2f", h[r] / 100.);
        std::printf("\n");
        hipMemcpy(ph, t + 64, sizeof(ph), hipMemcpyDeviceToHost);
        std::printf("  warm phases (us per rep): stage %.2f a-load %.2f chain %.2f store %.2f mfma %.2f tail %.2f\n",
                    ph[0] / 100. / (REPS - 1), ph[1] / 100. / (REPS - 1), ph[2] / 100. / (REPS - 1),
                    ph[3] / 100. / (REPS - 1), ph[4] / 100. / (REPS - 1), ph[5] / 100. / (REPS - 1));
    }
    return 0;
}
