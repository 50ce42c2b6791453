// Microbenchmark: the blocked augmented pivot chain of mmba_bcr_dev.h
// (bcr_chol_aug_blk<24, PW>) in isolation, one to four waves per workgroup
// each running its own chain, shader clock cycles (clock64) and wall-clock ns
// per 24 x 24 augmented factorisation; variant "+stores" adds the 24
// write-through (sc1) stores per right-hand-side lane that k_pcr_solve
// issues after its chain.  Build (from this directory):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../mayamatchmovesolver_amd/csrc \
//     chain_dev.hip -o chain_dev
#include "mmba_bcr_dev.h"

#include <cstdio>

using namespace mmba;
constexpr int K = 24, REPS = 64;

template <int PW, bool ST>
__global__ void __launch_bounds__(256) kchain(double *out, long long *cyc, double *gst) {
    __shared__ double plw[4][64 * 24];
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
        bcr_chol_aug_blk<K, PW>(a, nullptr, pl, bad);
        if (ST && lane >= K && lane < 2 * K) {
            double *dst = gst + (threadIdx.x >> 6) * K * K + (lane - K) * K;
#pragma unroll
            for (int i = 0; i < K; ++i) bcr_st(dst + i, a[i]);
        }
        sink += a[K - 1] + a[3];
    }
    if (ST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    long long t1 = clock64(), w1 = wall_clock64();
    out[threadIdx.x] = sink + bad;
    if (threadIdx.x == 0) {
        cyc[0] = (t1 - t0) / REPS;
        cyc[1] = (w1 - w0) * 10 / REPS;  // ns
    }
}

template <int PW, bool ST>
void run(const char *nm, double *d, long long *c, double *g, int nw) {
    long long h[2];
    for (int w = 0; w < 3; ++w) kchain<PW, ST><<<1, 64 * nw>>>(d, c, g);
    hipDeviceSynchronize();
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("  %-22s %7lld cycles %6lld ns per factorisation (%.1f cycles per step)\n", nm, h[0],
                h[1], h[0] / 24.);
}

int main() {
    double *d, *g;
    long long *c;
    hipMalloc(&d, 256 * sizeof(double));
    hipMalloc(&g, 4 * K * K * sizeof(double));
    hipMalloc(&c, 2 * sizeof(long long));
    for (int nw = 1; nw <= 4; nw *= 2) {
        std::printf("%d wave(s), each its own chain:\n", nw);
        run<4, false>("PW=4", d, c, g, nw);
        run<6, false>("PW=6", d, c, g, nw);
        run<8, false>("PW=8", d, c, g, nw);
        run<12, false>("PW=12", d, c, g, nw);
        run<6, true>("PW=6 +stores", d, c, g, nw);
    }
    return 0;
}
