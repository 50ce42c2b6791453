// Microbenchmark: the BCR pivot-chain variants of mmba_bcr.hip in isolation
// (one wave, 24 x 24 block in lanes 0..23, right-hand sides in lanes 24..63),
// shader cycles (s_memtime) per factorisation.  Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../mayamatchmovesolver_amd/csrc \
//     bcr_chain.hip -L../../mayamatchmovesolver_amd/csrc -lmmba -o bcr_chain
#include "mmba_bcr.hip"

#include <cstdio>

using namespace mmba;
constexpr int K = 24, REPS = 64;

template <int V>
__global__ void __launch_bounds__(256) kchain(double *out, long long *cyc) {
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
    long long t0 = clock64(), w0 = wall_clock64();
    long long tf = 0;
    for (int r = 0; r < REPS; ++r) {
        if (r == 1) tf = clock64() - t0;  // first (cold instruction cache) factorisation
        double a[K];
#pragma unroll
        for (int c = 0; c < K; ++c) a[c] = a0[c] + sink * 1e-300;
        if (V == 0) bcr_chol_aug_blk<K, 8>(a, nullptr, pl, bad);
        if (V == 1) bcr_chol_aug_blk<K, 4>(a, nullptr, pl, bad);
        if (V == 2) bcr_chol_aug_blk<K, 12>(a, nullptr, pl, bad);
        if (V == 3) bcr_chol_aug_blk<K, 24>(a, nullptr, pl, bad);
        if (V == 4) bcr_chol_aug_wave<K>(a, nullptr, pl, bad);
        sink += a[K - 1] + a[3];
    }
    long long t1 = clock64(), w1 = wall_clock64();
    out[threadIdx.x] = sink + bad;
    if (threadIdx.x == 0) {
        cyc[V] = (t1 - t0 - tf) / (REPS - 1);
        cyc[16 + V] = tf;
        cyc[8 + V] = (w1 - w0) * 10 / REPS;  // ns
    }
}

int main() {
    double *d;
    long long *c, h[24] = {};
    hipMalloc(&d, 256 * sizeof(double));
    hipMalloc(&c, 24 * sizeof(long long));
    for (int nw = 1; nw <= 4; nw *= 2) {
    std::printf("%d wave(s) per workgroup, each its own chain:\n", nw);
    for (int w = 0; w < 1; ++w) {
        kchain<0><<<1, 64 * nw>>>(d, c);
        kchain<1><<<1, 64 * nw>>>(d, c);
        kchain<2><<<1, 64 * nw>>>(d, c);
        kchain<3><<<1, 64 * nw>>>(d, c);
        kchain<4><<<1, 64 * nw>>>(d, c);
        hipDeviceSynchronize();
    }
    hipMemcpy(h, c, sizeof(h), hipMemcpyDeviceToHost);
    const char *nm[5] = {"blk PW=8", "blk PW=4", "blk PW=12", "blk PW=24 (all readlane)", "LDS chain"};
    for (int v = 0; v < 5; ++v)
        std::printf("%-28s %8lld cycles %7lld ns per 24x24 augmented factorisation (%.1f cycles "
                    "per step, %.2f GHz); first (cold) %lld cycles\n", nm[v], h[v], h[8 + v], h[v] / 24.,
                    (double)h[v] / h[8 + v] * (REPS - 1) / REPS, h[16 + v]);
    }
    return 0;
}
