// Microbenchmark: k_dgemm_nt (mmba_gemm.hip) on the C3 dense reduced solve's
// update shapes -- the rank-512 SYRK of the trailing matrix and the panel
// GEMMs -- warm, HIP-event time per launch and fp64 TFLOP/s.  Build (from this
// directory):
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I../../mayamatchmovesolver_amd/csrc \
//     dgemm_probe.hip -o dgemm_probe
#include "mmba_gemm.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace mmba;

static double run(bool tri, int M, int N, int Kd, int reps) {
    const int ld = M + 64;
    double *A, *B, *Cm;
    hipMalloc(&A, sizeof(double) * (size_t)ld * Kd);
    hipMalloc(&B, sizeof(double) * (size_t)(N + 64) * Kd);
    hipMalloc(&Cm, sizeof(double) * (size_t)ld * N);
    std::vector<double> h((size_t)ld * Kd);
    for (size_t i = 0; i < h.size(); ++i) h[i] = 1e-3 * (double)((i * 2654435761u) % 1000);
    hipMemcpy(A, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice);
    hipMemcpy(B, h.data(), sizeof(double) * std::min(h.size(), (size_t)(N + 64) * Kd),
              hipMemcpyHostToDevice);
    hipMemset(Cm, 0, sizeof(double) * (size_t)ld * N);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int it = 0; it < reps; ++it) {
        hipEventRecord(a);
        launch_dgemm_nt(nullptr, tri, M, N, Kd, A, ld, tri ? A : B, tri ? ld : N + 64, Cm, ld,
                        -1.0, 1.0);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0.f;
        hipEventElapsedTime(&ms, a, b);
        if (it > 0) best = std::min(best, ms);
    }
    const double flop = tri ? (double)M * (M + 1) * Kd : 2.0 * M * N * Kd;
    const double tf = flop / (best * 1e-3) / 1e12;
    std::printf("%s M %6d N %6d K %4d: %8.3f ms  %6.2f TF/s  (%.1f %% of 78.6)\n",
                tri ? "SYRK" : "GEMM", M, N, Kd, best, tf, 100. * tf / 78.6);
    hipFree(A);
    hipFree(B);
    hipFree(Cm);
    return tf;
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 6;
    for (int M : {29504, 20480, 10240, 4096}) run(true, M, M, 512, reps);
    for (int M : {29504, 10240}) run(false, M, 512, 512, reps);
    run(false, 29504, 64, 64, reps);
    return 0;
}
