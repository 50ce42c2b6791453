// Hand-back probe (C2's three output lists: 3.2 + 3.2 + 1.6 MB device ->
// page-locked host): wall time from enqueue to completion of
//   seq     three hipMemcpyAsync on one stream (the plan's hand-back)
//   par     the three copies on three streams (separate DMA queues)
//   kern    one kernel storing the three lists straight into the page-locked
//           buffers (host-mapped, coalesced 16-B stores per lane)
//   kern+g  the same kernel gathering through a permutation (the unpermute)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_store(const double *__restrict__ a, const double *__restrict__ b, const double *__restrict__ c,
                        const int *__restrict__ perm, size_t n2, size_t n1, double *ha, double *hb, double *hc) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < n1; r += stride) {
        const size_t d = perm ? (size_t)perm[r] : r;
        double2 va = {a[2 * d], a[2 * d + 1]}, vb = {b[2 * d], b[2 * d + 1]};
        reinterpret_cast<double2 *>(ha)[r] = va;
        reinterpret_cast<double2 *>(hb)[r] = vb;
        hc[r] = c[d];
    }
    (void)n2;
}

int main() {
    const size_t M = 199680, m = 2 * M;
    double *da, *db, *dc, *ha, *hb, *hc;
    int *perm;
    CK(hipMalloc(&da, m * 8));
    CK(hipMalloc(&db, m * 8));
    CK(hipMalloc(&dc, M * 8));
    CK(hipMalloc(&perm, M * 4));
    std::vector<int> hp(M);
    for (size_t i = 0; i < M; ++i) hp[i] = (int)((i * 7919) % M);
    CK(hipMemcpy(perm, hp.data(), M * 4, hipMemcpyHostToDevice));
    CK(hipMemset(da, 0, m * 8));
    CK(hipMemset(db, 0, m * 8));
    CK(hipMemset(dc, 0, M * 8));
    CK(hipHostMalloc(&ha, m * 8, hipHostMallocDefault));
    CK(hipHostMalloc(&hb, m * 8, hipHostMallocDefault));
    CK(hipHostMalloc(&hc, M * 8, hipHostMallocDefault));
    hipStream_t s[3];
    for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    hipEvent_t ev;
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    printf("%.1f MB per hand-back\n", (2 * m + M) * 8 / 1e6);
    for (int mode = 0; mode < 5; ++mode) {
        double best = 1e9, sum = 0.;
        const int reps = 30;
        for (int r = 0; r < reps + 3; ++r) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            if (mode == 0) {
                CK(hipMemcpyAsync(ha, da, m * 8, hipMemcpyDeviceToHost, s[0]));
                CK(hipMemcpyAsync(hb, db, m * 8, hipMemcpyDeviceToHost, s[0]));
                CK(hipMemcpyAsync(hc, dc, M * 8, hipMemcpyDeviceToHost, s[0]));
                CK(hipStreamSynchronize(s[0]));
            } else if (mode == 1) {
                CK(hipMemcpyAsync(ha, da, m * 8, hipMemcpyDeviceToHost, s[0]));
                CK(hipMemcpyAsync(hb, db, m * 8, hipMemcpyDeviceToHost, s[1]));
                CK(hipMemcpyAsync(hc, dc, M * 8, hipMemcpyDeviceToHost, s[2]));
                for (auto &x : s) CK(hipStreamSynchronize(x));
            } else if (mode == 4) {
                // two halves of each list on two streams
                CK(hipMemcpyAsync(ha, da, m * 4, hipMemcpyDeviceToHost, s[0]));
                CK(hipMemcpyAsync(ha + m / 2, da + m / 2, m * 4, hipMemcpyDeviceToHost, s[1]));
                CK(hipMemcpyAsync(hb, db, m * 4, hipMemcpyDeviceToHost, s[2]));
                CK(hipMemcpyAsync(hb + m / 2, db + m / 2, m * 4, hipMemcpyDeviceToHost, s[0]));
                CK(hipMemcpyAsync(hc, dc, M * 4, hipMemcpyDeviceToHost, s[1]));
                CK(hipMemcpyAsync(hc + M / 2, dc + M / 2, M * 4, hipMemcpyDeviceToHost, s[2]));
                for (auto &x : s) CK(hipStreamSynchronize(x));
            } else {
                const int grid = mode == 2 ? 1024 : 2048;
                k_store<<<grid, 256, 0, s[0]>>>(da, db, dc, mode == 3 ? perm : nullptr, m, M, ha, hb, hc);
                CK(hipEventRecord(ev, s[0]));
                while (hipEventQuery(ev) == hipErrorNotReady) {
                }
            }
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            if (r >= 3) {
                sum += us;
                if (us < best) best = us;
            }
        }
        const char *nm[] = {"seq", "par", "kern", "kern+g", "par6"};
        printf("%-7s avg %7.1f us  best %7.1f us  %5.1f GB/s (avg)\n", nm[mode], sum / reps, best,
               (2 * m + M) * 8 / (sum / reps) / 1e3);
    }
    return 0;
}
