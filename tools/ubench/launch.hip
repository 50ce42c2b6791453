// Host cost of one kernel launch by argument size (the library's kernels take
// DevProblem, 792 B, and NeEpi, 312 B, by value): a stream kept busy by a
// long kernel, then N launches of an empty kernel with 16 B / 256 B / 1 KB /
// 2 KB of arguments -- host wall time per launch call, and the same through
// one pointer argument to a device-resident copy.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NB>
struct Blob {
    double v[NB / 8];
};

template <int NB>
__global__ void k_arg(const Blob<NB> b, double *out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[NB / 8 - 1] == 12345.) out[0] = b.v[0];
}

__global__ void k_spin(long long cycles) {
    const long long t0 = clock64();
    while (clock64() - t0 < cycles) {
    }
}

template <int NB>
double per_launch(hipStream_t s, double *out, int n) {
    Blob<NB> b{};
    k_spin<<<1, 64, 0, s>>>(200000000LL);  // keep the queue busy: launches only enqueue
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) k_arg<NB><<<256, 64, 0, s>>>(b, out);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    (void)hipStreamSynchronize(s);
    return us / n;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    double *out;
    CK(hipMalloc(&out, 64));
    per_launch<16>(s, out, 100);  // warm
    for (int rep = 0; rep < 2; ++rep) {
        printf("args   16 B: %6.2f us per launch\n", per_launch<16>(s, out, 200));
        printf("args  256 B: %6.2f us per launch\n", per_launch<256>(s, out, 200));
        printf("args 1024 B: %6.2f us per launch\n", per_launch<1024>(s, out, 200));
        printf("args 2048 B: %6.2f us per launch\n", per_launch<2048>(s, out, 200));
    }
    return 0;
}
