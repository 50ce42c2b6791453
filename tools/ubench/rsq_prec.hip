// Microbenchmark: accuracy of v_rsq_f64 (__builtin_amdgcn_rsq) with 0, 1 and
// 2 Newton steps against the correctly rounded 1 / sqrt(d) (computed in long
// double on the host), and the dependent-chain latency of each form (one
// wave, s_memtime cycles per link).  Build:
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off rsq_prec.hip -o rsq_prec
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__device__ __forceinline__ double newton(double d, double y) {
    const double h = 0.5 * d;
    return y * fma(-h * y, y, 1.5);
}

__global__ void krsq(const double *d, double *y0, double *y1, double *y2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = d[i];
    const double r = __builtin_amdgcn_rsq(v);
    y0[i] = r;
    const double r1 = newton(v, r);
    y1[i] = r1;
    y2[i] = newton(v, r1);
}

template <int NW>
__global__ void kchain(double *out, long long *cyc, double seed) {
    double v = seed + threadIdx.x * 1e-3;
    const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 1024; ++i) {
        double r = __builtin_amdgcn_rsq(v);
        if (NW >= 1) r = newton(v, r);
        if (NW >= 2) r = newton(v, r);
        v = fma(r, 1e-9, v);  // next link depends on this one
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = v;
    if (threadIdx.x == 0) cyc[NW] = t1 - t0;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> h(n);
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> u(-20.0, 20.0);
    for (int i = 0; i < n; ++i) h[i] = std::exp(u(g));
    double *d, *y[3];
    hipMalloc(&d, n * sizeof(double));
    for (auto &p : y) hipMalloc(&p, n * sizeof(double));
    hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice);
    krsq<<<n / 256, 256>>>(d, y[0], y[1], y[2], n);
    std::vector<double> r(n);
    for (int k = 0; k < 3; ++k) {
        hipMemcpy(r.data(), y[k], n * sizeof(double), hipMemcpyDeviceToHost);
        double maxrel = 0, maxulp = 0;
        long exact = 0;
        for (int i = 0; i < n; ++i) {
            const long double t = 1.0L / std::sqrt((long double)h[i]);
            const double tr = (double)t;
            const double rel = std::fabs((double)((r[i] - t) / t));
            maxrel = std::max(maxrel, rel);
            maxulp = std::max(maxulp, std::fabs(r[i] - tr) / (std::nextafter(tr, 1e300) - tr));
            exact += r[i] == tr;
        }
        std::printf("newton steps %d: max rel err %.3e, max %.2f ulp, correctly rounded %.4f\n", k,
                    maxrel, maxulp, exact / (double)n);
    }
    long long *cyc, hc[3];
    double *o;
    hipMalloc(&cyc, 3 * sizeof(long long));
    hipMalloc(&o, 64 * sizeof(double));
    for (int rep = 0; rep < 2; ++rep) {
        kchain<0><<<1, 64>>>(o, cyc, 2.0);
        kchain<1><<<1, 64>>>(o, cyc, 2.0);
        kchain<2><<<1, 64>>>(o, cyc, 2.0);
        hipDeviceSynchronize();
    }
    hipMemcpy(hc, cyc, sizeof(hc), hipMemcpyDeviceToHost);
    for (int k = 0; k < 3; ++k)
        std::printf("dependent link rsq + %d Newton + fma: %.1f s_memtime ticks per link\n", k,
                    hc[k] / 1024.0);
    return 0;
}
