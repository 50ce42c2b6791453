// Microbenchmark: per-step latency of the Cholesky pivot chain pieces on one
// wave (gfx950).  Each variant runs STEPS dependent steps; cycles from
// clock64 (s_memtime) around the loop, wall time from hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int STEPS = 24 * 64;

__device__ __forceinline__ double rdl(double v, int l) {
    const long long x = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double rsq2(double d) {
    double y = __builtin_amdgcn_rsq(d);
    const double h = 0.5 * d;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

template <int V>
__global__ void k(double *out, long long *cyc, double seed) {
    const int lane = threadIdx.x;
    double a = seed + lane * 1e-3, acc = 0.;
    long long t0 = clock64();
#pragma unroll 8
    for (int s = 0; s < STEPS; ++s) {
        if (V == 0) {  // full pivot step: readlane -> check -> rsq2 -> mul -> readlane -> fma
            double d = rdl(a, s & 31);
            if (!(d > 0.) || !isfinite(d)) d = 1.;
            const double rs = rsq2(d);
            const double l = a * rs;
            const double lj = rdl(l, (s + 1) & 31);
            a = fma(-l, lj * 1e-3, a) + 1.0;
        } else if (V == 1) {  // rsq2 chain only (uniform value)
            a = rsq2(a) + 1.0;
        } else if (V == 2) {  // v_rsq only
            a = __builtin_amdgcn_rsq(a) + 1.0;
        } else if (V == 3) {  // readlane round trip + fma
            a = fma(rdl(a, s & 31), 1e-3, 1.0);
        } else if (V == 4) {  // dependent fma chain
            a = fma(a, 0.999, 1e-3);
        } else if (V == 5) {  // sqrt (library) chain
            a = sqrt(a) + 1.0;
        }
    }
    long long t1 = clock64();
    out[lane] = a + acc;
    if (lane == 0) cyc[0] = t1 - t0;
}

template <int V>
void run(const char *name, double *dout, long long *dcyc) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    k<V><<<1, 64>>>(dout, dcyc, 2.0);  // warm
    hipEventRecord(e0);
    k<V><<<1, 64>>>(dout, dcyc, 2.0);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    long long c = 0;
    hipMemcpy(&c, dcyc, sizeof(c), hipMemcpyDeviceToHost);
    printf("%-34s %8.1f ns/step  %8.1f clk/step\n", name, ms * 1e6 / STEPS, (double)c / STEPS);
}

int main() {
    double *dout;
    long long *dcyc;
    hipMalloc(&dout, 64 * sizeof(double));
    hipMalloc(&dcyc, sizeof(long long));
    run<4>("fma chain", dout, dcyc);
    run<2>("v_rsq_f64 chain", dout, dcyc);
    run<1>("rsq + 2 Newton chain", dout, dcyc);
    run<3>("readlane + fma chain", dout, dcyc);
    run<5>("sqrt() chain", dout, dcyc);
    run<0>("full pivot step", dout, dcyc);
    return 0;
}
