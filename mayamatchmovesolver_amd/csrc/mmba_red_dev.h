// Device helpers shared by the kernel translation units: write-through /
// L1-bypassing scalar accesses and the fixed-tree row reduction of
// k_reduce_multi (every launch that reduces a partial row in its own extra
// workgroups uses this one, so the slots get the same bits whichever launch
// carries them).
#pragma once
#include <hip/hip_runtime.h>

#include "mmba_kernels.h"

namespace mmba {

typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void st_sc1(double *p, double v) {  // write-through store
    __hip_atomic_store((gu64_t *)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double *p) {  // L1-bypassing load
    return __longlong_as_double((long long)__hip_atomic_load(
        (gu64_t *)const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// One partial row reduced by one 256-thread workgroup: k_reduce_multi's
// arithmetic (thread t sums entries t, t + 256, ..., then the fixed tree).
template <bool SC1>
__device__ __forceinline__ double reduce_row_block(const double *partial, const RedRow &rw,
                                                   double *red) {
    const bool mx = rw.is_max != 0;
    double s = 0.;
    for (int i = threadIdx.x; i < rw.n; i += blockDim.x) {
        const double q = SC1 ? ld_sc1(&partial[rw.off + i]) : partial[rw.off + i];
        s = mx ? fmax(s, q) : s + q;
    }
    red[threadIdx.x] = s;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (threadIdx.x < w)
            red[threadIdx.x] = mx ? fmax(red[threadIdx.x], red[threadIdx.x + w])
                                  : red[threadIdx.x] + red[threadIdx.x + w];
        __syncthreads();
    }
    const double v = red[0];
    __syncthreads();
    return v;
}

}  // namespace mmba
