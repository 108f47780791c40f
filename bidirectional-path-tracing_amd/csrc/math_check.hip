// Diagnostic kernel for bdpt_debug_math (include/bdpt_amd.h): evaluates the
// device restatements of glibc's sinf / cosf / powf and the sincos pair the
// warps use, element-wise, so tests can compare them bit for bit against the
// host libm the reference links (std::sinf / cosf / powf, src/core/math.h).
#include <hip/hip_runtime.h>

#include "device_math.hpp"

namespace bdpt {
namespace dev {

__global__ __launch_bounds__(256) void math_check_kernel(int32_t fn, const float* __restrict__ x,
                                                         const float* __restrict__ y, float* __restrict__ out,
                                                         int64_t n) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n) return;
    const float a = x[i];
    float r;
    switch (fn) {
        case 0: r = glibc_sinf(a); break;
        case 1: r = glibc_cosf(a); break;
        case 2: r = glibc_powf(a, y[i]); break;
        case 3: r = glibc_sincosf2(a).s; break;
        default: r = glibc_sincosf2(a).c; break;
    }
    out[i] = r;
}

}  // namespace dev

hipError_t launch_math_check(int32_t fn, const float* x, const float* y, float* out, int64_t n, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
    hipLaunchKernelGGL(dev::math_check_kernel, dim3(blocks), dim3(256), 0, st, fn, x, y, out, n);
    return hipGetLastError();
}

}  // namespace bdpt
