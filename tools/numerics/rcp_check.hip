// Exhaustive check of the short reciprocal sequence (v_rcp_f32 + one FMA Newton
// step) against the correctly rounded 1.0f / x over all 2^32 float inputs, and
// a randomized check of the division built on it. Prints mismatch counts per
// input exponent band. Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ __forceinline__ float rcp_nr(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float div_nr(float a, float b) {
    const float r = rcp_nr(b);
    const float q = a * r;
    const float rem = __builtin_fmaf(-b, q, a);
    return __builtin_fmaf(rem, r, q);
}

__global__ void rcp_all(uint32_t hi, unsigned long long* bad) {  // hi = top 16 bits of the input
    const uint32_t i = (hi << 16) | (blockIdx.x * blockDim.x + threadIdx.x);
    const float x = __uint_as_float(i);
    const float ref = 1.0f / x, got = rcp_nr(x);
    const bool same = (__float_as_uint(ref) == __float_as_uint(got)) || (ref != ref && got != got);
    if (!same) atomicAdd(bad + ((i >> 23) & 0xff), 1ull);
}

__device__ __forceinline__ uint32_t hash(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
// a, b with exponents in [-40, 40] (b) and [-60, 60] (a): the path's range
__global__ void div_rand(uint32_t seed, unsigned long long* bad, float* ex) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t h1 = hash(t * 2 + seed * 0x9e3779b9u), h2 = hash(t * 2 + 1 + seed * 0x85ebca6bu);
    const uint32_t eb = 127 - 40 + (h1 >> 24) % 81, ea = 127 - 60 + (h2 >> 24) % 121;
    const float b = __uint_as_float((h1 & 0x807fffffu) | (eb << 23));
    const float a = __uint_as_float((h2 & 0x807fffffu) | (ea << 23));
    const float ref = a / b, got = div_nr(a, b);
    if (__float_as_uint(ref) != __float_as_uint(got)) {
        const unsigned long long k = atomicAdd(bad, 1ull);
        if (k < 4) ex[2 * k] = a, ex[2 * k + 1] = b;
    }
}

int main() {
    unsigned long long* bad;
    float* ex;
    hipMalloc(&bad, 257 * 8);
    hipMalloc(&ex, 64);
    hipMemset(bad, 0, 257 * 8);
    for (uint32_t hi = 0; hi < 65536; hi++) rcp_all<<<256, 256>>>(hi, bad);
    unsigned long long h[257];
    hipMemcpy(h, bad, 257 * 8, hipMemcpyDeviceToHost);
    unsigned long long tot = 0, mid = 0;
    for (int e = 0; e < 256; e++) {
        tot += h[e];
        if (e >= 2 && e <= 252) mid += h[e];
        if (h[e]) printf("rcp exponent field %3d: %llu mismatches\n", e, h[e]);
    }
    printf("rcp: %llu mismatches over 2^32 inputs, %llu with exponent field in [2, 252]\n", tot, mid);
    hipMemset(bad, 0, 8);
    for (uint32_t s = 0; s < 256; s++) div_rand<<<65536, 256>>>(s, bad, ex);
    hipMemcpy(h, bad, 8, hipMemcpyDeviceToHost);
    float e4[8];
    hipMemcpy(e4, ex, 32, hipMemcpyDeviceToHost);
    printf("div: %llu mismatches over 2^32 random pairs\n", h[0]);
    for (int k = 0; k < 4 && k < (int)h[0]; k++) printf("  e.g. %a / %a\n", e4[2 * k], e4[2 * k + 1]);
    return 0;
}
