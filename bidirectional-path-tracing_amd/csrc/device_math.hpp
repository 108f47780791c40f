// Device math for the BDPT kernels, bit-faithful to the reference's x86 build.
//
// Every float operation here must round exactly like the reference's g++ -O2
// SSE2 code: the kernels are compiled with -ffp-contract=off (no a*b+c fusion)
// and HIP's default correctly-rounded f32 division and square root. glm's
// operation order is mirrored explicitly (externals/glm/glm/detail/
// func_geometric.inl: dot = (x*x' + y*y') + z*z', normalize = v * (1/sqrt(dot)),
// cross as written at :74-83).
//
// The transcendental functions reproduce glibc 2.35's x86_64 FMA-multiarch
// sinf / cosf / powf (the ARM optimized-routines algorithms: double-precision
// polynomials on a 16/32-entry table), which is what the reference's
// std::sinf / std::cosf / std::powf calls (src/core/math.h:125-242,
// src/bsdfs/mixture.h:70) resolve to on an FMA+AVX2 host. CDNA4 has full-rate
// enough FP64 FMA for this to cost a few dozen cycles per call.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bdpt {
namespace dev {

// Large, rarely-divergent helpers are real calls: one copy of their code in the
// megakernel instead of one per call site (i-cache and register pressure).
#define BDPT_NOINLINE __attribute__((noinline))

// Relaxed agent-scope atomic adds on pointers named global (global_atomic_*):
// HIP's atomicAdd on a generic pointer the compiler cannot place becomes a FLAT
// atomic, which also makes the wave's next waits cover LDS (lgkmcnt) too.
typedef __attribute__((address_space(1))) float gfloat_t;
typedef __attribute__((address_space(1))) uint32_t gu32_t;
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
__device__ __forceinline__ void gadd(float* p, float v) {
    __hip_atomic_fetch_add((gfloat_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t gadd(uint32_t* p, uint32_t v) {
    return __hip_atomic_fetch_add((gu32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long gadd(unsigned long long* p, unsigned long long v) {
    return __hip_atomic_fetch_add((gu64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gmax(unsigned long long* p, unsigned long long v) {
    __hip_atomic_fetch_max((gu64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void gmin(unsigned long long* p, unsigned long long v) {
    __hip_atomic_fetch_min((gu64_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------- float3
struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float div_cr(float a, float b);
__device__ __forceinline__ float rcp_cr(float x);
__device__ __forceinline__ f3 operator/(f3 a, float s) { return mk(div_cr(a.x, s), div_cr(a.y, s), div_cr(a.z, s)); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
__device__ __forceinline__ float sqrt_cr(float x) { return __builtin_sqrtf(x); }

// Correctly rounded reciprocal and division in a few instructions instead of
// the ~10 of the IEEE division sequence. rcp: v_rcp_f32 (1 ulp) plus one FMA
// Newton step, equal to 1.0f / x for every x with 2^-126 <= |x| < 2^126
// (checked on the GPU over all 2^32 inputs, tools/numerics/rcp_check.hip).
// div: q = a * rcp(b) corrected by one FMA residual step (Markstein), equal to
// a / b when the reciprocal is correctly rounded and nothing over/underflows;
// the guard keeps |a| in [2^-60, 2^60] and |b| in [2^-40, 2^40] (0 mismatches
// over 2^32 random pairs there). Anything else takes the IEEE division, so both
// return exactly what `/` returns.
__device__ __forceinline__ float rcp_nr(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
}
#ifndef BDPT_FAST_DIV
#define BDPT_FAST_DIV 0  // 1: rcp_cr / div_cr take the short sequences (measured: no gain in the shading code)
#endif
__device__ __forceinline__ float rcp_cr(float x) {
    if (!BDPT_FAST_DIV) return 1.0f / x;
    const float ax = __builtin_fabsf(x);
    if (__builtin_expect(ax >= 0x1p-126f && ax < 0x1p126f, 1)) return rcp_nr(x);
    return 1.0f / x;
}
// The triangle test's 1 / det: |det| >= 1e-8 is known, so only the upper bound is checked.
#ifndef BDPT_FAST_TRI_RCP
#define BDPT_FAST_TRI_RCP 1
#endif
__device__ __forceinline__ float rcp_det(float det) {
    if (!BDPT_FAST_TRI_RCP) return 1.0f / det;
    if (__builtin_expect(__builtin_fabsf(det) < 0x1p126f, 1)) return rcp_nr(det);
    return 1.0f / det;
}
__device__ __forceinline__ float div_cr(float a, float b) {
    if (!BDPT_FAST_DIV) return a / b;
    const float aa = __builtin_fabsf(a), ab = __builtin_fabsf(b);
    if (__builtin_expect(aa >= 0x1p-60f && aa <= 0x1p60f && ab >= 0x1p-40f && ab <= 0x1p40f, 1)) {
        const float r = rcp_nr(b);
        const float q = a * r;
        return __builtin_fmaf(__builtin_fmaf(-b, q, a), r, q);
    }
    return a / b;
}
__device__ __forceinline__ f3 normalize(f3 v) { return v * rcp_cr(sqrt_cr(dot(v, v))); }

// Arithmetic that only WEIGHTS a path — the MIS recursion (vc, vcm), pdf ratios,
// throughput and contributions — and never steers it (no direction, hit, pixel or
// random-number decision depends on it; a cosine sign computed from a direction
// normalized this way flips only where the connection's contribution is 0). With
// BDPT_FAST_WEIGHTS these take the hardware's 1-ulp v_rcp_f32 / v_sqrt_f32 /
// v_rsq_f32 instead of the correctly rounded ~11-instruction sequences: every
// sample still follows the reference's path bit for bit, its contributions differ
// by a few ulp (per-pixel ~1e-6 relative, against the 1e-4 bound). The frame
// kernels without Russian roulette build with it (bdpt_kernels.hip); the Russian-
// roulette build (whose throughput steers the roulette) and the single-sample and
// per-function kernels keep the IEEE operations.
#ifndef BDPT_FAST_WEIGHTS
#define BDPT_FAST_WEIGHTS 0
#endif
__device__ __forceinline__ float rcp_w(float x) { return BDPT_FAST_WEIGHTS ? __builtin_amdgcn_rcpf(x) : rcp_cr(x); }
__device__ __forceinline__ float div_w(float a, float b) { return BDPT_FAST_WEIGHTS ? a * __builtin_amdgcn_rcpf(b) : div_cr(a, b); }
__device__ __forceinline__ float sqrt_w(float x) { return BDPT_FAST_WEIGHTS ? __builtin_amdgcn_sqrtf(x) : sqrt_cr(x); }
__device__ __forceinline__ float rsqrt_w(float x) { return BDPT_FAST_WEIGHTS ? __builtin_amdgcn_rsqf(x) : rcp_cr(sqrt_cr(x)); }
__device__ __forceinline__ bool is_zero(f3 v) { return v.x == 0.f && v.y == 0.f && v.z == 0.f; }
__device__ __forceinline__ f3 xyz(float4 q) { return mk(q.x, q.y, q.z); }

// glibc 2.35 x86_64 fmaxf / fminf (maxss / minss): the second operand wins ties.
__device__ __forceinline__ float glibc_fmaxf(float x, float y) {
    if (x != x) return y;
    if (y != y) return x;
    return x > y ? x : y;
}
__device__ __forceinline__ float glibc_fminf(float x, float y) {
    if (x != x) return y;
    if (y != y) return x;
    return x < y ? x : y;
}

// static_cast<int>(float) as x86 cvttss2si: NaN / out of range -> INT_MIN.
__device__ __forceinline__ int x86_trunc_i32(float f) {
    if (!(f > -2147483648.f && f < 2147483648.f)) return INT32_MIN;
    return static_cast<int>(f);
}

// ------------------------------------------------------------- sin / cos
// glibc __inv_pio4: bits of 4/pi.
static __constant__ uint32_t kInvPio4[24] = {0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44,
                               0x6e4e4415, 0x4e441529, 0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1,
                               0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0, 0x34ddc0db, 0xddc0db62,
                               0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041};

// glibc __powf_log2_data (POWF_LOG2_TABLE_BITS = 4): {invc, logc}
static __constant__ double kPowfLog2Tab[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2}};

// glibc __exp2f_data (EXP2F_TABLE_BITS = 5).
static __constant__ uint64_t kExp2fTab[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51, 0x3fef72b83c7d517b,
    0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1, 0x3fef06fe0a31b715, 0x3feef1a7373aa9cb,
    0x3feedea64c123422, 0x3feece086061892d, 0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429,
    0x3feea47eb03a5585, 0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d, 0x3feee89f995ad3ad,
    0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069, 0x3fef5818dcfba487, 0x3fef7c97337b9b5f,
    0x3fefa4afa2a490da, 0x3fefd0765b6e4540};

__device__ __forceinline__ uint32_t f2u(float f) { return __float_as_uint(f); }
__device__ __forceinline__ uint32_t abstop12(float x) { return (f2u(x) >> 20) & 0x7ff; }

// glibc sincosf.h tables, in its field order {c0, c1, s1, c2, s2, c3, s3, c4}.
struct SinCosPoly {
    double c0, c1, s1, c2, s2, c3, s3, c4;
};
__device__ __forceinline__ SinCosPoly sincos_poly_table(bool negate_cos) {
    const double c0 = 0x1p+0, c1 = -0x1.ffffffd0c621cp-2, c2 = 0x1.55553e1068f19p-5, c3 = -0x1.6c087e89a359dp-10,
                 c4 = 0x1.99343027bf8c3p-16;
    const double s1 = -0x1.555545995a603p-3, s2 = 0x1.1107605230bc4p-7, s3 = -0x1.994eb3774cf24p-13;
    if (negate_cos) return SinCosPoly{-c0, -c1, s1, -c2, s2, -c3, s3, -c4};
    return SinCosPoly{c0, c1, s1, c2, s2, c3, s3, c4};
}

// sinf_poly: even n -> sine polynomial of x, odd n -> cosine polynomial.
__device__ __forceinline__ float sincos_poly(double x, double x2, const SinCosPoly& p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = __builtin_fma(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = __builtin_fma(x3, p.s1, x);
        return static_cast<float>(__builtin_fma(x7, s1, s));
    }
    double x4 = x2 * x2;
    double c2 = __builtin_fma(x2, p.c4, p.c3);
    double c1 = __builtin_fma(x2, p.c1, p.c0);
    double x6 = x4 * x2;
    double c = __builtin_fma(x4, p.c2, c1);
    return static_cast<float>(__builtin_fma(x6, c2, c));
}

// reduce_large for |x| >= 120 (4/pi bit table, 2^-62 pi scale).
__device__ __noinline__ double sincos_reduce_large(uint32_t xi, int* np) {
    const uint32_t* arr = &kInvPio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    uint64_t res0 = static_cast<uint32_t>(xi * arr[0]);
    uint64_t res1 = static_cast<uint64_t>(xi) * arr[4];
    uint64_t res2 = static_cast<uint64_t>(xi) * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    uint64_t n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    *np = static_cast<int>(n);
    return static_cast<double>(static_cast<int64_t>(res0)) * 0x1.921fb54442d18p-62;
}

// which = 0: sinf, 1: cosf
__device__ BDPT_NOINLINE float glibc_sincosf(float y, int which) {
    double x = y;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return which ? 1.0f : y;
        return sincos_poly(x, x2, sincos_poly_table(false), which);
    }
    int n;
    double s;
    bool neg;
    if (abstop12(y) < abstop12(120.0f)) {
        double r = x * 0x1.45f306dc9c883p+23;
        n = (static_cast<int32_t>(r) + 0x800000) >> 24;
        x = __builtin_fma(-static_cast<double>(n), 0x1.921fb54442d18p+0, x);
        s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
        neg = (n & 2) != 0;
    } else if (abstop12(y) < abstop12(__builtin_inff())) {
        uint32_t xi = f2u(y);
        int sign = xi >> 31;
        x = sincos_reduce_large(xi, &n);
        int q = n + sign;
        s = ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0;
        neg = (q & 2) != 0;
    } else {
        return (y - y) / (y - y);
    }
    return sincos_poly(x * s, x * x, sincos_poly_table(neg), which ? (n ^ 1) : n);
}

struct SinCos {
    float s, c;
};
#ifndef BDPT_SINCOS_ATTR
#define BDPT_SINCOS_ATTR __forceinline__  // branch-free below 120: inline costs fewer registers than a call
#endif
// |y| >= 120, inf, NaN: reduce_large (never reached by the warps' angles).
__device__ __noinline__ SinCos glibc_sincosf2_large(float y) {
    if (abstop12(y) >= abstop12(__builtin_inff())) {
        const float nan = (y - y) / (y - y);
        return SinCos{nan, nan};
    }
    int n;
    const uint32_t xi = f2u(y);
    const int sign = xi >> 31;
    const double x = sincos_reduce_large(xi, &n);
    const int q = n + sign;
    const double s = ((q & 3) == 1 || (q & 3) == 2) ? -1.0 : 1.0;
    const SinCosPoly p = sincos_poly_table((q & 2) != 0);
    return SinCos{sincos_poly(x * s, x * x, p, n), sincos_poly(x * s, x * x, p, n ^ 1)};
}
// sinf(y) and cosf(y) from one range reduction, each bit-identical to the
// single calls above, without divergent branches for |y| < 120 (every angle the
// warps produce): glibc's reduce_fast path, with both polynomials evaluated once
// and assigned by the quadrant's parity. It also covers glibc's two small-
// argument paths: for |y| < pi/4 the reduction gives n = 0 and x = y exactly
// (the same polynomial call), and for |y| < 2^-12 both polynomials round to
// glibc's (y, 1.0f) (the terms past x / 1 are below half an ulp; only the sign
// of a zero sine needs the explicit select). A negated
// cosine table negates the polynomial's value exactly (fma is sign-symmetric
// under round-to-nearest), so the quadrant's sign is applied to the float.
// tools/numerics/sincos_check.hip compares it with the branchy form over every
// float with |y| < 120.
__device__ BDPT_SINCOS_ATTR SinCos glibc_sincosf2(float y) {
    if (abstop12(y) >= abstop12(120.0f)) return glibc_sincosf2_large(y);
    double x = y;
    const double r = x * 0x1.45f306dc9c883p+23;
    const int n = (static_cast<int32_t>(r) + 0x800000) >> 24;
    x = __builtin_fma(-static_cast<double>(n), 0x1.921fb54442d18p+0, x);
    const double xs = ((n & 3) == 1 || (n & 3) == 2) ? -x : x;
    const double x2 = x * x;
    const SinCosPoly p = sincos_poly_table(false);
    float sp = sincos_poly(xs, x2, p, 0);  // sine polynomial
    sp = (y == 0.f) ? y : sp;              // sinf(-0) = -0 (glibc's tiny-argument path)
    float cp = sincos_poly(xs, x2, p, 1);        // cosine polynomial
    cp = (n & 2) ? -cp : cp;
    return (n & 1) ? SinCos{cp, sp} : SinCos{sp, cp};
}

__device__ __forceinline__ float glibc_sinf(float x) { return glibc_sincosf(x, 0); }
__device__ __forceinline__ float glibc_cosf(float x) { return glibc_sincosf(x, 1); }

// ------------------------------------------------------------------ powf
__device__ __forceinline__ double d_from_u(uint64_t u) { return __longlong_as_double(static_cast<long long>(u)); }
__device__ __forceinline__ uint64_t u_from_d(double d) { return static_cast<uint64_t>(__double_as_longlong(d)); }

__device__ __forceinline__ double powf_log2(uint32_t ix) {
    const double A0 = 0x1.27616c9496e0bp-2, A1 = -0x1.71969a075c67ap-2, A2 = 0x1.ec70a6ca7baddp-2,
                 A3 = -0x1.7154748bef6c8p-1, A4 = 0x1.71547652ab82bp+0;
    uint32_t tmp = ix - 0x3f330000;
    int i = static_cast<int>((tmp >> 19) % 16);
    uint32_t top = tmp & 0xff800000;
    uint32_t iz = ix - top;
    int k = static_cast<int32_t>(top) >> 23;
    double z = static_cast<double>(__uint_as_float(iz));
    double r = __builtin_fma(z, kPowfLog2Tab[i][0], -1.0);
    double y0 = kPowfLog2Tab[i][1] + static_cast<double>(k);
    double r2 = r * r;
    double y = __builtin_fma(A0, r, A1);
    double p = __builtin_fma(A2, r, A3);
    double r4 = r2 * r2;
    double q = __builtin_fma(A4, r, y0);
    q = __builtin_fma(p, r2, q);
    return __builtin_fma(y, r4, q);
}

__device__ __forceinline__ float powf_exp2(double xd, uint32_t sign_bias) {
    // !TOINT_INTRINSICS path of glibc exp2_inline.
    const double shift = 0x1.8p+47;
    double kd = xd + shift;
    uint64_t ki = u_from_d(kd);
    kd -= shift;
    double r = xd - kd;
    uint64_t t = kExp2fTab[ki % 32];
    t += (ki + sign_bias) << 47;
    double s = d_from_u(t);
    double z = __builtin_fma(0x1.c6af84b912394p-5, r, 0x1.ebfce50fac4f3p-3);
    double r2 = r * r;
    double y = __builtin_fma(0x1.62e42ff0c52d6p-1, r, 1.0);
    y = __builtin_fma(z, r2, y);
    return static_cast<float>(y * s);
}

__device__ __forceinline__ int powf_checkint(uint32_t iy) {
    int e = iy >> 23 & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
__device__ __forceinline__ bool powf_zeroinfnan(uint32_t i) { return 2 * i - 1 >= 2u * 0x7f800000 - 1; }
__device__ __forceinline__ float powf_xflow(uint32_t sign, float y) { return (sign ? -y : y) * y; }

__device__ __noinline__ float powf_special(float x, float y, uint32_t ix, uint32_t iy, bool* done, uint32_t* ix_out,
                                          uint32_t* sign_bias) {
    *done = true;
    if (powf_zeroinfnan(iy)) {
        if (2 * iy == 0) return 1.0f;  // (signalling-NaN x is not produced by the BDPT path)
        if (ix == 0x3f800000) return 1.0f;
        if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
        if (2 * ix == 2 * 0x3f800000) return 1.0f;
        if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
        return y * y;
    }
    if (powf_zeroinfnan(ix)) {
        float x2 = x * x;
        uint32_t sb = 0;
        if ((ix & 0x80000000) && powf_checkint(iy) == 1) {
            x2 = -x2;
            sb = 1;
        }
        if (2 * ix == 0 && (iy & 0x80000000)) return powf_xflow(sb, 1.0f) / 0.0f;
        return (iy & 0x80000000) ? 1 / x2 : x2;
    }
    *done = false;
    if (ix & 0x80000000) {
        int yint = powf_checkint(iy);
        if (yint == 0) {
            *done = true;
            return (x - x) / (x - x);
        }
        if (yint == 1) *sign_bias = 1u << 16;
        ix &= 0x7fffffff;
    }
    if (ix < 0x00800000) {
        ix = f2u(x * 0x1p23f);
        ix &= 0x7fffffff;
        ix -= 23 << 23;
    }
    *ix_out = ix;
    return 0.f;
}

#ifndef BDPT_POWF_ATTR
#define BDPT_POWF_ATTR BDPT_NOINLINE
#endif
__device__ BDPT_POWF_ATTR float glibc_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = f2u(x), iy = f2u(y);
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || powf_zeroinfnan(iy)) {
        bool done;
        float r = powf_special(x, y, ix, iy, &done, &ix, &sign_bias);
        if (done) return r;
    }
    double ylogx = static_cast<double>(y) * powf_log2(ix);
    if (((u_from_d(ylogx) >> 47) & 0xffff) >= (u_from_d(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return powf_xflow(sign_bias, 0x1p97f);
        if (ylogx <= -150.0) return powf_xflow(sign_bias, 0x1p-95f);
        if (ylogx < -149.0) return powf_xflow(sign_bias, 0x1.4p-75f);
    }
    return powf_exp2(ylogx, sign_bias);
}

// x^y for a Phong lobe's value or pdf (weights only, see rcp_w): with
// BDPT_FAST_WEIGHTS exp2(y * log2(x)) on the hardware's v_log_f32 / v_exp_f32,
// else glibc's powf. The callers pass x in [0, 1] (or just above 1 by rounding)
// and y = the exponent >= 0; the relative error y * |log2 x| * ~2^-22 is largest
// where x^y is tiny. y == 0 gives 1 as powf does (also for x == 0).
#ifndef BDPT_FAST_POW
#define BDPT_FAST_POW BDPT_FAST_WEIGHTS
#endif
__device__ __forceinline__ float pow_w(float x, float y) {
#if BDPT_FAST_POW
    return y == 0.f ? 1.f : __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#else
    return glibc_powf(x, y);
#endif
}

}  // namespace dev
}  // namespace bdpt
