/* TEST INFRASTRUCTURE (oracle) — see tr_mathf.h for provenance.
 * Restatement of glibc 2.35's sinf/cosf/powf (x86_64 fma multiarch variant).
 * Tables: glibc __sincosf_table, __inv_pio4, __powf_log2_data, __exp2f_data
 * (published constants of the ARM optimized-routines implementation). */
#include "tr_mathf.h"

#include <math.h>
#include <string.h>

static inline uint32_t asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint64_t asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
static inline double asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

/* ---------------------------------------------------------------- sin/cos */
/* sincos_t as laid out in glibc 2.35: sign[4], hpi_inv, hpi, c0, c1, s1, c2,
 * s2, c3, s3, c4 (sincosf.h, s_sincosf_data.c). Index 1 negates the cosine
 * polynomial (used for quadrants with n & 2). */
typedef struct {
    double sign[4];
    double hpi_inv, hpi;
    double c0, c1, s1, c2, s2, c3, s3, c4;
} sincos_t;

static const sincos_t SINCOSF_TABLE[2] = {
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     0x1p+0, -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, 0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16},
    {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
     -0x1p+0, 0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3, -0x1.55553e1068f19p-5,
     0x1.1107605230bc4p-7, 0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, -0x1.99343027bf8c3p-16},
};

/* 4/pi bits (glibc __inv_pio4). */
static const uint32_t INV_PIO4[24] = {
    0xa2,       0xa2f9,     0xa2f983,   0xa2f9836e, 0xf9836e4e, 0x836e4e44, 0x6e4e4415, 0x4e441529,
    0x441529fc, 0x1529fc27, 0x29fc2757, 0xfc2757d1, 0x2757d1f5, 0x57d1f534, 0xd1f534dd, 0xf534ddc0,
    0x34ddc0db, 0xddc0db62, 0xc0db6295, 0xdb629599, 0x6295993c, 0x95993c43, 0x993c4390, 0x3c439041,
};
static const double PI63 = 0x1.921fb54442d18p-62;

static inline uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

/* sincosf.h sinf_poly: even n -> sine polynomial, odd n -> cosine polynomial. */
static inline float sinf_poly(double x, double x2, const sincos_t* p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma(x2, p->s3, p->s2);
        double x7 = x3 * x2;
        double s = fma(x3, p->s1, x);
        return (float)fma(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = fma(x2, p->c4, p->c3);
        double c1 = fma(x2, p->c1, p->c0);
        double x6 = x4 * x2;
        double c = fma(x4, p->c2, c1);
        return (float)fma(x6, c2, c);
    }
}

/* sincosf.h reduce_fast, !TOINT_INTRINSICS form. */
static inline double reduce_fast(double x, const sincos_t* p, int* np) {
    double r = x * p->hpi_inv;
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, p->hpi, x);
}

/* sincosf.h reduce_large (|x| >= 120). */
static inline double reduce_large(uint32_t xi, int* np) {
    const uint32_t* arr = &INV_PIO4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = (uint32_t)(xi * arr[0]);
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * PI63;
}

float tr_sinf(float y) {
    double x = y;
    const sincos_t* p = &SINCOSF_TABLE[0];
    int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double s = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return y;
        return sinf_poly(x, s, p, 0);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, p, &n);
        double s = p->sign[n & 3];
        if (n & 2) p = &SINCOSF_TABLE[1];
        return sinf_poly(x * s, x * x, p, n);
    } else if (abstop12(y) < abstop12(INFINITY)) {
        uint32_t xi = asuint(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        double s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &SINCOSF_TABLE[1];
        return sinf_poly(x * s, x * x, p, n);
    }
    return (y - y) / (y - y); /* __math_invalidf */
}

float tr_cosf(float y) {
    double x = y;
    const sincos_t* p = &SINCOSF_TABLE[0];
    int n;
    if (abstop12(y) < abstop12(0x1.921FB6p-1f)) {
        double x2 = x * x;
        if (abstop12(y) < abstop12(0x1p-12f)) return 1.0f;
        return sinf_poly(x, x2, p, 1);
    } else if (abstop12(y) < abstop12(120.0f)) {
        x = reduce_fast(x, p, &n);
        double s = p->sign[n & 3];
        if (n & 2) p = &SINCOSF_TABLE[1];
        return sinf_poly(x * s, x * x, p, n ^ 1);
    } else if (abstop12(y) < abstop12(INFINITY)) {
        uint32_t xi = asuint(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        double s = p->sign[(n + sign) & 3];
        if ((n + sign) & 2) p = &SINCOSF_TABLE[1];
        return sinf_poly(x * s, x * x, p, n ^ 1);
    }
    return (y - y) / (y - y);
}

/* ------------------------------------------------------------------ powf */
/* __powf_log2_data: 16 x {invc, logc}, poly[5] (POWF_SCALE_BITS = 0). */
static const double POWF_LOG2_TAB[16][2] = {
    {0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2}, {0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2},
    {0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2}, {0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2},
    {0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2}, {0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3}, {0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4},
    {0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4},  {0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3},
    {0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2},
    {0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2},  {0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2},
};
static const double POWF_LOG2_POLY[5] = {
    0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2, 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1, 0x1.71547652ab82bp+0,
};
/* __exp2f_data: tab[32], shift_scaled, poly_scaled[3] (EXP2F_TABLE_BITS = 5). */
static const uint64_t EXP2F_TAB[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51, 0x3fef72b83c7d517b,
    0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1, 0x3fef06fe0a31b715, 0x3feef1a7373aa9cb,
    0x3feedea64c123422, 0x3feece086061892d, 0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429,
    0x3feea47eb03a5585, 0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d, 0x3feee89f995ad3ad,
    0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069, 0x3fef5818dcfba487, 0x3fef7c97337b9b5f,
    0x3fefa4afa2a490da, 0x3fefd0765b6e4540,
};
static const double EXP2F_SHIFT = 0x1.8p+47;
static const double EXP2F_POLY[3] = {0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3, 0x1.62e42ff0c52d6p-1};
#define POWF_SIGN_BIAS (1u << 16)

static inline double log2_inline(uint32_t ix) {
    uint32_t tmp = ix - 0x3f330000;
    int i = (int)((tmp >> 19) % 16);
    uint32_t top = tmp & 0xff800000;
    uint32_t iz = ix - top;
    int k = (int32_t)top >> 23;
    double invc = POWF_LOG2_TAB[i][0];
    double logc = POWF_LOG2_TAB[i][1];
    double z = (double)asfloat(iz);
    double r = fma(z, invc, -1.0);
    double y0 = logc + (double)k;
    double r2 = r * r;
    double y = fma(POWF_LOG2_POLY[0], r, POWF_LOG2_POLY[1]);
    double p = fma(POWF_LOG2_POLY[2], r, POWF_LOG2_POLY[3]);
    double r4 = r2 * r2;
    double q = fma(POWF_LOG2_POLY[4], r, y0);
    q = fma(p, r2, q);
    y = fma(y, r4, q);
    return y;
}

static inline float exp2_inline(double xd, uint32_t sign_bias) {
    double kd = xd + EXP2F_SHIFT;
    uint64_t ki = asuint64(kd);
    kd -= EXP2F_SHIFT;
    double r = xd - kd;
    uint64_t t = EXP2F_TAB[ki % 32];
    uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    double s = asdouble(t);
    double z = fma(EXP2F_POLY[0], r, EXP2F_POLY[1]);
    double r2 = r * r;
    double y = fma(EXP2F_POLY[2], r, 1.0);
    y = fma(z, r2, y);
    y = y * s;
    return (float)y;
}

static inline int checkint(uint32_t iy) {
    int e = iy >> 23 & 0xff;
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}
static inline int zeroinfnan(uint32_t ix) { return 2 * ix - 1 >= 2u * 0x7f800000 - 1; }
static inline int issignalingf(float x) { return 2 * (asuint(x) ^ 0x00400000) > 2u * 0x7fc00000; }
static float xflowf(uint32_t sign, float y) {
    volatile float a = sign ? -y : y;
    return a * y;
}

float tr_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = asuint(x), iy = asuint(y);
    if (ix - 0x00800000 >= 0x7f800000 - 0x00800000 || zeroinfnan(iy)) {
        if (zeroinfnan(iy)) {
            if (2 * iy == 0) return issignalingf(x) ? x + y : 1.0f;
            if (ix == 0x3f800000) return issignalingf(y) ? x + y : 1.0f;
            if (2 * ix > 2u * 0x7f800000 || 2 * iy > 2u * 0x7f800000) return x + y;
            if (2 * ix == 2 * 0x3f800000) return 1.0f;
            if ((2 * ix < 2 * 0x3f800000) == !(iy & 0x80000000)) return 0.0f;
            return y * y;
        }
        if (zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000) && checkint(iy) == 1) {
                x2 = -x2;
                sign_bias = 1;
            }
            if (2 * ix == 0 && (iy & 0x80000000)) return xflowf(sign_bias, 1.0f) / 0.0f; /* __math_divzerof */
            return (iy & 0x80000000) ? 1 / x2 : x2;
        }
        if (ix & 0x80000000) {
            int yint = checkint(iy);
            if (yint == 0) return (x - x) / (x - x); /* __math_invalidf */
            if (yint == 1) sign_bias = POWF_SIGN_BIAS;
            ix &= 0x7fffffff;
        }
        if (ix < 0x00800000) {
            ix = asuint(x * 0x1p23f);
            ix &= 0x7fffffff;
            ix -= 23 << 23;
        }
    }
    double logx = log2_inline(ix);
    double ylogx = (double)y * logx;
    if (((asuint64(ylogx) >> 47) & 0xffff) >= (asuint64(126.0) >> 47)) {
        if (ylogx > 0x1.fffffffd1d571p+6) return xflowf(sign_bias, 0x1p97f);   /* __math_oflowf */
        if (ylogx <= -150.0) return xflowf(sign_bias, 0x1p-95f);             /* __math_uflowf */
        if (ylogx < -149.0) return xflowf(sign_bias, 0x1.4p-75f);            /* __math_may_uflowf */
    }
    return exp2_inline(ylogx, sign_bias);
}

float tr_fmaxf(float x, float y) {
    if (x != x) return y;
    if (y != y) return x;
    return x > y ? x : y;
}

float tr_fminf(float x, float y) {
    if (x != x) return y;
    if (y != y) return x;
    return x < y ? x : y;
}
