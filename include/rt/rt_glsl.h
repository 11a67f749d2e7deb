/*
 * rt_glsl.h — the GLSL 4.30 built-in functions the reference shader relies on,
 * defined once, deterministically, for both sides of the parity check.
 *
 * In the reference the built-ins (sin, cos, log, acos, atan, pow, sqrt,
 * normalize, reflect, refract, mix, fract, mod, dot, cross, texture2D ...) are
 * implemented by the GPU vendor's GLSL compiler (SURVEY §8c "Third-party
 * arithmetic"), so their bits are unpinned.  This header *is* our definition of
 * them.  Every function uses only IEEE-754 binary32 +,-,*,/, sqrt, fma, floor,
 * rint and exact integer/bit operations, so the same source compiled by g++
 * (oracle, x86-64 SSE) and by hipcc (gfx950 kernel) produces identical bits as
 * long as both are built with -ffp-contract=off and without fast-math
 * (correctly-rounded f32 div/sqrt is hipcc's default).  tests/test_oracle.py
 * pins each transcendental against libm in double precision (ulp bounds).
 *
 * Shared by: oracle/rt_oracle.cpp (CPU restatement, test infrastructure) and
 * raytracing-book_amd/csrc/rt_kernel.hip (the product).  Nothing above the
 * built-in level (traversal, shading, sampling) lives here.
 */
#ifndef RT_GLSL_H
#define RT_GLSL_H

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#include <string.h>
#define RT_HD static inline
#endif

/* compute.glsl:7 — "INFINITY" is FLT_MAX-ish, not IEEE inf. */
#define RT_INFINITY 3.402823E+38f
/* math.glsl:1 — const float PI = 3.14159265359 (rounds to 0x40490fdb). */
#define RT_PI 3.14159265359f

/* ---------------------------------------------------------------- bits */
RT_HD uint32_t rt_f2u(float f) {
#if defined(__HIPCC__)
    return __float_as_uint(f);
#else
    uint32_t u; memcpy(&u, &f, 4); return u;
#endif
}
RT_HD float rt_u2f(uint32_t u) {
#if defined(__HIPCC__)
    return __uint_as_float(u);
#else
    float f; memcpy(&f, &u, 4); return f;
#endif
}
RT_HD int rt_isnan(float x) { return x != x; }

/* float -> int with C truncation; NaN -> 0, saturating outside int range.
 * (GLSL leaves out-of-range conversion undefined; this is our definition.) */
RT_HD int rt_f2i(float x) {
    if (!(x == x)) return 0;
    if (x >= 2147483520.0f) return 2147483647;
    if (x <= -2147483648.0f) return (-2147483647 - 1);
    return (int)x;
}

/* GLSL 4.30 §8.3: min(x,y) = y < x ? y : x ; max(x,y) = x < y ? y : x */
RT_HD float g_min(float x, float y) { return (y < x) ? y : x; }
RT_HD float g_max(float x, float y) { return (x < y) ? y : x; }
RT_HD float g_fract(float x) { return x - floorf(x); }
/* GLSL mod(x,y) = x - y*floor(x/y) */
RT_HD float g_mod(float x, float y) { return x - y * floorf(x / y); }
/* GLSL normalize() applied to a scalar (pdf.glsl:33): x/|x| = sign, NaN at 0 */
RT_HD float g_normalize1(float x) { return x / fabsf(x); }

/* ---------------------------------------------------------------- vec */
struct v3 { float x, y, z; };
struct v2 { float x, y; };

RT_HD v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
RT_HD v3 mk3s(float s) { return mk3(s, s, s); }
RT_HD v3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }
RT_HD v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
RT_HD v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
RT_HD v3 mul3(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
RT_HD v3 div3(v3 a, v3 b) { return mk3(a.x / b.x, a.y / b.y, a.z / b.z); }
RT_HD v3 scale3(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }   /* a*s and s*a */
/* vec3 / float (hitting.glsl:40, compute.glsl:339): one IEEE reciprocal, then three products
 * (round 4 definition; GLSL leaves division to 2.5 ulp) */
RT_HD v3 divs3(v3 a, float s) { const float r = 1.0f / s; return mk3(a.x * r, a.y * r, a.z * r); }
RT_HD v3 neg3(v3 a) { return mk3(-a.x, -a.y, -a.z); }
RT_HD float comp3(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

/* dot: fused chain x, then y, then z (our definition of GLSL dot) */
RT_HD float g_dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
RT_HD float g_dot2(v2 a, v2 b) { return fmaf(a.y, b.y, a.x * b.x); }
RT_HD v3 g_cross(v3 a, v3 b) {
    return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
RT_HD float g_length(v3 a) { return sqrtf(g_dot(a, a)); }
/* GLSL inversesqrt (round 4; GLSL 4.60 §4.7.1 allows 2 ulp): the bit-level first guess
 * 0x5f375a86 - bits(x)/2 (relative error below 3.5e-2), then three Newton steps
 * y <- y + y*(1/2 - (x/2)*y*y), fused the same way on both sides (relative error 1.8e-3, 4.6e-6,
 * then below float rounding: within 2 ulp for normal x, test_oracle.py).  Special inputs as
 * 1/sqrt(x): +-0 -> +-inf, +inf -> +0, x < 0 and NaN -> NaN.  About a dozen operations where
 * the IEEE 1/sqrtf(x) takes two correctly rounded operations of ~13 each on gfx950. */
RT_HD float g_inversesqrt(float x) {
    /* a subnormal x is scaled by 2^24 first (exact) and the result by 2^12: the bit-level guess
     * is far off below FLT_MIN, where three Newton steps would not converge; normal
     * inputs take the same operations as before (scale 1) */
    const int sub = x < 1.17549435e-38f;
    const float xs = sub ? x * 16777216.0f : x;
    float y = rt_u2f(0x5f375a86u - (rt_f2u(xs) >> 1));
    const float h = 0.5f * xs;
    y = fmaf(y, fmaf(-h, y * y, 0.5f), y);
    y = fmaf(y, fmaf(-h, y * y, 0.5f), y);
    y = fmaf(y, fmaf(-h, y * y, 0.5f), y);
    y = y * (sub ? 4096.0f : 1.0f);
    if (x == 0.0f) y = rt_u2f(rt_f2u(x) | 0x7f800000u);   /* +-inf with x's sign */
    if (x == __builtin_inff()) y = 0.0f;
    if (!(x >= 0.0f)) y = __builtin_nanf("");              /* x < 0 or NaN (-0 passes: -inf above) */
    return y;
}
/* normalize(a) = a * inversesqrt(dot(a, a)) */
RT_HD v3 g_normalize(v3 a) { return scale3(a, g_inversesqrt(g_dot(a, a))); }
/* GLSL reflect(I,N) = I - 2*dot(N,I)*N */
RT_HD v3 g_reflect(v3 i, v3 n) { float d2 = 2.0f * g_dot(n, i); return sub3(i, scale3(n, d2)); }
/* GLSL refract(I,N,eta) */
RT_HD v3 g_refract(v3 i, v3 n, float eta) {
    float d = g_dot(n, i);
    float k = 1.0f - (eta * eta) * (1.0f - d * d);
    if (k < 0.0f) return mk3s(0.0f);
    float s = eta * d + sqrtf(k);
    return sub3(scale3(i, eta), scale3(n, s));
}
/* GLSL mix(x,y,a) = x*(1-a) + y*a */
RT_HD float g_mix(float x, float y, float a) { return x * (1.0f - a) + y * a; }
/* mat3(c0,c1,c2) * v */
RT_HD v3 g_mat3_mul(v3 c0, v3 c1, v3 c2, v3 v) {
    return mk3(fmaf(c2.x, v.z, fmaf(c1.x, v.y, c0.x * v.x)),
               fmaf(c2.y, v.z, fmaf(c1.y, v.y, c0.y * v.x)),
               fmaf(c2.z, v.z, fmaf(c1.z, v.y, c0.z * v.x)));
}

/* ------------------------------------------------------ transcendentals */
/* sin/cos (round 4): reduction by pi -- x = j*pi + r, |r| <= pi/2, Cody-Waite in three fma
 * steps -- then one odd degree-9 polynomial for sin(r) (coefficients tuned in float32: within
 * 1.51 ulp of sin on [-pi/2, pi/2]) and the sign of (-1)^j.  cos(x) = (-1)^(j+1) sin(r) with
 * x = (j + 1/2) pi + r.  Every GLSL sin() / cos() of the reference is one of these (rand()'s
 * hash, the cosine and sphere-light directions, the marble texture); round 3 reduced by pi/2
 * and evaluated both a sine and a cosine polynomial with a quadrant select for every call,
 * ~25 operations against ~15 here.  The parity of j is taken in float (j/2 against its floor):
 * exact below 2^24, and every float from 2^24 up is an even integer; NaN and +-inf give NaN.
 * Deterministic and branch-free on both sides; accurate to ~1e-7 absolute for |x| < 2^20. */
RT_HD float rt_sin_poly(float r) {
    const float z = r * r;
    const float p = fmaf(fmaf(fmaf(2.6000548132287804e-06f, z, -1.9806638010777533e-04f), z,
                              8.333016186952591e-03f), z, -1.6666656732559204e-01f);
    return fmaf(p, z * r, r);
}
RT_HD float rt_neg_if_odd(float s, float j) {
    const float h = j * 0.5f;
    return (h != floorf(h)) ? -s : s;
}
RT_HD float g_sin(float x) {
    const float j = rintf(x * 0x1.45f306p-2f);                  /* 1/pi */
    float r = fmaf(j, -0x1.921fb6p+1f, x);                       /* pi = A + B + C */
    r = fmaf(j, 0x1.777a5cp-24f, r);
    r = fmaf(j, 0x1.ee59dap-49f, r);
    return rt_neg_if_odd(rt_sin_poly(r), j);
}
RT_HD float g_cos(float x) {
    const float j = rintf(fmaf(x, 0x1.45f306p-2f, -0.5f));      /* x = (j + 1/2) pi + r */
    const float jh = j + 0.5f;
    float r = fmaf(jh, -0x1.921fb6p+1f, x);
    r = fmaf(jh, 0x1.777a5cp-24f, r);
    r = fmaf(jh, 0x1.ee59dap-49f, r);
    return rt_neg_if_odd(-rt_sin_poly(r), j);
}
RT_HD void g_sincos(float x, float* s_out, float* c_out) { *s_out = g_sin(x); *c_out = g_cos(x); }

/* natural log: exponent/mantissa split (m in [sqrt(1/2), sqrt(2))), degree-9
 * polynomial for log(1+f), Cody–Waite ln2 split. */
RT_HD float g_log(float x) {
    /* the finite positive path on every input, the special cases selected at the end
     * (NaN or x < 0 -> NaN, +-0 -> -inf, +inf -> +inf): no branches */
    const uint32_t u0 = rt_f2u(x);
    const int sub = u0 < 0x00800000u;             /* +0 and subnormals: scale by 2^23 */
    const uint32_t u = sub ? rt_f2u(x * 8388608.0f) : u0;
    int e = (sub ? -23 : 0) + (int)(u >> 23) - 126;   /* x = m * 2^e, m in [0.5,1) */
    float m = rt_u2f((u & 0x007fffffu) | 0x3f000000u);
    if (m < 0.707106781186547524f) { e -= 1; m = m + m - 1.0f; }
    else { m = m - 1.0f; }
    float z = m * m;
    float y = fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(fmaf(7.0376836292e-2f, m, -1.1514610310e-1f), m,
                  1.1676998740e-1f), m, -1.2420140846e-1f), m, 1.4249322787e-1f), m,
                  -1.6668057665e-1f), m, 2.0000714765e-1f), m, -2.4999993993e-1f), m,
                  3.3333331174e-1f);
    y = (y * m) * z;
    float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    float r = m + y;
    r = fmaf(fe, 0.693359375f, r);
    r = (x == rt_u2f(0x7f800000u)) ? x : r;
    r = (x == 0.0f) ? rt_u2f(0xff800000u) : r;
    return (!(x == x) || x < 0.0f) ? rt_u2f(0x7fc00000u) : r;
}

/* asin core on [0, 0.5]: x + x*z*P(z), z = x*x */
RT_HD float rt_asin_core(float x, float z) {
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                   7.4953002686e-2f), z, 1.6666752422e-1f);
    return fmaf(p * z, x, x);
}
RT_HD float g_acos(float x) {
    float a = fabsf(x);
    if (!(a <= 1.0f)) return rt_u2f(0x7fc00000u);
    if (a > 0.5f) {
        float z = 0.5f * (1.0f - a);
        float s = sqrtf(z);
        float r = 2.0f * rt_asin_core(s, z);        /* acos(|x|) */
        return (x < 0.0f) ? (3.14159274101257324f - r) + (-8.74227766e-8f) : r;
    }
    float p = rt_asin_core(a, a * a);
    float asn = (x < 0.0f) ? -p : p;
    return (1.57079637050628662f - asn) + (-4.37113883e-8f);
}
/* atan on all reals (range-reduced at tan(3pi/8), tan(pi/8)) */
RT_HD float rt_atan(float x) {
    float a = fabsf(x);
    float y0 = 0.0f, t = a;
    if (a > 2.414213562373095f) { y0 = 1.57079637050628662f; t = -1.0f / a; }
    else if (a > 0.4142135623730950f) { y0 = 0.785398185253143311f; t = (a - 1.0f) / (a + 1.0f); }
    float z = t * t;
    float p = fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                   -3.33329491539e-1f);
    float r = y0 + fmaf(p * z, t, t);
    return (x < 0.0f) ? -r : r;
}
/* GLSL atan(y, x) with IEEE signed-zero quadrant rules (needed by the
 * get_sphere_uv known-answer table, texture.glsl:100-102). */
RT_HD float g_atan2(float y, float x) {
    if (!(x == x) || !(y == y)) return rt_u2f(0x7fc00000u);
    int yneg = (rt_f2u(y) >> 31) != 0;
    int xneg = (rt_f2u(x) >> 31) != 0;
    if (y == 0.0f) {
        if (xneg) return yneg ? -3.14159274101257324f : 3.14159274101257324f;
        return y;                                   /* ±0 */
    }
    if (x == 0.0f) return yneg ? -1.57079637050628662f : 1.57079637050628662f;
    float z = rt_atan(y / x);
    if (x < 0.0f) z = yneg ? z - 3.14159274101257324f : z + 3.14159274101257324f;
    return z;
}
/* pow(x, 5.0) as used by Schlick (scatter.glsl:21) */
RT_HD float g_pow5(float x) { float x2 = x * x; return (x2 * x2) * x; }

/* unorm8 -> float, GL conversion c/255 */
RT_HD float rt_unorm8(uint32_t c) { return (float)c / 255.0f; }

#endif /* RT_GLSL_H */
