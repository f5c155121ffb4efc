/*
 * rt2_pinned_math.h — the transcendental functions of the render path, pinned.
 *
 * compute.glsl calls cos/sin (randomDirection2D, :161-165), acos/exp (the
 * sky, :216-273) and pow (toSRGB, :656-658).  GLSL only bounds their error,
 * and the host libm and the device ocml return different last bits, so a CPU
 * render and a GPU render of the same seed would differ in the last ulp of
 * those terms — and through the defocus disk, in the paths themselves.
 *
 * These implementations (Cephes single-precision polynomials, explicit fmaf
 * Horner steps, bit-exact range reduction) are the render path's libm.  They
 * use only IEEE-754 operations that are correctly rounded on both x86-64
 * (SSE/FMA) and gfx950 (v_fma_f32, v_mul/v_add, v_cvt), so the same code gives
 * the same bits on the host and on the device.  Accuracy (checked against the
 * system libm in tests/test_oracle_kat.py) is within a few ulp, well inside
 * GLSL's own allowance.
 *
 * This header is the product's own libm (like <math.h>), shared by the HIP
 * kernel and by any CPU restatement of the path.  It compiles as C99 (gcc) and
 * as HIP device/host code (hipcc).
 */
#ifndef RT2_PINNED_MATH_H
#define RT2_PINNED_MATH_H

#include <stdint.h>

#if defined(__HIPCC__)
#define RT2PM_FN static inline __host__ __device__
#else
#define RT2PM_FN static inline
#endif

#define RT2PM_FMA(a, b, c) __builtin_fmaf((a), (b), (c))

RT2PM_FN uint32_t rt2pm_f2u(float f) {
    union { float f; uint32_t u; } v;
    v.f = f;
    return v.u;
}
RT2PM_FN float rt2pm_u2f(uint32_t u) {
    union { float f; uint32_t u; } v;
    v.u = u;
    return v.f;
}

/* 2^k for -126 <= k <= 127, exact. */
RT2PM_FN float rt2pm_pow2i(int k) { return rt2pm_u2f((uint32_t)(k + 127) << 23); }

/* y * 2^k with a single rounding (k in [-200, 254]). */
RT2PM_FN float rt2pm_ldexp(float y, int k) {
    if (k > 127) return (y * rt2pm_pow2i(127)) * rt2pm_pow2i(k - 127);
    if (k < -126) return (y * rt2pm_pow2i(k + 64)) * rt2pm_pow2i(-64);
    return y * rt2pm_pow2i(k);
}

/* exp(x): Cephes expf.  |error| <= 2 ulp for normal results. */
RT2PM_FN float rt2pm_expf(float x) {
    if (x != x) return x;
    if (x > 88.7228317f) return rt2pm_u2f(0x7f800000u);
    if (x < -103.972076f) return 0.0f;
    float k = __builtin_rintf(x * 1.44269504088896341f);
    float r = RT2PM_FMA(k, -0.693359375f, x);
    r = RT2PM_FMA(k, 2.12194440e-4f, r);
    float z = r * r;
    float p = 1.9875691500e-4f;
    p = RT2PM_FMA(p, r, 1.3981999507e-3f);
    p = RT2PM_FMA(p, r, 8.3334519073e-3f);
    p = RT2PM_FMA(p, r, 4.1665795894e-2f);
    p = RT2PM_FMA(p, r, 1.6666665459e-1f);
    p = RT2PM_FMA(p, r, 5.0000001201e-1f);
    float y = RT2PM_FMA(p, z, r) + 1.0f;
    return rt2pm_ldexp(y, (int)k);
}

/* log(x): Cephes logf.  x <= 0 -> -inf (0) / NaN (< 0). */
RT2PM_FN float rt2pm_logf(float x) {
    if (x != x) return x;
    if (x < 0.0f) return rt2pm_u2f(0x7fc00000u);
    if (x == 0.0f) return rt2pm_u2f(0xff800000u);
    if (x == rt2pm_u2f(0x7f800000u)) return x;
    int e = 0;
    uint32_t u = rt2pm_f2u(x);
    if (u < 0x00800000u) { /* subnormal: scale into the normal range (exact) */
        x = x * 8388608.0f;
        e = -23;
        u = rt2pm_f2u(x);
    }
    e += (int)((u >> 23) & 0xffu) - 126;               /* x = m * 2^e, m in [0.5, 1) */
    float m = rt2pm_u2f((u & 0x807fffffu) | 0x3f000000u);
    if (m < 0.707106781186547524f) {
        e -= 1;
        m = (m + m) - 1.0f;
    } else {
        m = m - 1.0f;
    }
    float z = m * m;
    float y = 7.0376836292e-2f;
    y = RT2PM_FMA(y, m, -1.1514610310e-1f);
    y = RT2PM_FMA(y, m, 1.1676998740e-1f);
    y = RT2PM_FMA(y, m, -1.2420140846e-1f);
    y = RT2PM_FMA(y, m, 1.4249322787e-1f);
    y = RT2PM_FMA(y, m, -1.6668057665e-1f);
    y = RT2PM_FMA(y, m, 2.0000714765e-1f);
    y = RT2PM_FMA(y, m, -2.4999993993e-1f);
    y = RT2PM_FMA(y, m, 3.3333331174e-1f);
    y = (y * m) * z;
    float fe = (float)e;
    y = RT2PM_FMA(fe, -2.12194440e-4f, y);
    y = RT2PM_FMA(z, -0.5f, y);
    float r = m + y;
    return RT2PM_FMA(fe, 0.693359375f, r);
}

/* pow(x, y) for x >= 0 (GLSL leaves x < 0 undefined): exp(y * log(x)). */
RT2PM_FN float rt2pm_powf(float x, float y) {
    if (x == 0.0f) return y > 0.0f ? 0.0f : (y == 0.0f ? 1.0f : rt2pm_u2f(0x7f800000u));
    if (x == 1.0f) return 1.0f;
    return rt2pm_expf(y * rt2pm_logf(x));
}

/* asin core on |x| <= 0.5 (Cephes asinf). */
RT2PM_FN float rt2pm_asin_core(float x) {
    float z = x * x;
    float p = 4.2163199048e-2f;
    p = RT2PM_FMA(p, z, 2.4181311049e-2f);
    p = RT2PM_FMA(p, z, 4.5470025998e-2f);
    p = RT2PM_FMA(p, z, 7.4953002686e-2f);
    p = RT2PM_FMA(p, z, 1.6666752422e-1f);
    return RT2PM_FMA(p * z, x, x);
}

/* acos(x) on [-1, 1]: Cephes acosf. */
RT2PM_FN float rt2pm_acosf(float x) {
    if (!(x >= -1.0f && x <= 1.0f)) return rt2pm_u2f(0x7fc00000u);
    if (x < -0.5f) return 3.14159265358979323846f - 2.0f * rt2pm_asin_core(__builtin_sqrtf(0.5f * (1.0f + x)));
    if (x > 0.5f) return 2.0f * rt2pm_asin_core(__builtin_sqrtf(0.5f * (1.0f - x)));
    return 1.57079632679489661923f - rt2pm_asin_core(x);
}

/* sin/cos polynomials on |x| <= pi/4 (Cephes sinf/cosf). */
RT2PM_FN float rt2pm_sin_poly(float x) {
    float z = x * x;
    float p = -1.9515295891e-4f;
    p = RT2PM_FMA(p, z, 8.3321608736e-3f);
    p = RT2PM_FMA(p, z, -1.6666654611e-1f);
    return RT2PM_FMA(p * z, x, x);
}
RT2PM_FN float rt2pm_cos_poly(float x) {
    float z = x * x;
    float p = 2.443315711809948e-5f;
    p = RT2PM_FMA(p, z, -1.388731625493765e-3f);
    p = RT2PM_FMA(p, z, 4.166664568298827e-2f);
    float y = (p * z) * z;
    y = RT2PM_FMA(z, -0.5f, y);
    return y + 1.0f;
}

/* Cody-Waite reduction by pi/4 (Cephes DP1..DP3); valid for |x| < 8192. */
RT2PM_FN float rt2pm_reduce(float ax, int* quadrant) {
    int j = (int)(ax * 1.27323954473516f);
    float y = (float)j;
    if (j & 1) {
        j += 1;
        y += 1.0f;
    }
    *quadrant = j & 7;
    float r = RT2PM_FMA(y, -0.78515625f, ax);
    r = RT2PM_FMA(y, -2.4187564849853515625e-4f, r);
    r = RT2PM_FMA(y, -3.77489497744594108e-8f, r);
    return r;
}

RT2PM_FN float rt2pm_sinf(float x) {
    if (x != x) return x;
    int sign = x < 0.0f;
    float ax = sign ? -x : x;
    int q;
    float r = rt2pm_reduce(ax, &q);
    if (q > 3) {
        sign = !sign;
        q -= 4;
    }
    float y = (q == 1 || q == 2) ? rt2pm_cos_poly(r) : rt2pm_sin_poly(r);
    return sign ? -y : y;
}

RT2PM_FN float rt2pm_cosf(float x) {
    if (x != x) return x;
    float ax = x < 0.0f ? -x : x;
    int q;
    float r = rt2pm_reduce(ax, &q);
    int sign = 0;
    if (q > 3) {
        sign = 1;
        q -= 4;
    }
    if (q > 1) sign = !sign;
    float y = (q == 1 || q == 2) ? rt2pm_sin_poly(r) : rt2pm_cos_poly(r);
    return sign ? -y : y;
}

#endif /* RT2_PINNED_MATH_H */
