// Device-side math of the render path: the GLSL built-ins compute.glsl uses,
// evaluated in the pinned form documented in DESIGN.md §Numerics (the file is
// compiled with -ffp-contract=off; the only fused operations are the explicit
// fmaf of dot() and cross()):
//   dot(a,b)    = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
//   cross(a,b)  = (fma(a.y,b.z,-(a.z*b.y)), fma(a.z,b.x,-(a.x*b.z)), fma(a.x,b.y,-(a.y*b.x)))
//   normalize   = v / sqrt(dot(v,v))      (IEEE / and sqrt)
//   reflect     = I - (2*dot(N,I)) * N
//   mix(x,y,a)  = x*(1-a) + y*a
//   cos/sin/acos/exp/pow from include/rt2_pinned_math.h
#pragma once

#include <hip/hip_runtime.h>

#include "../../../include/rt2_pinned_math.h"

namespace rt2d {

struct f3 {
    float x, y, z;
};

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 add(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 mul(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 muls(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 divs(f3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ f3 neg(f3 a) { return mk(-a.x, -a.y, -a.z); }
__device__ __forceinline__ float dot(f3 a, f3 b) {
    return __builtin_fmaf(a.z, b.z, __builtin_fmaf(a.y, b.y, a.x * b.x));
}
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return mk(__builtin_fmaf(a.y, b.z, -(a.z * b.y)), __builtin_fmaf(a.z, b.x, -(a.x * b.z)),
              __builtin_fmaf(a.x, b.y, -(a.y * b.x)));
}
__device__ __forceinline__ float length(f3 a) { return __builtin_sqrtf(dot(a, a)); }
__device__ __forceinline__ f3 normalize(f3 a) { return divs(a, length(a)); }
__device__ __forceinline__ f3 reflect(f3 i, f3 n) { return sub(i, muls(n, 2.0f * dot(n, i))); }
__device__ __forceinline__ f3 mixs(f3 x, f3 y, float a) { return add(muls(x, 1.0f - a), muls(y, a)); }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ float smoothstep(float e0, float e1, float x) {
    float t = clampf((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}

// Reciprocal sequences built on v_rcp_f32 (<= 1 ulp) + FMA Newton/quotient
// refinement (the f32 fdiv expansion of the AMDGPU backend without its
// div_scale/div_fixup range handling).  rcp_variant(x, 3) is bit-identical to
// IEEE 1.0f/x for every x whose reciprocal is a normal number — checked
// exhaustively on the device over all such bit patterns
// (tests/test_gpu_numerics.py::test_rcp_exhaustive).
__device__ __forceinline__ float rcp_variant(float x, int v) {
    float r = __builtin_amdgcn_rcpf(x);
    if (v == 0) return r;
    float e = __builtin_fmaf(-x, r, 1.0f);
    r = __builtin_fmaf(e, r, r);
    if (v == 1) return r;
    float q = r;
    float rem = __builtin_fmaf(-x, q, 1.0f);
    q = __builtin_fmaf(rem, r, q);
    if (v == 2) return q;
    rem = __builtin_fmaf(-x, q, 1.0f);
    return __builtin_fmaf(rem, r, q);
}

// random, compute.glsl:148-154 — PCG-RXS-M-XS, result / 2^32
__device__ __forceinline__ float rnd(uint32_t& state) {
    state = state * 747796405u + 2891336453u;
    uint32_t r = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    r = (r >> 22u) ^ r;
    return (float)r / 4294967296.0f;
}

// randomDirection, compute.glsl:174-185
__device__ __forceinline__ f3 rnd_dir(uint32_t& state) {
    for (int i = 0; i < 100; i++) {
        float x = rnd(state) * 2.0f - 1.0f;
        float y = rnd(state) * 2.0f - 1.0f;
        float z = rnd(state) * 2.0f - 1.0f;
        f3 p = mk(x, y, z);
        if (length(p) < 1.0f) return normalize(p);
    }
    return mk(0.0f, 0.0f, 0.0f);
}

// refract_, compute.glsl:201-214
__device__ __forceinline__ f3 refract_(f3 I, f3 N, float eta, bool& isRefracted) {
    float k = 1.0f - eta * eta * (1.0f - dot(N, I) * dot(N, I));
    if (k < 0.0f) {
        isRefracted = false;
        return reflect(I, N);
    }
    isRefracted = true;
    return sub(muls(I, eta), muls(N, eta * dot(N, I) + __builtin_sqrtf(k)));
}

// getEnvironmentalLight, compute.glsl:216-273
__device__ __noinline__ f3 sky(f3 dir) {
    f3 sunDir = normalize(mk(0.6f, 0.3f, -0.2f));
    float sunDot = dot(dir, sunDir);
    float horizonDot = dir.y;
    const f3 zenithColor = mk(0.15f, 0.25f, 0.65f);
    const f3 deepOrange = mk(1.2f, 0.4f, 0.1f);
    const f3 yellow = mk(1.0f, 0.8f, 0.3f);
    const f3 coolBlue = mk(0.3f, 0.4f, 0.7f);
    const f3 groundColor = mk(0.2f, 0.15f, 0.1f);
    float sunToOpposite = (dot(dir, neg(sunDir)) + 1.0f) * 0.5f;
    f3 horizonColor = sunToOpposite < 0.5f ? mixs(deepOrange, yellow, sunToOpposite * 2.0f)
                                           : mixs(yellow, coolBlue, (sunToOpposite - 0.5f) * 2.0f);
    float skyGradient = smoothstep(-0.2f, 0.8f, horizonDot);
    f3 baseColor = mixs(horizonColor, zenithColor, skyGradient);
    const f3 sunCenter = mk(15.0f, 15.0f, 10.0f);
    float sunAngle = rt2pm_acosf(clampf(sunDot, -1.0f, 1.0f));
    float glow1 = rt2pm_expf(-sunAngle * 600.0f);
    float glow2 = rt2pm_expf(-sunAngle * 150.0f) * 0.3f;
    float glow3 = rt2pm_expf(-sunAngle * 60.0f) * 0.1f;
    float glow4 = rt2pm_expf(-sunAngle * 15.0f) * 0.03f;
    float totalGlow = glow1 + glow2 + glow3 + glow4;
    f3 finalColor = add(baseColor, muls(sunCenter, totalGlow));
    if (horizonDot < 0.0f) {
        float groundBlend = smoothstep(-0.1f, 0.0f, horizonDot);
        finalColor = mixs(groundColor, finalColor, groundBlend);
        float groundSunGlow = rt2pm_expf(-sunAngle * 15.0f) * 0.2f;
        finalColor = add(finalColor, muls(muls(sunCenter, groundSunGlow), 0.05f));
    }
    return finalColor;
}

// tonemapACES + toSRGB, compute.glsl:647-658
__device__ __forceinline__ float aces1(float x) {
    const float a = 2.51f, b = 0.03f, c = 2.43f, d = 0.59f, e = 0.14f;
    return clampf((x * (a * x + b)) / (x * (c * x + d) + e), 0.0f, 1.0f);
}
__device__ __forceinline__ float srgb1(float x) { return rt2pm_powf(x, 1.0f / 2.2f); }

}  // namespace rt2d
