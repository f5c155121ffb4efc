/*
 * rt_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
 * render kernel, RayTracing/Assets/Shaders/compute.glsl (the reference has no
 * CPU render path: SURVEY.md §0 fact 1).  Used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg as the checker /
 * baseline; never linked into the product (raytracing2-fork_amd/).
 *
 * It follows compute.glsl line by line; every function cites the lines it
 * restates.  Floating-point evaluation is pinned (the GLSL leaves it open):
 *   - no contraction: built with -ffp-contract=off, every a*b+c below is two
 *     roundings unless written fmaf();
 *   - dot(a,b)   = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))   (a fused evaluation
 *     GLSL permits without `precise`, GLSL 4.30 §4.7.1);
 *   - cross(a,b) = (fma(a.y,b.z,-(a.z*b.y)), fma(a.z,b.x,-(a.x*b.z)),
 *                   fma(a.x,b.y,-(a.y*b.x)));
 *   - normalize(v) = v / sqrt(dot(v,v)) (GLSL 4.30 §8.5 definition), IEEE
 *     correctly-rounded / and sqrt;
 *   - cos/sin/acos/exp/pow = include/rt2_pinned_math.h.
 * The GLSL driver the reference ran on is unknown (SURVEY.md §8c "Pins"), so
 * this file, not a GLSL run, is the definition the HIP kernel is held to.
 *
 * Two traversals:
 *   mode 0 "brute": closest hit over all triangles in array order, strict <
 *                   (the kernel's algorithm; same result as the BVH except on
 *                   exact distance ties);
 *   mode 1 "bvh"  : calculateRayCollisionBVH, compute.glsl:410-460, over the
 *                   node array of BVH.h.
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rt2_pinned_math.h"

/* Material types, compute.glsl:7-13 */
enum { DIFFUSE = 0, SPECULAR = 1, LIGHT = 2, CHECKER = 3, GLASS = 4, TEXTURE = 5, GLASS_HIGHLIGHT = 6 };

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 cross(v3 a, v3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}
static inline float length(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize(v3 a) { return divs(a, length(a)); }
/* GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N */
static inline v3 reflect(v3 i, v3 n) { return sub(i, muls(n, 2.0f * dot(n, i))); }
/* GLSL mix(x, y, a) = x * (1 - a) + y * a */
static inline v3 mixs(v3 x, v3 y, float a) { return add(muls(x, 1.0f - a), muls(y, a)); }
static inline v3 mixv(v3 x, v3 y, v3 a) {
    return mk(x.x * (1.0f - a.x) + y.x * a.x, x.y * (1.0f - a.y) + y.y * a.y, x.z * (1.0f - a.z) + y.z * a.z);
}
static inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
static inline float smoothstep(float e0, float e1, float x) {
    float t = clampf((x - e0) / (e1 - e0), 0.0f, 1.0f);
    return t * t * (3.0f - 2.0f * t);
}
static inline v3 v4xyz(const float* p) { return mk(p[0], p[1], p[2]); }

/* ---- random, compute.glsl:148-159 ------------------------------------- */
static inline float rnd(uint32_t* state) {
    *state = *state * 747796405u + 2891336453u;
    uint32_t result = ((*state >> ((*state >> 28u) + 4u)) ^ *state) * 277803737u;
    result = (result >> 22u) ^ result;
    /* `result / 4294967295.0`: uint -> float conversion, divided by the float
     * literal, which rounds to 2^32 (exact power-of-two scaling). */
    return (float)result / 4294967296.0f;
}
static inline float rnd_range(float left, float right, uint32_t* state) {
    return left + (right - left) * rnd(state);
}

/* randomDirection2D, compute.glsl:161-165 */
static inline void rnd_dir2d(uint32_t* state, float* c, float* s) {
    float angle = rnd(state);
    *c = rt2pm_cosf(angle);
    *s = rt2pm_sinf(angle);
}

/* randomDirection, compute.glsl:174-185 */
static inline v3 rnd_dir(uint32_t* state) {
    for (int i = 0; i < 100; i++) {
        float x = rnd(state) * 2.0f - 1.0f;
        float y = rnd(state) * 2.0f - 1.0f;
        float z = rnd(state) * 2.0f - 1.0f;
        v3 p = mk(x, y, z);
        if (length(p) < 1.0f) return normalize(p);
    }
    return mk(0.0f, 0.0f, 0.0f);
}

/* refract_, compute.glsl:201-214 */
static inline v3 refract_(v3 I, v3 N, float eta, int* isRefracted) {
    float k = 1.0f - eta * eta * (1.0f - dot(N, I) * dot(N, I));
    if (k < 0.0f) {
        *isRefracted = 0;
        return reflect(I, N);
    }
    *isRefracted = 1;
    return sub(muls(I, eta), muls(N, eta * dot(N, I) + sqrtf(k)));
}

/* getEnvironmentalLight, compute.glsl:216-273 */
static v3 sky(v3 dir) {
    v3 sunDir = normalize(mk(0.6f, 0.3f, -0.2f));
    float sunDot = dot(dir, sunDir);
    float horizonDot = dir.y;
    v3 zenithColor = mk(0.15f, 0.25f, 0.65f);
    v3 deepOrange = mk(1.2f, 0.4f, 0.1f);
    v3 yellow = mk(1.0f, 0.8f, 0.3f);
    v3 coolBlue = mk(0.3f, 0.4f, 0.7f);
    v3 groundColor = mk(0.2f, 0.15f, 0.1f);
    float sunToOpposite = (dot(dir, neg(sunDir)) + 1.0f) * 0.5f;
    v3 horizonColor;
    if (sunToOpposite < 0.5f)
        horizonColor = mixs(deepOrange, yellow, sunToOpposite * 2.0f);
    else
        horizonColor = mixs(yellow, coolBlue, (sunToOpposite - 0.5f) * 2.0f);
    float skyGradient = smoothstep(-0.2f, 0.8f, horizonDot);
    v3 baseColor = mixs(horizonColor, zenithColor, skyGradient);
    v3 sunCenter = mk(15.0f, 15.0f, 10.0f);
    float sunAngle = rt2pm_acosf(clampf(sunDot, -1.0f, 1.0f));
    float glow1 = rt2pm_expf(-sunAngle * 600.0f);
    float glow2 = rt2pm_expf(-sunAngle * 150.0f) * 0.3f;
    float glow3 = rt2pm_expf(-sunAngle * 60.0f) * 0.1f;
    float glow4 = rt2pm_expf(-sunAngle * 15.0f) * 0.03f;
    float totalGlow = glow1 + glow2 + glow3 + glow4;
    v3 finalColor = add(baseColor, muls(sunCenter, totalGlow));
    if (horizonDot < 0.0f) {
        float groundBlend = smoothstep(-0.1f, 0.0f, horizonDot);
        finalColor = mixs(groundColor, finalColor, groundBlend);
        float groundSunGlow = rt2pm_expf(-sunAngle * 15.0f) * 0.2f;
        finalColor = add(finalColor, muls(muls(sunCenter, groundSunGlow), 0.05f));
    }
    return finalColor;
}

/* ---- intersection ------------------------------------------------------- */
typedef struct {
    int didHit;
    float dst;
    int tri;
} hit_t;

/* rayTriangleIntersect, compute.glsl:302-340 — decision part.  Returns 1 and
 * dst on a hit. */
static inline int tri_test(v3 o, v3 d, const oracle_triangle* t, float* dst_out) {
    v3 a = v4xyz(t->a), b = v4xyz(t->b), c = v4xyz(t->c);
    v3 e0 = sub(b, a);
    v3 e1 = sub(c, a);
    v3 cross01 = cross(e0, e1);
    float det = -dot(d, cross01);
    if ((det < 1e-10f && det > -1e-10f) || det < 0.0f) return 0;
    float invDet = 1.0f / det;
    v3 ao = sub(o, a);
    float dst = dot(ao, cross01) * invDet;
    if (dst <= 1e-6f) return 0;
    v3 dirCrossAO = cross(d, ao);
    float u = -dot(e1, dirCrossAO) * invDet;
    float v = dot(e0, dirCrossAO) * invDet;
    if (u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f) return 0;
    *dst_out = dst;
    return 1;
}

/* rayBoundsIntersect, compute.glsl:382-408 */
static inline float ray_bounds(v3 o, v3 d, const oracle_node* nd) {
    float tMin = -1e32f, tMax = 1e32f;
    float oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    for (int i = 0; i < 3; i++) {
        if (!(dd[i] < 1e-6f && dd[i] > -1e-6f)) {
            float t0 = (nd->bmin[i] - oo[i]) / dd[i];
            float t1 = (nd->bmax[i] - oo[i]) / dd[i];
            if (t0 > t1) { float tmp = t0; t0 = t1; t1 = tmp; }
            if (tMin < t0) tMin = t0;
            if (tMax > t1) tMax = t1;
            if (tMin >= tMax || tMax < 0.0f) return 1e38f;
        }
    }
    return tMin;
}

typedef struct {
    const oracle_triangle* tris;
    int32_t n_tris;
    const oracle_material* mats;
    int32_t n_mats;
    const oracle_node* nodes;
    int32_t n_nodes;
    const oracle_uniforms* u;
    int mode;
} ctx_t;

/* Closest hit.  Brute force: every triangle in array order, `dst < best`
 * (compute.glsl:432-434).  BVH: compute.glsl:410-460. */
static hit_t closest(const ctx_t* c, v3 o, v3 d, uint64_t* tests) {
    hit_t r;
    r.didHit = 0;
    r.dst = 1e38f;
    r.tri = -1;
    if (c->mode == 0) {
        for (int i = 0; i < c->n_tris; i++) {
            float dst;
            if (tri_test(o, d, &c->tris[i], &dst) && dst < r.dst) {
                r.didHit = 1;
                r.dst = dst;
                r.tri = i;
            }
        }
        *tests += (uint64_t)c->n_tris;
        return r;
    }
    int stack[64];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        sp -= 1;
        const oracle_node* node = &c->nodes[stack[sp]];
        if (node->childIndex == -1) {
            for (int i = node->triangleIndex; i < node->triangleIndex + node->triangleCount; i++) {
                float dst;
                *tests += 1;
                if (tri_test(o, d, &c->tris[i], &dst) && dst < r.dst) {
                    r.didHit = 1;
                    r.dst = dst;
                    r.tri = i;
                }
            }
        } else {
            int ia = node->childIndex, ib = node->childIndex + 1;
            float dstA = ray_bounds(o, d, &c->nodes[ia]);
            float dstB = ray_bounds(o, d, &c->nodes[ib]);
            int nearA = dstA < dstB;
            float dstNear = nearA ? dstA : dstB;
            float dstFar = nearA ? dstB : dstA;
            int iNear = nearA ? ia : ib;
            int iFar = nearA ? ib : ia;
            if (dstFar < r.dst && sp < 64) stack[sp++] = iFar;
            if (dstNear < r.dst && sp < 64) stack[sp++] = iNear;
        }
    }
    return r;
}

/* ---- textures (getTriangleTextureColor, compute.glsl:342-368) ------------
 * Set by oracle_set_textures from stb-layout images (w, h, n, bytes); held as
 * RGBA8 after GL's unpack (GL_UNPACK_ALIGNMENT 4: rows every align4(w*n)
 * bytes, bytes past the buffer read as 0) and Texture2D's swizzles
 * (textureClass.cpp:70-90: 1 channel -> r,r,r,1; GL_RG -> r,g,0,1). */
typedef struct {
    int32_t w, h;
    uint8_t* rgba;
} otex_t;
static otex_t g_tex[64];
static int32_t g_ntex = 0;

int oracle_set_textures(const int32_t* whn, const uint8_t* const* pixels, int32_t n) {
    for (int i = 0; i < g_ntex; i++) free(g_tex[i].rgba);
    g_ntex = 0;
    if (n < 0 || n > 64) return -1;
    for (int i = 0; i < n; i++) {
        const int32_t w = whn[3 * i], h = whn[3 * i + 1], ch = whn[3 * i + 2];
        if (w < 1 || h < 1 || ch < 1 || ch > 4) return -1;
        const size_t stride = ((size_t)w * ch + 3) & ~(size_t)3, total = (size_t)w * h * ch;
        uint8_t* q = (uint8_t*)malloc((size_t)w * h * 4);
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                uint8_t c[4] = {0, 0, 0, 255};
                for (int k = 0; k < ch; k++) {
                    const size_t at = (size_t)y * stride + (size_t)x * ch + k;
                    c[k] = at < total ? pixels[i][at] : 0;
                }
                uint8_t* o = q + ((size_t)y * w + x) * 4;
                if (ch == 1) {
                    o[0] = o[1] = o[2] = c[0];
                    o[3] = 255;
                } else if (ch == 2) {
                    o[0] = c[0];
                    o[1] = c[1];
                    o[2] = 0;
                    o[3] = 255;
                } else {
                    o[0] = c[0];
                    o[1] = c[1];
                    o[2] = c[2];
                    o[3] = ch == 4 ? c[3] : 255;
                }
            }
        g_tex[i].w = w;
        g_tex[i].h = h;
        g_tex[i].rgba = q;
        g_ntex = i + 1;
    }
    return 0;
}

static int tex_wrap(float f, int n) {
    const int i = (f >= -1073741824.0f && f <= 1073741824.0f) ? (int)f : 0;
    const int r = i % n;
    return r < 0 ? r + n : r;
}

/* texture(sampler2D, uv): GL_LINEAR (no mipmaps) + GL_REPEAT, GL 4.3 §8.14.2,
 * unorm8 texels c/255, evaluated in binary32 as written. */
static v3 tex_sample(const otex_t* t, float s, float tc) {
    const float u = s * (float)t->w - 0.5f;
    const float v = tc * (float)t->h - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float a = u - fu, b = v - fv;
    const int i0 = tex_wrap(fu, t->w), j0 = tex_wrap(fv, t->h);
    const int i1 = i0 + 1 == t->w ? 0 : i0 + 1, j1 = j0 + 1 == t->h ? 0 : j0 + 1;
    const uint8_t* T00 = t->rgba + ((size_t)j0 * t->w + i0) * 4;
    const uint8_t* T10 = t->rgba + ((size_t)j0 * t->w + i1) * 4;
    const uint8_t* T01 = t->rgba + ((size_t)j1 * t->w + i0) * 4;
    const uint8_t* T11 = t->rgba + ((size_t)j1 * t->w + i1) * 4;
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float r[3];
    for (int k = 0; k < 3; k++)
        r[k] = w00 * ((float)T00[k] / 255.0f) + w10 * ((float)T10[k] / 255.0f) + w01 * ((float)T01[k] / 255.0f) +
               w11 * ((float)T11[k] / 255.0f);
    return mk(r[0], r[1], r[2]);
}

/* getTriangleTextureColor at the closest hit of (o, d) on triangle t: the
 * barycentrics of rayTriangleIntersect (:307-338, w = 1 - u - v),
 * uv = aTex*u + bTex*v + cTex*w. */
static v3 texture_color(const ctx_t* c, int tex_index, const oracle_triangle* t, v3 o, v3 d) {
    if (tex_index < 0 || tex_index >= c->u->numTextures) return mk(0.0f, 0.0f, 0.0f);
    if (tex_index > 4) return mk(1.0f, 0.0f, 1.0f);
    if (tex_index >= g_ntex) return mk(0.0f, 0.0f, 0.0f);
    v3 a = v4xyz(t->a), b = v4xyz(t->b), cc = v4xyz(t->c);
    v3 e0 = sub(b, a), e1 = sub(cc, a);
    v3 cross01 = cross(e0, e1);
    float det = -dot(d, cross01);
    float invDet = 1.0f / det;
    v3 ao = sub(o, a);
    v3 q = cross(d, ao);
    float u = -dot(e1, q) * invDet;
    float v = dot(e0, q) * invDet;
    float w = 1.0f - u - v;
    float s = t->aTex[0] * u + t->bTex[0] * v + t->cTex[0] * w;
    float tc = t->aTex[1] * u + t->bTex[1] * v + t->cTex[1] * w;
    return tex_sample(&g_tex[tex_index], s, tc);
}

/* trace, compute.glsl:472-563 */
static v3 trace(const ctx_t* c, v3 origin, v3 dir, uint32_t* rng, uint64_t* segs, uint64_t* tests) {
    v3 rayColor = mk(1.0f, 1.0f, 1.0f);
    v3 incomingLight = mk(0.0f, 0.0f, 0.0f);
    int insideGlass = 0;
    int bounceCount = 0;
    while (bounceCount < c->u->maxBounceCount) {
        bounceCount++;
        *segs += 1;
        hit_t h = closest(c, origin, dir, tests);
        if (h.didHit) {
            const oracle_triangle* t = &c->tris[h.tri];
            v3 a = v4xyz(t->a), b = v4xyz(t->b), cc = v4xyz(t->c);
            v3 cross01 = cross(sub(b, a), sub(cc, a));
            v3 normal = normalize(cross01);
            v3 hitPoint = add(origin, muls(dir, h.dst));
            int mi = t->materialIndex;
            const oracle_material* m = &c->mats[mi];
            v3 tex = m->materialType == TEXTURE ? texture_color(c, m->textureIndex, t, origin, dir)
                                                : mk(0.0f, 0.0f, 0.0f);
            if (m->materialType != GLASS)
                origin = sub(hitPoint, muls(muls(dir, h.dst), -1e-3f));
            else
                origin = add(hitPoint, muls(muls(dir, h.dst), -1e-3f));
            v3 attenuation = mk(0.0f, 0.0f, 0.0f);
            v3 prevDirection = dir;
            switch (m->materialType) {
            case DIFFUSE:
            case TEXTURE:
                dir = normalize(add(normal, rnd_dir(rng)));
                attenuation = m->materialType == DIFFUSE ? v4xyz(m->color) : tex;
                break;
            case SPECULAR: {
                v3 diffuseDirection = normalize(add(normal, rnd_dir(rng)));
                v3 specularDirection = reflect(dir, normal);
                int isSpecularBounce = m->specularProbability > rnd(rng);
                dir = mixs(diffuseDirection, specularDirection, isSpecularBounce ? m->smoothness : 0.0f);
                attenuation = isSpecularBounce ? mk(1.0f, 1.0f, 1.0f) : v4xyz(m->color);
                break;
            }
            case LIGHT: {
                v3 emitted = muls(v4xyz(m->emissionColor), m->emissionStrength);
                incomingLight = add(incomingLight, mul(emitted, rayColor));
                return incomingLight;
            }
            case CHECKER: {
                dir = normalize(add(normal, rnd_dir(rng)));
                float s = m->checkerScale;
                int black = 0;
                if (s > 0.0f) {
                    float sum = floorf(origin.x * s) + floorf(origin.y * s) + floorf(origin.z * s);
                    float md = sum - 2.0f * floorf(sum / 2.0f); /* GLSL mod(x, 2) */
                    black = md == 0.0f;
                }
                attenuation = black ? mk(0.0f, 0.0f, 0.0f) : mk(1.0f, 1.0f, 1.0f);
                break;
            }
            case GLASS: {
                float eta = insideGlass ? m->refractiveIndex : 1.0f / m->refractiveIndex;
                int isRefracted;
                dir = refract_(dir, normal, eta, &isRefracted);
                insideGlass = isRefracted != insideGlass;
                attenuation = v4xyz(m->color);
                break;
            }
            default:
                return mk(1.0f, 0.0f, 1.0f);
            }
            if (m->isEdgeHighlight && bounceCount > 1)
                dir = prevDirection;
            else
                rayColor = mul(rayColor, attenuation);
            float p = fmaxf(rayColor.x, fmaxf(rayColor.y, rayColor.z));
            if (rnd(rng) > p) break;
            rayColor = muls(rayColor, 1.0f / p);
        } else {
            if (c->u->environmentalLight) incomingLight = add(incomingLight, mul(sky(dir), rayColor));
            return incomingLight;
        }
    }
    return incomingLight;
}

/* normalizeColor, compute.glsl:462-470 */
static inline v3 normalize_color(v3 c) {
    float m = fmaxf(fmaxf(c.x, c.y), c.z);
    if (m > 1.0f) return divs(c, m);
    return c;
}

/* traceBasic, compute.glsl:565-645 — the interactive one-ray preview.  `Ray
 * ray;` leaves insideGlass uninitialised in the shader (:674); it starts false
 * here. */
static v3 trace_basic(const ctx_t* c, v3 origin, v3 dir, uint64_t* segs, uint64_t* tests) {
    v3 colorCumulative = mk(0.0f, 0.0f, 0.0f);
    int insideGlass = 0;
    int bounceCount = 0;
    while (bounceCount < c->u->maxBounceCount) {
        bounceCount++;
        *segs += 1;
        hit_t h = closest(c, origin, dir, tests);
        if (h.didHit) {
            const oracle_triangle* t = &c->tris[h.tri];
            v3 a = v4xyz(t->a), b = v4xyz(t->b), cc = v4xyz(t->c);
            v3 normal = normalize(cross(sub(b, a), sub(cc, a)));
            v3 hitPoint = add(origin, muls(dir, h.dst));
            const oracle_material* m = &c->mats[t->materialIndex];
            v3 tex = m->materialType == TEXTURE ? texture_color(c, m->textureIndex, t, origin, dir)
                                                : mk(0.0f, 0.0f, 0.0f);
            origin = sub(hitPoint, muls(normal, 1e-4f));
            switch (m->materialType) {
            case SPECULAR:
                colorCumulative = add(colorCumulative, v4xyz(m->color));
                dir = reflect(dir, normal);
                break;
            case DIFFUSE:
            case TEXTURE:
            case CHECKER: {
                v3 color;
                if (m->materialType == TEXTURE) {
                    color = tex;
                } else if (m->materialType == DIFFUSE) {
                    color = v4xyz(m->color);
                } else {
                    float s = m->checkerScale;
                    int black = 0;
                    if (s > 0.0f) {
                        float sum = floorf(origin.x * s) + floorf(origin.y * s) + floorf(origin.z * s);
                        black = (sum - 2.0f * floorf(sum / 2.0f)) == 0.0f;
                    }
                    color = black ? mk(0.0f, 0.0f, 0.0f) : mk(1.0f, 1.0f, 1.0f);
                }
                colorCumulative = add(colorCumulative, color);
                if (c->u->basicShadingShadow) {
                    v3 toLight = normalize(sub(v4xyz(c->u->basicShadingLightPosition), hitPoint));
                    *segs += 1;
                    hit_t h2 = closest(c, origin, toLight, tests);
                    v3 r = h2.didHit ? divs(colorCumulative, 5.0f) : colorCumulative;
                    return divs(r, (float)bounceCount);
                }
                return divs(colorCumulative, (float)bounceCount);
            }
            case LIGHT:
                return normalize_color(v4xyz(m->emissionColor));
            case GLASS: {
                float eta = insideGlass ? m->refractiveIndex : 1.0f / m->refractiveIndex;
                int isRefracted;
                dir = refract_(dir, normal, eta, &isRefracted);
                insideGlass = isRefracted != insideGlass;
                colorCumulative = v4xyz(m->color);
                break;
            }
            case GLASS_HIGHLIGHT:
                break; /* `if (bounceCount == 0)` never holds after bounceCount++ */
            default:
                return mk(1.0f, 0.0f, 1.0f);
            }
        } else {
            colorCumulative = add(colorCumulative, sky(dir));
            break;
        }
    }
    return divs(colorCumulative, (float)bounceCount);
}

/* tonemapACES + toSRGB, compute.glsl:647-658 */
static inline float aces1(float x) {
    const float a = 2.51f, b = 0.03f, cc = 2.43f, d = 0.59f, e = 0.14f;
    return clampf((x * (a * x + b)) / (x * (cc * x + d) + e), 0.0f, 1.0f);
}
static inline float srgb1(float x) { return rt2pm_powf(x, 1.0f / 2.2f); }

/* main(), compute.glsl:660-701, one (pixel, frame). */
static v3 render_pixel_frame(const ctx_t* c, int tx, int ty, uint32_t frame, uint64_t* segs, uint64_t* tests) {
    const oracle_uniforms* u = c->u;
    int W = (int)u->width, H = (int)u->height;
    float x = (float)(tx * 2 - W) / (float)W;
    float y = (float)(ty * 2 - H) / (float)H;
    uint32_t seed = (uint32_t)tx + (uint32_t)ty * (uint32_t)W + frame * 968824447u;
    v3 cam = v4xyz(u->cameraPos);
    if (u->basicShading) { /* compute.glsl:672-678: no jitter, no RNG, no tonemap */
        v3 dir = normalize(add(add(v4xyz(u->viewportFront), muls(v4xyz(u->viewportRight), x)),
                               muls(v4xyz(u->viewportUp), y)));
        return trace_basic(c, cam, dir, segs, tests);
    }
    v3 endPoint = add(add(add(cam, v4xyz(u->viewportFront)), muls(v4xyz(u->viewportRight), x)),
                      muls(v4xyz(u->viewportUp), y));
    v3 colorCumulative = mk(0.0f, 0.0f, 0.0f);
    for (int i = 0; i < u->numRaysPerPixel; i++) {
        float cs, sn;
        rnd_dir2d(&seed, &cs, &sn);
        v3 origin = add(add(cam, muls(v4xyz(u->defocusDiskRight), cs)), muls(v4xyz(u->defocusDiskUp), sn));
        float jr = rnd_range(-0.5f, 0.5f, &seed);
        float ju = rnd_range(-0.5f, 0.5f, &seed);
        v3 endJ = add(add(endPoint, muls(v4xyz(u->pixelRight), jr)), muls(v4xyz(u->pixelUp), ju));
        v3 dir = normalize(sub(endJ, origin));
        colorCumulative = add(colorCumulative, trace(c, origin, dir, &seed, segs, tests));
    }
    v3 color = divs(colorCumulative, (float)u->numRaysPerPixel);
    return mk(srgb1(aces1(color.x)), srgb1(aces1(color.y)), srgb1(aces1(color.z)));
}

/* ---- threaded driver ----------------------------------------------------- */
typedef struct {
    const ctx_t* c;
    const int32_t* px; /* (x, y) pairs */
    int64_t n_px;
    uint32_t frame_begin, frame_count;
    float* out_rgba;
    uint32_t* out_acc8;
    atomic_llong next_unit;
    atomic_ullong segs, tests;
} job_t;

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    const ctx_t* c = j->c;
    uint64_t segs = 0, tests = 0;
    const int64_t chunk = 32; /* work unit: 32 consecutive list pixels */
    for (;;) {
        int64_t p0 = atomic_fetch_add(&j->next_unit, 1) * chunk;
        if (p0 >= j->n_px) break;
        int64_t p1 = p0 + chunk < j->n_px ? p0 + chunk : j->n_px;
        for (int64_t p = p0; p < p1; p++) {
            const int tx = j->px[2 * p], ty = j->px[2 * p + 1];
            float acc[3] = {0.0f, 0.0f, 0.0f};
            uint32_t a8[3] = {0, 0, 0};
            for (uint32_t f = 0; f < j->frame_count; f++) {
                v3 col = render_pixel_frame(c, tx, ty, j->frame_begin + f, &segs, &tests);
                acc[0] += col.x;
                acc[1] += col.y;
                acc[2] += col.z;
                float cc[3] = {col.x, col.y, col.z};
                for (int k = 0; k < 3; k++) {
                    /* GL float -> unorm8 (GL 4.3 §2.3.5.2, round to nearest) */
                    float q = clampf(cc[k], 0.0f, 1.0f) * 255.0f + 0.5f;
                    a8[k] += (uint32_t)q;
                }
            }
            size_t o = (size_t)p * 4;
            if (j->out_rgba) {
                j->out_rgba[o + 0] = acc[0];
                j->out_rgba[o + 1] = acc[1];
                j->out_rgba[o + 2] = acc[2];
                j->out_rgba[o + 3] = (float)j->frame_count;
            }
            if (j->out_acc8) {
                j->out_acc8[o + 0] = a8[0];
                j->out_acc8[o + 1] = a8[1];
                j->out_acc8[o + 2] = a8[2];
                j->out_acc8[o + 3] = j->frame_count;
            }
        }
    }
    atomic_fetch_add(&j->segs, segs);
    atomic_fetch_add(&j->tests, tests);
    return NULL;
}

/* Renders an arbitrary list of pixels ((x, y) pairs); out_accum / out_acc8
 * hold n_px * 4 entries in list order. */
int oracle_render_pixels(const oracle_triangle* tris, int32_t n_tris, const oracle_material* mats, int32_t n_mats,
                         const oracle_node* nodes, int32_t n_nodes, const oracle_uniforms* u, uint32_t frame_begin,
                         uint32_t frame_count, const int32_t* px, int64_t n_px, int32_t mode, int32_t threads,
                         float* out_accum, uint32_t* out_acc8, uint64_t* out_segments, uint64_t* out_tests) {
    if (!tris || !mats || !u || (!px && n_px > 0) || n_px < 0 || n_tris < 0) return -1;
    if (mode == 1 && (!nodes || n_nodes < 1)) return -2;
    if (!u->basicShading && u->numRaysPerPixel < 1) return -3;
    for (int i = 0; i < n_tris; i++)
        if (tris[i].materialIndex < 0 || tris[i].materialIndex >= n_mats) return -4;
    for (int64_t i = 0; i < n_px; i++)
        if (px[2 * i] < 0 || px[2 * i] >= (int32_t)u->width || px[2 * i + 1] < 0 || px[2 * i + 1] >= (int32_t)u->height)
            return -5;
    ctx_t c = {tris, n_tris, mats, n_mats, nodes, n_nodes, u, mode};
    job_t j;
    j.c = &c;
    j.px = px;
    j.n_px = n_px;
    j.frame_begin = frame_begin;
    j.frame_count = frame_count;
    j.out_rgba = out_accum;
    j.out_acc8 = out_acc8;
    atomic_init(&j.next_unit, 0);
    atomic_init(&j.segs, 0);
    atomic_init(&j.tests, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int i = 1; i < threads; i++) pthread_create(&th[i], NULL, worker, &j);
    worker(&j);
    for (int i = 1; i < threads; i++) pthread_join(th[i], NULL);
    if (out_segments) *out_segments = atomic_load(&j.segs);
    if (out_tests) *out_tests = atomic_load(&j.tests);
    return 0;
}

/* Whole rows: out_accum / out_acc8 are [n_rows][W][4]. */
int oracle_render(const oracle_triangle* tris, int32_t n_tris, const oracle_material* mats, int32_t n_mats,
                  const oracle_node* nodes, int32_t n_nodes, const oracle_uniforms* u, uint32_t frame_begin,
                  uint32_t frame_count, const int32_t* rows, int32_t n_rows, int32_t mode, int32_t threads,
                  float* out_accum, uint32_t* out_acc8, uint64_t* out_segments, uint64_t* out_tests) {
    if (!u || !rows || n_rows < 0) return -1;
    const int64_t W = (int64_t)u->width;
    int32_t* px = (int32_t*)malloc(sizeof(int32_t) * 2 * (size_t)(W * n_rows + 1));
    if (!px) return -6;
    for (int64_t r = 0; r < n_rows; r++)
        for (int64_t x = 0; x < W; x++) {
            px[2 * (r * W + x)] = (int32_t)x;
            px[2 * (r * W + x) + 1] = rows[r];
        }
    int rc = oracle_render_pixels(tris, n_tris, mats, n_mats, nodes, n_nodes, u, frame_begin, frame_count, px,
                                  W * n_rows, mode, threads, out_accum, out_acc8, out_segments, out_tests);
    free(px);
    return rc;
}

/* Single-call helpers for known-answer tests. */
uint32_t oracle_pcg_next(uint32_t* state, float* out) {
    float f = rnd(state);
    if (out) *out = f;
    uint32_t s = *state;
    uint32_t result = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (result >> 22u) ^ result;
}

int oracle_ray_triangle(const float o[3], const float d[3], const oracle_triangle* t, float* dst) {
    return tri_test(mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), t, dst);
}

void oracle_sky(const float d[3], float out[3]) {
    v3 s = sky(mk(d[0], d[1], d[2]));
    out[0] = s.x;
    out[1] = s.y;
    out[2] = s.z;
}

float oracle_tonemap_srgb(float x) { return srgb1(aces1(x)); }

float oracle_pinned(int which, float x) {
    switch (which) {
    case 0: return rt2pm_expf(x);
    case 1: return rt2pm_logf(x);
    case 2: return rt2pm_acosf(x);
    case 3: return rt2pm_cosf(x);
    case 4: return rt2pm_sinf(x);
    case 5: return rt2pm_powf(x, 1.0f / 2.2f);
    default: return 0.0f;
    }
}
