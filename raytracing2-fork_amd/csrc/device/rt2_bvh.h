// BVH render kernels (calculateRayCollisionBVH, compute.glsl:410-460): v1
// (node array, also the traceBasic walk), v2 and v3 (child-pair records, exact
// Markstein division; v3 is the product kernel) and the division check.
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

// Slab-test division of render_bvh3 (all exact: RN32(n/d) bit for bit).
enum class Slab : int {
    Markstein = 0,  // two Markstein corrections of RN(n * RN(1/d)) (default)
    Binary64 = 1,   // RN32(RN64(n * RN64(1/d)))
    Filtered = 2,   // approximate t, exact slab only on near-ties
};
struct Bvh3Spec {
    int block;
    int thresh;  // finished lanes of a wave that end its traversal phase
    Slab slab;
    int waves;   // minimum waves per SIMD the register allocation must allow (1 = unconstrained)
    bool diag;   // diagnostic build: occupancy tallies of the traversal loop
};
struct Bvh2Spec {
    int block;
    int thresh;
};
struct BvhSpec {
    int block;
};

// ---------------------------------------------------------------------------
// BVH traversal: calculateRayCollisionBVH, compute.glsl:410-460, per lane.
// Stack in LDS (slot-major [slot][thread]: conflict-free), near child pushed
// last so it is popped first, far/near pushed only if their box distance is
// below the running best — the reference's visiting order exactly, so ties
// resolve as in the reference (and as the oracle's bvh mode).
// ---------------------------------------------------------------------------

// rayBoundsIntersect, compute.glsl:382-408.  The per-axis early return is
// folded into one final test: tMin only grows and tMax only shrinks, so a
// failed check stays failed (and |d| = 1 guarantees an unskipped axis).
__device__ __forceinline__ float ray_bounds(const f3& o, const f3& d, bool sx, bool sy, bool sz, const float* bmin,
                                            const float* bmax) {
    float tMin = -1e32f, tMax = 1e32f;
    if (!sx) {
        float t0 = (bmin[0] - o.x) / d.x, t1 = (bmax[0] - o.x) / d.x;
        if (t0 > t1) { const float t = t0; t0 = t1; t1 = t; }
        if (tMin < t0) tMin = t0;
        if (tMax > t1) tMax = t1;
    }
    if (!sy) {
        float t0 = (bmin[1] - o.y) / d.y, t1 = (bmax[1] - o.y) / d.y;
        if (t0 > t1) { const float t = t0; t0 = t1; t1 = t; }
        if (tMin < t0) tMin = t0;
        if (tMax > t1) tMax = t1;
    }
    if (!sz) {
        float t0 = (bmin[2] - o.z) / d.z, t1 = (bmax[2] - o.z) / d.z;
        if (t0 > t1) { const float t = t0; t0 = t1; t1 = t; }
        if (tMin < t0) tMin = t0;
        if (tMax > t1) tMax = t1;
    }
    return (tMin >= tMax || tMax < 0.0f) ? 1e38f : tMin;
}

template <int BLOCK>
__device__ __forceinline__ void closest_bvh(const f3& o, const f3& d, const rt2_node* __restrict__ nodes,
                                            const float4* __restrict__ tri, int* stack, int stack_slots,
                                            float& best, int& bi, uint32_t& tests, uint32_t& visits) {
    const bool sx = d.x < 1e-6f && d.x > -1e-6f;
    const bool sy = d.y < 1e-6f && d.y > -1e-6f;
    const bool sz = d.z < 1e-6f && d.z > -1e-6f;
    float bestK = best * 1.0009765625f;
    int* st = stack + threadIdx.x;
    int sp = 0;
    st[0] = 0;
    sp = 1;
    while (sp > 0) {
        sp -= 1;
        const int ni = st[sp * BLOCK];
        const int4 meta = *reinterpret_cast<const int4*>(&nodes[ni].triangleIndex);
        if (meta.z == -1) {  // leaf: compute.glsl:429-435
            tests += (uint32_t)max(meta.y, 0);
            for (int i = meta.x; i < meta.x + meta.y; i++) {
                const float4* t = tri + 3 * i;
                const MtQ q = mt_quantities(o, d, t[0], t[1], t[2]);
                if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
            }
        } else {  // compute.glsl:441-456
            visits++;
            const int ia = meta.z, ib = meta.z + 1;
            const float dA = ray_bounds(o, d, sx, sy, sz, nodes[ia].bmin, nodes[ia].bmax);
            const float dB = ray_bounds(o, d, sx, sy, sz, nodes[ib].bmin, nodes[ib].bmax);
            const bool nearA = dA < dB;
            const float dNear = nearA ? dA : dB;
            const float dFar = nearA ? dB : dA;
            const int iNear = nearA ? ia : ib;
            const int iFar = nearA ? ib : ia;
            if (dFar < best && sp < stack_slots) st[(sp++) * BLOCK] = iFar;
            if (dNear < best && sp < stack_slots) st[(sp++) * BLOCK] = iNear;
        }
    }
}

// BVH: per-lane traversal of the reference's node array (nodes uploaded with
// the scene).  Dynamic LDS = stack_slots * BLOCK ints.
template <BvhSpec S>
__global__ __launch_bounds__(S.block) void render_bvh(RenderParams p) {
    constexpr int BLOCK = S.block;
    extern __shared__ int bvh_stack[];
    Lane L;
    lane_init(L);
    uint32_t tests = 0, visits = 0;
    for (;;) {
        advance(L, p);
        if (!__any(L.st == ST_TRACE)) break;
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            float best = 1e38f;
            int bi = -1;
            closest_bvh<BLOCK>(L.o, L.d, p.nodes, p.tri, bvh_stack, p.stack_slots, best, bi, tests, visits);
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
    unsigned long long t = tests, v = visits;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_xor(t, off);
        v += __shfl_xor(v, off);
    }
    if (lane_id() == 0) {
        atomicAdd(p.seg_counter + 1, t);  // leaf triangle tests
        atomicAdd(p.seg_counter + 2, v);  // interior node visits (diagnostic)
    }
}

// ---------------------------------------------------------------------------
// BVH traversal, v2: the same visiting order as closest_bvh, restructured for
// SIMT efficiency.
//  * Child-pair records (host-built, bvh_records): one 64-B record per
//    interior node holds both children's boxes and their stack entries, so a
//    pop costs one 64-B load instead of a meta load followed by two box loads.
//    A stack entry >= 0 is an interior record; < 0 is ~(start << 5 | count)
//    for a leaf (count 31 = look the range up in the node array).
//  * Exact slab divisions without the IEEE divide sequence: with y = RN(1/d)
//    computed once per segment, q0 = RN(n*y), r = fma(-q0, d, n) (exact),
//    q1 = RN(q0 + r*y), repeated once more, is RN(n/d) (Markstein) for
//    2^-60 <= |n| <= 2^60 (or n = 0) and 1e-6 <= |d| <= 1; a wave with any
//    numerator outside that range takes the IEEE division for the node
//    (verified against IEEE division by tests/test_gpu_bvh.py's check).
//  * While-while scheduling: lanes traverse independently; a lane whose
//    segment is finished idles until at least `T` lanes of the wave are
//    finished (or none traverses), then those lanes shade, start their next
//    segment or next ray together.  A heavy-tailed ray no longer holds the
//    whole wave at the segment boundary.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float div_mk(float n, float d, float y) {
    float q = n * y;
    float r = fmaf(-q, d, n);
    q = fmaf(r, y, q);
    r = fmaf(-q, d, n);
    return fmaf(r, y, q);
}
__device__ __forceinline__ bool div_mk_ok(float n) {
    const float a = fabsf(n);
    return (a <= 0x1p60f && a >= 0x1p-60f) || a == 0.0f;
}

struct SlabRay {
    f3 o, d, y;  // y = RN(1/d) on unskipped axes
    bool sx, sy, sz;
};

// rayBoundsIntersect (compute.glsl:382-408) on box (b0, b1), exact.
template <bool IEEE>
__device__ __forceinline__ float slab(const SlabRay& R, float b0x, float b0y, float b0z, float b1x, float b1y,
                                      float b1z) {
    float tMin = -1e32f, tMax = 1e32f;
#define RT2_SLAB_AXIS(S, B0, B1, O, D, Y)                                  \
    if (!S) {                                                              \
        float t0, t1;                                                      \
        if constexpr (IEEE) {                                              \
            t0 = (B0 - O) / D;                                             \
            t1 = (B1 - O) / D;                                             \
        } else {                                                           \
            t0 = div_mk(B0 - O, D, Y);                                     \
            t1 = div_mk(B1 - O, D, Y);                                     \
        }                                                                  \
        if (t0 > t1) { const float t_ = t0; t0 = t1; t1 = t_; }            \
        if (tMin < t0) tMin = t0;                                          \
        if (tMax > t1) tMax = t1;                                          \
    }
    RT2_SLAB_AXIS(R.sx, b0x, b1x, R.o.x, R.d.x, R.y.x)
    RT2_SLAB_AXIS(R.sy, b0y, b1y, R.o.y, R.d.y, R.y.y)
    RT2_SLAB_AXIS(R.sz, b0z, b1z, R.o.z, R.d.z, R.y.z)
#undef RT2_SLAB_AXIS
    return (tMin >= tMax || tMax < 0.0f) ? 1e38f : tMin;
}

__device__ __forceinline__ bool slab_numerators_ok(const SlabRay& R, const float4& r0, const float4& r1,
                                                   const float4& r2) {
    bool ok = true;
    if (!R.sx) ok = ok && div_mk_ok(r0.x - R.o.x) && div_mk_ok(r0.w - R.o.x) && div_mk_ok(r1.z - R.o.x) &&
                    div_mk_ok(r2.y - R.o.x);
    if (!R.sy) ok = ok && div_mk_ok(r0.y - R.o.y) && div_mk_ok(r1.x - R.o.y) && div_mk_ok(r1.w - R.o.y) &&
                    div_mk_ok(r2.z - R.o.y);
    if (!R.sz) ok = ok && div_mk_ok(r0.z - R.o.z) && div_mk_ok(r1.y - R.o.z) && div_mk_ok(r2.x - R.o.z) &&
                    div_mk_ok(r2.w - R.o.z);
    return ok;
}

struct TravState {
    int sp;  // > 0 traversing, 0 idle, -1 finished (awaiting shade)
    float best, bestK;
    int bi;
    SlabRay R;
};

__device__ __forceinline__ void begin_segment(Lane& L, TravState& T, int* st, int root) {
    L.bounce += 1;
    L.segs += 1;
    T.best = 1e38f;
    T.bestK = 1e38f * 1.0009765625f;
    T.bi = -1;
    T.R.o = L.o;
    T.R.d = L.d;
    T.R.sx = L.d.x < 1e-6f && L.d.x > -1e-6f;
    T.R.sy = L.d.y < 1e-6f && L.d.y > -1e-6f;
    T.R.sz = L.d.z < 1e-6f && L.d.z > -1e-6f;
    T.R.y = mk(T.R.sx ? 0.0f : 1.0f / L.d.x, T.R.sy ? 0.0f : 1.0f / L.d.y, T.R.sz ? 0.0f : 1.0f / L.d.z);
    st[0] = root;
    T.sp = 1;
}

// One pop of the lane's stack (compute.glsl:419-457).
template <int BLOCK>
__device__ __forceinline__ void bvh_step(TravState& T, int* st, const float4* __restrict__ recs,
                                         const rt2_node* __restrict__ nodes, const float4* __restrict__ tri,
                                         int stack_slots, uint32_t& tests, uint32_t& visits) {
    T.sp -= 1;
    const int e = st[T.sp * BLOCK];
    if (e < 0) {  // leaf: compute.glsl:429-435
        const int v = ~e;
        int start = v >> 5, cnt = v & 31;
        if (cnt == 31) {
            const int4 meta = *reinterpret_cast<const int4*>(&nodes[start].triangleIndex);
            start = meta.x;
            cnt = max(meta.y, 0);
        }
        tests += (uint32_t)cnt;
        for (int i = start; i < start + cnt; i++) {
            const float4* t = tri + 3 * i;
            const MtQ q = mt_quantities(T.R.o, T.R.d, t[0], t[1], t[2]);
            if (mt_pass(q, T.bestK)) mt_exact(q, i, T.best, T.bi, T.bestK);
        }
    } else {  // compute.glsl:437-456
        visits++;
        const float4* rp = recs + 4 * e;
        const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
        const float4 r3 = rp[3];
        float dA, dB;
        if (__builtin_expect(__all(slab_numerators_ok(T.R, r0, r1, r2)), 1)) {
            dA = slab<false>(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
            dB = slab<false>(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
        } else {
            dA = slab<true>(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
            dB = slab<true>(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
        }
        const int eA = __float_as_int(r3.x), eB = __float_as_int(r3.y);
        const bool nearA = dA < dB;
        const float dNear = nearA ? dA : dB;
        const float dFar = nearA ? dB : dA;
        const int iNear = nearA ? eA : eB;
        const int iFar = nearA ? eB : eA;
        if (dFar < T.best && T.sp < stack_slots) st[(T.sp++) * BLOCK] = iFar;
        if (dNear < T.best && T.sp < stack_slots) st[(T.sp++) * BLOCK] = iNear;
    }
    if (T.sp == 0) T.sp = -1;
}

template <Bvh2Spec S>
__global__ __launch_bounds__(S.block) void render_bvh2(RenderParams p) {
    constexpr int BLOCK = S.block, THRESH = S.thresh;
    extern __shared__ int bvh_stack[];
    int* st = bvh_stack + threadIdx.x;
    const float4* __restrict__ recs = p.bvh_recs;
    Lane L;
    lane_init(L);
    TravState T;
    T.sp = 0;
    T.best = T.bestK = 1e38f;
    T.bi = -1;
    uint32_t tests = 0, visits = 0;
    for (;;) {
        // phase A: finished lanes shade; lanes between rays advance; new segments start
        if (T.sp < 0) {
            shade(L, p, T.best, T.bi);
            T.sp = 0;
        }
        advance(L, p);
        if (L.st == ST_TRACE && T.sp == 0) begin_segment(L, T, st, p.bvh_root);
        if (!__any(T.sp > 0)) break;
        // phase B: traverse until THRESH lanes have finished (or none traverses)
        for (;;) {
            if (T.sp > 0) bvh_step<BLOCK>(T, st, recs, p.nodes, p.tri, p.stack_slots, tests, visits);
            const unsigned long long fin = __ballot(T.sp < 0);
            if (!__any(T.sp > 0) || __popcll(fin) >= (unsigned)THRESH) break;
        }
    }
    flush_counters(L, p);
    unsigned long long t = tests, v = visits;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_xor(t, off);
        v += __shfl_xor(v, off);
    }
    if (lane_id() == 0) {
        atomicAdd(p.seg_counter + 1, t);  // leaf triangle tests
        atomicAdd(p.seg_counter + 2, v);  // interior node visits (diagnostic)
    }
}

// ---------------------------------------------------------------------------
// BVH traversal, v3 (render_bvh3): v2 plus
//  * a wave-uniform fast path: when every lane's segment has no skipped axis
//    (|d_i| >= 1e-6) and satisfies the Markstein preconditions by
//    construction — origin components and (host-checked, p.recs_ok) box
//    coordinates in {0} U [2^-37, 2^59], so every numerator b - o is 0 or in
//    [2^-60, 2^60], and |d_i| <= 2 — the slab test runs branch-free with no
//    per-numerator checks; otherwise the node takes the IEEE slab<true>;
//  * one interior pop AND one leaf pop per lane per iteration (the leaf
//    sub-step sees the near child just pushed), so the leaf body runs for
//    more lanes at once.  The per-lane pop order is unchanged.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool mk_coord_ok(float c) {
    const float a = fabsf(c);
    return a == 0.0f || (a >= 0x1p-37f && a <= 0x1p59f);
}

struct TravState3 {
    int sp;  // > 0 traversing, 0 idle, -1 finished (awaiting shade)
    float best, bestK;
    int bi;
    bool fast;  // no skipped axis, Markstein preconditions hold
    SlabRay R;
    double yx, yy, yz;  // DIV64: RN64(1/d) on unskipped axes
};

template <int DIV>
__device__ __forceinline__ void begin_segment3(Lane& L, TravState3& T, int* st, int root) {
    L.bounce += 1;
    L.segs += 1;
    T.best = 1e38f;
    T.bestK = 1e38f * 1.0009765625f;
    T.bi = -1;
    T.R.o = L.o;
    T.R.d = L.d;
    T.R.sx = L.d.x < 1e-6f && L.d.x > -1e-6f;
    T.R.sy = L.d.y < 1e-6f && L.d.y > -1e-6f;
    T.R.sz = L.d.z < 1e-6f && L.d.z > -1e-6f;
    T.R.y = mk(T.R.sx ? 0.0f : 1.0f / L.d.x, T.R.sy ? 0.0f : 1.0f / L.d.y, T.R.sz ? 0.0f : 1.0f / L.d.z);
    if constexpr (DIV == 1) {
        T.fast = !(T.R.sx || T.R.sy || T.R.sz);
        T.yx = 1.0 / (double)L.d.x;
        T.yy = 1.0 / (double)L.d.y;
        T.yz = 1.0 / (double)L.d.z;
    } else {
        T.fast = !(T.R.sx || T.R.sy || T.R.sz) && mk_coord_ok(L.o.x) && mk_coord_ok(L.o.y) &&
                 mk_coord_ok(L.o.z) && fabsf(L.d.x) <= 2.0f && fabsf(L.d.y) <= 2.0f && fabsf(L.d.z) <= 2.0f;
    }
    st[0] = root;
    T.sp = 1;
}

// Branch-free exact slab for the fast path (all axes live, div_mk valid).
__device__ __forceinline__ float slab_fast(const SlabRay& R, float b0x, float b0y, float b0z, float b1x, float b1y,
                                           float b1z) {
    float tMin = -1e32f, tMax = 1e32f;
#define RT2_SLAB_FAST(B0, B1, O, D, Y)                          \
    {                                                           \
        float t0 = div_mk(B0 - O, D, Y);                        \
        float t1 = div_mk(B1 - O, D, Y);                        \
        if (t0 > t1) { const float t_ = t0; t0 = t1; t1 = t_; } \
        if (tMin < t0) tMin = t0;                               \
        if (tMax > t1) tMax = t1;                               \
    }
    RT2_SLAB_FAST(b0x, b1x, R.o.x, R.d.x, R.y.x)
    RT2_SLAB_FAST(b0y, b1y, R.o.y, R.d.y, R.y.y)
    RT2_SLAB_FAST(b0z, b1z, R.o.z, R.d.z, R.y.z)
#undef RT2_SLAB_FAST
    return (tMin >= tMax || tMax < 0.0f) ? 1e38f : tMin;
}

// Exact RN32(n/d) through binary64: with yd = RN64(1/d),
// RN32(RN64(n*yd)) = RN32(n/d) for every float n and normal d: n*yd is within
// 2^-52 relative of n/d, i.e. 2^-28 ulp32, while a quotient of two floats is
// never closer than 2^-25 ulp32 to a binary32 rounding boundary (midpoint).
__device__ __forceinline__ float div64(float n, double yd) { return (float)((double)n * yd); }

__device__ __forceinline__ float slab64(const TravState3& T, float b0x, float b0y, float b0z, float b1x, float b1y,
                                        float b1z) {
    float tMin = -1e32f, tMax = 1e32f;
#define RT2_SLAB64(B0, B1, O, Y)                                \
    {                                                           \
        float t0 = div64(B0 - O, Y);                            \
        float t1 = div64(B1 - O, Y);                            \
        if (t0 > t1) { const float t_ = t0; t0 = t1; t1 = t_; } \
        if (tMin < t0) tMin = t0;                               \
        if (tMax > t1) tMax = t1;                               \
    }
    RT2_SLAB64(b0x, b1x, T.R.o.x, T.yx)
    RT2_SLAB64(b0y, b1y, T.R.o.y, T.yy)
    RT2_SLAB64(b0z, b1z, T.R.o.z, T.yz)
#undef RT2_SLAB64
    return (tMin >= tMax || tMax < 0.0f) ? 1e38f : tMin;
}

// DIV == 2: decision filter for the slab tests.  t' = RN(n*y) is within
// 2^-21 * max(|t|, |t'|) of the exact t = RN(n/d) (y = RN(1/d): |n*y - n/d| <=
// 2^-24 |n/d|, plus two half-ulp roundings), has the same sign, and is 0 iff
// t is; min/max keep that bound.  Every decision the traversal takes from the
// box distances (a box missed: tMin >= tMax or tMax < 0; near/far: dA < dB;
// push: d < best) is taken from the t' values when the two compared numbers
// are further apart than 2^-19 * (|a| + |b|) — then the exact values order
// the same way — and the lane re-runs the exact slab_fast otherwise.
__device__ __forceinline__ void slab_approx(const SlabRay& R, float b0x, float b0y, float b0z, float b1x, float b1y,
                                            float b1z, float& tMin, float& tMax) {
    const float x0 = (b0x - R.o.x) * R.y.x, x1 = (b1x - R.o.x) * R.y.x;
    const float y0 = (b0y - R.o.y) * R.y.y, y1 = (b1y - R.o.y) * R.y.y;
    const float z0 = (b0z - R.o.z) * R.y.z, z1 = (b1z - R.o.z) * R.y.z;
    tMin = fmaxf(fmaxf(fmaxf(-1e32f, fminf(x0, x1)), fminf(y0, y1)), fminf(z0, z1));
    tMax = fminf(fminf(fminf(1e32f, fmaxf(x0, x1)), fmaxf(y0, y1)), fmaxf(z0, z1));
}
__device__ __forceinline__ bool near_tie(float a, float b) { return fabsf(a - b) <= (fabsf(a) + fabsf(b)) * 0x1p-19f; }

template <int BLOCK, int DIV>
__device__ __forceinline__ void bvh_interior3(TravState3& T, int* st, int e, const float4* __restrict__ recs,
                                              bool fast, int stack_slots, uint32_t& visits, uint32_t& refined) {
    visits++;
    const float4* rp = recs + 4 * e;
    const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
    const float4 r3 = rp[3];
    float dA = 1e38f, dB = 1e38f;  // set by the filter (DIV 2) or the exact forms below
    bool exact = true;
    if (fast && DIV == 2) {
        float aMin, aMax, bMin, bMax;
        slab_approx(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, aMin, aMax);
        slab_approx(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w, bMin, bMax);
        const bool hitA = !(aMin >= aMax || aMax < 0.0f), hitB = !(bMin >= bMax || bMax < 0.0f);
        dA = hitA ? aMin : 1e38f;
        dB = hitB ? bMin : 1e38f;
        // a box flat on some axis (bmin == bmax there) is missed in both
        // arithmetics: that axis puts the same t into tMin's max and tMax's min
        const bool flatA = (r0.x == r0.w) | (r0.y == r1.x) | (r0.z == r1.y);
        const bool flatB = (r1.z == r2.y) | (r1.w == r2.z) | (r2.x == r2.w);
        bool amb = (int)(near_tie(aMin, aMax) & !flatA) | (int)(near_tie(bMin, bMax) & !flatB);  // branch-free
        amb |= hitA & hitB & near_tie(dA, dB);
        amb |= hitA & near_tie(dA, T.best);
        amb |= hitB & near_tie(dB, T.best);
        exact = amb;
        refined += amb ? 1u : 0u;
    }
    if (!exact) {
        // decisions taken from the filtered distances
    } else if (fast && DIV == 1) {
        dA = slab64(T, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
        dB = slab64(T, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
    } else if (fast) {
        dA = slab_fast(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
        dB = slab_fast(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
    } else {
        dA = slab<true>(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
        dB = slab<true>(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
    }
    const int eA = __float_as_int(r3.x), eB = __float_as_int(r3.y);
    const bool nearA = dA < dB;
    const float dNear = nearA ? dA : dB;
    const float dFar = nearA ? dB : dA;
    const int iNear = nearA ? eA : eB;
    const int iFar = nearA ? eB : eA;
    if (dFar < T.best && T.sp < stack_slots) st[(T.sp++) * BLOCK] = iFar;
    if (dNear < T.best && T.sp < stack_slots) st[(T.sp++) * BLOCK] = iNear;
}

__device__ __forceinline__ void bvh_leaf3(TravState3& T, int e, const rt2_node* __restrict__ nodes,
                                          const float4* __restrict__ tri, uint32_t& tests) {
    const int v = ~e;
    int start = v >> 5, cnt = v & 31;
    if (cnt == 31) {
        const int4 meta = *reinterpret_cast<const int4*>(&nodes[start].triangleIndex);
        start = meta.x;
        cnt = max(meta.y, 0);
    }
    tests += (uint32_t)cnt;
    for (int i = start; i < start + cnt; i++) {
        const float4* t = tri + 3 * i;
        const MtQ q = mt_quantities(T.R.o, T.R.d, t[0], t[1], t[2]);
        if (mt_pass3(q, T.bestK)) mt_exact(q, i, T.best, T.bi, T.bestK);
    }
}

template <Bvh3Spec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_bvh3(RenderParams p) {
    constexpr int BLOCK = S.block, THRESH = S.thresh, DIV = (int)S.slab;
    constexpr bool DIAG = S.diag;
    extern __shared__ int bvh_stack[];
    int* st = bvh_stack + threadIdx.x;
    const float4* __restrict__ recs = p.bvh_recs;
    Lane L;
    lane_init(L);
    TravState3 T;
    T.sp = 0;
    T.best = T.bestK = 1e38f;
    T.bi = -1;
    T.fast = true;
    T.yx = T.yy = T.yz = 0.0;
    uint32_t tests = 0, visits = 0, refined = 0;
    // DIAG: wave-uniform tallies (lane 0 publishes them): [0] inner iterations,
    // [1] lanes in the interior sub-step, [2] lanes in the leaf sub-step,
    // [3] finished lanes waiting, [4] DONE lanes, [5] outer iterations,
    // [6] lanes shading, [7] iterations running the interior body
    unsigned long long dg[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (;;) {
        if constexpr (DIAG) {
            dg[5] += 1;
            dg[6] += __popcll(__ballot(T.sp < 0));
        }
        if (T.sp < 0) {
            shade(L, p, T.best, T.bi);
            T.sp = 0;
        }
        advance(L, p);
        if (L.st == ST_TRACE && T.sp == 0) begin_segment3<DIV>(L, T, st, p.bvh_root);
        if (!__any(T.sp > 0)) break;
        const bool fast = (DIV == 1 || p.recs_ok) && __all(T.fast || T.sp <= 0);
        for (;;) {
            if constexpr (DIAG) {
                dg[0] += 1;
                const bool in = T.sp > 0 && st[(T.sp - 1) * BLOCK] >= 0;
                const unsigned long long bi = __ballot(in);
                dg[1] += __popcll(bi);
                dg[7] += bi ? 1 : 0;
                dg[3] += __popcll(__ballot(T.sp < 0));
                dg[4] += __popcll(__ballot(L.st == ST_DONE));
            }
            // interior sub-step
            if (T.sp > 0) {
                const int e = st[(T.sp - 1) * BLOCK];
                if (e >= 0) {
                    T.sp -= 1;
                    bvh_interior3<BLOCK, DIV>(T, st, e, recs, fast, p.stack_slots, visits, refined);
                    if (T.sp == 0) T.sp = -1;
                }
            }
            // leaf sub-step
            if constexpr (DIAG) dg[2] += __popcll(__ballot(T.sp > 0 && st[(T.sp - 1) * BLOCK] < 0));
            if (T.sp > 0) {
                const int e = st[(T.sp - 1) * BLOCK];
                if (e < 0) {
                    T.sp -= 1;
                    bvh_leaf3(T, e, p.nodes, p.tri, tests);
                    if (T.sp == 0) T.sp = -1;
                }
            }
            const unsigned long long fin = __ballot(T.sp < 0);
            if (!__any(T.sp > 0) || __popcll(fin) >= (unsigned)THRESH) break;
        }
    }
    flush_counters(L, p);
    unsigned long long t = tests, v = visits, rf = refined;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_xor(t, off);
        v += __shfl_xor(v, off);
        rf += __shfl_xor(rf, off);
    }
    if (lane_id() == 0) {
        atomicAdd(p.seg_counter + 1, t);   // leaf triangle tests
        atomicAdd(p.seg_counter + 2, v);   // interior node visits (diagnostic)
        atomicAdd(p.seg_counter + 3, rf);  // DIV 2: visits re-run exactly (diagnostic)
        if constexpr (DIAG)
            for (int k = 0; k < 8; k++) atomicAdd(p.seg_counter + 7 + k, dg[k]);  // counters [8..15]
        // wave finish-time spread (diagnostic): [6] earliest, [7] latest wave end, 10 ns ticks
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        atomicMin(p.seg_counter + 5, t_end);
        atomicMax(p.seg_counter + 6, t_end);
    }
}

// ---------------------------------------------------------------------------
// BVH traversal, v4 (render_bvh4): v3 with the entry to visit next kept in a
// register.  The reference pushes far then near and pops near at once; v4
// continues with near in the register and pushes only far, popping when the
// register is consumed — the same visiting order, one LDS store and load less
// per interior visit, and at most depth - 1 stack entries (one pending far
// child per level), so the LDS stack is `depth` slots instead of depth + 2:
// config C's depth-32 tree fits 5 workgroups of 256 lanes per CU (5 waves per
// SIMD, the register limit) instead of 4.
// ---------------------------------------------------------------------------
struct TravState4 {
    int state;  // 1 traversing (cur valid), 0 idle, -1 finished (awaiting shade)
    int cur;    // entry to visit next (record index >= 0, or ~leaf)
    int sp;     // LDS stack entries
    float best, bestK;
    int bi;
    bool fast;
    SlabRay R;
};

__device__ __forceinline__ void begin_segment4(Lane& L, TravState4& T, int root) {
    L.bounce += 1;
    L.segs += 1;
    T.best = 1e38f;
    T.bestK = 1e38f * 1.0009765625f;
    T.bi = -1;
    T.R.o = L.o;
    T.R.d = L.d;
    T.R.sx = L.d.x < 1e-6f && L.d.x > -1e-6f;
    T.R.sy = L.d.y < 1e-6f && L.d.y > -1e-6f;
    T.R.sz = L.d.z < 1e-6f && L.d.z > -1e-6f;
    T.R.y = mk(T.R.sx ? 0.0f : 1.0f / L.d.x, T.R.sy ? 0.0f : 1.0f / L.d.y, T.R.sz ? 0.0f : 1.0f / L.d.z);
    T.fast = !(T.R.sx || T.R.sy || T.R.sz) && mk_coord_ok(L.o.x) && mk_coord_ok(L.o.y) && mk_coord_ok(L.o.z) &&
             fabsf(L.d.x) <= 2.0f && fabsf(L.d.y) <= 2.0f && fabsf(L.d.z) <= 2.0f;
    T.cur = root;
    T.sp = 0;
    T.state = 1;
}

// next entry: the top of the LDS stack, or the end of the traversal
template <int BLOCK>
__device__ __forceinline__ void bvh_pop4(TravState4& T, const int* st) {
    if (T.sp > 0) {
        T.sp -= 1;
        T.cur = st[T.sp * BLOCK];
    } else {
        T.state = -1;
    }
}

template <int BLOCK>
__device__ __forceinline__ void bvh_interior4(TravState4& T, int* st, const float4* __restrict__ recs, bool fast,
                                              int stack_slots, uint32_t& visits) {
    visits++;
    const float4* rp = recs + 4 * T.cur;
    const float4 r0 = rp[0], r1 = rp[1], r2 = rp[2];
    const float4 r3 = rp[3];
    float dA, dB;
    if (fast) {
        dA = slab_fast(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
        dB = slab_fast(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
    } else {
        dA = slab<true>(T.R, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y);
        dB = slab<true>(T.R, r1.z, r1.w, r2.x, r2.y, r2.z, r2.w);
    }
    const int eA = __float_as_int(r3.x), eB = __float_as_int(r3.y);
    const bool nearA = dA < dB;
    const float dNear = nearA ? dA : dB;
    const float dFar = nearA ? dB : dA;
    const int iNear = nearA ? eA : eB;
    const int iFar = nearA ? eB : eA;
    // the reference's two pushes (far, then near) and the pop that follows
    // (a valid tree never needs more than depth - 1 < stack_slots entries;
    // the bound only keeps the store inside the lane's slots)
    const bool pushFar = dFar < T.best;
    const bool pushNear = dNear < T.best;
    if (pushNear) {
        if (pushFar && T.sp < stack_slots) st[(T.sp++) * BLOCK] = iFar;
        T.cur = iNear;
    } else if (pushFar) {
        T.cur = iFar;
    } else {
        bvh_pop4<BLOCK>(T, st);
    }
}

template <Bvh3Spec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_bvh4(RenderParams p) {
    constexpr int BLOCK = S.block, THRESH = S.thresh;
    extern __shared__ int bvh_stack[];
    int* st = bvh_stack + threadIdx.x;
    const float4* __restrict__ recs = p.bvh_recs;
    Lane L;
    lane_init(L);
    TravState4 T;
    T.state = 0;
    T.cur = 0;
    T.sp = 0;
    T.best = T.bestK = 1e38f;
    T.bi = -1;
    T.fast = true;
    uint32_t tests = 0, visits = 0;
    for (;;) {
        if (T.state < 0) {
            shade(L, p, T.best, T.bi);
            T.state = 0;
        }
        advance(L, p);
        if (L.st == ST_TRACE && T.state == 0) begin_segment4(L, T, p.bvh_root);
        if (!__any(T.state > 0)) break;
        const bool fast = p.recs_ok && __all(T.fast || T.state <= 0);
        for (;;) {
            // interior sub-step
            if (T.state > 0 && T.cur >= 0) bvh_interior4<BLOCK>(T, st, recs, fast, p.stack_slots, visits);
            // leaf sub-step (sees the near child just taken)
            if (T.state > 0 && T.cur < 0) {
                TravState3 t3;  // bvh_leaf3's view of the lane
                t3.R = T.R;
                t3.best = T.best;
                t3.bestK = T.bestK;
                t3.bi = T.bi;
                bvh_leaf3(t3, T.cur, p.nodes, p.tri, tests);
                T.best = t3.best;
                T.bestK = t3.bestK;
                T.bi = t3.bi;
                bvh_pop4<BLOCK>(T, st);
            }
            const unsigned long long fin = __ballot(T.state < 0);
            if (!__any(T.state > 0) || __popcll(fin) >= (unsigned)THRESH) break;
        }
    }
    flush_counters(L, p);
    unsigned long long t = tests, v = visits;
    for (int off = 32; off > 0; off >>= 1) {
        t += __shfl_xor(t, off);
        v += __shfl_xor(v, off);
    }
    if (lane_id() == 0) {
        atomicAdd(p.seg_counter + 1, t);  // leaf triangle tests
        atomicAdd(p.seg_counter + 2, v);  // interior node visits (diagnostic)
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        atomicMin(p.seg_counter + 5, t_end);
        atomicMax(p.seg_counter + 6, t_end);
    }
}

// Division check for div_mk (test hook): n, d drawn from the ranges above.
__global__ void div_check_kernel(uint32_t seed, unsigned long long count, int mode, unsigned long long* bad,
                                 uint32_t* first) {
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    unsigned long long nbad = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
        uint32_t h = (uint32_t)i * 2654435761u ^ seed;
        h ^= h >> 16;
        h *= 0x7feb352du;
        h ^= h >> 15;
        h *= 0x846ca68bu;
        h ^= h >> 16;
        uint32_t g = h * 747796405u + 2891336453u;
        g = ((g >> ((g >> 28u) + 4u)) ^ g) * 277803737u;
        g ^= g >> 22;
        // n: |n| in [2^-60, 2^60], random sign/mantissa; d: |d| in [1e-6, 2]
        // mode 1 (div64): any finite n, subnormals included
        const uint32_t ne = mode == 1 ? (h % 255u) : 127 - 60 + (h % 121u);
        const float n = __uint_as_float((h & 0x80000000u) | (ne << 23) | (g & 0x7fffffu));
        const uint32_t de = 127 - 20 + ((g >> 23) % 22u);
        float d = __uint_as_float(((g << 8) & 0x80000000u) | (de << 23) | ((h * 2246822519u) & 0x7fffffu));
        if (fabsf(d) < 1e-6f) d = copysignf(1e-6f, d);
        if (fabsf(d) > 2.0f) d = copysignf(2.0f, d);
        float q;
        if (mode == 1) {
            q = div64(n, 1.0 / (double)d);
        } else {
            q = div_mk(n, d, 1.0f / d);
        }
        const float ref = n / d;
        if (__float_as_uint(q) != __float_as_uint(ref)) {
            nbad++;
            atomicCAS(first, 0xffffffffu, (uint32_t)i);
        }
    }
    if (nbad) atomicAdd(bad, nbad);
}

}  // namespace
