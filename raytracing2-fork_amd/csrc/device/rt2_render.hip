// MI355X (gfx950) render path: the per-pixel Monte-Carlo loop of
// RayTracing/Assets/Shaders/compute.glsl:472-701 as a persistent HIP kernel.
//
// Unit of work ("item") = one pixel of the shard; an item runs frames
// frame_begin.. in order, each frame numRaysPerPixel rays in order, exactly
// like one compute.glsl invocation per frame (the rays of a pixel-frame share
// one sequential RNG stream, compute.glsl:668/683, so they cannot be split).
//
// Execution model:
//   - one lane = one item at a time; every loop iteration each lane traces ONE
//     segment (closest-hit query + scatter) of its current ray;
//   - a lane whose path ends starts the next ray / frame of its item itself;
//     a lane whose item ends is refilled from a global item counter with one
//     wave-level __ballot + popcount + mbcnt prefix sum + one atomicAdd per
//     wave (ray regeneration: lanes never idle while items remain);
//   - closest hit = brute force over all triangles in array order (strict <,
//     so the lowest index wins a tie).  Triangles are pre-transformed on the
//     device to {a, e0 = b-a, e1 = c-a, n = cross(e0,e1)} (48 B, bit-identical
//     to computing them per test) and staged in LDS:
//       RESIDENT: the whole array fits in LDS, loaded once per workgroup, and
//                 waves then run independently (no barriers);
//       TILED:    the array is streamed through LDS in tiles; the workgroup
//                 sweeps every tile in lockstep once per segment.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/rt2.h"
#include "rt2_math.h"

using namespace rt2d;

namespace {


struct RenderParams {
    const float4* tri;  // 3 float4 per triangle: {ax ay az e0x} {e0y e0z e1x e1y} {e1z nx ny nz}
    const int* tri_mtl;
    const rt2_material* mats;
    int n_tris;
    int n_mats;
    int W, H;
    int maxBounce, R, envLight;
    float cam[3], vpRight[3], vpUp[3], vpFront[3], pixR[3], pixU[3], defR[3], defU[3];
    uint32_t frame_begin, frame_count;
    int tile_rows, rank, nranks;
    unsigned long long n_items;  // work items: pixels, or frames x pixels when frame_split
    unsigned long long n_pix;    // pixels of the shard
    int frame_split;             // 1: item = (frame, pixel), frame-major; colours -> frame_buf
    const uint32_t* order;       // nullable: run rank -> run of 64 pixels (most expensive first)
    uint32_t n_runs;             // full 64-pixel runs covered by `order` (the partial last run keeps its place)
    uint32_t* cost_out;          // nullable: per-pixel item cost (shader clocks) for the next launch's order
    float4* frame_buf;           // frame_split: [frame_count][n_pix] per-frame colours
    float4* accum;
    uint4* accum8;
    unsigned long long* item_counter;
    unsigned long long* seg_counter;
    int tile_tris;  // TILED: triangles per LDS tile
    const rt2_node* nodes;  // BVH traversal
    int stack_slots;        // BVH: per-lane stack entries (tree depth + 2)
    int basicShadow;        // traceBasic: basicShadingShadow
    float light[3];         // traceBasic: basicShadingLightPosition.xyz
    const float4* bvh_recs; // BVH v2: child-pair records (4 float4 each)
    int bvh_root;           // BVH v2: stack entry of node 0
    int recs_ok;            // BVH v3: every record coordinate in {0} U [2^-37, 2^59]
    const rt2_triangle* raw;     // as uploaded (texture coordinates)
    const uchar4* texels;        // all textures, RGBA8 after GL unpack + swizzle
    const int4* tex_desc;        // per texture {width, height, offset lo, offset hi}
    int n_tex;                   // textures uploaded
    int num_textures;            // uniforms.numTextures
};

enum : int { ST_NEED_ITEM = 0, ST_NEW_FRAME = 1, ST_NEW_RAY = 2, ST_TRACE = 3, ST_DONE = 4 };

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 xyz4(const rt2_vec4& v) { return mk(v.x, v.y, v.z); }

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int shard_row(int local_row, int tile_rows, int rank, int nranks) {
    int t = local_row / tile_rows;
    return (t * nranks + rank) * tile_rows + local_row % tile_rows;
}

// One Möller–Trumbore test (compute.glsl:302-340) against a pre-transformed
// triangle; updates the running closest hit (compute.glsl:432-434).
__device__ __forceinline__ void mt_test(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2, int idx,
                                        float& best, int& best_i) {
    const f3 a = mk(t0.x, t0.y, t0.z);
    const f3 e0 = mk(t0.w, t1.x, t1.y);
    const f3 e1 = mk(t1.z, t1.w, t2.x);
    const f3 n = mk(t2.y, t2.z, t2.w);
    float det = -dot(d, n);
    bool ok = !((det < 1e-10f && det > -1e-10f) || det < 0.0f);
    float inv = 1.0f / det;
    f3 ao = sub(o, a);
    float dst = dot(ao, n) * inv;
    ok = ok && !(dst <= 1e-6f);
    f3 q = cross(d, ao);
    float u = -dot(e1, q) * inv;
    float v = dot(e0, q) * inv;
    ok = ok && !(u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f);
    if (ok && dst < best) {
        best = dst;
        best_i = idx;
    }
}

// Filtered Möller–Trumbore: same decision as mt_test, bit for bit.
//
// With det = -dot(d,n), inv = RN(1/det), the reference updates the closest hit
// iff det >= 1e-10, dst = RN(tnum*inv) > 1e-6, u = RN(-U*inv) >= 0,
// v = RN(V*inv) >= 0, RN(RN(1-u)-v) >= 0 and dst < best, where tnum =
// dot(o-a, n), U = dot(e1, q), V = dot(e0, q), q = cross(d, o-a).  The filter
// F below uses only those exact intermediates (no division) and is false only
// when the update is impossible ("Exactness of the
// filter"): for det > 0, inv > 0, so
//   tnum <= 0                      => dst <= 0                (reject)
//   U > det*2^-60                  => u <= -2^-61 < 0         (reject)
//   V < -det*2^-60                 => v < 0                   (reject)
//   RN(V-U) > RN(det*(1+2^-10))    => w < 0 (u, v >= -2^-60)  (reject)
//   tnum > RN(det*RN(best*(1+2^-10))) => dst >= best          (no update)
// det < 0, det = 0 and NaN fail `tnum > 0 && tnum <= det*bestK`; 0 < det <
// 1e-10 and det = +inf pass F and are rejected by the exact path, as in the
// reference.  Only F-survivors (a few per mille of pairs) pay for the IEEE
// division.
__device__ __forceinline__ void mt_test_filtered(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2, int idx,
                                                 float& best, int& best_i, float& bestK) {
    const f3 a = mk(t0.x, t0.y, t0.z);
    const f3 e0 = mk(t0.w, t1.x, t1.y);
    const f3 e1 = mk(t1.z, t1.w, t2.x);
    const f3 n = mk(t2.y, t2.z, t2.w);
    const float det = -dot(d, n);
    const f3 ao = sub(o, a);
    const float tnum = dot(ao, n);
    const f3 q = cross(d, ao);
    const float U = dot(e1, q);
    const float V = dot(e0, q);
    const float B = det * 0x1p-60f;
    const bool F = (tnum > 0.0f) & (U <= B) & (V >= -B) & ((V - U) <= det * 1.0009765625f) & (tnum <= det * bestK);
    if (F) {
        // compute.glsl:312-327, exactly as written
        if (!((det < 1e-10f && det > -1e-10f) || det < 0.0f)) {
            const float inv = 1.0f / det;
            const float dst = tnum * inv;
            const float u = -U * inv;
            const float v = V * inv;
            if (!(dst <= 1e-6f) && !(u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f) && dst < best) {
                best = dst;
                best_i = idx;
                bestK = best * 1.0009765625f;
            }
        }
    }
}

// Filter part of mt_test_filtered only (branch-free): true when triangle
// {t0,t1,t2} may update the closest hit.
__device__ __forceinline__ bool mt_filter(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2, float bestK) {
    const f3 a = mk(t0.x, t0.y, t0.z);
    const f3 e0 = mk(t0.w, t1.x, t1.y);
    const f3 e1 = mk(t1.z, t1.w, t2.x);
    const f3 n = mk(t2.y, t2.z, t2.w);
    const float det = -dot(d, n);
    const f3 ao = sub(o, a);
    const float tnum = dot(ao, n);
    const f3 q = cross(d, ao);
    const float U = dot(e1, q);
    const float V = dot(e0, q);
    const float B = det * 0x1p-60f;
    return (tnum > 0.0f) & (U <= B) & (V >= -B) & ((V - U) <= det * 1.0009765625f) & (tnum <= det * bestK);
}

// Two-phase sweep over [begin, end) of the LDS array (triangle indices base+k):
// phase 1 evaluates the filter of G triangles branch-free (G independent
// dependency chains, 3G LDS reads in flight), phase 2 runs the exact test
// (mt_test_filtered) for the surviving bits in increasing index order — the
// same update sequence as testing every triangle in order.
// Diagnostic counters of the grouped sweep (STATS variants only).
struct SweepStats {
    uint32_t groups = 0;         // phase-1 groups evaluated (per wave)
    uint32_t groups_exact = 0;   // groups where some lane had a survivor (per wave)
    uint32_t exact_iters = 0;    // phase-2 iterations executed by the wave
    uint32_t lane_survivors = 0; // survivor bits summed over lanes
};

template <int G, bool STATS = false>
__device__ __forceinline__ void sweep_grouped(const f3& o, const f3& d, const float4* lds, int count, int base,
                                              float& best, int& bi, float& bestK, SweepStats* ss = nullptr) {
    int i = 0;
    for (; i + G <= count; i += G) {
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < G; k++) {
            const float4* t = lds + 3 * (i + k);
            m |= (uint32_t)mt_filter(o, d, t[0], t[1], t[2], bestK) << k;
        }
        if constexpr (STATS) {
            ss->groups += 1;
            ss->lane_survivors += __popc(m);
            if (__any(m != 0)) ss->groups_exact += 1;
            uint32_t mm = m;
            while (__any(mm != 0)) {
                ss->exact_iters += 1;
                mm &= mm - 1;
            }
        }
        while (m) {
            const int k = __builtin_ctz(m);
            m &= m - 1;
            const float4* t = lds + 3 * (i + k);
            mt_test_filtered(o, d, t[0], t[1], t[2], base + i + k, best, bi, bestK);
        }
    }
    for (; i < count; i++) {
        const float4* t = lds + 3 * i;
        mt_test_filtered(o, d, t[0], t[1], t[2], base + i, best, bi, bestK);
    }
}

// Scalar-path sweep: the triangle records are wave-uniform, so they are read
// with scalar loads (constant address space -> s_load_dwordx4 into SGPRs,
// through the scalar cache) and fed to the VALU as SGPR operands; no LDS, no
// VGPRs for triangle data.  Same two-phase structure as sweep_grouped.
typedef const __attribute__((address_space(4))) float cfloat;
__device__ __forceinline__ float4 ldc4(cfloat* p) { return make_float4(p[0], p[1], p[2], p[3]); }
template <int G>
__device__ __forceinline__ void sweep_smem(const f3& o, const f3& d, cfloat* tri, int count, float& best, int& bi,
                                           float& bestK) {
    int i = 0;
    for (; i + G <= count; i += G) {
        uint32_t m = 0;
#pragma unroll
        for (int k = 0; k < G; k++) {
            cfloat* t = tri + 12 * (i + k);
            m |= (uint32_t)mt_filter(o, d, ldc4(t), ldc4(t + 4), ldc4(t + 8), bestK) << k;
        }
        while (m) {
            const int k = __builtin_ctz(m);
            m &= m - 1;
            cfloat* t = tri + 12 * (i + k);
            mt_test_filtered(o, d, ldc4(t), ldc4(t + 4), ldc4(t + 8), i + k, best, bi, bestK);
        }
    }
    for (; i < count; i++) {
        cfloat* t = tri + 12 * i;
        mt_test_filtered(o, d, ldc4(t), ldc4(t + 4), ldc4(t + 8), i, best, bi, bestK);
    }
}

// Exact intermediates of one test (phase 1 output, reused by phase 2).
struct MtQ {
    float det, tnum, U, V;
};
__device__ __forceinline__ MtQ mt_quantities(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2) {
    const f3 a = mk(t0.x, t0.y, t0.z);
    const f3 e0 = mk(t0.w, t1.x, t1.y);
    const f3 e1 = mk(t1.z, t1.w, t2.x);
    const f3 n = mk(t2.y, t2.z, t2.w);
    MtQ r;
    r.det = -dot(d, n);
    const f3 ao = sub(o, a);
    r.tnum = dot(ao, n);
    const f3 q = cross(d, ao);
    r.U = dot(e1, q);
    r.V = dot(e0, q);
    return r;
}
__device__ __forceinline__ bool mt_pass(const MtQ& q, float bestK) {
    const float B = q.det * 0x1p-60f;
    return (q.tnum > 0.0f) & (q.U <= B) & (q.V >= -B) & ((q.V - q.U) <= q.det * 1.0009765625f) &
           (q.tnum <= q.det * bestK);
}
// compute.glsl:312-327 on the phase-1 intermediates (exactly the reference arithmetic).
__device__ __forceinline__ void mt_exact(const MtQ& q, int idx, float& best, int& bi, float& bestK) {
    if (!((q.det < 1e-10f && q.det > -1e-10f) || q.det < 0.0f)) {
        const float inv = 1.0f / q.det;
        const float dst = q.tnum * inv;
        const float u = -q.U * inv;
        const float v = q.V * inv;
        if (!(dst <= 1e-6f) && !(u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f) && dst < best) {
            best = dst;
            bi = idx;
            bestK = best * 1.0009765625f;
        }
    }
}

// Masked two-phase sweep: phase 1 computes the intermediates and the filter of
// G triangles (the G predicates stay wave lane-masks in SGPR pairs, no
// per-lane bit packing); phase 2 runs mt_exact under each mask in index order
// (skipped by a scalar branch when the mask is empty).  SMEM selects the
// scalar-load path for the triangle records instead of LDS.
template <int G, bool SMEM>
__device__ __forceinline__ void sweep_masked(const f3& o, const f3& d, const float4* lds, const float* gtri,
                                             int count, int base, float& best, int& bi, float& bestK) {
    int i = 0;
    for (; i + G <= count; i += G) {
        MtQ q[G];
        bool f[G];
#pragma unroll
        for (int k = 0; k < G; k++) {
            float4 t0, t1, t2;
            if constexpr (SMEM) {
                cfloat* t = (cfloat*)gtri + 12 * (i + k);
                t0 = ldc4(t);
                t1 = ldc4(t + 4);
                t2 = ldc4(t + 8);
            } else {
                const float4* t = lds + 3 * (i + k);
                t0 = t[0];
                t1 = t[1];
                t2 = t[2];
            }
            q[k] = mt_quantities(o, d, t0, t1, t2);
            f[k] = mt_pass(q[k], bestK);
        }
#pragma unroll
        for (int k = 0; k < G; k++)
            if (f[k]) mt_exact(q[k], base + i + k, best, bi, bestK);
    }
    for (; i < count; i++) {
        float4 t0, t1, t2;
        if constexpr (SMEM) {
            cfloat* t = (cfloat*)gtri + 12 * i;
            t0 = ldc4(t);
            t1 = ldc4(t + 4);
            t2 = ldc4(t + 8);
        } else {
            const float4* t = lds + 3 * i;
            t0 = t[0];
            t1 = t[1];
            t2 = t[2];
        }
        const MtQ q = mt_quantities(o, d, t0, t1, t2);
        if (mt_pass(q, bestK)) mt_exact(q, base + i, best, bi, bestK);
    }
}

// Ballot sweep: phase 1 computes G filters and turns them into wave masks
// (__ballot); phase 2 runs only when any mask is set, one scalar branch per G
// triangles in the common case.
__device__ __forceinline__ void load_tri_smem(const float* gtri, int i, float4& t0, float4& t1, float4& t2) {
    cfloat* t = (cfloat*)gtri + 12 * i;
    t0 = ldc4(t);
    t1 = ldc4(t + 4);
    t2 = ldc4(t + 8);
}
template <int G>
__device__ __forceinline__ void sweep_ballot(const f3& o, const f3& d, const float* gtri, int count, float& best,
                                             int& bi, float& bestK) {
    int i = 0;
    const unsigned long long me = 1ull << lane_id();
    for (; i + G <= count; i += G) {
        MtQ q[G];
        unsigned long long m[G], any = 0;
#pragma unroll
        for (int k = 0; k < G; k++) {
            float4 t0, t1, t2;
            load_tri_smem(gtri, i + k, t0, t1, t2);
            q[k] = mt_quantities(o, d, t0, t1, t2);
            m[k] = __ballot(mt_pass(q[k], bestK));
            any |= m[k];
        }
        if (__builtin_expect(any != 0, 0)) {
#pragma unroll
            for (int k = 0; k < G; k++)
                if (m[k] & me) mt_exact(q[k], i + k, best, bi, bestK);
        }
    }
    for (; i < count; i++) {
        float4 t0, t1, t2;
        load_tri_smem(gtri, i, t0, t1, t2);
        const MtQ q = mt_quantities(o, d, t0, t1, t2);
        if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
    }
}

// VALU-only form of mt_pass: the five conditions as signed slacks whose
// minimum is >= 0 exactly when all hold (RN(x - y) has the sign of x - y;
// tnum > 0 as tnum - 2^-149 >= 0).  Conservative under flush-to-zero and NaN
// as well (both can only make it pass more).
__device__ __forceinline__ bool mt_pass_min(const MtQ& q, float bestK) {
    const float B = q.det * 0x1p-60f;
    const float D = q.det * 1.0009765625f;
    const float K = q.det * bestK;
    const float m1 = fminf(fminf(B - q.U, q.V + B), D - (q.V - q.U));
    const float m2 = fminf(K - q.tnum, q.tnum - 0x1p-149f);
    return fminf(m1, m2) >= 0.0f;
}
template <int G>
__device__ __forceinline__ void sweep_minfilter(const f3& o, const f3& d, const float* gtri, int count, float& best,
                                                int& bi, float& bestK) {
    int i = 0;
    const unsigned long long me = 1ull << lane_id();
    for (; i + G <= count; i += G) {
        MtQ q[G];
        unsigned long long m[G], any = 0;
#pragma unroll
        for (int k = 0; k < G; k++) {
            float4 t0, t1, t2;
            load_tri_smem(gtri, i + k, t0, t1, t2);
            q[k] = mt_quantities(o, d, t0, t1, t2);
            m[k] = __ballot(mt_pass_min(q[k], bestK));
            any |= m[k];
        }
        if (__builtin_expect(any != 0, 0)) {
#pragma unroll
            for (int k = 0; k < G; k++)
                if (m[k] & me) mt_exact(q[k], i + k, best, bi, bestK);
        }
    }
    for (; i < count; i++) {
        float4 t0, t1, t2;
        load_tri_smem(gtri, i, t0, t1, t2);
        const MtQ q = mt_quantities(o, d, t0, t1, t2);
        if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
    }
}

// Lean masked sweep: like sweep_masked, but phase 1 keeps ONLY the G filter
// lane-masks (SGPRs) live; phase 2 (entered for ~5% of groups on config B)
// reloads the surviving triangle and recomputes its intermediates.  Frees the
// 4*G VGPRs sweep_masked holds across the group.
__device__ __forceinline__ void load_tri(const float4* lds, const float* gtri, bool smem, int i, float4& t0,
                                         float4& t1, float4& t2) {
    if (smem) {
        cfloat* t = (cfloat*)gtri + 12 * i;
        t0 = ldc4(t);
        t1 = ldc4(t + 4);
        t2 = ldc4(t + 8);
    } else {
        const float4* t = lds + 3 * i;
        t0 = t[0];
        t1 = t[1];
        t2 = t[2];
    }
}
template <int G, bool SMEM>
__device__ __forceinline__ void sweep_lean(const f3& o, const f3& d, const float4* lds, const float* gtri, int count,
                                           int base, float& best, int& bi, float& bestK) {
    int i = 0;
    for (; i + G <= count; i += G) {
        bool f[G];
#pragma unroll
        for (int k = 0; k < G; k++) {
            float4 t0, t1, t2;
            load_tri(lds, gtri, SMEM, i + k, t0, t1, t2);
            f[k] = mt_pass(mt_quantities(o, d, t0, t1, t2), bestK);
        }
#pragma unroll
        for (int k = 0; k < G; k++) {
            if (f[k]) {
                // opaque index: force a reload + recompute instead of keeping
                // phase 1's intermediates live across the group
                int j = i + k;
                asm volatile("" : "+s"(j));
                float4 t0, t1, t2;
                load_tri(lds, gtri, SMEM, j, t0, t1, t2);
                mt_exact(mt_quantities(o, d, t0, t1, t2), base + j, best, bi, bestK);
            }
        }
    }
    for (; i < count; i++) {
        float4 t0, t1, t2;
        load_tri(lds, gtri, SMEM, i, t0, t1, t2);
        const MtQ q = mt_quantities(o, d, t0, t1, t2);
        if (mt_pass(q, bestK)) mt_exact(q, base + i, best, bi, bestK);
    }
}

// Cooperative closest hit for the drain phase: all 64 lanes sweep ONE ray
// (lane l tests triangles l, l+64, ... in increasing order with its own
// running best) and the wave reduces (dst, index) lexicographically.  The
// result equals the sequential strict-< scan: the minimum distance, and among
// exact ties the lowest index.  Triangle records are read from `tris`
// (LDS or global) with per-lane addresses.
__device__ __forceinline__ void coop_closest(const f3& o, const f3& d, const float4* tris, int n, float& best_out,
                                             int& bi_out) {
    const int lane = (int)lane_id();
    float best = 1e38f, bestK = 1e38f * 1.0009765625f;
    int bi = -1;
    for (int i = lane; i < n; i += 64) {
        const float4* t = tris + 3 * i;
        const MtQ q = mt_quantities(o, d, t[0], t[1], t[2]);
        if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        const bool take = (ob < best) || (ob == best && oi >= 0 && (bi < 0 || oi < bi));
        if (take) {
            best = ob;
            bi = oi;
        }
    }
    best_out = best;
    bi_out = bi;
}

// Team sweep (tail mode): the n live rays of a wave each get a team of
// k = 64 / 2^ceil(log2 n) lanes; member j of a team tests triangles j, j+k,
// j+2k, ... of its ray (vector loads: the k members read k consecutive
// records, every team the same ones), then the team reduces (dst, index)
// lexicographically — the sequential strict `dst < best` scan's result.  A
// segment of every live ray costs N/k tests per lane instead of N, so the
// last rays of a launch (and small per-GPU slabs) finish up to k times sooner.
// Returns the closest hit of the calling lane's own ray (live lanes).
__device__ __forceinline__ void team_closest(const f3& lo, const f3& ld, const float4* tris, int n_tris,
                                             unsigned long long act, float& best_out, int& bi_out) {
    const int n = __popcll(act);
    const int lg = n <= 1 ? 0 : 32 - __builtin_clz((unsigned)(n - 1));
    const int k = 64 >> lg;
    const int me = (int)lane_id();
    const int t = me / k, j = me - t * k;
    // the t-th live lane of the wave: the lane whose live-rank is t
    int leader = 0;
    {
        unsigned long long m = act;
        for (int r = 0; r < t && m; r++) m &= m - 1;
        leader = m ? __builtin_ctzll(m) : 0;
    }
    const bool member = t < n;
    const f3 o = mk(__shfl(lo.x, leader), __shfl(lo.y, leader), __shfl(lo.z, leader));
    const f3 d = mk(__shfl(ld.x, leader), __shfl(ld.y, leader), __shfl(ld.z, leader));
    float best = 1e38f, bestK = 1e38f * 1.0009765625f;
    int bi = -1;
    if (member) {
        for (int i = j; i < n_tris; i += k) {
            const float4* tp = tris + 3 * i;
            const MtQ q = mt_quantities(o, d, tp[0], tp[1], tp[2]);
            if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
        }
    }
    for (int off = 1; off < k; off <<= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        const bool take = (ob < best) || (ob == best && oi >= 0 && (bi < 0 || oi < bi));
        if (take) {
            best = ob;
            bi = oi;
        }
    }
    // each live lane reads its team's result (team index = its live rank)
    const int src = (int)lanes_below(act) * k;
    best_out = __shfl(best, src);
    bi_out = __shfl(bi, src);
}

template <int MT>
__device__ __forceinline__ void mt_dispatch(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2, int idx,
                                            float& best, int& best_i, float& bestK) {
    if constexpr (MT == 0)
        mt_test(o, d, t0, t1, t2, idx, best, best_i);
    else
        mt_test_filtered(o, d, t0, t1, t2, idx, best, best_i, bestK);
}

// Per-lane path state, kept small (VGPRs decide the waves per SIMD): the
// camera end point is recomputed per ray and the frame sums go straight to the
// accumulators in HBM (one read-modify-write per pixel-frame).
struct Lane {
    int st;
    uint32_t item;
    int x, y;
    uint32_t frame;  // frames done for this item
    uint32_t seed;
    int ray;
    int bounce;
    bool inside;
    f3 o, d, rayColor, incoming, colorCum;
    uint32_t segs;
    uint32_t t0;  // item start (s_memtime low bits), for the cost map
};

__device__ __forceinline__ void end_path(Lane& L, const RenderParams& p);

// Phase A: bring every lane to ST_TRACE or ST_DONE (wave-collective).
__device__ __forceinline__ void advance(Lane& L, const RenderParams& p) {
    for (;;) {
        const bool need = L.st == ST_NEED_ITEM;
        const unsigned long long m = __ballot(need);
        if (m) {
            unsigned long long base = 0;
            if (lane_id() == 0) base = atomicAdd(p.item_counter, (unsigned long long)__popcll(m));
            base = __shfl(base, 0);
            if (need) {
                unsigned long long it = base + lanes_below(m);
                if (it < p.n_items) {
                    // frame_split: item = frame * n_pix + pixel (frame-major), so the
                    // last items of a launch are single pixel-frames
                    // n_items < 2^32 (checked on the host): 32-bit arithmetic
                    const uint32_t it32 = (uint32_t)it, np32 = (uint32_t)p.n_pix;
                    const uint32_t f = p.frame_split ? it32 / np32 : 0u;
                    L.item = it32 - f * np32;
                    if (p.order && L.item < p.n_runs * 64u) L.item = p.order[L.item >> 6] * 64u + (L.item & 63u);
                    L.t0 = (uint32_t)__builtin_amdgcn_s_memtime();
                    int lr = (int)(L.item / (uint32_t)p.W);
                    L.x = (int)(L.item - (uint32_t)lr * (uint32_t)p.W);
                    L.y = shard_row(lr, p.tile_rows, p.rank, p.nranks);
                    L.frame = f;
                    L.st = ST_NEW_FRAME;
                } else {
                    L.st = ST_DONE;
                }
            }
        }
        if (L.st == ST_NEW_FRAME) {
            // compute.glsl:662-670
            const uint32_t f = p.frame_begin + L.frame;
            L.seed = (uint32_t)L.x + (uint32_t)L.y * (uint32_t)p.W + f * 968824447u;
            L.colorCum = mk(0.0f, 0.0f, 0.0f);
            L.ray = 0;
            L.st = ST_NEW_RAY;
        }
        if (L.st == ST_NEW_RAY) {
            // compute.glsl:665-670 (endPoint, recomputed per ray) and :685-690
            const float px = (float)(L.x * 2 - p.W) / (float)p.W;
            const float py = (float)(L.y * 2 - p.H) / (float)p.H;
            const f3 endPoint =
                add(add(add(ld3(p.cam), ld3(p.vpFront)), muls(ld3(p.vpRight), px)), muls(ld3(p.vpUp), py));
            float ang = rnd(L.seed);
            float cs = rt2pm_cosf(ang), sn = rt2pm_sinf(ang);
            L.o = add(add(ld3(p.cam), muls(ld3(p.defR), cs)), muls(ld3(p.defU), sn));
            float jr = -0.5f + (0.5f - -0.5f) * rnd(L.seed);
            float ju = -0.5f + (0.5f - -0.5f) * rnd(L.seed);
            f3 endJ = add(add(endPoint, muls(ld3(p.pixR), jr)), muls(ld3(p.pixU), ju));
            L.d = normalize(sub(endJ, L.o));
            L.inside = false;
            L.rayColor = mk(1.0f, 1.0f, 1.0f);
            L.incoming = mk(0.0f, 0.0f, 0.0f);
            L.bounce = 0;
            L.st = ST_TRACE;
            if (p.maxBounce <= 0) end_path(L, p);  // trace() returns 0 without tracing
        }
        if (!__any(L.st != ST_TRACE && L.st != ST_DONE)) break;
    }
}

// End of a path: colorCumulative += trace(...) (compute.glsl:692); next ray,
// or end of the frame (compute.glsl:696-700 + the screenshot accumulation).
__device__ __forceinline__ void end_path(Lane& L, const RenderParams& p) {
    L.colorCum = add(L.colorCum, L.incoming);
    L.ray += 1;
    if (L.ray < p.R) {
        L.st = ST_NEW_RAY;
        return;
    }
    f3 c = divs(L.colorCum, (float)p.R);
    c = mk(srgb1(aces1(c.x)), srgb1(aces1(c.y)), srgb1(aces1(c.z)));
    if (p.frame_split) {  // frame_accumulate adds the frames in order afterwards
        p.frame_buf[(size_t)L.frame * p.n_pix + L.item] = make_float4(c.x, c.y, c.z, 0.0f);
        if (p.cost_out) p.cost_out[L.item] = (uint32_t)__builtin_amdgcn_s_memtime() - L.t0;
        L.st = ST_NEED_ITEM;
        return;
    }
    // accumulate this frame in frame order: acc = acc + colour
    const float4 a = p.accum[L.item];
    p.accum[L.item] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
    if (p.accum8) {
        // GL float -> unorm8, round to nearest (GL 4.3 §2.3.5.2)
        const uint4 q = p.accum8[L.item];
        p.accum8[L.item] = make_uint4(q.x + (uint32_t)(clampf(c.x, 0.0f, 1.0f) * 255.0f + 0.5f),
                                      q.y + (uint32_t)(clampf(c.y, 0.0f, 1.0f) * 255.0f + 0.5f),
                                      q.z + (uint32_t)(clampf(c.z, 0.0f, 1.0f) * 255.0f + 0.5f), 0u);
    }
    L.frame += 1;
    L.st = L.frame < p.frame_count ? ST_NEW_FRAME : ST_NEED_ITEM;
    if (L.st == ST_NEED_ITEM && p.cost_out) p.cost_out[L.item] = (uint32_t)__builtin_amdgcn_s_memtime() - L.t0;
}

// texture(sampler2D, uv) with GL_LINEAR (no mipmaps) + GL_REPEAT, GL 4.3
// §8.14.2: u = s*w - 1/2, i0 = wrap(floor(u)), alpha = frac(u) (likewise v),
// tau = (1-a)(1-b) T00 + a(1-b) T10 + (1-a)b T01 + ab T11 with unorm8
// texels c/255.  Pinned in binary32, evaluated as written (oracle: same).
__device__ __forceinline__ int tex_wrap(float f, int n) {
    const int i = (f >= -1073741824.0f && f <= 1073741824.0f) ? (int)f : 0;  // NaN / huge -> 0
    const int r = i % n;
    return r < 0 ? r + n : r;
}
__device__ __forceinline__ f3 tex_sample(const RenderParams& p, int t, float s, float tc) {
    const int4 dsc = p.tex_desc[t];
    const int w = dsc.x, h = dsc.y;
    const unsigned long long off = (unsigned long long)(uint32_t)dsc.z | (unsigned long long)(uint32_t)dsc.w << 32;
    const float u = s * (float)w - 0.5f;
    const float v = tc * (float)h - 0.5f;
    const float fu = floorf(u), fv = floorf(v);
    const float a = u - fu, b = v - fv;
    const int i0 = tex_wrap(fu, w), j0 = tex_wrap(fv, h);
    const int i1 = i0 + 1 == w ? 0 : i0 + 1, j1 = j0 + 1 == h ? 0 : j0 + 1;
    const uchar4* T = p.texels + off;
    const uchar4 t00 = T[(size_t)j0 * w + i0], t10 = T[(size_t)j0 * w + i1];
    const uchar4 t01 = T[(size_t)j1 * w + i0], t11 = T[(size_t)j1 * w + i1];
    const float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
#define RT2_TEXCH(c) \
    (w00 * ((float)t00.c / 255.0f) + w10 * ((float)t10.c / 255.0f) + w01 * ((float)t01.c / 255.0f) + \
     w11 * ((float)t11.c / 255.0f))
    return mk(RT2_TEXCH(x), RT2_TEXCH(y), RT2_TEXCH(z));
#undef RT2_TEXCH
}

// getTriangleTextureColor (compute.glsl:342-368) at the closest hit of ray
// (o, d) on triangle bi: barycentrics recomputed with the test's own
// arithmetic (rayTriangleIntersect :322-338, w = 1 - u - v), uv = aTex*u +
// bTex*v + cTex*w.
__device__ __forceinline__ f3 texture_color(const RenderParams& p, int tex_index, int bi, const f3& o, const f3& d) {
    if (tex_index < 0 || tex_index >= p.num_textures) return mk(0.0f, 0.0f, 0.0f);
    if (tex_index > 4) return mk(1.0f, 0.0f, 1.0f);
    if (tex_index >= p.n_tex) return mk(0.0f, 0.0f, 0.0f);  // unit with no texture bound
    const MtQ q = mt_quantities(o, d, p.tri[3 * bi], p.tri[3 * bi + 1], p.tri[3 * bi + 2]);
    const float inv = 1.0f / q.det;
    const float u = -q.U * inv;
    const float v = q.V * inv;
    const float w = 1.0f - u - v;
    const rt2_triangle& t = p.raw[bi];
    const float s = t.aTex.x * u + t.bTex.x * v + t.cTex.x * w;
    const float tc = t.aTex.y * u + t.bTex.y * v + t.cTex.y * w;
    return tex_sample(p, tex_index, s, tc);
}

// Phase C: scatter at the closest hit (compute.glsl:485-559).
__device__ __forceinline__ void shade(Lane& L, const RenderParams& p, float best, int bi) {
    if (bi >= 0) {
        const int mi = p.tri_mtl[bi];
        // the texture lookup first, while little else is live (it needs the
        // segment's own origin, which the scatter below overwrites)
        f3 tex = mk(0.0f, 0.0f, 0.0f);
        if (p.mats[mi].materialType == RT2_TEXTURE) tex = texture_color(p, p.mats[mi].textureIndex, bi, L.o, L.d);
        const float4 t2 = p.tri[3 * bi + 2];
        const f3 normal = normalize(mk(t2.y, t2.z, t2.w));  // normalize(cross01), compute.glsl:331
        const f3 hitPoint = add(L.o, muls(L.d, best));      // compute.glsl:330
        const rt2_material m = p.mats[mi];
        if (m.materialType != RT2_GLASS)
            L.o = sub(hitPoint, muls(muls(L.d, best), -1e-3f));
        else
            L.o = add(hitPoint, muls(muls(L.d, best), -1e-3f));
        f3 atten = mk(0.0f, 0.0f, 0.0f);
        const f3 prevDir = L.d;
        switch (m.materialType) {
        case RT2_DIFFUSE:
        case RT2_TEXTURE:
            L.d = normalize(add(normal, rnd_dir(L.seed)));
            atten = m.materialType == RT2_DIFFUSE ? xyz4(m.color) : tex;
            break;
        case RT2_SPECULAR: {
            f3 diffuseDir = normalize(add(normal, rnd_dir(L.seed)));
            f3 specDir = reflect(L.d, normal);
            bool isSpec = m.specularProbability > rnd(L.seed);
            L.d = mixs(diffuseDir, specDir, isSpec ? m.smoothness : 0.0f);
            atten = isSpec ? mk(1.0f, 1.0f, 1.0f) : xyz4(m.color);
            break;
        }
        case RT2_LIGHT: {
            f3 emitted = muls(xyz4(m.emissionColor), m.emissionStrength);
            L.incoming = add(L.incoming, mul(emitted, L.rayColor));
            end_path(L, p);
            return;
        }
        case RT2_CHECKER: {
            L.d = normalize(add(normal, rnd_dir(L.seed)));
            float s = m.checkerScale;
            bool black = false;
            if (s > 0.0f) {
                float sum = floorf(L.o.x * s) + floorf(L.o.y * s) + floorf(L.o.z * s);
                float md = sum - 2.0f * floorf(sum / 2.0f);
                black = md == 0.0f;
            }
            atten = black ? mk(0.0f, 0.0f, 0.0f) : mk(1.0f, 1.0f, 1.0f);
            break;
        }
        case RT2_GLASS: {
            float eta = L.inside ? m.refractiveIndex : 1.0f / m.refractiveIndex;
            bool refr;
            L.d = refract_(L.d, normal, eta, refr);
            L.inside = refr != L.inside;
            atten = xyz4(m.color);
            break;
        }
        default:  // GLASS_HIGHLIGHT and unknown types: trace() returns magenta
            L.incoming = mk(1.0f, 0.0f, 1.0f);
            end_path(L, p);
            return;
        }
        if (m.isEdgeHighlight && L.bounce > 1)
            L.d = prevDir;
        else
            L.rayColor = mul(L.rayColor, atten);
        float pr = fmaxf(L.rayColor.x, fmaxf(L.rayColor.y, L.rayColor.z));
        if (rnd(L.seed) > pr) {
            end_path(L, p);
            return;
        }
        L.rayColor = muls(L.rayColor, 1.0f / pr);
        if (L.bounce >= p.maxBounce) end_path(L, p);
    } else {
        if (p.envLight) L.incoming = add(L.incoming, mul(sky(L.d), L.rayColor));
        end_path(L, p);
    }
}

__device__ __forceinline__ void lane_init(Lane& L) {
    L.st = ST_NEED_ITEM;
    L.item = 0;
    L.x = L.y = 0;
    L.frame = 0;
    L.seed = 0;
    L.ray = 0;
    L.bounce = 0;
    L.inside = false;
    L.o = L.d = L.rayColor = L.incoming = L.colorCum = mk(0.0f, 0.0f, 0.0f);
    L.segs = 0;
    L.t0 = 0;
}

__device__ __forceinline__ void flush_counters(const Lane& L, const RenderParams& p) {
    unsigned long long s = L.segs;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane_id() == 0) atomicAdd(p.seg_counter, s);
}

// RESIDENT: all triangles in LDS, waves independent after the initial load.
template <int BLOCK, int MT, int UNROLL>
__global__ __launch_bounds__(BLOCK) void render_resident(RenderParams p) {
    // UNROLL == 0 on a grouped variant = diagnostic build with sweep counters
    constexpr bool kStats = MT >= 2 && UNROLL == 0;
    SweepStats ss;
    extern __shared__ float4 lds[];
    const int n4 = 3 * p.n_tris;
    for (int i = threadIdx.x; i < n4; i += BLOCK) lds[i] = p.tri[i];
    __syncthreads();

    Lane L;
    lane_init(L);
    for (;;) {
        advance(L, p);
        if (!__any(L.st == ST_TRACE)) break;
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            float best = 1e38f, bestK = 1e38f * 1.0009765625f;
            int bi = -1;
            const f3 o = L.o, d = L.d;
            if constexpr (MT >= 200) {
                sweep_lean<MT - 200, false>(o, d, lds, nullptr, p.n_tris, 0, best, bi, bestK);
            } else if constexpr (MT >= 100) {
                sweep_masked<MT - 100, false>(o, d, lds, nullptr, p.n_tris, 0, best, bi, bestK);
            } else if constexpr (MT >= 2) {
                sweep_grouped<MT, kStats>(o, d, lds, p.n_tris, 0, best, bi, bestK, &ss);
            } else {
#pragma unroll UNROLL
                for (int i = 0; i < p.n_tris; i++) {
                    mt_dispatch<MT>(o, d, lds[3 * i], lds[3 * i + 1], lds[3 * i + 2], i, best, bi, bestK);
                }
            }
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
    if constexpr (kStats) {
        unsigned long long surv = ss.lane_survivors;
        for (int off = 32; off > 0; off >>= 1) surv += __shfl_xor(surv, off);
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();  // 100 MHz
        if (lane_id() == 0) {
            atomicAdd(p.seg_counter + 1, (unsigned long long)ss.groups);
            atomicAdd(p.seg_counter + 2, (unsigned long long)ss.groups_exact);
            atomicAdd(p.seg_counter + 3, (unsigned long long)ss.exact_iters);
            atomicAdd(p.seg_counter + 4, surv);
            // wave finish-time spread: [6] = earliest wave end, [5] = latest (ticks of 10 ns)
            atomicMin(p.seg_counter + 5, t_end);
            atomicMax(p.seg_counter + 4 + 2, t_end);
        }
    }
}

// TILED: triangles streamed through LDS; the workgroup sweeps in lockstep.
template <int BLOCK, int MT, int UNROLL>
__global__ __launch_bounds__(BLOCK) void render_tiled(RenderParams p) {
    extern __shared__ float4 lds[];
    __shared__ int block_any;
    Lane L;
    lane_init(L);
    const int T = p.tile_tris;
    for (;;) {
        advance(L, p);
        if (threadIdx.x == 0) block_any = 0;
        __syncthreads();
        if (L.st == ST_TRACE) block_any = 1;
        __syncthreads();
        if (!block_any) break;
        const bool tracing = L.st == ST_TRACE;
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        const f3 o = L.o, d = L.d;
        for (int base = 0; base < p.n_tris; base += T) {
            const int cnt = min(T, p.n_tris - base);
            __syncthreads();
            for (int i = threadIdx.x; i < 3 * cnt; i += BLOCK) lds[i] = p.tri[3 * base + i];
            __syncthreads();
            if (tracing) {
                if constexpr (MT >= 100) {
                    sweep_masked<MT - 100, false>(o, d, lds, nullptr, cnt, base, best, bi, bestK);
                } else if constexpr (MT >= 2) {
                    sweep_grouped<MT>(o, d, lds, cnt, base, best, bi, bestK);
                } else {
#pragma unroll UNROLL
                    for (int i = 0; i < cnt; i++)
                        mt_dispatch<MT>(o, d, lds[3 * i], lds[3 * i + 1], lds[3 * i + 2], base + i, best, bi, bestK);
                }
            }
        }
        if (tracing) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
}

// SMEM: no LDS; triangles reach the VALU through the scalar cache (sweep_smem).
// COOP > 0: drain mode — once the item pool is exhausted (some lane is DONE)
// and at most COOP lanes of the wave still trace, each live ray's closest hit
// is computed by the whole wave (coop_closest), one ray at a time.
template <int BLOCK, int G, int COOP, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void render_smem(RenderParams p) {
    cfloat* tri = (cfloat*)p.tri;
    Lane L;
    lane_init(L);
    for (;;) {
        advance(L, p);
        const unsigned long long act = __ballot(L.st == ST_TRACE);
        if (!act) break;
        if (COOP >= 100 && __popcll(act) <= (unsigned)(COOP - 100) && __any(L.st == ST_DONE)) {
            float b;
            int bidx;
            team_closest(L.o, L.d, p.tri, p.n_tris, act, b, bidx);
            if (L.st == ST_TRACE) {
                L.bounce += 1;
                L.segs += 1;
                shade(L, p, b, bidx);
            }
            continue;
        }
        if (COOP > 0 && COOP < 100 && __popcll(act) <= (unsigned)COOP && __any(L.st == ST_DONE)) {
            float mybest = 1e38f;
            int mybi = -1;
            unsigned long long m = act;
            while (m) {
                const int j = __builtin_ctzll(m);
                m &= m - 1;
                const f3 oj = mk(__shfl(L.o.x, j), __shfl(L.o.y, j), __shfl(L.o.z, j));
                const f3 dj = mk(__shfl(L.d.x, j), __shfl(L.d.y, j), __shfl(L.d.z, j));
                float b;
                int bidx;
                coop_closest(oj, dj, p.tri, p.n_tris, b, bidx);
                if ((int)lane_id() == j) {
                    mybest = b;
                    mybi = bidx;
                }
            }
            if (L.st == ST_TRACE) {
                L.bounce += 1;
                L.segs += 1;
                shade(L, p, mybest, mybi);
            }
            continue;
        }
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            float best = 1e38f, bestK = 1e38f * 1.0009765625f;
            int bi = -1;
            const f3 o = L.o, d = L.d;
            if constexpr (G >= 400)
                sweep_minfilter<G - 400>(o, d, (const float*)p.tri, p.n_tris, best, bi, bestK);
            else if constexpr (G >= 300)
                sweep_ballot<G - 300>(o, d, (const float*)p.tri, p.n_tris, best, bi, bestK);
            else if constexpr (G >= 200)
                sweep_lean<G - 200, true>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
            else if constexpr (G >= 100)
                sweep_masked<G - 100, true>(o, d, nullptr, p.tri ? (const float*)p.tri : nullptr, p.n_tris, 0, best,
                                            bi, bestK);
            else
                sweep_smem<G>(o, d, tri, p.n_tris, best, bi, bestK);
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
}

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
template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void render_bvh(RenderParams p) {
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

template <int BLOCK, int THRESH>
__global__ __launch_bounds__(BLOCK) void render_bvh2(RenderParams p) {
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
    float dA, dB;
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
        bool amb = (near_tie(aMin, aMax) & !flatA) | (near_tie(bMin, bMax) & !flatB);
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
        if (mt_pass(q, T.bestK)) mt_exact(q, i, T.best, T.bi, T.bestK);
    }
}

template <int BLOCK, int THRESH, int DIV, int WPE, int DIAG = 0>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void render_bvh3(RenderParams p) {
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

// ---------------------------------------------------------------------------
// traceBasic preview (compute.glsl:565-645 + main's basicShading branch,
// :672-678): one deterministic ray per pixel, no RNG, no tonemap.  One thread
// per pixel; the closest hit is the brute-force masked sweep (triangles through
// the scalar cache) or the BVH walk, whichever traversal the scene selects.
// ---------------------------------------------------------------------------
template <int BLOCK, bool BVH>
__device__ __forceinline__ void closest_any(const RenderParams& p, const f3& o, const f3& d, int* stack, float& best,
                                            int& bi, uint32_t& tests) {
    best = 1e38f;
    bi = -1;
    if constexpr (BVH) {
        uint32_t visits = 0;
        closest_bvh<BLOCK>(o, d, p.nodes, p.tri, stack, p.stack_slots, best, bi, tests, visits);
    } else {
        float bestK = 1e38f * 1.0009765625f;
        sweep_masked<8, true>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
    }
}

template <int BLOCK, bool BVH>
__device__ __forceinline__ f3 trace_basic(const RenderParams& p, f3 o, f3 d, int* stack, uint32_t& segs,
                                          uint32_t& tests) {
    f3 cum = mk(0.0f, 0.0f, 0.0f);
    bool inside = false;  // `Ray ray;` leaves insideGlass undefined (:674); false here and in the oracle
    int bc = 0;
    while (bc < p.maxBounce) {
        bc++;
        segs++;
        float best;
        int bi;
        closest_any<BLOCK, BVH>(p, o, d, stack, best, bi, tests);
        if (bi < 0) {
            cum = add(cum, sky(d));
            break;
        }
        const float4 t2 = p.tri[3 * bi + 2];
        const f3 normal = normalize(mk(t2.y, t2.z, t2.w));
        const f3 hitPoint = add(o, muls(d, best));
        const rt2_material mm = p.mats[p.tri_mtl[bi]];
        const f3 tex = mm.materialType == RT2_TEXTURE ? texture_color(p, mm.textureIndex, bi, o, d)
                                                      : mk(0.0f, 0.0f, 0.0f);
        o = sub(hitPoint, muls(normal, 1e-4f));  // :579
        const rt2_material m = p.mats[p.tri_mtl[bi]];
        switch (m.materialType) {
        case RT2_SPECULAR:
            cum = add(cum, xyz4(m.color));
            d = reflect(d, normal);
            break;
        case RT2_DIFFUSE:
        case RT2_TEXTURE:
        case RT2_CHECKER: {
            f3 color;
            if (m.materialType == RT2_TEXTURE) {
                color = tex;
            } else if (m.materialType == RT2_DIFFUSE) {
                color = xyz4(m.color);
            } else {
                const float s = m.checkerScale;
                bool black = false;
                if (s > 0.0f) {
                    const float sum = floorf(o.x * s) + floorf(o.y * s) + floorf(o.z * s);
                    black = sum - 2.0f * floorf(sum / 2.0f) == 0.0f;
                }
                color = black ? mk(0.0f, 0.0f, 0.0f) : mk(1.0f, 1.0f, 1.0f);
            }
            cum = add(cum, color);
            if (p.basicShadow) {  // :614-621, shadow ray toward the preview light
                const f3 toLight = normalize(sub(ld3(p.light), hitPoint));
                segs++;
                float b2;
                int bi2;
                closest_any<BLOCK, BVH>(p, o, toLight, stack, b2, bi2, tests);
                return divs(bi2 >= 0 ? divs(cum, 5.0f) : cum, (float)bc);
            }
            return divs(cum, (float)bc);
        }
        case RT2_LIGHT: {  // normalizeColor, :462-470
            const f3 e = xyz4(m.emissionColor);
            const float mx = fmaxf(fmaxf(e.x, e.y), e.z);
            return mx > 1.0f ? divs(e, mx) : e;
        }
        case RT2_GLASS: {
            const float eta = inside ? m.refractiveIndex : 1.0f / m.refractiveIndex;
            bool refr;
            d = refract_(d, normal, eta, refr);
            inside = refr != inside;
            cum = xyz4(m.color);
            break;
        }
        case RT2_GLASS_HIGHLIGHT:  // `if (bounceCount == 0)` never holds after bounceCount++
            break;
        default:
            return mk(1.0f, 0.0f, 1.0f);
        }
    }
    return divs(cum, (float)bc);
}

template <int BLOCK, bool BVH>
__global__ __launch_bounds__(BLOCK) void render_basic(RenderParams p) {
    extern __shared__ int basic_stack[];
    uint32_t segs = 0, tests = 0;
    const unsigned long long it = (unsigned long long)blockIdx.x * BLOCK + threadIdx.x;
    if (it < p.n_items) {
        const uint32_t item = (uint32_t)it;
        const int lr = (int)(item / (uint32_t)p.W);
        const int x = (int)(item - (uint32_t)lr * (uint32_t)p.W);
        const int y = shard_row(lr, p.tile_rows, p.rank, p.nranks);
        const float px = (float)(x * 2 - p.W) / (float)p.W;
        const float py = (float)(y * 2 - p.H) / (float)p.H;
        const f3 dir = normalize(add(add(ld3(p.vpFront), muls(ld3(p.vpRight), px)), muls(ld3(p.vpUp), py)));
        // frame-independent: traced once, accumulated frame_count times in order
        const f3 c = trace_basic<BLOCK, BVH>(p, ld3(p.cam), dir, basic_stack, segs, tests);
        float4 a = p.accum[item];
        for (uint32_t f = 0; f < p.frame_count; f++) a = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
        p.accum[item] = a;
        if (p.accum8) {
            const uint32_t qx = (uint32_t)(clampf(c.x, 0.0f, 1.0f) * 255.0f + 0.5f);
            const uint32_t qy = (uint32_t)(clampf(c.y, 0.0f, 1.0f) * 255.0f + 0.5f);
            const uint32_t qz = (uint32_t)(clampf(c.z, 0.0f, 1.0f) * 255.0f + 0.5f);
            const uint4 q = p.accum8[item];
            p.accum8[item] = make_uint4(q.x + qx * p.frame_count, q.y + qy * p.frame_count,
                                        q.z + qz * p.frame_count, 0u);
        }
    }
    // counters as the reference would do the work: once per frame
    unsigned long long s = (unsigned long long)segs * p.frame_count;
    unsigned long long t = (unsigned long long)tests * p.frame_count;
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off);
        t += __shfl_xor(t, off);
    }
    if (lane_id() == 0) {
        atomicAdd(p.seg_counter, s);
        if (BVH) atomicAdd(p.seg_counter + 1, t);
    }
}

// frame_split epilogue: acc += colour_f for f = 0 .. F-1 in frame order (the
// same float sums as the in-lane accumulation), plus the unorm8 path.
__global__ void frame_accumulate(const float4* __restrict__ fb, unsigned long long n_pix, uint32_t frames,
                                 float4* __restrict__ acc, uint4* __restrict__ acc8) {
    const unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pix) return;
    float4 a = acc[i];
    uint4 q = acc8 ? acc8[i] : make_uint4(0, 0, 0, 0);
    for (uint32_t f = 0; f < frames; f++) {
        const float4 c = fb[(size_t)f * n_pix + i];
        a = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
        q.x += (uint32_t)(clampf(c.x, 0.0f, 1.0f) * 255.0f + 0.5f);
        q.y += (uint32_t)(clampf(c.y, 0.0f, 1.0f) * 255.0f + 0.5f);
        q.z += (uint32_t)(clampf(c.z, 0.0f, 1.0f) * 255.0f + 0.5f);
    }
    acc[i] = a;
    if (acc8) acc8[i] = q;
}

// Cost-ordered scheduling: a counting sort of the pixels by the bit length of
// their previous item cost (32 buckets, most expensive first).  The order
// inside a bucket is whatever the atomics produce — it changes only which lane
// takes which pixel when, never a pixel's arithmetic.
// Runs of 64 consecutive pixels (one wave's worth of neighbouring pixels,
// so the lanes of a wave keep coherent rays) are the unit that is ordered.
__device__ __forceinline__ uint32_t run_cost(const uint32_t* __restrict__ cost, unsigned long long r) {
    uint32_t c = 0;
    for (int k = 0; k < 64; k++) c += cost[r * 64 + k] >> 8;
    return c;
}
__global__ void cost_histogram(const uint32_t* __restrict__ cost, unsigned long long n, uint32_t* __restrict__ hist) {
    __shared__ uint32_t h[32];
    if (threadIdx.x < 32) h[threadIdx.x] = 0;
    __syncthreads();
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t c = run_cost(cost, i);
        atomicAdd(&h[c ? 31 - __clz(c) : 0], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 32 && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}
__global__ void cost_offsets(uint32_t* hist) {  // one thread: descending exclusive scan, in place
    if (threadIdx.x != 0) return;
    uint32_t run = 0;
    for (int b = 31; b >= 0; b--) {
        const uint32_t c = hist[b];
        hist[b] = run;
        run += c;
    }
}
__global__ void cost_scatter(const uint32_t* __restrict__ cost, unsigned long long n, uint32_t* __restrict__ cursor,
                             uint32_t* __restrict__ order) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const uint32_t c = run_cost(cost, i);
        const uint32_t pos = atomicAdd(&cursor[c ? 31 - __clz(c) : 0], 1u);
        order[pos] = (uint32_t)i;
    }
}

// Pre-transform: RTXTriangle (80 B) -> {a, e0, e1, n} (48 B) + material index.
__global__ void prep_triangles(const rt2_triangle* tris, int n, float4* out, int* mtl) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const rt2_triangle t = tris[i];
    const f3 a = xyz4(t.a), b = xyz4(t.b), c = xyz4(t.c);
    const f3 e0 = sub(b, a), e1 = sub(c, a);
    const f3 nn = cross(e0, e1);
    out[3 * i + 0] = make_float4(a.x, a.y, a.z, e0.x);
    out[3 * i + 1] = make_float4(e0.y, e0.z, e1.x, e1.y);
    out[3 * i + 2] = make_float4(e1.z, nn.x, nn.y, nn.z);
    mtl[i] = t.materialIndex;
}

__global__ void resolve_kernel(const float4* acc, long long n, float inv_frames_dummy, float frames, float4* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    (void)inv_frames_dummy;
    float4 a = acc[i];
    out[i] = make_float4(a.x / frames, a.y / frames, a.z / frames, 1.0f);
}

// Numerics self-test: the IEEE primitives and pinned functions the path uses,
// evaluated on the device for comparison with the host (tests/test_gpu_numerics.py).
__global__ void selftest_kernel(const float* in, int n, float* out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = in[i];
    float y = in[(i * 7 + 3) % n];
    out[10 * i + 0] = x / y;
    out[10 * i + 1] = __builtin_sqrtf(fabsf(x));
    out[10 * i + 2] = __builtin_fmaf(x, y, x);
    out[10 * i + 3] = rt2pm_expf(x);
    out[10 * i + 4] = rt2pm_logf(fabsf(x));
    out[10 * i + 5] = rt2pm_acosf(fmaxf(-1.0f, fminf(1.0f, y)));
    out[10 * i + 6] = rt2pm_cosf(x);
    out[10 * i + 7] = rt2pm_sinf(x);
    out[10 * i + 8] = rt2pm_powf(fabsf(y), 1.0f / 2.2f);
    out[10 * i + 9] = 1.0f / x;
}

// Exhaustive check of the reciprocal sequences against IEEE 1.0f / x over a
// range of float bit patterns (test hook for the division-free exact path).
__global__ void rcp_check_kernel(uint32_t lo, unsigned long long count, int variant,
                                 unsigned long long* mismatches, uint32_t* first_bad) {
    unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
    unsigned long long bad = 0;
    for (; i < count; i += stride) {
        const uint32_t bits = lo + (uint32_t)i;
        const float x = __uint_as_float(bits);
        const float ref = 1.0f / x;
        float r = rcp_variant(x, variant);
        if (__float_as_uint(r) != __float_as_uint(ref)) {
            bad++;
            atomicMin(first_bad, bits);
        }
    }
    for (int off = 32; off > 0; off >>= 1) bad += __shfl_xor(bad, off);
    if ((threadIdx.x & 63) == 0 && bad) atomicAdd(mismatches, bad);
}

}  // namespace

/* =========================================================================
 * C-ABI, device half
 * ======================================================================= */
namespace rt2h {
void set_error(const std::string& msg);
}

#define HIPCHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) {                                                                \
            rt2h::set_error(std::string(#expr) + ": " + hipGetErrorString(e_));                \
            return -1;                                                                         \
        }                                                                                      \
    } while (0)

constexpr int kCounters = 32;  // [0] items, [1..7] stats + wave-end, [8..] kernel diagnostics
struct rt2_scene {
    int device = 0;
    int n_tris = 0, n_mats = 0, n_nodes = 0;
    rt2_triangle* d_raw = nullptr;
    float4* d_tri = nullptr;
    int* d_mtl = nullptr;
    rt2_material* d_mats = nullptr;
    rt2_node* d_nodes = nullptr;
    float4* d_recs = nullptr;                   // BVH v2 child-pair records
    float4* d_fb = nullptr;                     // frame_split scratch (per-frame colours)
    uchar4* d_texels = nullptr;                 // textures, RGBA8
    int4* d_tex_desc = nullptr;
    int n_tex = 0;
    size_t fb_bytes = 0;
    int bvh_root = 0;                           // BVH v2 stack entry of node 0
    int recs_ok = 0;                            // BVH v3 fast-path precondition on the boxes
    int split_frames = 1;                       // frame-major (frame, pixel) items when F > 1
    unsigned long long frame_scratch_cap = 2ull << 30;  // bytes of per-frame planes per launch
    int cost_order = 0;                         // order items by the previous launch's per-pixel cost (opt-in)
    uint32_t* d_cost = nullptr;                 // per-pixel cost map of the last launch
    uint32_t* d_order = nullptr;                // pixel order for the next launch
    uint32_t* d_hist = nullptr;                 // 32 counters
    unsigned long long cost_npix = 0;           // pixels the cost map describes (0 = none)
    unsigned long long cost_cap = 0;
    int cost_key[4] = {0, 0, 0, 0};             // W, tile_rows, rank, nranks the map belongs to
    hipEvent_t last_launch = nullptr;           // renders of one scene are ordered (shared scratch)
    bool last_launch_valid = false;
    unsigned long long* d_counters = nullptr;  // [0] item counter, [1] segments
    unsigned long long samples = 0, tests_per_seg = 0;
    int variant = 0;
    int last_variant = -1;
    int traversal = RT2_TRAVERSAL_BRUTE;
    int bvh_depth = 0;              // longest root-to-leaf path (nodes)
    int last_kind = 0;              // kind of the last launch (stats: tests)
    unsigned long long diag[kCounters] = {};
    int num_cus = 256;
    size_t max_lds = 65536;
};

// Validates a reference node array (BVH.h layout) against the triangle count
// and returns its depth; < 0 on a malformed array (child out of range, cycle,
// leaf range outside the triangles).
static int bvh_depth_check(const rt2_node* nodes, int n_nodes, int n_tris, std::string& err) {
    if (n_nodes < 1) {
        err = "empty node array";
        return -1;
    }
    std::vector<int> depth(n_nodes, 0);
    std::vector<int> stack;
    stack.push_back(0);
    depth[0] = 1;
    int maxd = 1;
    long long visited = 0;
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (++visited > n_nodes) {
            err = "node graph is not a tree";
            return -1;
        }
        const rt2_node& n = nodes[i];
        if (n.childIndex == -1) {
            if (n.triangleCount > 0 && (n.triangleIndex < 0 || (long long)n.triangleIndex + n.triangleCount > n_tris)) {
                err = "leaf " + std::to_string(i) + " references triangles outside [0, " + std::to_string(n_tris) + ")";
                return -1;
            }
            continue;
        }
        if (n.childIndex <= 0 || n.childIndex + 1 >= n_nodes) {
            err = "node " + std::to_string(i) + " has child index " + std::to_string(n.childIndex) + " out of range";
            return -1;
        }
        for (int c = n.childIndex; c <= n.childIndex + 1; c++) {
            depth[c] = depth[i] + 1;
            maxd = std::max(maxd, depth[c]);
            stack.push_back(c);
        }
    }
    return maxd;
}

// Child-pair records for render_bvh2 (layout: see bvh_step).  Interior nodes
// are numbered in depth-first pre-order (parents before children, left
// subtree first) so records of a subtree are contiguous.
static int bvh_records(const rt2_node* nodes, int n_nodes, std::vector<float4>& rec, int& root, std::string& err) {
    if (n_nodes >= (1 << 26)) {
        err = "more than 2^26 nodes";
        return -1;
    }
    std::vector<int> rid(n_nodes, -1);
    int n_int = 0;
    std::vector<int> stack{0};
    while (!stack.empty()) {
        const int i = stack.back();
        stack.pop_back();
        if (nodes[i].childIndex == -1) continue;
        rid[i] = n_int++;
        stack.push_back(nodes[i].childIndex + 1);
        stack.push_back(nodes[i].childIndex);
    }
    auto enc = [&](int i) -> int {
        const rt2_node& n = nodes[i];
        if (n.childIndex != -1) return rid[i];
        const int cnt = std::max(n.triangleCount, 0);
        const int start = cnt > 0 ? n.triangleIndex : 0;
        if (cnt <= 30 && start >= 0 && start < (1 << 26)) return ~((start << 5) | cnt);
        return ~((i << 5) | 31);
    };
    rec.assign((size_t)std::max(n_int, 1) * 4, make_float4(0.0f, 0.0f, 0.0f, 0.0f));
    for (int i = 0; i < n_nodes; i++) {
        if (rid[i] < 0) continue;
        const rt2_node& A = nodes[nodes[i].childIndex];
        const rt2_node& B = nodes[nodes[i].childIndex + 1];
        float4* r = &rec[(size_t)rid[i] * 4];
        r[0] = make_float4(A.bmin[0], A.bmin[1], A.bmin[2], A.bmax[0]);
        r[1] = make_float4(A.bmax[1], A.bmax[2], B.bmin[0], B.bmin[1]);
        r[2] = make_float4(B.bmin[2], B.bmax[0], B.bmax[1], B.bmax[2]);
        int e[4] = {enc(nodes[i].childIndex), enc(nodes[i].childIndex + 1), 0, 0};
        std::memcpy(&r[3], e, sizeof(e));
    }
    root = enc(0);
    return n_int;
}

// GL's unpack of a tightly packed stb image (GL_UNPACK_ALIGNMENT 4: rows
// start every align4(w*n) bytes; bytes past the buffer read as 0 — the
// reference reads past its allocation there) into RGBA8, with the swizzles of
// Texture2D(path) (1 channel: r,r,r,1; GL_RG: r,g,0,1; GL_RGB: r,g,b,1).
static void gl_unpack_rgba8(const rt2_image& im, uchar4* out) {
    const size_t n = (size_t)im.channels, stride = ((size_t)im.width * n + 3) & ~(size_t)3;
    const size_t total = (size_t)im.width * im.height * n;
    auto at = [&](size_t i) -> uint8_t { return i < total ? im.pixels[i] : (uint8_t)0; };
    for (int j = 0; j < im.height; j++)
        for (int i = 0; i < im.width; i++) {
            const size_t b = (size_t)j * stride + (size_t)i * n;
            uchar4 t;
            if (n == 1) t = make_uchar4(at(b), at(b), at(b), 255);
            else if (n == 2) t = make_uchar4(at(b), at(b + 1), 0, 255);
            else if (n == 3) t = make_uchar4(at(b), at(b + 1), at(b + 2), 255);
            else t = make_uchar4(at(b), at(b + 1), at(b + 2), at(b + 3));
            out[(size_t)j * im.width + i] = t;
        }
}

extern "C" int rt2_scene_set_textures(rt2_scene* s, const rt2_image* images, int32_t n) {
    if (!s || n < 0 || (n > 0 && !images)) {
        rt2h::set_error("rt2_scene_set_textures: bad argument");
        return -1;
    }
    size_t total = 0;
    for (int i = 0; i < n; i++) {
        const rt2_image& im = images[i];
        if (im.width < 1 || im.height < 1 || im.channels < 1 || im.channels > 4 || !im.pixels) {
            rt2h::set_error("rt2_scene_set_textures: image " + std::to_string(i) + " is empty or has " +
                            std::to_string(im.channels) + " channels");
            return -1;
        }
        total += (size_t)im.width * im.height;
    }
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipDeviceSynchronize());
    (void)hipFree(s->d_texels);
    (void)hipFree(s->d_tex_desc);
    s->d_texels = nullptr;
    s->d_tex_desc = nullptr;
    s->n_tex = 0;
    if (n == 0) return 0;
    std::vector<uchar4> host(total);
    std::vector<int4> desc(n);
    size_t off = 0;
    for (int i = 0; i < n; i++) {
        gl_unpack_rgba8(images[i], host.data() + off);
        desc[i] = make_int4(images[i].width, images[i].height, (int)(uint32_t)(off & 0xffffffffu), (int)(off >> 32));
        off += (size_t)images[i].width * images[i].height;
    }
    HIPCHECK(hipMalloc(&s->d_texels, total * sizeof(uchar4)));
    HIPCHECK(hipMalloc(&s->d_tex_desc, n * sizeof(int4)));
    HIPCHECK(hipMemcpy(s->d_texels, host.data(), total * sizeof(uchar4), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(s->d_tex_desc, desc.data(), n * sizeof(int4), hipMemcpyHostToDevice));
    s->n_tex = n;
    return 0;
}

// Not in rt2.h (test hook): bytes of per-frame colour planes one launch may use.
extern "C" int rt2_scene_set_frame_scratch_cap(rt2_scene* s, unsigned long long bytes) {
    if (!s || bytes == 0) return -1;
    s->frame_scratch_cap = bytes;
    return 0;
}

extern "C" int rt2_scene_set_cost_order(rt2_scene* s, int enable) {
    if (!s) {
        rt2h::set_error("rt2_scene_set_cost_order: null scene");
        return -1;
    }
    s->cost_order = enable ? 1 : 0;
    s->cost_npix = 0;  // forget the map
    return 0;
}

extern "C" int rt2_scene_set_frame_split(rt2_scene* s, int enable) {
    if (!s) {
        rt2h::set_error("rt2_scene_set_frame_split: null scene");
        return -1;
    }
    s->split_frames = enable ? 1 : 0;
    return 0;
}

extern "C" int rt2_scene_set_traversal(rt2_scene* s, int traversal) {
    if (!s || (traversal != RT2_TRAVERSAL_BRUTE && traversal != RT2_TRAVERSAL_BVH)) {
        rt2h::set_error("rt2_scene_set_traversal: bad argument");
        return -1;
    }
    if (traversal == RT2_TRAVERSAL_BVH && s->n_nodes == 0) {
        rt2h::set_error("rt2_scene_set_traversal: BVH traversal needs the node array (rt2_scene_create nodes)");
        return -1;
    }
    s->traversal = traversal;
    return 0;
}

extern "C" int rt2_scene_create(const rt2_triangle* tris, int32_t n_tris, const rt2_material* mats, int32_t n_mats,
                                const rt2_node* nodes, int32_t n_nodes, int32_t device, rt2_scene** out) {
    if (!out || n_tris < 0 || n_mats < 1 || !mats || (n_tris > 0 && !tris)) {
        rt2h::set_error("rt2_scene_create: bad argument");
        return -1;
    }
    for (int i = 0; i < n_tris; i++) {
        if (tris[i].materialIndex < 0 || tris[i].materialIndex >= n_mats) {
            rt2h::set_error("rt2_scene_create: triangle " + std::to_string(i) + " has material index " +
                            std::to_string(tris[i].materialIndex) + " outside [0, " + std::to_string(n_mats) + ")");
            return -1;
        }
    }
    int ndev = 0;
    HIPCHECK(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) {
        rt2h::set_error("rt2_scene_create: no HIP device " + std::to_string(device));
        return -1;
    }
    HIPCHECK(hipSetDevice(device));
    rt2_scene* s = new rt2_scene();
    s->device = device;
    s->n_tris = n_tris;
    s->n_mats = n_mats;
    s->n_nodes = nodes ? n_nodes : 0;
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device));
    s->num_cus = prop.multiProcessorCount;
    s->max_lds = prop.maxSharedMemoryPerMultiProcessor ? prop.maxSharedMemoryPerMultiProcessor : 65536;
    const size_t nt = (size_t)std::max(n_tris, 1);
    HIPCHECK(hipMalloc(&s->d_raw, nt * sizeof(rt2_triangle)));
    HIPCHECK(hipMalloc(&s->d_tri, nt * 3 * sizeof(float4)));
    HIPCHECK(hipMalloc(&s->d_mtl, nt * sizeof(int)));
    HIPCHECK(hipMalloc(&s->d_mats, (size_t)n_mats * sizeof(rt2_material)));
    HIPCHECK(hipMalloc(&s->d_counters, kCounters * sizeof(unsigned long long)));
    HIPCHECK(hipMemset(s->d_counters, 0, kCounters * sizeof(unsigned long long)));
    if (n_tris > 0) HIPCHECK(hipMemcpy(s->d_raw, tris, (size_t)n_tris * sizeof(rt2_triangle), hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(s->d_mats, mats, (size_t)n_mats * sizeof(rt2_material), hipMemcpyHostToDevice));
    if (s->n_nodes > 0) {
        std::string err;
        s->bvh_depth = bvh_depth_check(nodes, n_nodes, n_tris, err);
        if (s->bvh_depth < 0 || s->bvh_depth > 62) {
            if (s->bvh_depth > 62) err = "BVH deeper than compute.glsl's 64-entry stack";
            rt2h::set_error("rt2_scene_create: bad node array: " + err);
            delete s;
            return -1;
        }
        HIPCHECK(hipMalloc(&s->d_nodes, (size_t)n_nodes * sizeof(rt2_node)));
        HIPCHECK(hipMemcpy(s->d_nodes, nodes, (size_t)n_nodes * sizeof(rt2_node), hipMemcpyHostToDevice));
        std::vector<float4> rec;
        if (bvh_records(nodes, n_nodes, rec, s->bvh_root, err) < 0) {
            rt2h::set_error("rt2_scene_create: bad node array: " + err);
            delete s;
            return -1;
        }
        // the first three float4 of a record are box coordinates (the 4th: stack entries)
        s->recs_ok = 1;
        for (size_t i = 0; i < rec.size(); i++) {
            if (i % 4 == 3) continue;
            for (float c : {rec[i].x, rec[i].y, rec[i].z, rec[i].w})
                if (!(c == 0.0f || (std::fabs(c) >= 0x1p-37f && std::fabs(c) <= 0x1p59f))) s->recs_ok = 0;
        }
        HIPCHECK(hipMalloc(&s->d_recs, rec.size() * sizeof(float4)));
        HIPCHECK(hipMemcpy(s->d_recs, rec.data(), rec.size() * sizeof(float4), hipMemcpyHostToDevice));
    }
    if (n_tris > 0) {
        hipLaunchKernelGGL(prep_triangles, dim3((n_tris + 255) / 256), dim3(256), 0, 0, s->d_raw, n_tris, s->d_tri,
                           s->d_mtl);
        HIPCHECK(hipGetLastError());
    }
    HIPCHECK(hipDeviceSynchronize());
    *out = s;
    return 0;
}

extern "C" void rt2_scene_destroy(rt2_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    (void)hipFree(s->d_raw);
    (void)hipFree(s->d_tri);
    (void)hipFree(s->d_mtl);
    (void)hipFree(s->d_mats);
    (void)hipFree(s->d_nodes);
    (void)hipFree(s->d_recs);
    (void)hipFree(s->d_fb);
    (void)hipFree(s->d_cost);
    (void)hipFree(s->d_order);
    (void)hipFree(s->d_hist);
    if (s->last_launch) (void)hipEventDestroy(s->last_launch);
    (void)hipFree(s->d_texels);
    (void)hipFree(s->d_tex_desc);
    (void)hipFree(s->d_counters);
    delete s;
}

extern "C" int32_t rt2_shard_rows(int32_t height, rt2_shard sh) {
    if (sh.tile_rows < 1 || sh.nranks < 1 || sh.rank < 0 || sh.rank >= sh.nranks || height < 0) return -1;
    int32_t n = 0;
    for (int32_t t = sh.rank; (int64_t)t * sh.tile_rows < height; t += sh.nranks)
        n += std::min(sh.tile_rows, height - t * sh.tile_rows);
    return n;
}

extern "C" int32_t rt2_shard_row(int32_t local_row, rt2_shard sh) {
    int32_t t = local_row / sh.tile_rows;
    return (t * sh.nranks + sh.rank) * sh.tile_rows + local_row % sh.tile_rows;
}

extern "C" int rt2_scene_set_variant(rt2_scene* s, int variant) {
    if (!s) return -1;
    s->variant = variant;
    return variant;
}

namespace {
constexpr int kTileTris = 1024;  // 48 KiB of LDS per tile

// Kernel variants (rt2_scene_set_variant); 0 = auto = the default below.
enum Kind : int { K_RESIDENT = 0, K_TILED = 1, K_SMEM = 2, K_BVH = 3, K_BVH2 = 4, K_BVH3 = 5 };
struct Variant {
    int kind;
    int block;
    hipError_t (*launch)(const RenderParams&, int blocks, size_t lds, hipStream_t st);
    hipError_t (*occupancy)(int* occ, size_t lds);
    const char* name;
};

template <int KIND, int BLOCK, int MT, int UNROLL>
hipError_t launch_t(const RenderParams& p, int blocks, size_t lds, hipStream_t st) {
    if constexpr (KIND == K_TILED)
        hipLaunchKernelGGL((render_tiled<BLOCK, MT, UNROLL>), dim3(blocks), dim3(BLOCK), lds, st, p);
    else if constexpr (KIND == K_SMEM)
        hipLaunchKernelGGL((render_smem<BLOCK, MT % 1000, MT / 1000, UNROLL>), dim3(blocks), dim3(BLOCK), 0, st, p);
    else if constexpr (KIND == K_BVH)
        hipLaunchKernelGGL((render_bvh<BLOCK>), dim3(blocks), dim3(BLOCK), lds, st, p);
    else if constexpr (KIND == K_BVH2)
        hipLaunchKernelGGL((render_bvh2<BLOCK, MT>), dim3(blocks), dim3(BLOCK), lds, st, p);
    else if constexpr (KIND == K_BVH3)
        hipLaunchKernelGGL((render_bvh3<BLOCK, MT % 1000, (MT / 1000) % 10, UNROLL, MT / 10000>), dim3(blocks),
                           dim3(BLOCK), lds, st, p);
    else
        hipLaunchKernelGGL((render_resident<BLOCK, MT, UNROLL>), dim3(blocks), dim3(BLOCK), lds, st, p);
    return hipGetLastError();
}
template <int KIND, int BLOCK, int MT, int UNROLL>
hipError_t occ_t(int* occ, size_t lds) {
    if constexpr (KIND == K_TILED)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, render_tiled<BLOCK, MT, UNROLL>, BLOCK, lds);
    else if constexpr (KIND == K_SMEM)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, render_smem<BLOCK, MT % 1000, MT / 1000, UNROLL>,
                                                            BLOCK, 0);
    else if constexpr (KIND == K_BVH)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, render_bvh<BLOCK>, BLOCK, lds);
    else if constexpr (KIND == K_BVH2)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, render_bvh2<BLOCK, MT>, BLOCK, lds);
    else if constexpr (KIND == K_BVH3)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(
            occ, render_bvh3<BLOCK, MT % 1000, (MT / 1000) % 10, UNROLL, MT / 10000>, BLOCK, lds);
    else
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(occ, render_resident<BLOCK, MT, UNROLL>, BLOCK, lds);
}
#define RT2_VARIANT(T, B, M, U, NAME) Variant{T, B, launch_t<T, B, M, U>, occ_t<T, B, M, U>, NAME}

const Variant kVariants[] = {
    RT2_VARIANT(K_SMEM, 256, 32108, 1, "smem/256/masked8/coop32"),   // 0: default (<= kSmemMaxTris)
    RT2_VARIANT(K_RESIDENT, 256, 0, 4, "resident/256/plain/u4"),     // 1: round-1 v1 kernel
    RT2_VARIANT(K_TILED, 512, 4, 1, "tiled/512/grouped4"),           // 2: default (large scenes)
    RT2_VARIANT(K_RESIDENT, 256, 1, 4, "resident/256/filtered/u4"),  // 3
    RT2_VARIANT(K_RESIDENT, 1024, 1, 4, "resident/1024/filtered/u4"),// 4
    RT2_VARIANT(K_RESIDENT, 512, 1, 4, "resident/512/filtered/u4"),  // 5
    RT2_VARIANT(K_RESIDENT, 512, 1, 8, "resident/512/filtered/u8"),  // 6
    RT2_VARIANT(K_TILED, 256, 1, 4, "tiled/256/filtered/u4"),        // 7
    RT2_VARIANT(K_TILED, 1024, 4, 1, "tiled/1024/grouped4"),         // 8
    RT2_VARIANT(K_RESIDENT, 512, 4, 1, "resident/512/grouped4"),     // 9
    RT2_VARIANT(K_RESIDENT, 1024, 8, 1, "resident/1024/grouped8"),   // 10
    RT2_VARIANT(K_RESIDENT, 1024, 4, 1, "resident/1024/grouped4"),   // 11
    RT2_VARIANT(K_RESIDENT, 256, 4, 1, "resident/256/grouped4"),     // 12
    RT2_VARIANT(K_TILED, 512, 8, 1, "tiled/512/grouped8"),           // 13
    RT2_VARIANT(K_RESIDENT, 512, 2, 1, "resident/512/grouped2"),     // 14
    RT2_VARIANT(K_RESIDENT, 512, 4, 0, "resident/512/grouped4/STATS"), // 15: diagnostic counters
    RT2_VARIANT(K_SMEM, 256, 4, 1, "smem/256/grouped4"),             // 16
    RT2_VARIANT(K_SMEM, 512, 4, 1, "smem/512/grouped4"),             // 17
    RT2_VARIANT(K_SMEM, 1024, 4, 1, "smem/1024/grouped4"),           // 18
    RT2_VARIANT(K_SMEM, 512, 2, 1, "smem/512/grouped2"),             // 19
    RT2_VARIANT(K_SMEM, 512, 8, 1, "smem/512/grouped8"),             // 20
    RT2_VARIANT(K_RESIDENT, 512, 104, 1, "resident/512/masked4"),    // 21
    RT2_VARIANT(K_RESIDENT, 512, 108, 1, "resident/512/masked8"),    // 22
    RT2_VARIANT(K_SMEM, 256, 104, 1, "smem/256/masked4"),            // 23
    RT2_VARIANT(K_SMEM, 256, 108, 1, "smem/256/masked8"),            // 24
    RT2_VARIANT(K_SMEM, 512, 104, 1, "smem/512/masked4"),            // 25
    RT2_VARIANT(K_TILED, 512, 104, 1, "tiled/512/masked4"),          // 26
    RT2_VARIANT(K_SMEM, 256, 16108, 1, "smem/256/masked8/coop16"),   // 27
    RT2_VARIANT(K_SMEM, 256, 32108, 1, "smem/256/masked8/coop32"),   // 28
    RT2_VARIANT(K_SMEM, 256, 48108, 1, "smem/256/masked8/coop48"),   // 29
    RT2_VARIANT(K_SMEM, 256, 64108, 1, "smem/256/masked8/coop64"),   // 30
    RT2_VARIANT(K_SMEM, 256, 208, 1, "smem/256/lean8"),              // 31
    RT2_VARIANT(K_SMEM, 256, 204, 1, "smem/256/lean4"),              // 32
    RT2_VARIANT(K_RESIDENT, 1024, 208, 1, "resident/1024/lean8"),    // 33
    RT2_VARIANT(K_RESIDENT, 1024, 204, 1, "resident/1024/lean4"),    // 34
    RT2_VARIANT(K_RESIDENT, 512, 208, 1, "resident/512/lean8"),      // 35
    RT2_VARIANT(K_SMEM, 512, 208, 1, "smem/512/lean8"),              // 36
    RT2_VARIANT(K_BVH, 256, 0, 1, "bvh/256"),                        // 37: default (BVH traversal)
    RT2_VARIANT(K_BVH, 128, 0, 1, "bvh/128"),                        // 38
    RT2_VARIANT(K_BVH, 512, 0, 1, "bvh/512"),                        // 39
    RT2_VARIANT(K_BVH2, 256, 16, 1, "bvh2/256/t16"),                 // 40
    RT2_VARIANT(K_BVH2, 256, 8, 1, "bvh2/256/t8"),                   // 41
    RT2_VARIANT(K_BVH2, 256, 32, 1, "bvh2/256/t32"),                 // 42
    RT2_VARIANT(K_BVH2, 128, 16, 1, "bvh2/128/t16"),                 // 43
    RT2_VARIANT(K_BVH2, 64, 16, 1, "bvh2/64/t16"),                   // 44
    RT2_VARIANT(K_BVH2, 256, 1, 1, "bvh2/256/t1"),                   // 45
    RT2_VARIANT(K_BVH3, 256, 16, 1, "bvh3/256/t16"),                 // 46
    RT2_VARIANT(K_BVH3, 256, 8, 1, "bvh3/256/t8"),                   // 47
    RT2_VARIANT(K_BVH3, 256, 24, 1, "bvh3/256/t24"),                 // 48
    RT2_VARIANT(K_BVH3, 128, 16, 1, "bvh3/128/t16"),                 // 49
    RT2_VARIANT(K_BVH3, 256, 1016, 1, "bvh3/256/t16/div64"),         // 50
    RT2_VARIANT(K_BVH3, 256, 1008, 1, "bvh3/256/t8/div64"),          // 51
    RT2_VARIANT(K_SMEM, 256, 32108, 6, "smem/256/masked8/coop32/w6"), // 52
    RT2_VARIANT(K_BVH3, 256, 16, 5, "bvh3/256/t16/w5"),              // 53
    RT2_VARIANT(K_BVH3, 256, 8, 5, "bvh3/256/t8/w5"),                // 54
    RT2_VARIANT(K_BVH3, 256, 2016, 5, "bvh3/256/t16/filt/w5"),       // 55
    RT2_VARIANT(K_BVH3, 256, 2008, 5, "bvh3/256/t8/filt/w5"),        // 56
    RT2_VARIANT(K_BVH3, 256, 2016, 1, "bvh3/256/t16/filt"),          // 57
    RT2_VARIANT(K_BVH3, 256, 10016, 5, "bvh3/256/t16/w5/DIAG"),      // 58: diagnostic counters
    RT2_VARIANT(K_SMEM, 256, 32308, 1, "smem/256/ballot8/coop32"),   // 59
    RT2_VARIANT(K_SMEM, 256, 32408, 1, "smem/256/minfilt8/coop32"),  // 60
    RT2_VARIANT(K_SMEM, 256, 32304, 1, "smem/256/ballot4/coop32"),   // 61
    RT2_VARIANT(K_SMEM, 256, 32416, 1, "smem/256/minfilt16/coop32"), // 62
    RT2_VARIANT(K_SMEM, 256, 32404, 1, "smem/256/minfilt4/coop32"),  // 63
    RT2_VARIANT(K_SMEM, 256, 132108, 1, "smem/256/masked8/team32"),  // 64
    RT2_VARIANT(K_SMEM, 256, 148108, 1, "smem/256/masked8/team48"),  // 65
    RT2_VARIANT(K_SMEM, 256, 164108, 1, "smem/256/masked8/team64"),  // 66
};
constexpr int kNumVariants = sizeof(kVariants) / sizeof(kVariants[0]);
constexpr size_t kResidentMaxBytes = 112 * 1024;
constexpr int kSmemMaxTris = 16384;
constexpr int kDefaultBvhVariant = 53;
}  // namespace

extern "C" const char* rt2_variant_name(int v) { return v >= 0 && v < kNumVariants ? kVariants[v].name : nullptr; }

extern "C" int rt2_render(rt2_scene* s, const rt2_uniforms* u, uint32_t frame_begin, uint32_t frame_count,
                          rt2_shard sh, float* d_accum, uint32_t* d_accum8, void* stream) {
    if (!s || !u || !d_accum) {
        rt2h::set_error("rt2_render: null argument");
        return -1;
    }
    if ((!u->basicShading && u->numRaysPerPixel < 1) || u->width < 1 || u->height < 1) {
        rt2h::set_error("rt2_render: numRaysPerPixel, width and height must be >= 1");
        return -1;
    }
    const int rows = rt2_shard_rows((int)u->height, sh);
    if (rows < 0) {
        rt2h::set_error("rt2_render: bad shard");
        return -1;
    }
    if (frame_count == 0 || rows == 0) return 0;
    // frame-major items keep one colour plane per frame: beyond frame_scratch_cap
    // of planes (or 2^32 items), render consecutive frame chunks — the
    // accumulation stays in frame order, so the sums are unchanged
    if (!u->basicShading && s->split_frames && frame_count > 1) {
        const unsigned long long npix = (unsigned long long)rows * u->width;
        unsigned long long chunk = std::max<unsigned long long>(1, s->frame_scratch_cap / (npix * sizeof(float4)));
        chunk = std::min<unsigned long long>(chunk, 0xfffffffeull / std::max<unsigned long long>(npix, 1));
        if (chunk < frame_count) {
            for (unsigned long long f0 = 0; f0 < frame_count; f0 += chunk) {
                const uint32_t fc = (uint32_t)std::min<unsigned long long>(chunk, frame_count - f0);
                const int rc = rt2_render(s, u, frame_begin + (uint32_t)f0, fc, sh, d_accum, d_accum8, stream);
                if (rc != 0) return rc;
            }
            return 0;
        }
    }
    HIPCHECK(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)stream;

    RenderParams p;
    std::memset(&p, 0, sizeof(p));
    p.tri = s->d_tri;
    p.tri_mtl = s->d_mtl;
    p.raw = s->d_raw;
    p.texels = s->d_texels;
    p.tex_desc = s->d_tex_desc;
    p.n_tex = s->n_tex;
    p.num_textures = u->numTextures;
    p.mats = s->d_mats;
    p.n_tris = s->n_tris;
    p.n_mats = s->n_mats;
    p.W = (int)u->width;
    p.H = (int)u->height;
    p.maxBounce = u->maxBounceCount;
    p.R = u->numRaysPerPixel;
    p.envLight = u->environmentalLight;
    auto cp = [](float* d, const rt2_vec4& v) {
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
    };
    cp(p.cam, u->cameraPos);
    cp(p.vpRight, u->viewportRight);
    cp(p.vpUp, u->viewportUp);
    cp(p.vpFront, u->viewportFront);
    cp(p.pixR, u->pixelRight);
    cp(p.pixU, u->pixelUp);
    cp(p.defR, u->defocusDiskRight);
    cp(p.defU, u->defocusDiskUp);
    p.frame_begin = frame_begin;
    p.frame_count = frame_count;
    p.tile_rows = sh.tile_rows;
    p.rank = sh.rank;
    p.nranks = sh.nranks;
    p.n_pix = (unsigned long long)rows * (unsigned long long)p.W;
    p.n_items = p.n_pix;
    if (p.n_pix >= 0xffffffffull) {
        rt2h::set_error("rt2_render: more than 2^32-1 pixels in one shard");
        return -1;
    }
    p.accum = reinterpret_cast<float4*>(d_accum);
    p.accum8 = reinterpret_cast<uint4*>(d_accum8);
    p.item_counter = s->d_counters;
    p.seg_counter = s->d_counters + 1;
    p.tile_tris = kTileTris;

    // renders of one scene share its counters and scratch (frame planes, cost
    // map, pixel order): a render waits for the scene's previous one, whatever
    // stream that was issued on
    if (s->last_launch_valid) HIPCHECK(hipStreamWaitEvent(st, s->last_launch, 0));
    HIPCHECK(hipMemsetAsync(s->d_counters, 0, sizeof(unsigned long long), st));
    HIPCHECK(hipMemsetAsync(s->d_counters + 6, 0xff, sizeof(unsigned long long), st));  // diag: min wave end
    HIPCHECK(hipMemsetAsync(s->d_counters + 7, 0, sizeof(unsigned long long), st));     // diag: max wave end
    p.nodes = s->d_nodes;
    p.stack_slots = s->bvh_depth + 2;
    if (u->basicShading) {  // traceBasic preview: one thread per pixel
        p.basicShadow = u->basicShadingShadow;
        cp(p.light, u->basicShadingLightPosition);
        constexpr int kBasicBlock = 256;
        const unsigned long long blocks = (p.n_items + kBasicBlock - 1) / kBasicBlock;
        if (s->traversal == RT2_TRAVERSAL_BVH) {
            const size_t lds = (size_t)p.stack_slots * kBasicBlock * sizeof(int);
            hipLaunchKernelGGL((render_basic<kBasicBlock, true>), dim3((unsigned)blocks), dim3(kBasicBlock), lds, st,
                               p);
            s->last_kind = K_BVH;
        } else {
            hipLaunchKernelGGL((render_basic<kBasicBlock, false>), dim3((unsigned)blocks), dim3(kBasicBlock), 0, st,
                               p);
            s->last_kind = K_SMEM;
        }
        HIPCHECK(hipGetLastError());
        if (!s->last_launch) HIPCHECK(hipEventCreateWithFlags(&s->last_launch, hipEventDisableTiming));
        HIPCHECK(hipEventRecord(s->last_launch, st));
        s->last_launch_valid = true;
        s->last_variant = -1;
        s->samples += p.n_items * (unsigned long long)frame_count;
        s->tests_per_seg = (unsigned long long)s->n_tris;
        return 0;
    }
    // several frames: frame-major (frame, pixel) items into a scratch buffer,
    // then frame_accumulate (finer work items: a shorter tail)
    if (frame_count > 1 && s->split_frames && p.n_pix * frame_count < 0xffffffffull) {
        const size_t need = (size_t)p.n_pix * frame_count * sizeof(float4);
        if (need > s->fb_bytes) {
            if (s->d_fb) HIPCHECK(hipFree(s->d_fb));
            s->d_fb = nullptr;
            s->fb_bytes = 0;
            HIPCHECK(hipMalloc(&s->d_fb, need));
            s->fb_bytes = need;
        }
        p.frame_split = 1;
        p.frame_buf = s->d_fb;
        p.n_items = p.n_pix * frame_count;
    }
    // cost-ordered items: the previous launch's per-pixel costs (same slab)
    // give this launch's pixel order, most expensive first (a shorter tail)
    if (s->cost_order) {
        if (s->cost_cap < p.n_pix) {
            (void)hipFree(s->d_cost);
            (void)hipFree(s->d_order);
            s->d_cost = s->d_order = nullptr;
            s->cost_cap = 0;
            s->cost_npix = 0;
            HIPCHECK(hipMalloc(&s->d_cost, p.n_pix * sizeof(uint32_t)));
            HIPCHECK(hipMalloc(&s->d_order, p.n_pix * sizeof(uint32_t)));
            if (!s->d_hist) HIPCHECK(hipMalloc(&s->d_hist, 32 * sizeof(uint32_t)));
            s->cost_cap = p.n_pix;
        }
        const int key[4] = {(int)u->width, sh.tile_rows, sh.rank, sh.nranks};
        const bool valid = s->cost_npix == p.n_pix && std::memcmp(key, s->cost_key, sizeof(key)) == 0;
        const unsigned long long runs = p.n_pix / 64;
        if (valid && runs > 0) {
            const unsigned blocks = (unsigned)std::min<unsigned long long>((runs + 255) / 256, 2048);
            HIPCHECK(hipMemsetAsync(s->d_hist, 0, 32 * sizeof(uint32_t), st));
            hipLaunchKernelGGL(cost_histogram, dim3(blocks), dim3(256), 0, st, s->d_cost, runs, s->d_hist);
            hipLaunchKernelGGL(cost_offsets, dim3(1), dim3(64), 0, st, s->d_hist);
            hipLaunchKernelGGL(cost_scatter, dim3(blocks), dim3(256), 0, st, s->d_cost, runs, s->d_hist, s->d_order);
            HIPCHECK(hipGetLastError());
            p.order = s->d_order;
            p.n_runs = (uint32_t)runs;
        }
        p.cost_out = s->d_cost;
        s->cost_npix = p.n_pix;
        std::memcpy(s->cost_key, key, sizeof(key));
    }
    const size_t resident_bytes = (size_t)3 * sizeof(float4) * (size_t)std::max(s->n_tris, 1);
    const bool fits = resident_bytes <= kResidentMaxBytes;
    int vi = s->variant;
    // auto: scalar-path kernel for small scenes (config B: 1,208 triangles),
    // LDS-tiled sweep for large ones (config C/E: 100k-1M triangles)
    if (s->traversal == RT2_TRAVERSAL_BVH) {
        if (vi <= 0 || vi >= kNumVariants || kVariants[vi].kind < K_BVH)
            vi = kDefaultBvhVariant;
    } else {
        if (vi <= 0 || vi >= kNumVariants || kVariants[vi].kind >= K_BVH)
            vi = s->n_tris <= kSmemMaxTris ? 0 : 2;
        if (kVariants[vi].kind == K_RESIDENT && !fits) vi = 2;  // a resident variant cannot hold this scene
    }
    const Variant& V = kVariants[vi];
    size_t lds = 0;
    if (V.kind == K_TILED)
        lds = (size_t)3 * sizeof(float4) * kTileTris;
    else if (V.kind == K_RESIDENT)
        lds = resident_bytes;
    else if (V.kind >= K_BVH)
        lds = (size_t)p.stack_slots * V.block * sizeof(int);
    p.bvh_recs = s->d_recs;
    p.bvh_root = s->bvh_root;
    p.recs_ok = s->recs_ok;
    s->last_kind = V.kind >= K_BVH ? K_BVH : V.kind;
    int occ = 0;
    HIPCHECK(V.occupancy(&occ, lds));
    occ = std::max(occ, 1);
    unsigned long long blocks = (unsigned long long)s->num_cus * occ;
    blocks = std::min(blocks, (p.n_items + V.block - 1) / V.block);
    blocks = std::max(blocks, 1ull);
    s->last_variant = vi;
    HIPCHECK(V.launch(p, (int)blocks, lds, st));
    HIPCHECK(hipGetLastError());
    if (p.frame_split) {
        hipLaunchKernelGGL(frame_accumulate, dim3((unsigned)((p.n_pix + 255) / 256)), dim3(256), 0, st, p.frame_buf,
                           p.n_pix, frame_count, p.accum, p.accum8);
        HIPCHECK(hipGetLastError());
    }
    if (!s->last_launch) HIPCHECK(hipEventCreateWithFlags(&s->last_launch, hipEventDisableTiming));
    HIPCHECK(hipEventRecord(s->last_launch, st));
    s->last_launch_valid = true;
    s->samples += p.n_pix * (unsigned long long)p.R * (unsigned long long)frame_count;
    s->tests_per_seg = (unsigned long long)s->n_tris;
    return 0;
}

extern "C" int rt2_scene_stats(rt2_scene* s, rt2_stats* out, int reset) {
    if (!s || !out) {
        rt2h::set_error("rt2_scene_stats: null argument");
        return -1;
    }
    HIPCHECK(hipSetDevice(s->device));
    HIPCHECK(hipDeviceSynchronize());
    unsigned long long c[kCounters];
    HIPCHECK(hipMemcpy(c, s->d_counters, sizeof(c), hipMemcpyDeviceToHost));
    std::memcpy(s->diag, c, sizeof(c));
    out->samples = s->samples;
    out->segments = c[1];
    // brute force tests every triangle per segment; the BVH kernel counts its
    // leaf tests in c[2]
    out->tests = s->last_kind == 3 ? c[2] : c[1] * (unsigned long long)s->n_tris;
    out->node_visits = s->last_kind == 3 ? c[3] : 0;
    if (reset) {
        s->samples = 0;
        HIPCHECK(hipMemset(s->d_counters, 0, sizeof(c)));
    }
    return 0;
}

extern "C" int rt2_resolve_rgba32f(const float* d_accum, int64_t n, uint32_t frames, float* d_out, void* stream) {
    if (!d_accum || !d_out || n < 0 || frames == 0) {
        rt2h::set_error("rt2_resolve_rgba32f: bad argument");
        return -1;
    }
    if (n == 0) return 0;
    hipLaunchKernelGGL(resolve_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       reinterpret_cast<const float4*>(d_accum), (long long)n, 0.0f, (float)frames,
                       reinterpret_cast<float4*>(d_out));
    HIPCHECK(hipGetLastError());
    return 0;
}

extern "C" int rt2_resolve_rgb8_reference(const uint32_t* acc8, int64_t n, uint32_t frames, uint8_t* out) {
    if (!acc8 || !out || n < 0 || frames == 0) {
        rt2h::set_error("rt2_resolve_rgb8_reference: bad argument");
        return -1;
    }
    const float F = (float)frames;
    for (int64_t i = 0; i < n; i++)
        for (int c = 0; c < 3; c++) {
            float v = std::min(255.0f, (float)acc8[4 * i + c] / F);
            out[3 * i + c] = (uint8_t)v;
        }
    return 0;
}

extern "C" int rt2_render_host(rt2_scene* s, const rt2_uniforms* u, uint32_t frame_begin, uint32_t frame_count,
                               rt2_shard sh, float* out_rgba, uint8_t* out_rgb8) {
    if (!s || !u) {
        rt2h::set_error("rt2_render_host: null argument");
        return -1;
    }
    const int rows = rt2_shard_rows((int)u->height, sh);
    if (rows < 0) {
        rt2h::set_error("rt2_render_host: bad shard");
        return -1;
    }
    const size_t n = (size_t)rows * u->width;
    HIPCHECK(hipSetDevice(s->device));
    float* acc = nullptr;
    float* res = nullptr;
    uint32_t* acc8 = nullptr;
    HIPCHECK(hipMalloc(&acc, std::max(n, (size_t)1) * 16));
    HIPCHECK(hipMalloc(&res, std::max(n, (size_t)1) * 16));
    HIPCHECK(hipMemset(acc, 0, std::max(n, (size_t)1) * 16));
    if (out_rgb8) {
        HIPCHECK(hipMalloc(&acc8, std::max(n, (size_t)1) * 16));
        HIPCHECK(hipMemset(acc8, 0, std::max(n, (size_t)1) * 16));
    }
    int rc = rt2_render(s, u, frame_begin, frame_count, sh, acc, acc8, nullptr);
    if (rc == 0 && out_rgba && n) {
        rc = rt2_resolve_rgba32f(acc, (int64_t)n, frame_count, res, nullptr);
        if (rc == 0) {
            hipError_t e = hipMemcpy(out_rgba, res, n * 16, hipMemcpyDeviceToHost);
            if (e != hipSuccess) {
                rt2h::set_error(std::string("hipMemcpy: ") + hipGetErrorString(e));
                rc = -1;
            }
        }
    }
    if (rc == 0 && out_rgb8 && n) {
        std::vector<uint32_t> h8(n * 4);
        hipError_t e = hipMemcpy(h8.data(), acc8, n * 16, hipMemcpyDeviceToHost);
        if (e != hipSuccess) {
            rt2h::set_error(std::string("hipMemcpy: ") + hipGetErrorString(e));
            rc = -1;
        } else {
            rc = rt2_resolve_rgb8_reference(h8.data(), (int64_t)n, frame_count, out_rgb8);
        }
    }
    hipError_t e = hipDeviceSynchronize();
    if (rc == 0 && e != hipSuccess) {
        rt2h::set_error(std::string("render: ") + hipGetErrorString(e));
        rc = -1;
    }
    (void)hipFree(acc);
    (void)hipFree(res);
    (void)hipFree(acc8);
    return rc;
}

// Not in rt2.h (diagnostics): counters of the last rt2_scene_stats call
// [1] segments, [2] groups, [3] groups with survivors, [4] exact iterations,
// [5] lane survivors (STATS variants only), and the variant last launched.
// Not in rt2.h (diagnostics): all kCounters counters of the last stats call.
extern "C" int rt2_scene_diag_ex(rt2_scene* s, unsigned long long* out, int n) {
    if (!s || !out || n < 0) return -1;
    std::memcpy(out, s->diag, sizeof(unsigned long long) * (size_t)std::min(n, kCounters));
    return std::min(n, kCounters);
}

extern "C" int rt2_scene_diag(rt2_scene* s, unsigned long long* out8, int* last_variant) {
    if (!s || !out8) return -1;
    std::memcpy(out8, s->diag, 8 * sizeof(unsigned long long));
    if (last_variant) *last_variant = s->last_variant;
    return 0;
}

// Not in rt2.h (test hook): exhaustive reciprocal check over [lo, hi] bit patterns.
extern "C" int rt2_device_rcp_check(uint32_t lo, uint32_t hi, int variant, unsigned long long* mismatches,
                                    uint32_t* first_bad) {
    unsigned long long* d = nullptr;
    HIPCHECK(hipMalloc(&d, 16));
    HIPCHECK(hipMemset(d, 0, 8));
    uint32_t init = 0xffffffffu;
    HIPCHECK(hipMemcpy((char*)d + 8, &init, 4, hipMemcpyHostToDevice));
    const unsigned long long count = (unsigned long long)hi - lo + 1;
    hipLaunchKernelGGL(rcp_check_kernel, dim3(4096), dim3(256), 0, 0, lo, count, variant, d, (uint32_t*)((char*)d + 8));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(mismatches, d, 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(first_bad, (char*)d + 8, 4, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

// Not in rt2.h (test hook): div_mk (mode 0) or div64 (mode 1) against IEEE
// division on `count` random (n, d) pairs of the ranges the kernels use them on.
extern "C" int rt2_device_div_check(uint32_t seed, unsigned long long count, int mode,
                                    unsigned long long* mismatches, uint32_t* first_bad) {
    unsigned long long* d = nullptr;
    HIPCHECK(hipMalloc(&d, 16));
    HIPCHECK(hipMemset(d, 0, 8));
    uint32_t init = 0xffffffffu;
    HIPCHECK(hipMemcpy((char*)d + 8, &init, 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(div_check_kernel, dim3(8192), dim3(256), 0, 0, seed, count, mode, d,
                       (uint32_t*)((char*)d + 8));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(mismatches, d, 8, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(first_bad, (char*)d + 8, 4, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}

// Not in rt2.h (test hook): device numerics self-test, host in/out arrays.
extern "C" int rt2_device_selftest(const float* in, int32_t n, float* out10) {
    float *din = nullptr, *dout = nullptr;
    HIPCHECK(hipMalloc(&din, (size_t)n * 4));
    HIPCHECK(hipMalloc(&dout, (size_t)n * 40));
    HIPCHECK(hipMemcpy(din, in, (size_t)n * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(selftest_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, din, n, dout);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(out10, dout, (size_t)n * 40, hipMemcpyDeviceToHost));
    (void)hipFree(din);
    (void)hipFree(dout);
    return 0;
}
