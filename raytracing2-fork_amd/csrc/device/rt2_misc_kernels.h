// traceBasic preview, frame accumulation, cost-ordered scheduling, triangle
// preparation, resolve to 8-bit and self-test kernels.
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

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

// sweep_plk records (rt2_sweep.h) from the pre-transformed triangles, in
// binary64: p0 = a×e0, p1 = a×e1 and a·n are rounded once to binary32 after
// the exact power-of-two scale s (s·max(|e0|,|e1|,|n|)∞ in [1,2)).  The
// filter's error bound holds for |a_i| <= 2^20, every component of e0/e1/n 0
// or in [2^-100, 2^20], and max(|e0|,|e1|,|n|)∞ >= 2^-30; a triangle outside
// that range (or non-finite, or degenerate) gets the all-zero record, which
// always passes (the exact test decides), and is counted in flags[0].
// flags[1] = max |a_i| over the in-range triangles (float bits: an atomic max
// over non-negative floats).
__global__ void prep_plk(const float4* tri, int n, float4* out, uint32_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 t0 = tri[3 * i], t1 = tri[3 * i + 1], t2 = tri[3 * i + 2];
    const float a[3] = {t0.x, t0.y, t0.z}, e0[3] = {t0.w, t1.x, t1.y}, e1[3] = {t1.z, t1.w, t2.x},
                nn[3] = {t2.y, t2.z, t2.w};
    bool ok = true;
    float A = 0.0f, M = 0.0f;
    for (int k = 0; k < 3; k++) {
        ok = ok && fabsf(a[k]) <= 0x1p20f;  // false for NaN
        A = fmaxf(A, fabsf(a[k]));
        for (float x : {e0[k], e1[k], nn[k]}) {
            const float ax = fabsf(x);
            ok = ok && (x == 0.0f || (ax >= 0x1p-100f && ax <= 0x1p20f));
            M = fmaxf(M, ax);
        }
    }
    ok = ok && M >= 0x1p-30f;
    float r[16];
    for (int k = 0; k < 16; k++) r[k] = 0.0f;
    if (ok) {
        int ex;
        (void)frexpf(M, &ex);  // M = f * 2^ex, f in [0.5, 1)
        const double s = ldexp(1.0, 1 - ex);
        auto D = [](float x) { return (double)x; };
        const double p0[3] = {D(a[1]) * e0[2] - D(a[2]) * e0[1], D(a[2]) * e0[0] - D(a[0]) * e0[2],
                              D(a[0]) * e0[1] - D(a[1]) * e0[0]};
        const double p1[3] = {D(a[1]) * e1[2] - D(a[2]) * e1[1], D(a[2]) * e1[0] - D(a[0]) * e1[2],
                              D(a[0]) * e1[1] - D(a[1]) * e1[0]};
        const double an = D(a[0]) * nn[0] + D(a[1]) * nn[1] + D(a[2]) * nn[2];
        for (int k = 0; k < 3; k++) {
            r[k] = (float)(nn[k] * s);
            r[4 + k] = (float)(e0[k] * s);
            r[10 + k] = (float)(e1[k] * s);
        }
        r[3] = (float)(-an * s);
        r[7] = (float)(-p0[0] * s);
        r[8] = (float)(-p0[1] * s);
        r[9] = (float)(-p0[2] * s);
        r[13] = (float)(-p1[0] * s);
        r[14] = (float)(-p1[1] * s);
        r[15] = (float)(-p1[2] * s);
        atomicMax(&flags[1], __float_as_uint(A));
    } else {
        atomicAdd(&flags[0], 1u);
    }
    for (int k = 0; k < 4; k++) out[4 * i + k] = make_float4(r[4 * k], r[4 * k + 1], r[4 * k + 2], r[4 * k + 3]);
}

__global__ void resolve_kernel(const float4* acc, long long n, float inv_frames_dummy, float frames, float4* out) {
    long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    (void)inv_frames_dummy;
    float4 a = acc[i];
    out[i] = make_float4(a.x / frames, a.y / frames, a.z / frames, 1.0f);
}

// The reference screenshot's 8-bit average (rayTracing.cpp:248-250) on the
// device: u8(min(255, float(sum) / frames)) per channel, rgba sums -> rgb
// bytes; the same operations as the host rt2_resolve_rgb8_reference.
__global__ void resolve_rgb8_kernel(const uint4* acc8, long long n, float frames, uint8_t* out) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint4 q = acc8[i];
    out[3 * i + 0] = (uint8_t)fminf(255.0f, (float)q.x / frames);
    out[3 * i + 1] = (uint8_t)fminf(255.0f, (float)q.y / frames);
    out[3 * i + 2] = (uint8_t)fminf(255.0f, (float)q.z / frames);
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
