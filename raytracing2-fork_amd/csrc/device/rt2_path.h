// Per-lane path state and shading: ray generation, scatter, sky and
// accumulation (compute.glsl:472-701), textures (getTriangleTextureColor).
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

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
};

// S > 1: split mode (render_split) — the S waves of a workgroup hold the same
// lanes (same items, same RNG streams, identical arithmetic) and each sweeps
// 1/S of the triangles; wave 0 alone takes items and writes results.
template <int S = 1>
__device__ __forceinline__ bool split_writer() {
    return S == 1 || threadIdx.x < 64;
}
template <int S = 1>
__device__ __forceinline__ void end_path(Lane& L, const RenderParams& p);

// The pixel of item `item` (row-major in the slab; rows interleaved over
// ranks in tiles)
__device__ __forceinline__ void item_xy(uint32_t item, const RenderParams& p, int& x, int& y) {
    const uint32_t W = opaque((uint32_t)p.W);
    const int lr = (int)(item / W);
    x = (int)(item - (uint32_t)lr * W);
    y = shard_row(lr, p.tile_rows, p.rank, p.nranks);
}

// Phase A: bring every lane to ST_TRACE or ST_DONE (wave-collective; with
// S > 1 workgroup-collective, every wave of the group on the same path).
// XY = false: L.x, L.y are not kept across calls (recomputed from L.item
// where a new frame or ray needs them: two VGPRs less live across the sweep
// of the register-bound resident kernel)
template <int S = 1, bool XY = true>
__device__ __forceinline__ void advance(Lane& L, const RenderParams& p) {
    for (;;) {
        const bool need = L.st == ST_NEED_ITEM;
        unsigned long long m = __ballot(need);
        if (m) {
            unsigned long long it = ~0ull;  // this lane's item (~0: none left)
            if constexpr (S == 1) {
                if (p.region_ctr) {
                    // 8 contiguous item regions, one per workgroup group b % 8
                    // (the workgroups that share an XCD's L2): a group takes
                    // items from its own region first, then from the others
                    const uint32_t g0 = blockIdx.x & 7u;
#pragma unroll 1
                    for (uint32_t k = 0; k < 8u && m; k++) {
                        const uint32_t r = (g0 + k) & 7u;
                        const unsigned long long lo = p.n_items * r / 8u, hi = p.n_items * (r + 1u) / 8u;
                        unsigned long long base = 0;
                        if (lane_id() == 0) base = atomicAdd(p.region_ctr + 16u * r, (unsigned long long)__popcll(m));
                        base = __shfl(base, 0);
                        if ((m >> lane_id()) & 1ull) {
                            const unsigned long long j = lo + base + lanes_below(m);
                            if (j < hi) it = j;
                        }
                        m = __ballot(need && it == ~0ull);
                    }
                } else {
                    unsigned long long base = 0;
                    if (lane_id() == 0) base = atomicAdd(p.item_counter, (unsigned long long)__popcll(m));
                    base = __shfl(base, 0);
                    if (need) it = base + lanes_below(m);
                }
            } else {
                __shared__ unsigned long long split_base;
                if (threadIdx.x == 0) split_base = atomicAdd(p.item_counter, (unsigned long long)__popcll(m));
                __syncthreads();
                if (need) it = split_base + lanes_below(m);
                __syncthreads();
            }
            if (need) {
                if (it < p.n_items) {
                    // frame_split: item = frame * n_pix + pixel (frame-major), so the
                    // last items of a launch are single pixel-frames
                    // n_items < 2^32 (checked on the host): 32-bit arithmetic
                    const uint32_t it32 = (uint32_t)it, np32 = opaque((uint32_t)p.n_pix);
                    const uint32_t f = p.frame_split ? it32 / np32 : 0u;
                    L.item = it32 - f * np32;
                    if (p.order && L.item < p.n_runs * 64u) L.item = p.order[L.item >> 6] * 64u + (L.item & 63u);
                    // cost map (opt-in): the item's start clock waits in its own
                    // slot (no register of the lane carries it); with frame-major
                    // items only frame 0 of a pixel measures (one writer per
                    // slot: the pixel's other frames run at the same time)
                    if (p.cost_out && split_writer<S>() && f == 0u)
                        p.cost_out[L.item] = (uint32_t)__builtin_amdgcn_s_memtime();
                    if constexpr (XY) item_xy(L.item, p, L.x, L.y);
                    L.frame = f;
                    L.st = ST_NEW_FRAME;
                } else {
                    L.st = ST_DONE;
                }
            }
        }
        if constexpr (!XY)
            if (L.st == ST_NEW_FRAME || L.st == ST_NEW_RAY) item_xy(L.item, p, L.x, L.y);
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
            if (p.maxBounce <= 0) end_path<S>(L, p);  // trace() returns 0 without tracing
        }
        if (!__any(L.st != ST_TRACE && L.st != ST_DONE)) break;
    }
}

// End of a path: colorCumulative += trace(...) (compute.glsl:692); next ray,
// or end of the frame (compute.glsl:696-700 + the screenshot accumulation).
template <int S>
__device__ __forceinline__ void end_path(Lane& L, const RenderParams& p) {
    L.colorCum = add(L.colorCum, L.incoming);
    L.ray += 1;
    if (L.ray < p.R) {
        L.st = ST_NEW_RAY;
        return;
    }
    f3 c = divs(L.colorCum, (float)p.R);
    c = mk(srgb1(aces1(c.x)), srgb1(aces1(c.y)), srgb1(aces1(c.z)));
    const bool writer = split_writer<S>();
    if (p.frame_split) {  // frame_accumulate adds the frames in order afterwards
        if (writer) p.frame_buf[(size_t)L.frame * p.n_pix + L.item] = make_float4(c.x, c.y, c.z, 0.0f);
        if (writer && p.cost_out && L.frame == 0)
            p.cost_out[L.item] = (uint32_t)__builtin_amdgcn_s_memtime() - p.cost_out[L.item];
        L.st = ST_NEED_ITEM;
        return;
    }
    // accumulate this frame in frame order: acc = acc + colour
    if (writer) {
        const float4 a = p.accum[L.item];
        p.accum[L.item] = make_float4(a.x + c.x, a.y + c.y, a.z + c.z, 0.0f);
        if (p.accum8) {
            // GL float -> unorm8, round to nearest (GL 4.3 §2.3.5.2)
            const uint4 q = p.accum8[L.item];
            p.accum8[L.item] = make_uint4(q.x + (uint32_t)(clampf(c.x, 0.0f, 1.0f) * 255.0f + 0.5f),
                                          q.y + (uint32_t)(clampf(c.y, 0.0f, 1.0f) * 255.0f + 0.5f),
                                          q.z + (uint32_t)(clampf(c.z, 0.0f, 1.0f) * 255.0f + 0.5f), 0u);
        }
    }
    L.frame += 1;
    L.st = L.frame < p.frame_count ? ST_NEW_FRAME : ST_NEED_ITEM;
    if (L.st == ST_NEED_ITEM && writer && p.cost_out)
        p.cost_out[L.item] = (uint32_t)__builtin_amdgcn_s_memtime() - p.cost_out[L.item];
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
template <int S = 1>
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
            end_path<S>(L, p);
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
            end_path<S>(L, p);
            return;
        }
        if (m.isEdgeHighlight && L.bounce > 1)
            L.d = prevDir;
        else
            L.rayColor = mul(L.rayColor, atten);
        float pr = fmaxf(L.rayColor.x, fmaxf(L.rayColor.y, L.rayColor.z));
        if (rnd(L.seed) > pr) {
            end_path<S>(L, p);
            return;
        }
        L.rayColor = muls(L.rayColor, 1.0f / pr);
        if (L.bounce >= p.maxBounce) end_path<S>(L, p);
    } else {
        if (p.envLight) L.incoming = add(L.incoming, mul(sky(L.d), L.rayColor));
        end_path<S>(L, p);
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
}

template <int S = 1>
__device__ __forceinline__ void flush_counters(const Lane& L, const RenderParams& p) {
    unsigned long long s = L.segs;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    if (lane_id() == 0 && split_writer<S>()) atomicAdd(p.seg_counter, s);
}

}  // namespace
