// Brute-force render kernels (the north-star path): every segment's closest hit
// is a sweep over all triangles in array order (compute.glsl:410-460 with the
// BVH replaced by the full triangle list; the same hit except on exact distance
// ties, which keep the lowest index).
//
// Each kernel is parameterised by a named spec (C++20 class template argument):
//   SmemSpec     records through the scalar data cache (product default)
//   SplitSpec    several waves per 64 rays, each sweeping a share of the triangles
//   TiledSpec    records streamed through LDS tiles (large scenes)
//   ResidentSpec whole scene resident in LDS (experiment builds)
// The assist kernel (idle waves help busy ones; multi-GPU slabs) is in
// rt2_assist.h.  Included by rt2_render.hip only (one translation unit;
// internal linkage).
#pragma once

namespace {

struct SmemSpec {
    int block;       // threads per workgroup
    int group;       // triangles per filter group (phase 1 width)
    Filter filter;
    Tail tail;       // drain-phase mode
    int tail_lanes;  // the tail mode starts when at most this many lanes trace
    int waves;       // minimum waves per SIMD the register allocation must allow (1 = unconstrained)
    bool stats;      // diagnostic build: filter survivor counters
    bool lockstep = false;  // one workgroup barrier per segment: the waves start their sweeps together
};
struct SplitSpec {
    int waves_per_ray;  // S: waves that trace the same 64 rays (1/S of the triangles each)
    int group;
    Filter filter;
    int waves;
};
struct TiledSpec {
    int block;
    int group;
    Filter filter;
};
struct ResidentSpec {
    int block;
    int group;
    Filter filter;
};

// RESIDENT: all triangles in LDS, waves independent after the initial load.
template <ResidentSpec S>
__global__ __launch_bounds__(S.block) void render_resident(RenderParams p) {
    extern __shared__ float4 lds[];
    const int n4 = 3 * p.n_tris;
    for (int i = threadIdx.x; i < n4; i += S.block) lds[i] = p.tri[i];
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
            sweep_masked<S.group, false, S.filter>(L.o, L.d, lds, nullptr, p.n_tris, 0, best, bi, bestK);
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
}

// TILED: triangles streamed through LDS in tiles of p.tile_tris (coalesced
// 16-B loads); the workgroup sweeps each tile in lockstep, so one tile serves
// all S.block lanes.
template <TiledSpec S>
__global__ __launch_bounds__(S.block) void render_tiled(RenderParams p) {
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
            for (int i = threadIdx.x; i < 3 * cnt; i += S.block) lds[i] = p.tri[3 * base + i];
            __syncthreads();
            if (tracing) sweep_masked<S.group, false, S.filter>(o, d, lds, nullptr, cnt, base, best, bi, bestK);
        }
        if (tracing) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
}

// SMEM: no LDS; triangles reach the VALU through the scalar cache.  With a
// tail mode, once the item pool is exhausted (some lane is DONE) and at most
// S.tail_lanes lanes of the wave still trace, the live rays' closest hits are
// computed by several lanes each (coop_closest / team_closest).  Lockstep:
// the workgroup's waves start every segment's sweep together (one barrier per
// segment), so the record lines one wave brings into the scalar cache serve
// the others (config B: 521-523 vs 520-557 ms free-running, same bits).
template <SmemSpec S>
__device__ __forceinline__ void smem_body(const RenderParams& p) {
    FiltStats fs;
    Lane L;
    lane_init(L);
    for (;;) {
        advance(L, p);
        const unsigned long long act = __ballot(L.st == ST_TRACE);
        if constexpr (S.lockstep) {
            if (!__syncthreads_or(act != 0)) break;
            if (!act) continue;
        } else {
            if (!act) break;
        }
        if constexpr (S.tail == Tail::Team) {
            if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE)) {
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
        }
        if constexpr (S.tail == Tail::Coop) {
            if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE)) {
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
        }
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            float best = 1e38f, bestK = 1e38f * 1.0009765625f;
            int bi = -1;
            const f3 o = L.o, d = L.d;
            if constexpr (S.filter == Filter::Plk) {
                // per-ray precomputed filter when the scene and every tracing
                // lane of the wave are inside its validated range
                if (p.plk && __ballot(!plk_lane_ok(o, d)) == 0)
                    sweep_plk<S.group, S.stats>(o, d, (const float*)p.plk, (const float*)p.tri, p.n_tris, p.plk_A,
                                                best, bi, bestK, &fs);
                else
                    sweep_masked<8, true, Filter::Max3, S.stats>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0,
                                                                 best, bi, bestK, &fs);
            } else {
                sweep_masked<S.group, true, S.filter, S.stats>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best,
                                                               bi, bestK, &fs);
            }
            shade(L, p, best, bi);
        }
    }
    if constexpr (S.stats) fs.flush(p.seg_counter + 20);
    flush_counters(L, p);
}

template <SmemSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_smem(RenderParams p) {
    smem_body<S>(p);
}

// SPLIT: the S waves of a workgroup trace the same 64 rays (same items, same
// RNG streams, identical shading); wave w sweeps the w-th contiguous 1/S of the
// triangle array, and the partial closest hits are combined through LDS in
// wave order with strict < (a lower range wins a tie): the sequential scan's
// (dst, index).  Per-ray latency falls by ~S at the same lane efficiency, for
// launches with few items per lane (a 1/8 slab of config B on 8 GPUs).
template <SplitSpec S>
__global__ __launch_bounds__(64 * S.waves_per_ray) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_split(
    RenderParams p) {
    constexpr int NW = S.waves_per_ray;
    __shared__ float part_best[NW][64];
    __shared__ int part_bi[NW][64];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform: scalar loads below
    const int lane = (int)(threadIdx.x & 63);
    const int per = ((p.n_tris + NW - 1) / NW + S.group - 1) / S.group * S.group;  // whole groups per wave
    const int lo = min(w * per, p.n_tris), hi = min(lo + per, p.n_tris);
    const float* tri = (const float*)p.tri + 12 * (size_t)lo;
    Lane L;
    lane_init(L);
    for (;;) {
        advance<NW>(L, p);
        if (!__any(L.st == ST_TRACE)) break;  // the same in every wave of the group
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        if (L.st == ST_TRACE) sweep_masked<S.group, true, S.filter>(L.o, L.d, nullptr, tri, hi - lo, lo, best, bi, bestK);
        part_best[w][lane] = best;
        part_bi[w][lane] = bi;
        __syncthreads();
        best = part_best[0][lane];
        bi = part_bi[0][lane];
#pragma unroll
        for (int k = 1; k < NW; k++) {
            const float ob = part_best[k][lane];
            if (ob < best) {
                best = ob;
                bi = part_bi[k][lane];
            }
        }
        __syncthreads();
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            shade<NW>(L, p, best, bi);
        }
    }
    flush_counters<NW>(L, p);
}

}  // namespace
