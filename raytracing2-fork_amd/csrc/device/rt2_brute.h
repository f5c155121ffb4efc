// Brute-force render kernels: RESIDENT, TILED and SMEM (north-star path).
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

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
                if constexpr (MT >= 500) {
                    sweep_masked<MT - 500, false, 1>(o, d, lds, nullptr, cnt, base, best, bi, bestK);
                } else if constexpr (MT >= 100) {
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
template <int BLOCK, int G, int COOP>
__device__ __forceinline__ void smem_body(const RenderParams& p) {
    cfloat* tri = (cfloat*)p.tri;
    constexpr bool kStats = G >= 700 && G < 900;  // diagnostic builds: filter survivor counters
    FiltStats fs;
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
            if constexpr (G >= 800) {
                sweep_masked<G - 800, true, 1, true>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK,
                                                    &fs);
            } else if constexpr (G >= 700) {
                if (p.plk && __ballot(!plk_lane_ok(o, d)) == 0)
                    sweep_plk<G - 700, true>(o, d, (const float*)p.plk, (const float*)p.tri, p.n_tris, p.plk_A, best,
                                             bi, bestK, &fs);
                else
                    sweep_masked<8, true, 1, true>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK,
                                                   &fs);
            } else if constexpr (G >= 600) {
                // per-ray precomputed filter when the scene and every tracing
                // lane of the wave are inside its validated range
                if (p.plk && __ballot(!plk_lane_ok(o, d)) == 0)
                    sweep_plk<G - 600>(o, d, (const float*)p.plk, (const float*)p.tri, p.n_tris, p.plk_A, best, bi,
                                       bestK);
                else
                    sweep_masked<8, true, 1>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
            } else if constexpr (G >= 500)
                sweep_masked<G - 500, true, 1>(o, d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
            else if constexpr (G >= 400)
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
    if constexpr (kStats) fs.flush(p.seg_counter + 20);
    flush_counters(L, p);
}

template <int BLOCK, int G, int COOP, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void render_smem(RenderParams p) {
    smem_body<BLOCK, G, COOP>(p);
}
// SPLIT: the S waves of a workgroup trace the same 64 rays (same items, same
// RNG streams, identical shading); wave w sweeps the w-th contiguous 1/S of the
// triangle array, and the partial closest hits are combined through LDS in
// wave order with strict < (a lower range wins a tie): the sequential scan's
// (dst, index).  Per-ray latency falls by ~S at the same lane efficiency, for
// launches with few items per lane (a 1/8 slab of config B on 8 GPUs).
template <int S, int G, int FILT, int WPE>
__global__ __launch_bounds__(64 * S) __attribute__((amdgpu_waves_per_eu(WPE))) void render_split(RenderParams p) {
    __shared__ float part_best[S][64];
    __shared__ int part_bi[S][64];
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform: scalar loads below
    const int lane = (int)(threadIdx.x & 63);
    const int per = ((p.n_tris + S - 1) / S + G - 1) / G * G;  // whole groups of G per wave
    const int lo = min(w * per, p.n_tris), hi = min(lo + per, p.n_tris);
    const float* tri = (const float*)p.tri + 12 * (size_t)lo;
    Lane L;
    lane_init(L);
    for (;;) {
        advance<S>(L, p);
        if (!__any(L.st == ST_TRACE)) break;  // the same in every wave of the group
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        if (L.st == ST_TRACE) sweep_masked<G, true, FILT>(L.o, L.d, nullptr, tri, hi - lo, lo, best, bi, bestK);
        part_best[w][lane] = best;
        part_bi[w][lane] = bi;
        __syncthreads();
        best = part_best[0][lane];
        bi = part_bi[0][lane];
#pragma unroll
        for (int k = 1; k < S; k++) {
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
            shade<S>(L, p, best, bi);
        }
    }
    flush_counters<S>(L, p);
}

}  // namespace
