// Experiment (variants 269/270): the LDS record tiles of rt2_k5_tiles.h with
// the per-tile workgroup barrier replaced by per-buffer LDS counters, so that
// a wave waits only for what it needs.  Included by rt2_render.hip only.
//
// Why: in render_mfma_k5t every wave passes one __syncthreads per tile, so
// each tile costs the workgroup its slowest wave's time on it — a wave whose
// rays hit many groups (exact phase) holds the other eleven.  The PMC of the
// default kernel (217, config C) has the waves waiting on a counter or a
// barrier in 46 % of their cycles.
//
// How (double buffering, tile g of the workgroup's sequence in buffer g & 1):
//   land[b]: +1 per wave once its LDS-DMA pieces of the buffer's tile landed;
//            tile g is readable when land[b] = NW (g / 2 + 1);
//   done[b]: +1 per wave once it has read the buffer's tile; tile g + 2 may
//            be issued into it when done[b] = NW (g / 2 + 1).
// A wave issues its pieces of tile t + 1 as soon as every wave has finished
// tile t - 1 (checked between groups, waited for at the end of tile t) and
// signals their landing one group later, so a fast wave runs up to one tile
// ahead of the slowest instead of meeting it at every tile.  The segment's
// vote barrier (block_any) still joins all waves between segments, and every
// wave (sweeping or not) issues, signals and counts every tile, so each
// counter reaches its target: a wave waiting for tile t needs only waves that
// are at tile t - 1 or later, which can always proceed.
//
// Arithmetic: sweep_k5_tiles's cthr group (k5_cthr_group) and exact phase,
// unchanged: the image is the sequential strict `dst < best` scan's.
#pragma once

namespace {

struct TileSync {
    uint32_t land[2], done[2];
};

__device__ __forceinline__ uint32_t lds_load_acq(uint32_t* c) {
    return (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}
__device__ __forceinline__ void lds_wait_geq(uint32_t* c, uint32_t target) {
    while (lds_load_acq(c) < target) __builtin_amdgcn_s_sleep(1);
}
// +1 by this wave, after its earlier LDS / LDS-DMA work is complete
__device__ __forceinline__ void lds_signal(uint32_t* c) {
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane_id() == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <MfmaSpec S, class SH>
__device__ __forceinline__ bool sweep_k5_dtiles(const RenderParams& p, SH& sh, K5Tiles<S.tile_groups, 2>& tl,
                                                TileSync& ts, uint32_t& gbase, const f3& o, const f3& d, float& best,
                                                int& bi, float& bestK, MfmaDiag& dg, bool sweeping, bool upper) {
    static_assert(S.k5 && S.no_tn && S.cthr && S.rows80 && S.tile_bufs == 2 && S.tile_groups > 0, "the cthr tile form");
    constexpr int K = S.tile_groups, NW = S.block / 64;
    constexpr int YO = 16;
    const int lane = (int)lane_id();
    const int r32 = lane & 31, hl = lane >> 5, wave = (int)(threadIdx.x >> 6);
    MfmaScale sc{0.0f, 0.0f, 0.0f};
    float zlo = 0.0f, zhi = 0.0f;
    h8 a0[2], y1[2];
    ThrBits thr = {};
    bool compute = false, in_range = true;
    auto write_y = [&](float bkv) {
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bkv, sc.sigma, sc.Bmax);
        h8* row = reinterpret_cast<h8*>(&sh.ray[lane][YO]);
        row[0] = h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
        row[1] = h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]};
    };
    auto read_y = [&]() {
#pragma unroll
        for (int R = 0; R < 2; R++) y1[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][YO + 8 * hl]);
    };
    if (sweeping) {
        const f3 m = cross(d, o);
        in_range = mfma_scale<S>(p.mfma_A, o, d, m, sc);
        if (in_range) {
            mfma_main_row_half(&sh.ray[lane][0], d, m, sc.sigma);
            const float vz = m.z * sc.sigma;
            const _Float16 hz = (_Float16)vz;
            const _Float16 lz = (_Float16)(vz - (float)hz);
            zhi = wave_max_s<S>(fabsf((float)hz));
            zlo = wave_max_s<S>(fabsf((float)lz));
            thr = mfma_thr_bits(sc.Tw, zlo, zhi);
            write_y(bestK);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int R = 0; R < 2; R++) a0[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][8 * hl]);
            read_y();
            compute = true;
        }
    }
    const int ng = (p.n_tris + 31) >> 5, nt = (ng + K - 1) / K;
    const uint32_t g0 = gbase;
    gbase += (uint32_t)nt;
    const h8* gsrc = reinterpret_cast<const h8*>(p.mfma_k16_frag);
    // this wave's LDS-DMA pieces of segment tile t (global tile g0 + t, buffer
    // (g0 + t) & 1): 4 record pieces of 1 KiB per group, round-robin
    auto issue = [&](int t) {
        const int gg = t * K, gn = min(K, ng - gg), nrec = gn * 4;
        const uint32_t b = (g0 + (uint32_t)t) & 1u;
        for (int pc = wave; pc < nrec; pc += NW) {
            const int gi = pc >> 2, op = 2 * (pc & 3);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(gsrc + ((size_t)(gg + gi) * kK16Ops + op) * 64 + lane),
                (__attribute__((address_space(3))) void*)&tl.rec[b][pc * 64], 16, 0, 0);
        }
    };
    // every wave has read global tile g (its buffer's (g / 2 + 1)-th use)
    auto read_by_all = [&](uint32_t g) { return lds_load_acq(&ts.done[g & 1u]) >= (uint32_t)NW * (g / 2u + 1u); };
    int issued = 0, signalled = 0;
    bool fresh = false;  // a tile was issued since the last landing check
    // the segment's first two tiles: their buffers' earlier tiles were read by
    // every wave before the segment's vote barrier
    issue(0);
    issued = 1;
    if (nt > 1) {
        issue(1);
        issued = 2;
    }
    lds_signal(&ts.land[g0 & 1u]);
    signalled = 1;
    if (nt > 1) {
        lds_signal(&ts.land[(g0 + 1u) & 1u]);
        signalled = 2;
    }
    // between groups of tile t: issue tile t + 1 once tile t - 1 is read by
    // every wave; signal an issued tile's landing one call later
    auto progress = [&](int t) {
        if (signalled < issued && !fresh) {
            lds_signal(&ts.land[(g0 + (uint32_t)signalled) & 1u]);
            signalled++;
        }
        fresh = false;
        if (issued == t + 1 && t + 1 < nt && read_by_all(g0 + (uint32_t)t - 1u)) {
            issue(t + 1);
            issued++;
            fresh = true;
        }
    };
    for (int t = 0; t < nt; t++) {
        const uint32_t g = g0 + (uint32_t)t, b = g & 1u;
        lds_wait_geq(&ts.land[b], (uint32_t)NW * (g / 2u + 1u));
        if (compute) {
            const int gn = min(K, ng - t * K);
            for (int gi = 0; gi < gn; gi++) {
                if (t >= 1) progress(t);
                const int G = t * K + gi;
                const h8* tb = &tl.rec[b][gi * 4 * 64 + lane];
                const h8 b0 = tb[0], b2 = tb[64], b4 = tb[128], b6 = tb[192];
                const unsigned long long M = k5_cthr_group<S>(thr, a0, y1, b0, b2, b4, b6, upper, sh);
                if constexpr (S.diag) dg.groups += 1;
                if (M) {
                    if constexpr (S.diag) dg.hot += 1;
                    uint32_t m32 = (uint32_t)(M | M >> 32);
                    const float bk0 = bestK;
                    while (m32) {
                        const int tt = __builtin_ctz(m32);
                        m32 &= m32 - 1;
                        const int idx = 32 * G + tt;
                        if (idx >= p.n_tris) break;
                        if constexpr (S.diag) dg.exact += 1;
                        cfloat* tp = (cfloat*)p.tri + 12 * idx;
                        const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                        if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
                    }
                    if (__ballot(bestK != bk0)) {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        write_y(bestK);
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();
                        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                        read_y();
                    }
                }
            }
        }
        lds_signal(&ts.done[b]);  // this wave has read tile g
        if (t + 1 < nt) {
            // tile t + 1 issued (its buffer's tile t - 1 read by every wave)
            // and its landing signalled before this wave moves on
            if (issued == t + 1) {
                while (!read_by_all(g - 1u)) __builtin_amdgcn_s_sleep(1);
                issue(t + 1);
                issued++;
            }
            if (signalled == t + 1) {
                lds_signal(&ts.land[(g + 1u) & 1u]);
                signalled++;
            }
        }
        fresh = false;
    }
    return in_range;
}

// render_mfma_k5t's segment loop around sweep_k5_dtiles (path state in
// registers, 80-B rows).
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_k5d(RenderParams p_arg) {
    static_assert(S.lane_lds == 0 && S.rows80 && S.lockstep, "lockstep segments, path state in registers");
    constexpr int NW = S.block / 64;
    __shared__ MfmaK5rLds wl[NW];
    __shared__ K5Tiles<S.tile_groups, 2> tl;
    __shared__ TileSync ts;
    __shared__ BlockVote<NW> vote;
    uint32_t vote_parity = 0, gbase = 0;
    MfmaK5rLds& sh = wl[threadIdx.x >> 6];
    if (threadIdx.x < 4) (&ts.land[0])[threadIdx.x] = 0u;
    __syncthreads();
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    for (;;) {
        const RenderParams& p = kargs<RenderParams>();
        advance(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        if (!block_any<NW>(act != 0, vote, vote_parity)) break;
        const bool coop = act != 0 && __popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE);
        const bool sweeping = act != 0 && !coop;
        bool upper = true;
        if constexpr (S.compact) {
            if (sweeping && __popcll(act) <= 32) {
                if (act >> 32) {
                    const uint32_t l = lane_id(), nl = (uint32_t)__popcll(act);
                    const bool live = (act >> l) & 1ull;
                    const int to = 4 * (int)(live ? lanes_below(act) : nl + lanes_below(~act));
                    lane_permute(L, to);
                    act = __ballot(L.st == ST_TRACE);
                }
                upper = false;
            }
        }
        const bool mine = L.st == ST_TRACE;
        if (sweeping) {
            const int j0 = __builtin_ctzll(act);
            const f3 o = mk(__shfl(L.o.x, j0), __shfl(L.o.y, j0), __shfl(L.o.z, j0));
            const f3 dd = mk(__shfl(L.d.x, j0), __shfl(L.d.y, j0), __shfl(L.d.z, j0));
            if (!mine) {
                L.o = o;
                L.d = dd;
            }
        }
        const f3 ro = L.o, rd = L.d;
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        const bool swept = sweep_k5_dtiles<S>(p, sh, tl, ts, gbase, ro, rd, best, bi, bestK, dg, sweeping, upper);
        L.o = ro;
        L.d = rd;
        if (coop) {
            float mybest = 1e38f;
            int mybi = -1;
            coop_each(act, L.o, L.d, p, mybest, mybi);
            if (mine) {
                L.bounce += 1;
                L.segs += 1;
                shade(L, p, mybest, mybi);
            }
            continue;
        }
        if (!act) continue;
        if (!swept) coop_each(act, ro, rd, p, best, bi);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    const RenderParams& p = kargs<RenderParams>();
    flush_counters(L, p);
}

}  // namespace
