// The 5-product matrix filter (rt2_mfma.h, MfmaSpec::k5) with its record
// operands streamed through workgroup-shared LDS tiles: the north star's
// "triangle arrays streamed from HBM in coalesced tiles and staged in LDS".
// Included by rt2_render.hip only (one translation unit; internal linkage).
//
// What it replaces: in render_mfma every wave loads its own copy of each
// 32-triangle group's records (4 operands x 1 KiB + tau + the m.z bound) from
// L2/MALL — for a 100k-triangle scene 12.8 MB per wave-segment, about 2 B per
// (ray, triangle) pair, half of it missing the L2 (DESIGN.md, config C PMC).
// The reference reads `triangles[i]` from SSBO 1 in every leaf test
// (compute.glsl:429-431, block :75-78).
//
// Here the NW waves of a workgroup (one workgroup per CU) sweep the same
// records in the same order, so each tile of K groups is brought into LDS
// once per workgroup and segment, by LDS-DMA (global_load_lds_dwordx4: 1-KiB
// coalesced pieces, no VGPRs), split across the waves and double-buffered:
// tile t+1 is in flight while tile t is swept.  One barrier per tile.  The
// record traffic from L2 falls NW-fold.  The arithmetic of every product,
// threshold and exact test is sweep_k16's 5-product form term for term, so
// the result is the sequential strict `dst < best` scan's bit for bit.
//
// Register budget: the k16 tiled attempt (render_mfma_tiled) kept the path
// state in VGPRs across the tile loop and spilled 45 of them.  The first form
// here (MfmaSpec::lane_lds = 2, variant 252) parks it in LDS (the packed
// 15-word stash of the 4-wave build); with round 4's register changes and
// 80-B fragment rows it fits in registers (lane_lds = 0, rows80: variants
// 213 and 217, 10-group tiles), and with MfmaSpec::cthr the threshold rides
// in the products' accumulator (k5_cthr_group), so the tiles carry no bounds
// or scales.
#pragma once

namespace {

// LDS of one workgroup's record tiles: 2 buffers x K groups x the 4 operands
// the 5-product form reads (U0, V0, X0, T1: k16 ops 0, 2, 4, 6) as 64 lanes x
// 16 B, the per-triangle scale tau and the m.z residual bound.
template <int K, int NB = 2, bool SCALES = true>
struct K5Tiles {
    h8 rec[NB][K * 4 * 64];
    float tau[NB][K * 32];
    float2 bnd[NB][K * 32];
};
// MfmaSpec::cthr: the -tn record carries the threshold, the tiles hold the
// records alone
template <int K, int NB>
struct K5Tiles<K, NB, false> {
    h8 rec[NB][K * 4 * 64];
};

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// wait until at most n of this wave's vector-memory operations are in flight
// (the youngest n: the pieces of the tiles issued after the awaited one)
__device__ __forceinline__ void wait_vm(int n) {
    if (n <= 0)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (n == 1)
        asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if (n == 2)
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else
        asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
}

// Closest hit of every lane's ray over all triangles, or (sweeping = false)
// only the workgroup's tile traffic and barriers: every wave of the workgroup
// calls it in every segment the workgroup runs.  Returns false when the wave's
// rays are outside the filter's range (nothing computed; wave-uniform).
template <MfmaSpec S, class SH>
__device__ __forceinline__ bool sweep_k5_tiles(const RenderParams& p, SH& sh,
                                               K5Tiles<S.tile_groups, S.tile_bufs, !(S.cthr || S.kthr)>& tl,
                                               const f3& o, const f3& d, float& best, int& bi, float& bestK,
                                               MfmaDiag& dg, bool sweeping, bool upper) {
    static_assert(S.k5 && S.ymma && S.imax && S.minred && S.tile_groups > 0, "the 5-product form");
    static_assert(!S.rows80 || S.no_tn, "80-B rows hold the first K-half of the main fragment only");
    static_assert(S.tile_bufs >= 2 && S.tile_bufs <= 3, "double or triple buffering");
    constexpr int K = S.tile_groups, NW = S.block / 64, NB = S.tile_bufs;
    constexpr int YO = S.rows80 ? 16 : 32;  // the Y slots' offset in a row
    const int lane = (int)lane_id();
    const int r32 = lane & 31, hl = lane >> 5, wave = (int)(threadIdx.x >> 6);
    MfmaScale sc{0.0f, 0.0f, 0.0f};
    float zlo = 0.0f, zhi = 0.0f;
    h8 a0[2], a1[2], y1[2];
    [[maybe_unused]] ThrBits thr = {};
    [[maybe_unused]] _Float16 tw16 = (_Float16)0.0f;  // kthr: Tw' for the Y rebuilds
    bool compute = false, in_range = true;
    auto write_y = [&](float bkv) {
        if constexpr (S.kthr) {
            kt_y(d, o, bkv, sc, tw16, y1);
            return;
        }
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bkv, sc.sigma, sc.Bmax);
        if constexpr (S.perm_frag) {
            frag_pair(s, y1);  // in registers: no rows, no wave barrier
        } else {
            h8* row = reinterpret_cast<h8*>(&sh.ray[lane][YO]);
            row[0] = h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
            row[1] = h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]};
        }
    };
    auto read_y = [&]() {
        if constexpr (!S.perm_frag) {
#pragma unroll
            for (int R = 0; R < 2; R++) y1[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][YO + 8 * hl]);
        }
    };
    if (sweeping) {
        const f3 m = cross(d, o);
        in_range = mfma_scale<S>(p.mfma_A, o, d, m, sc);
        if (in_range && S.kthr) {
            // MfmaSpec::kthr: the threshold in the K-slots (register fragments)
            kt_frags<S>(d, m, sc, a0, tw16);
            write_y(bestK);
            compute = true;
        } else if (in_range && S.perm_frag) {
            // MfmaSpec::perm_frag: the fragments built in registers by
            // v_permlane32_swap (rt2_k5_resident.h frag_pair), no LDS rows
            _Float16 s[18];
            mfma_main_half_slots(s, d, m, sc.sigma);
            frag_pair(s, a0);
            const float vz = m.z * sc.sigma;
            const _Float16 hz = (_Float16)vz;
            const _Float16 lz = (_Float16)(vz - (float)hz);
            zhi = wave_max_s<S>(fabsf((float)hz));
            zlo = wave_max_s<S>(fabsf((float)lz));
            if constexpr (S.cthr) thr = mfma_thr_bits(sc.Tw, zlo, zhi);
            write_y(bestK);
            compute = true;
        } else if (in_range) {
            if constexpr (S.rows80)
                mfma_main_row_half(&sh.ray[lane][0], d, m, sc.sigma);
            else
                mfma_main_row(&sh.ray[lane][0], d, m, o, sc.sigma);
            // the wave's largest |ray lo| and |ray hi| of m.z (sweep_k16's k5 bound)
            const float vz = m.z * sc.sigma;
            const _Float16 hz = (_Float16)vz;
            const _Float16 lz = (_Float16)(vz - (float)hz);
            zhi = wave_max_s<S>(fabsf((float)hz));
            zlo = wave_max_s<S>(fabsf((float)lz));
            if constexpr (S.cthr) thr = mfma_thr_bits(sc.Tw, zlo, zhi);
            write_y(bestK);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int R = 0; R < 2; R++) {
                a0[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][8 * hl]);
                if constexpr (!S.no_tn) a1[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][16 + 8 * hl]);
            }
            read_y();
            compute = true;
        }
    }
    const int ng = (p.n_tris + 31) >> 5, nt = (ng + K - 1) / K;
    const h8* gsrc = reinterpret_cast<const h8*>(S.kthr ? p.mfma_kt_frag : p.mfma_k16_frag);
    // LDS-DMA of tile t into buffer t % NB, round-robin over the waves: 4 record
    // pieces per group (1 KiB each: a lane's 16 B land at base + 16 lane),
    // then the groups' bounds (256 B per group) and scales (128 B per group)
    // as 16-B pieces with the lanes past the tile's end masked off
    auto issue = [&](int t) {
        const int g0 = t * K, gn = min(K, ng - g0);
        // cthr: the -tn record carries the threshold; no bounds or scales
        const int nrec = gn * 4, nbnd = (S.cthr || S.kthr) ? 0 : (gn * 16 + 63) / 64, ntau = (S.cthr || S.kthr) ? 0 : (gn * 8 + 63) / 64;
        const int b = t % NB;
        for (int pc = wave; pc < nrec + nbnd + ntau; pc += NW) {
            if (pc < nrec) {
                const int gi = pc >> 2, op = S.kthr ? (pc & 3) : 2 * (pc & 3);  // kt: 4 contiguous ops per group
                __builtin_amdgcn_global_load_lds(
                    (const __attribute__((address_space(1))) void*)(gsrc + ((size_t)(g0 + gi) * (S.kthr ? kKtOps : kK16Ops) + op) * 64 + lane),
                    (__attribute__((address_space(3))) void*)&tl.rec[b][pc * 64], 16, 0, 0);
            } else if constexpr (S.cthr || S.kthr) {
                // (no bound or scale pieces)
            } else if (pc < nrec + nbnd) {
                const int q = pc - nrec;
                if (64 * q + lane < gn * 16)
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(reinterpret_cast<const float4*>(
                                                                            p.mfma_k16_bnd + 32 * (size_t)g0) +
                                                                        64 * q + lane),
                        (__attribute__((address_space(3))) void*)&tl.bnd[b][128 * q], 16, 0, 0);
            } else {
                const int q = pc - nrec - nbnd;
                if (64 * q + lane < gn * 8)
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void*)(reinterpret_cast<const float4*>(
                                                                            p.mfma_k16_tau + 32 * (size_t)g0) +
                                                                        64 * q + lane),
                        (__attribute__((address_space(3))) void*)&tl.tau[b][256 * q], 16, 0, 0);
            }
        }
    };
    // this wave's pieces of tile t (issued round-robin: pc = wave, wave + NW, ...)
    auto my_pieces = [&](int t) {
        const int gn = min(K, ng - t * K);
        const int n = gn * 4 + ((S.cthr || S.kthr) ? 0 : (gn * 16 + 63) / 64 + (gn * 8 + 63) / 64);
        return wave < n ? (n - wave + NW - 1) / NW : 0;
    };
    for (int t = 0; t < NB - 1 && t < nt; t++) issue(t);
    for (int t = 0; t < nt; t++) {
        // this wave's pieces of tile t have landed (the tiles issued after it
        // may still be in flight: NB = 3 keeps tile t + 1's)
        if constexpr (NB == 2)
            wait_vm0();
        else
            wait_vm(t + 1 < nt ? my_pieces(t + 1) : 0);
        __syncthreads();  // every wave's have; every wave is done with buffer (t + NB - 1) % NB (tile t - 1)
        if (t + NB - 1 < nt) issue(t + NB - 1);
        if (!compute) continue;
        const int b = t % NB, gn = min(K, ng - t * K);
        // a group's operands from the tile; MfmaSpec::prefetch: the next
        // group's are read (into a second register set) before this group's
        // products, so the LDS latency overlaps them
        h8 nb[4];
        float ntau = 0.0f;
        float2 nbnd = make_float2(0.0f, 0.0f);
        auto lds_fetch = [&](int gi) {
            const h8* tb = &tl.rec[b][gi * 4 * 64 + lane];
            nb[0] = tb[0];
            nb[1] = tb[64];
            nb[2] = tb[128];
            nb[3] = tb[192];
            if constexpr (!(S.cthr || S.kthr)) {
                ntau = tl.tau[b][gi * 32 + r32];
                nbnd = tl.bnd[b][gi * 32 + r32];
            }
        };
        if constexpr (S.prefetch) lds_fetch(0);
        for (int gi = 0; gi < gn; gi++) {
            const int G = t * K + gi;
            if constexpr (!S.prefetch) lds_fetch(gi);
            const h8 b0 = nb[0], b2 = nb[1], b4 = nb[2], b6 = nb[3];
            const float tau = ntau;
            const float2 bnd = nbnd;
            if constexpr (S.prefetch)
                if (gi + 1 < gn) lds_fetch(gi + 1);
            // sweep_k16's threshold: tau T + the bound of the left-out m.z
            // slots, padded by 2^-10 for its own rounding ("The
            // 5-product form")
            unsigned long long M;
            if constexpr (S.kthr) {
                M = kt_group<S>(a0, y1, b0, b2, b4, b6, upper);
            } else if constexpr (S.cthr) {
                M = k5_cthr_group<S>(thr, a0, y1, b0, b2, b4, b6, upper, sh);
            } else {
            const float Tl = tau * sc.Tw + (bnd.x * zlo + bnd.y * zhi) * 1.0009765625f;
            int tmin = 0x7fffffff;
#pragma unroll
            for (int R = 0; R < 2; R++) {
                if (R == 1 && !upper) break;
                const f16v zero = {};
                const f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b0, zero, 0, 0, 0);
                const f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b2, zero, 0, 0, 0);
                const f16v X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b4, zero, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                int t3[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    t3[i] = max(max(__float_as_int(U[i]), __float_as_int(V[i])), __float_as_int(X[i]));
                __builtin_amdgcn_sched_barrier(0);
                f16v T = {};
                if constexpr (!S.no_tn) T = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b6, zero, 0, 0, 0);
                const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], b6, zero, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    if constexpr (S.no_tn)
                        tmin = min(tmin, max(t3[i], __float_as_int(Y[i])));
                    else
                        tmin = min(tmin, max(max(t3[i], __float_as_int(T[i])), __float_as_int(Y[i])));
                }
                if (R == 1) __builtin_amdgcn_sched_barrier(0);
            }
            M = __ballot(tmin <= __float_as_int(Tl));
            }
            if constexpr (S.diag) dg.groups += 1;
            if (M) {
                if constexpr (S.diag) dg.hot += 1;
                // triangles of the group with a passing pair: the exact phase, in index order
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
                    if constexpr (S.perm_frag) {
                        write_y(bestK);
                    } else {
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                        __builtin_amdgcn_wave_barrier();  // every lane has read the rows' previous Y slots
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
    }
    return in_range;
}

// MfmaSpec::tile_flow — the record tiles as a stream with LDS counters instead
// of a workgroup barrier per tile (round 6; DESIGN.md "LDS record tiles").
// With one barrier per tile the 12 waves meet 165 times per config C segment
// and wait for the slowest of them every time.  Here a wave waits only for
// the tile it is about to read: the waves drift apart by up to a tile and a
// wave that is behind is not waited for until it holds the stream up.
//
// Every wave walks the same stream of tiles (stream index s: tile s % nt of
// the segment, buffer s % NB; a segment is nt consecutive indices, so the
// index runs on across segments) and, per tile: waits until all NW shares of
// tile s have landed in buffer b (landed[b] == NW * (s / NB + 1)), sweeps it
// (when it has rays), and releases it (rel[b] += 1).  Each wave issues its own
// share of each tile's LDS-DMA pieces (pc = wave, wave + NW, ...) once every
// wave has released the buffer's previous tile (rel[b] == NW * (s / NB)), and
// publishes the share (landed[b] += 1) after its own `s_waitcnt vmcnt(0)`, two
// groups later or at once when it is waiting anyway.  No wave reads a buffer
// before every share of its tile has landed, and no DMA overwrites a buffer
// before all NW waves released it.  MfmaSpec::flow_prio: a wave's issue
// priority for the next tile follows its finishing rank in this one (the
// last to finish take the SIMD's issue slots first).
template <int NB>
struct TileFlow {
    uint32_t landed[NB];  // per buffer: shares landed so far (NW per tile)
    uint32_t rel[NB];     // per buffer: releases so far (NW per tile)
};
// the wave's place in the stream (wave-uniform; kept across segments)
struct FlowWave {
    uint32_t next = 0;        // stream index of the next tile this wave reads
    uint32_t next_issue = 0;  // ... of the next tile this wave issues its share of
    int pend = -1;            // a share issued whose landing is not published yet
    int age = 0;              // groups swept since that share was issued
};

__device__ __forceinline__ uint32_t lds_acquire(uint32_t* a) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
}

template <MfmaSpec S, class TL, class FL>
__device__ __forceinline__ bool sweep_kt_flow(const RenderParams& p, TL& tl, FL& fl, FlowWave& fw, const f3& o,
                                              const f3& d, float& best, int& bi, float& bestK, MfmaDiag& dg,
                                              bool sweeping, bool upper) {
    static_assert(S.kthr && S.perm_frag && S.tile_groups > 0, "the kthr form with register fragments");
    constexpr int K = S.tile_groups, NW = S.block / 64, NB = S.tile_bufs;
    static_assert((NB & (NB - 1)) == 0 && NW % 2 == 0, "stream counters: NB a power of two, NW even (wrap-safe)");
    const int lane = (int)lane_id(), wave = (int)(threadIdx.x >> 6);
    // MfmaSpec::diag: shader clocks per phase (MfmaDiag t_wait / t_filt / t_exact / t_swp)
    [[maybe_unused]] unsigned long long tc = 0, tsw = 0;
    if constexpr (S.diag) tsw = tc = __builtin_amdgcn_s_memtime();
    auto stamp = [&](unsigned long long& acc) {
        if constexpr (S.diag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc += t - tc;
            tc = t;
        }
    };
    MfmaScale sc{0.0f, 0.0f, 0.0f};
    h8 a0[2], y1[2];
    _Float16 tw16 = (_Float16)0.0f;
    bool compute = false, in_range = true;
    if (sweeping) {
        const f3 m = cross(d, o);
        in_range = mfma_scale<S>(p.mfma_A, o, d, m, sc);
        if (in_range) {
            kt_frags<S>(d, m, sc, a0, tw16);
            kt_y(d, o, bestK, sc, tw16, y1);
            compute = true;
        }
    }
    const int ng = (p.n_tris + 31) >> 5, nt = (ng + K - 1) / K;
    const h8* gsrc = reinterpret_cast<const h8*>(p.mfma_kt_frag) + lane;
    // this wave's share of stream index s: pieces pc = wave, wave + NW, ...
    // (4 per group, 1 KiB each: a lane's 16 B land at base + 16 lane); the kt
    // records of a tile are contiguous
    auto issue_share = [&](uint32_t s) {
        const int g0 = (int)(s % (uint32_t)nt) * K, gn = min(K, ng - g0), b = (int)(s % NB);
        const h8* src = gsrc + (size_t)g0 * (kKtOps * 64);
        for (int pc = wave; pc < kKtOps * gn; pc += NW)
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + pc * 64),
                                             (__attribute__((address_space(3))) void*)&tl.rec[b][pc * 64], 16, 0, 0);
    };
    // the wave's part of the stream's upkeep: publish a share that has had
    // time to land (`force`: now), then issue the next share once every wave
    // has released that tile's buffer
    auto upkeep = [&](bool force, bool try_issue) {
        if (fw.pend >= 0 && (force || fw.age >= 2)) {
            [[maybe_unused]] unsigned long long t0 = 0;
            if constexpr (S.diag) t0 = __builtin_amdgcn_s_memtime();
            wait_vm0();  // this wave's pieces (its only vector-memory operations in flight) have landed
            if constexpr (S.diag) dg.t_pub += __builtin_amdgcn_s_memtime() - t0;
            if (lane == 0)
                __hip_atomic_fetch_add(&fl.landed[fw.pend % NB], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            fw.pend = -1;
        }
        if (fw.pend < 0 && try_issue) {
            const uint32_t s = fw.next_issue;
            if (lds_acquire(&fl.rel[s % NB]) == (uint32_t)NW * (s / NB)) {
                [[maybe_unused]] unsigned long long t0 = 0;
                if constexpr (S.diag) t0 = __builtin_amdgcn_s_memtime();
                issue_share(s);
                if constexpr (S.diag) {
                    dg.t_issue += __builtin_amdgcn_s_memtime() - t0;
                    dg.claims += 1;
                }
                fw.pend = (int)s;
                fw.age = 0;
                fw.next_issue = s + 1u;
            }
        }
    };
    for (int t = 0; t < nt; t++) {
        const uint32_t s = fw.next++;
        const int b = (int)(s % NB), gn = min(K, ng - t * K);
        stamp(dg.t_exact);
        upkeep(true, true);
        // (wrap-safe: the counters and stream index are 32-bit and may wrap in
        // a launch of hours; NB and NW even keep NW * (s / NB) consistent mod 2^32)
        // (bounded: a wait of 2^24 sleeps, ~1 s, cannot be a slow wave — a
        // tile takes ~20-40 k clocks — so the kernel traps instead of hanging)
        uint32_t spins = 0;
        while ((int32_t)(lds_acquire(&fl.landed[b]) - (uint32_t)NW * (s / NB + 1u)) < 0) {
            upkeep(true, true);
            __builtin_amdgcn_s_sleep(1);
            if (++spins == (1u << 24)) __builtin_trap();
        }
        stamp(dg.t_wait);
        if (compute) {
            const h8* tb = &tl.rec[b][lane];
            for (int gi = 0; gi < gn; gi++) {
                const int G = t * K + gi;
                const h8 b0 = tb[0], b1 = tb[64], b2 = tb[128], b3 = tb[192];
                tb += kKtOps * 64;
                fw.age++;
                upkeep(false, gi == K / 2);
                const unsigned long long M = kt_group<S>(a0, y1, b0, b1, b2, b3, upper);
                if constexpr (S.diag) dg.groups += 1;
                stamp(dg.t_filt);
                if (M) {
                    if constexpr (S.diag) dg.hot += 1;
                    // the exact phase, in index order (compute.glsl:302-340, strict `dst < best`)
                    uint32_t m32 = (uint32_t)(M | M >> 32);
                    const float bk0 = bestK;
                    while (m32) {
                        const int idx = 32 * G + __builtin_ctz(m32);
                        m32 &= m32 - 1;
                        if (idx >= p.n_tris) break;
                        if constexpr (S.diag) dg.exact += 1;
                        cfloat* tp = (cfloat*)p.tri + 12 * idx;
                        const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                        if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
                    }
                    if (__ballot(bestK != bk0)) kt_y(d, o, bestK, sc, tw16, y1);
                    stamp(dg.t_exact);
                }
            }
        }
        // done with buffer b (the LDS executes this wave's reads before the add)
        uint32_t r_old = 0;
        if (lane == 0) r_old = __hip_atomic_fetch_add(&fl.rel[b], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if constexpr (S.flow_prio) {
            const int rank = (int)(__builtin_amdgcn_readfirstlane(r_old) - (uint32_t)NW * (s / NB));
            const int q = rank * 4 / NW;
            if (q >= 3)
                __builtin_amdgcn_s_setprio(3);
            else if (q == 2)
                __builtin_amdgcn_s_setprio(2);
            else if (q == 1)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
    }
    if constexpr (S.flow_prio) __builtin_amdgcn_s_setprio(0);
    stamp(dg.t_exact);
    if constexpr (S.diag) dg.t_swp += __builtin_amdgcn_s_memtime() - tsw;
    return in_range;
}

// render_mfma's lockstep segment loop around sweep_k5_tiles: every wave of the
// workgroup takes part in every tile barrier of every segment the workgroup
// runs (block_any decides, workgroup-uniformly, whether it runs one), sweeping
// only when it has rays and is not in the cooperative drain.  With lane_lds ==
// 2 (experiment variants 250/252) the path state waits in LDS
// (lane_stash_packed) across the tile loop, and the launcher's "llds2" name
// check keeps those variants to launches the packed fields hold; the default
// (217, lane_lds == 0) keeps the path state in registers and has no such limit.
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_k5t(RenderParams p_arg) {
    static_assert((S.lane_lds == 2 || (S.lane_lds == 0 && S.rows80)) && S.lockstep, "lockstep segments");
    static_assert(!S.perm_frag || S.lane_lds == 0, "register fragments: the path state stays in registers too");
    constexpr int NW = S.block / 64;
    constexpr bool stash = S.lane_lds == 2;  // the path state waits in LDS across the tile loop
    using WL = std::conditional_t<S.rows80, std::conditional_t<stash, MfmaK5nLds, MfmaK5rLds>, MfmaK16PackedLds>;
    // MfmaSpec::perm_frag: no fragment rows (one row array serves as a dummy
    // the sweep never touches)
    __shared__ WL wl[S.perm_frag ? 1 : NW];
    __shared__ K5Tiles<S.tile_groups, S.tile_bufs, !(S.cthr || S.kthr)> tl;
    __shared__ BlockVote<NW> vote;
    // MfmaSpec::tile_flow: the tile stream's counters (sweep_kt_flow)
    __shared__ TileFlow<S.tile_bufs> flow;
    FlowWave fw;
    if constexpr (S.tile_flow) {
        if (threadIdx.x == 0) {
            for (int b = 0; b < S.tile_bufs; b++) flow.landed[b] = flow.rel[b] = 0;
        }
        __syncthreads();
    }
    uint32_t vote_parity = 0;
    WL& sh = wl[S.perm_frag ? 0 : threadIdx.x >> 6];
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    [[maybe_unused]] unsigned long long t_start = 0;
    if constexpr (S.diag) t_start = __builtin_amdgcn_s_memtime();
    // MfmaSpec::lean (as in render_mfma_k5r): x, y recomputed from the item,
    // the wave counts its lanes' segments
    [[maybe_unused]] unsigned long long segs_w = 0;
    for (;;) {
        const RenderParams& p = kargs<RenderParams>();
        advance<1, !S.lean>(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        if (!block_any<NW>(act != 0, vote, vote_parity)) break;
        if constexpr (S.lean) segs_w += (unsigned long long)__popcll(act);
        const bool coop = act != 0 && __popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE);
        const bool sweeping = act != 0 && !coop;
        bool upper = true;
        if constexpr (S.compact) {
            if (sweeping && __popcll(act) <= 32) {
                if (act >> 32) {
                    const uint32_t l = lane_id(), nl = (uint32_t)__popcll(act);
                    const bool live = (act >> l) & 1ull;
                    const int to = 4 * (int)(live ? lanes_below(act) : nl + lanes_below(~act));
                    lane_permute<!S.lean, !S.lean>(L, to);
                    act = __ballot(L.st == ST_TRACE);
                }
                upper = false;
            }
        }
        const bool mine = L.st == ST_TRACE;
        if (sweeping) {
            // lanes without a ray carry the first live lane's (ST_DONE lanes
            // never read their o, d again)
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
        if constexpr (stash) {
            lane_stash_packed(L, sh.lane, (int)lane_id());
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        }
        bool swept;
        if constexpr (S.tile_flow)
            swept = sweep_kt_flow<S>(p, tl, flow, fw, ro, rd, best, bi, bestK, dg, sweeping, upper);
        else
            swept = sweep_k5_tiles<S>(p, sh, tl, ro, rd, best, bi, bestK, dg, sweeping, upper);
        if constexpr (stash) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            lane_unstash_packed(L, sh.lane, (int)lane_id());
        }
        L.o = ro;
        L.d = rd;
        if (coop) {
            float mybest = 1e38f;
            int mybi = -1;
            coop_each(act, L.o, L.d, p, mybest, mybi);
            if (mine) {
                L.bounce += 1;
                if constexpr (!S.lean) L.segs += 1;
                shade(L, p, mybest, mybi);
            }
            continue;
        }
        if (!act) continue;
        if (!swept) coop_each(act, ro, rd, p, best, bi);
        if (mine) {
            L.bounce += 1;
            if constexpr (!S.lean) L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    // tile_flow: a share of the next segment's first tiles may still be in
    // flight; it must land before the workgroup's LDS is given back
    if constexpr (S.tile_flow) wait_vm0();
    const RenderParams& p = kargs<RenderParams>();
    if constexpr (S.lean) {
        if (lane_id() == 0) atomicAdd(p.seg_counter, segs_w);
    } else {
        flush_counters(L, p);
    }
    if constexpr (S.diag)
        if (lane_id() == 0) {
            atomicAdd(p.seg_counter + 1, dg.groups);  // (wave, triangle group) sweeps
            atomicAdd(p.seg_counter + 2, dg.hot);     // ... with a passing pair
            atomicAdd(p.seg_counter + 3, dg.exact);   // (wave, triangle) exact tests
            if constexpr (S.tile_flow) {
                atomicAdd(p.seg_counter + 12, dg.t_wait);  // shader clocks: waiting for tiles
                atomicAdd(p.seg_counter + 13, dg.t_filt);  // ... products + record reads
                atomicAdd(p.seg_counter + 14, dg.t_exact); // ... exact phase + Y rebuilds (+ loop)
                atomicAdd(p.seg_counter + 15, dg.t_swp);   // ... whole sweeps
                atomicAdd(p.seg_counter + 16, __builtin_amdgcn_s_memtime() - t_start);  // ... the wave's life
                atomicAdd(p.seg_counter + 17, dg.t_issue);  // ... issuing claimed tiles (inside wait / filter)
                atomicAdd(p.seg_counter + 18, dg.t_pub);    // ... a claimer's wait for its pieces (inside wait)
                atomicAdd(p.seg_counter + 19, dg.claims);   // tiles claimed
            }
        }
}

}  // namespace
