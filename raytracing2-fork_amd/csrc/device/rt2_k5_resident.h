// The matrix filter for scenes whose records fit the LDS: every 32-triangle
// group's four record operands (4 KiB) are brought into the workgroup's LDS
// ONCE per launch and every wave sweeps them from there for the rest of the
// launch.  Two arithmetic forms (rt2_mfma.h): the 5-product form without -tn
// with the threshold in the accumulator (MfmaSpec::k5 / no_tn / cthr: records
// U0, V0, X0, T1 of the k16 layout; variants 282 / 298, round 5) and the
// threshold in the K-slots (MfmaSpec::kthr: the kt records; round 6).
// Included by rt2_render.hip only (one translation unit; internal linkage).
//
// Why: the 4-wave register kernel (render_mfma, variant 263) re-reads the
// whole scene's records from L2 in every wave-segment — config B's 38 groups
// are 152 KiB per wave and segment, 16 waves per CU — and 38 % of its wave
// cycles wait on those loads or the segment barrier (PMC of 263);
// the LDS-tiled kernel (render_mfma_k5t) shares them per segment but pays a
// workgroup barrier per tile.  Here the 152 KiB stay in LDS: no record
// traffic to L2 after the launch's first microseconds, no barrier after the
// initial one (waves run free: each leaves when its own lanes are done and
// the item pool is dry), and a group's operands are 4 conflict-free
// ds_read_b128 per lane (~100 cycles) instead of L2 loads.  MfmaSpec::res_l2
// (kthr): a scene of more than res_groups groups keeps its first res_groups
// resident and reads the rest per wave from L2 after them (up to 256 groups).
//
// The LDS then has no room for fragment rows, so the ray fragments are built
// in registers: each lane forms its own ray's 16 k-slots (the rows' exact
// f16 values) and one v_permlane32_swap per dword exchanges halves between
// lanes l and l + 32, which yields the MFMA A-operand layout of both 32-ray
// blocks at once (frag_pair).  The Y fragment is rebuilt the same way when a
// lane's bound improves: no LDS, no wave barrier.
//
// The filter only decides which (wave, triangle) pairs skip the exact test;
// the exact phase is the reference arithmetic in index order, so the image is
// the sequential strict `dst < best` scan's bit for bit.  Reference:
// compute.glsl:429-434 (the `triangles[i]` loop this sweep replaces).
#pragma once

namespace {

// LDS of the resident records: NG groups x the 4 operands x 64 lanes x 16 B
template <int NG>
struct K5Resident {
    h8 rec[NG * 4 * 64];
};

// The exact phase of one group: the triangles with a passing pair (ballot M)
// in index order, mt_pass3 + mt_exact (compute.glsl:302-340, strict `dst <
// best`).  Returns whether some lane's bound improved.
template <MfmaSpec S>
__device__ __forceinline__ bool exact_group(unsigned long long M, int G, int n_tris, cfloat* tri, const f3& o,
                                            const f3& d, float& best, int& bi, float& bestK, MfmaDiag& dg) {
    if constexpr (S.diag) dg.hot += 1;
    uint32_t m32 = (uint32_t)(M | M >> 32);
    const float bk0 = bestK;
    if constexpr (S.exact_pf) {
        // MfmaSpec::exact_pf: the next triangle's record is requested (vector
        // loads of one uniform address: in-order vmcnt, unlike the scalar
        // cache's) before this one is tested, so its latency overlaps the test
        const float4* tv = reinterpret_cast<const float4*>((const float*)tri);
        int tt = __builtin_ctz(m32);
        m32 &= m32 - 1;
        int idx = 32 * G + tt;
        if (idx >= n_tris) return false;
        float4 c0 = tv[3 * idx], c1 = tv[3 * idx + 1], c2 = tv[3 * idx + 2];
        for (;;) {
            int nidx = n_tris;
            float4 n0 = c0, n1 = c1, n2 = c2;
            if (m32) {
                nidx = 32 * G + __builtin_ctz(m32);
                m32 &= m32 - 1;
                if (nidx < n_tris) n0 = tv[3 * nidx], n1 = tv[3 * nidx + 1], n2 = tv[3 * nidx + 2];
            }
            if constexpr (S.diag) dg.exact += 1;
            const MtQ qq = mt_quantities(o, d, c0, c1, c2);
            if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
            if (nidx >= n_tris) break;
            idx = nidx;
            c0 = n0, c1 = n1, c2 = n2;
        }
        return __ballot(bestK != bk0) != 0;
    }
    while (m32) {
        const int tt = __builtin_ctz(m32);
        m32 &= m32 - 1;
        const int idx = 32 * G + tt;
        if (idx >= n_tris) break;
        if constexpr (S.diag) dg.exact += 1;
        cfloat* tp = tri + 12 * idx;
        const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
        if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
    }
    return __ballot(bestK != bk0) != 0;
}

// MfmaSpec::phase_prio: the wave's issue priority by its phase (the SIMD's
// arbiter issues by priority, then age): 1 = the products' phase high, the
// exact phase and shading low; 2 = the exact phase high; 3 = shading high;
// 4 = both VALU phases (exact phase, shading) high
template <MfmaSpec S>
__device__ __forceinline__ void phase_prio(int phase) {  // 0 products, 1 exact phase, 2 shading
    if constexpr (S.phase_prio > 0) {
        const bool hi = (S.phase_prio == 1 && phase == 0) || (S.phase_prio == 2 && phase == 1) ||
                        (S.phase_prio == 3 && phase == 2) || (S.phase_prio == 4 && phase != 0);
        if (hi)
            __builtin_amdgcn_s_setprio(1);
        else
            __builtin_amdgcn_s_setprio(0);
    }
}

// Closest hit of every lane's ray over all triangles, cthr records from LDS.
// Returns false (wave-uniform, nothing computed) when a ray is outside the
// filter's range.
template <MfmaSpec S>
__device__ __forceinline__ bool sweep_k5_res(const RenderParams& p, const h8* rec, const f3& o, const f3& d,
                                             float& best, int& bi, float& bestK, MfmaDiag& dg, bool upper) {
    static_assert(S.k5 && S.no_tn && S.cthr && S.ymma && S.imax && S.minred && S.ylds == 0, "the cthr 4-product form");
    const int lane = (int)lane_id();
    const f3 m = cross(d, o);
    MfmaScale sc;
    if (!mfma_scale<S>(p.mfma_A, o, d, m, sc)) return false;
    h8 a0[2], y1[2];
    {
        _Float16 s[18];
        mfma_main_half_slots(s, d, m, sc.sigma);
        frag_pair(s, a0);
    }
    // the wave's largest |ray lo| and |ray hi| of m.z (sweep_k16's k5 bound)
    const float vz = m.z * sc.sigma;
    const _Float16 hz = (_Float16)vz;
    const _Float16 lz = (_Float16)(vz - (float)hz);
    const float zhi = wave_max_s<S>(fabsf((float)hz));
    const float zlo = wave_max_s<S>(fabsf((float)lz));
    const ThrBits thr = mfma_thr_bits(sc.Tw, zlo, zhi);
    auto build_y = [&](float bkv) {
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bkv, sc.sigma, sc.Bmax);
        frag_pair(s, y1);
    };
    build_y(bestK);
    // MfmaSpec::thr_hoist: the threshold fragment once per sweep
    [[maybe_unused]] const h8 tfh = S.thr_hoist ? mfma_thr_frag(thr) : h8{};
    const int ng = (p.n_tris + 31) >> 5, n_tris = p.n_tris;
    cfloat* const tri = (cfloat*)p.tri;  // held across the sweep (not re-read from the kernel arguments per hot group)
    const h8* tb = rec + lane;
    for (int G = 0; G < ng; G++) {
        const h8 b0 = tb[0], b2 = tb[64], b4 = tb[128], b6 = tb[192];
        tb += 4 * 64;
        const unsigned long long M = k5_cthr_group<S>(thr, a0, y1, b0, b2, b4, b6, upper, 0, tfh);
        if constexpr (S.diag) dg.groups += 1;
        if (M && exact_group<S>(M, G, n_tris, tri, o, d, best, bi, bestK, dg)) build_y(bestK);
    }
    return true;
}

// The same with the threshold in the K-slots (MfmaSpec::kthr, kt records):
// 8 independent products per group with a zero accumulator.  res_l2: groups
// [res_groups, ng) are read from the scene's kt records in L2 after the
// resident ones, in the same (index) order.
template <MfmaSpec S>
__device__ __forceinline__ bool sweep_kt_res(const RenderParams& p, const h8* rec, const f3& o, const f3& d,
                                             float& best, int& bi, float& bestK, MfmaDiag& dg, bool upper) {
    static_assert(S.kthr > 0 && S.ymma, "the kthr form");
    const int lane = (int)lane_id();
    // MfmaSpec::diag: shader clocks of the ray setup (t_wait), the products
    // with their record reads (t_filt), the exact phase with the Y rebuilds
    // (t_exact) and the whole sweep (t_swp)
    [[maybe_unused]] unsigned long long tc = 0, tsw = 0;
    if constexpr (S.diag) tsw = tc = __builtin_amdgcn_s_memtime();
    auto stamp = [&](unsigned long long& acc) {
        if constexpr (S.diag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc += t - tc;
            tc = t;
        }
    };
    const f3 m = cross(d, o);
    MfmaScale sc;
    if (!mfma_scale<S>(p.mfma_A, o, d, m, sc)) return false;
    h8 a0[2], y1[2];
    _Float16 tw16;
    kt_frags<S>(d, m, sc, a0, tw16);
    kt_y(d, o, bestK, sc, tw16, y1);
    stamp(dg.t_wait);
    const int ng = (p.n_tris + 31) >> 5, n_tris = p.n_tris;
    const int nres = S.res_l2 ? min(ng, S.res_groups) : ng;
    cfloat* const tri = (cfloat*)p.tri;
    const h8* tb = rec + lane;
    if constexpr (S.prefetch) {
        // MfmaSpec::prefetch: the next group's operands are read from LDS
        // while this group's products run (a second register set)
        h8 n0 = tb[0], n1 = tb[64], n2 = tb[128], n3 = tb[192];
        for (int G = 0; G < nres; G++) {
            const h8 b0 = n0, b1 = n1, b2 = n2, b3 = n3;
            tb += kKtOps * 64;
            if (G + 1 < nres) n0 = tb[0], n1 = tb[64], n2 = tb[128], n3 = tb[192];
            const unsigned long long M = kt_group<S>(a0, y1, b0, b1, b2, b3, upper);
            if constexpr (S.diag) dg.groups += 1;
            if (M && exact_group<S>(M, G, n_tris, tri, o, d, best, bi, bestK, dg)) kt_y(d, o, bestK, sc, tw16, y1);
        }
    } else {
        for (int G = 0; G < nres; G++) {
            const h8 b0 = tb[0], b1 = tb[64], b2 = tb[128], b3 = tb[192];
            tb += kKtOps * 64;
            const unsigned long long M = kt_group<S>(a0, y1, b0, b1, b2, b3, upper);
            if constexpr (S.diag) dg.groups += 1;
            stamp(dg.t_filt);
            if constexpr (S.sol == 2) {
                // speed-of-light probe (WRONG images): no exact phase
                if (M == 0x123456789ull) best = -best;
                continue;
            }
            if (M) {
                phase_prio<S>(1);
                if (exact_group<S>(M, G, n_tris, tri, o, d, best, bi, bestK, dg)) kt_y(d, o, bestK, sc, tw16, y1);
                phase_prio<S>(0);
            }
            stamp(dg.t_exact);
        }
    }
    if constexpr (S.res_l2) {
        const h8* gb = reinterpret_cast<const h8*>(p.mfma_kt_frag) + (size_t)nres * (kKtOps * 64) + lane;
        for (int G = nres; G < ng; G++) {
            const h8 b0 = gb[0], b1 = gb[64], b2 = gb[128], b3 = gb[192];
            gb += kKtOps * 64;
            const unsigned long long M = kt_group<S>(a0, y1, b0, b1, b2, b3, upper);
            if constexpr (S.diag) dg.groups += 1;
            if (M && exact_group<S>(M, G, n_tris, tri, o, d, best, bi, bestK, dg)) kt_y(d, o, bestK, sc, tw16, y1);
        }
    }
    if constexpr (S.diag) dg.t_swp += __builtin_amdgcn_s_memtime() - tsw;
    return true;
}

// render_mfma's segment loop (free-running waves: no barrier after the
// records have landed) around sweep_k5_res / sweep_kt_res.  The launcher takes
// it only for scenes of at most S.res_groups groups (res_l2: at most 256).
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_k5r(RenderParams p_arg) {
    static_assert(S.res_groups > 0 && !S.lockstep, "records resident in LDS; free-running waves");
    static_assert(!S.res_l2 || S.kthr, "L2 groups beyond the resident ones: the kthr form");
    constexpr int NW = S.block / 64;
    __shared__ K5Resident<S.res_groups> rs;
    {
        // every resident group's 4 operands by LDS-DMA (1-KiB pieces, coalesced
        // 16 B per lane, no VGPRs), dealt round-robin over the waves; then one
        // barrier: every wave's pieces have landed
        const RenderParams& p = kargs<RenderParams>();
        const int ng = min((p.n_tris + 31) >> 5, S.res_groups);
        const int lane = (int)lane_id(), wave = (int)(threadIdx.x >> 6);
        for (int pc = wave; pc < 4 * ng; pc += NW) {
            const h8* src;
            if constexpr (S.kthr)
                src = reinterpret_cast<const h8*>(p.mfma_kt_frag) + (size_t)pc * 64 + lane;  // [G][4 ops] contiguous
            else
                src = reinterpret_cast<const h8*>(p.mfma_k16_frag) + ((size_t)(pc >> 2) * kK16Ops + 2 * (pc & 3)) * 64 +
                      lane;  // ops 0, 2, 4, 6 of the k16 layout
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)&rs.rec[pc * 64], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    const int wave = (int)(threadIdx.x >> 6);
    // MfmaSpec::lean: the wave counts its lanes' segments (no per-lane counter)
    [[maybe_unused]] unsigned long long segs_w = 0;
    // diag wave timeline (p.wave_log, render_mfma's 10-word layout: start,
    // first lane out of items, end, segment rounds with two 32-ray blocks /
    // one / - / cooperative drain, HW_ID | XCC_ID << 32, shader clocks)
    [[maybe_unused]] unsigned long long wl_t0 = 0, wl_c0 = 0, wl_dry = 0, wl_r2 = 0, wl_r1 = 0, wl_coop = 0;
    if constexpr (S.diag) {
        wl_t0 = __builtin_amdgcn_s_memrealtime();
        wl_c0 = __builtin_amdgcn_s_memtime();
    }
    for (;;) {
        const RenderParams& p = kargs<RenderParams>();
        advance<1, !S.lean>(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        if constexpr (S.lean) segs_w += (unsigned long long)__popcll(act);
        if constexpr (S.diag) {
            if (!wl_dry && __any(L.st == ST_DONE)) wl_dry = __builtin_amdgcn_s_memrealtime();
            if (act) {
                if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE))
                    wl_coop++;
                else if (__popcll(act) <= 32)
                    wl_r1++;
                else
                    wl_r2++;
            }
        }
        if (!act) break;  // every lane is done and the pool is dry
        if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE)) {
            float mybest = 1e38f;
            int mybi = -1;
            coop_each(act, L.o, L.d, p, mybest, mybi);
            if (L.st == ST_TRACE) {
                L.bounce += 1;
                if constexpr (!S.lean) L.segs += 1;
                shade(L, p, mybest, mybi);
            }
            continue;
        }
        if constexpr (S.fair_prio) {
            // MfmaSpec::fair_prio.  A SIMD's four waves start together, and
            // in a rank slab each lane holds about one item (a pixel's 64
            // rays, one after another): the SIMD is done when its slowest
            // wave is.  The arbiter issues by priority, then age, so with
            // equal priorities the oldest wave runs ahead and the youngest
            // ends alone, latency-bound, for ~3 ms of a 25-ms 1/8 slab.  Here
            // a wave's priority rises with the rays its slowest lane has left
            // (quartiles of the rays per pixel): waves that fall behind take
            // the issue slots back, and the SIMD's waves end together.
            const float left = wave_max((float)(L.st == ST_TRACE ? p.R - L.ray : 0));
            const int q = (int)(left * 4.0f - 1.0f) / p.R;
            if (q >= 3)
                __builtin_amdgcn_s_setprio(3);
            else if (q == 2)
                __builtin_amdgcn_s_setprio(2);
            else if (q == 1)
                __builtin_amdgcn_s_setprio(1);
            else
                __builtin_amdgcn_s_setprio(0);
        }
        bool upper = true;
        if constexpr (S.compact) {
            // at most 32 live rays: move them to lanes 0..31 and sweep the
            // first 32-ray block only
            if (__popcll(act) <= 32) {
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
        // lanes without a ray carry the first live lane's (ST_DONE lanes never
        // read their o, d again)
        const int j0 = __builtin_ctzll(act);
        const bool mine = L.st == ST_TRACE;
        {
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
        bool swept;
        phase_prio<S>(0);
        if constexpr (S.kthr)
            swept = sweep_kt_res<S>(p, rs.rec, ro, rd, best, bi, bestK, dg, upper);
        else
            swept = sweep_k5_res<S>(p, rs.rec, ro, rd, best, bi, bestK, dg, upper);
        // a ray outside the filter's range (wave-uniform): the drain's code
        if (!swept) coop_each(act, ro, rd, p, best, bi);
        phase_prio<S>(2);
        if (mine) {
            L.bounce += 1;
            if constexpr (!S.lean) L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    const RenderParams& p = kargs<RenderParams>();
    if constexpr (S.lean) {
        if (lane_id() == 0) atomicAdd(p.seg_counter, segs_w);
    } else {
        flush_counters(L, p);
    }
    if constexpr (S.diag)
        if (p.wave_log) {
            const uint32_t gw = blockIdx.x * NW + (uint32_t)wave;
            const unsigned long long c1 = __builtin_amdgcn_s_memtime();
            const unsigned long long hw = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |
                                          (unsigned long long)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32;
            if (lane_id() == 0 && gw < p.wave_log_n) {
                unsigned long long* e = p.wave_log + 10 * (size_t)gw;
                e[0] = wl_t0;
                e[1] = wl_dry;
                e[2] = __builtin_amdgcn_s_memrealtime();
                e[3] = wl_r2;
                e[4] = wl_r1;
                e[5] = 0;
                e[6] = wl_coop;
                e[7] = hw;
                e[8] = wl_c0;
                e[9] = c1;
            }
        }
    if constexpr (S.diag)
        if (lane_id() == 0) {
            atomicAdd(p.seg_counter + 1, dg.groups);  // (wave, triangle group) sweeps
            atomicAdd(p.seg_counter + 2, dg.hot);     // ... with a passing pair
            atomicAdd(p.seg_counter + 3, dg.exact);   // (wave, triangle) exact tests
            if constexpr (S.kthr) {
                atomicAdd(p.seg_counter + 12, dg.t_wait);  // shader clocks: the sweep's ray setup
                atomicAdd(p.seg_counter + 13, dg.t_filt);  // ... products + record reads
                atomicAdd(p.seg_counter + 14, dg.t_exact); // ... exact phase + Y rebuilds
                atomicAdd(p.seg_counter + 15, dg.t_swp);   // ... whole sweeps
                atomicAdd(p.seg_counter + 16, __builtin_amdgcn_s_memtime() - wl_c0);  // ... the wave's life
            }
        }
}

}  // namespace
