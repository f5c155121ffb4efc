// The 5-product matrix filter without -tn and with the threshold in the
// accumulator (rt2_mfma.h: MfmaSpec::k5 / no_tn / cthr) for scenes whose
// records fit the LDS: every 32-triangle group's four record operands (U0,
// V0, X0, T1: 4 KiB) are brought into the workgroup's LDS ONCE per launch and
// every wave sweeps them from there for the rest of the launch.  Included by
// rt2_render.hip only (one translation unit; internal linkage).
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
// ds_read_b128 per lane (~100 cycles) instead of L2 loads.
//
// The LDS then has no room for fragment rows, so the ray fragments are built
// in registers: each lane forms its own ray's 16 k-slots (the rows' exact
// f16 values) and one v_permlane32_swap per dword exchanges halves between
// lanes l and l + 32, which yields the MFMA A-operand layout of both 32-ray
// blocks at once (frag_pair).  The Y fragment is rebuilt the same way when a
// lane's bound improves: no LDS, no wave barrier.
//
// The arithmetic of every product, threshold and exact test is sweep_k16's
// (5-product form, cthr) term for term, so the image is the sequential strict
// `dst < best` scan's bit for bit.  Reference: compute.glsl:429-434 (the
// `triangles[i]` loop this sweep replaces).
#pragma once

namespace {

// LDS of the resident records: NG groups x the 4 operands x 64 lanes x 16 B
template <int NG>
struct K5Resident {
    h8 rec[NG * 4 * 64];
};

// Closest hit of every lane's ray over all triangles, records from LDS.
// Returns false (wave-uniform, nothing computed) when a ray is outside the
// filter's range.
template <MfmaSpec S>
__device__ __forceinline__ bool sweep_k5_res(const RenderParams& p, const h8* rec, const f3& o, const f3& d,
                                             float& best, int& bi, float& bestK, MfmaDiag& dg, bool upper, int G0 = 0,
                                             int G1 = -1) {
    // [G0, G1): the 32-triangle groups to sweep (all by default; a range when
    // the groups of one wave's segment are split into tail-job units)
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
    const int ng = G1 < 0 ? (p.n_tris + 31) >> 5 : G1, n_tris = p.n_tris;
    cfloat* const tri = (cfloat*)p.tri;  // held across the sweep (not re-read from the kernel arguments per hot group)
    const h8* tb = rec + (size_t)G0 * (4 * 64) + lane;
    for (int G = G0; G < ng; G++) {
        const h8 b0 = tb[0], b2 = tb[64], b4 = tb[128], b6 = tb[192];
        tb += 4 * 64;
        const unsigned long long M = k5_cthr_group<S>(thr, a0, y1, b0, b2, b4, b6, upper, 0, tfh);
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
                if (idx >= n_tris) break;
                if constexpr (S.diag) dg.exact += 1;
                cfloat* tp = tri + 12 * idx;
                const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
            }
            if (__ballot(bestK != bk0)) build_y(bestK);
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// Tail jobs (MfmaSpec::tail_jobs): once the item pool is dry, a wave whose
// lanes are all done does not leave; it helps the waves of its workgroup that
// still trace.  A pixel-frame's rays share one RNG stream, so a launch ends
// with whole items whose segments run one after another on one lane; at the
// end a lone wave sweeps all groups for its last few rays while the other
// waves of its CU idle (the last ~13 % of a config B launch, more
// of a 1/N rank slab).  A wave with <= 32 live rays (after compaction) posts
// its segment as a JOB in the LDS left beside the records: its rays, a 64-bit
// key per ray, and a ticket; the groups are cut into one unit per helper
// (at most tail_jobs), which the helpers claim by compare-and-swap on the
// ticket and sweep for the job's rays from scratch (bound = none), folding
// each ray's result into its
// key with an LDS atomic minimum on (dst bits << 32 | triangle index).  A hit
// has dst > 1e-6 > 0, and positive binary32 values order like their bit
// patterns, so the minimum key is the lexicographic (dst, index) minimum: the
// smallest distance and, among exact ties, the lowest index — what the
// sequential strict `dst < best` scan keeps.  Each unit's sweep starts from
// no bound, for which the filter is still conservative (it only rejects what
// the exact test rejects); the exact test is the reference arithmetic.  So
// the result is bit-identical to the one-wave sweep (and to the oracle).
// Termination: an owner posts only when helpers exist, and a helper leaves
// only when no wave of the workgroup traces any more (busy == 0), which a wave
// signals after its last job has completed; a claimed unit finishes without
// waiting on anything, so the owner's wait for its units ends.  The owner
// itself serves no unit: a form in which it served its own units (a call
// inside its segment loop) returned correct keys but a corrupted image unless
// further code followed the call — a code-generation effect around the call
// that we did not isolate ("Tail jobs"); owners that only wait are
// bit-exact.
constexpr int kTailSlots = 6;  // jobs at once per workgroup (the LDS beside config B's 152 KiB of records)
struct TailBoard {
    float4 ray[kTailSlots][32][2];            // o (xyz), d (xyz) of the job's 32 rays (lanes 0..31 after compaction)
    unsigned long long key[kTailSlots][32];   // (dst bits << 32 | index) minimum over the units; ~0 = no hit
    uint32_t ticket[kTailSlots];              // epoch:24 | units:4 | next unit:4
    uint32_t done[kTailSlots];                // units finished
    uint32_t owner[kTailSlots];               // 0 = free, wave + 1
    uint32_t busy;                            // waves of the workgroup that may still post jobs
};
__device__ __forceinline__ uint32_t lds_load_acq(uint32_t* a) {
    return __hip_atomic_load(a, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Sweeps unit u of nu of job j for the job's rays (lanes 0..31; lanes 32..63
// carry ray 0, as a compacted owner's do) and folds the results into the keys.
template <MfmaSpec S>
__device__ __attribute__((noinline)) void serve_unit(const RenderParams& p, const h8* rec, TailBoard& tb, int j, int u,
                                                    int nu, MfmaDiag& dg) {
    const int lane = (int)lane_id(), src = lane < 32 ? lane : 0;
    const float4 ro = tb.ray[j][src][0], rdv = tb.ray[j][src][1];
    const f3 o = mk(ro.x, ro.y, ro.z), d = mk(rdv.x, rdv.y, rdv.z);
    const int ng = (p.n_tris + 31) >> 5;
    const int G0 = u * ng / nu, G1 = (u + 1) * ng / nu;
    float best = 1e38f, bestK = 1e38f * 1.0009765625f;
    int bi = -1;
    (void)sweep_k5_res<S>(p, rec, o, d, best, bi, bestK, dg, false, G0, G1);  // in range: the owner checked these rays
    if (lane < 32 && bi >= 0)
        atomicMin(&tb.key[j][lane], (unsigned long long)__float_as_uint(best) << 32 | (uint32_t)bi);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(&tb.done[j], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// One claim on job j: the unit index (and the job's unit count), or -1 when
// every unit is claimed.  Lane 0 runs the compare-and-swap; the outcome is
// broadcast to the whole wave (wave-uniform control flow).
__device__ __forceinline__ int claim_unit(TailBoard& tb, int j, int& nu) {
    uint32_t got = 0xffffffffu;
    if (lane_id() == 0) {
        uint32_t t = lds_load_acq(&tb.ticket[j]);
        while ((t & 15u) < ((t >> 4) & 15u)) {
            if (__hip_atomic_compare_exchange_strong(&tb.ticket[j], &t, t + 1u, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP)) {
                got = t;
                break;
            }
        }
    }
    got = (uint32_t)__builtin_amdgcn_readfirstlane((int)got);
    if (got == 0xffffffffu) return -1;
    nu = (int)((got >> 4) & 15u);
    return (int)(got & 15u);
}

// render_mfma's segment loop (free-running waves: no barrier after the
// records have landed) around sweep_k5_res.  The launcher takes it only for
// scenes of at most S.res_groups groups (rt2_render).
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_k5r(RenderParams p_arg) {
    static_assert(S.res_groups > 0 && !S.lockstep, "records resident in LDS; free-running waves");
    constexpr int NW = S.block / 64;
    __shared__ K5Resident<S.res_groups> rs;
    [[maybe_unused]] TailBoard* tbp = nullptr;
    if constexpr (S.tail_jobs > 0) {
        __shared__ TailBoard board;
        tbp = &board;
        if (threadIdx.x < kTailSlots) {
            board.ticket[threadIdx.x] = 0u;
            board.done[threadIdx.x] = 0u;
            board.owner[threadIdx.x] = 0u;
        }
        if (threadIdx.x == 0) board.busy = NW;
    }
    {
        // every group's 4 operands by LDS-DMA (1-KiB pieces, coalesced 16 B
        // per lane, no VGPRs), dealt round-robin over the waves; then one
        // barrier: every wave's pieces have landed
        const RenderParams& p = kargs<RenderParams>();
        const int ng = min((p.n_tris + 31) >> 5, S.res_groups);
        const h8* gsrc = reinterpret_cast<const h8*>(p.mfma_k16_frag);
        const int lane = (int)lane_id(), wave = (int)(threadIdx.x >> 6);
        for (int pc = wave; pc < 4 * ng; pc += NW) {
            const int gi = pc >> 2, op = 2 * (pc & 3);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(gsrc + ((size_t)gi * kK16Ops + op) * 64 + lane),
                (__attribute__((address_space(3))) void*)&rs.rec[pc * 64], 16, 0, 0);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    [[maybe_unused]] int slot = -1;          // tail jobs: this wave's job slot once it has one
    [[maybe_unused]] uint32_t epoch = 0;
    const int wave = (int)(threadIdx.x >> 6);
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
        advance(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
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
        if (!act) {
            if constexpr (S.tail_jobs > 0) {
                // every lane is done and the pool is dry: help the waves that
                // still trace, until none does
                TailBoard& tb = *tbp;
                if (lane_id() == 0) {
                    if (slot >= 0) __hip_atomic_store(&tb.owner[slot], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __hip_atomic_fetch_add(&tb.busy, 0xffffffffu, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                for (;;) {
                    bool served = false;
                    for (int j = 0; j < kTailSlots; j++) {
                        int nu = 0;
                        const int u = claim_unit(tb, j, nu);
                        if (u >= 0) {
                            serve_unit<S>(p, rs.rec, tb, j, u, nu, dg);
                            served = true;
                        }
                    }
                    if (!served) {
                        const uint32_t b = (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_load_acq(&tb.busy));
                        if (b == 0) break;
                        __builtin_amdgcn_s_sleep(2);
                    }
                }
            }
            break;
        }
        if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE)) {
            float mybest = 1e38f;
            int mybi = -1;
            coop_each(act, L.o, L.d, p, mybest, mybi);
            if (L.st == ST_TRACE) {
                L.bounce += 1;
                L.segs += 1;
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
                    lane_permute(L, to);
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
        bool swept = false;
        if constexpr (S.tail_jobs > 0) {
            // the pool is dry, <= 32 live rays (lanes 0..31), the rays in the
            // filter's range, and the workgroup has waves that only help: the
            // segment becomes a job of nu units
            TailBoard& tb = *tbp;
            const uint32_t helpers = NW - (uint32_t)__builtin_amdgcn_readfirstlane((int)lds_load_acq(&tb.busy));
            if (!upper && helpers > 0 && __any(L.st == ST_DONE) &&
                !__ballot(!(abs_max3(ro) <= 0x1p20f && abs_max3(rd) <= 1.0001f))) {
                if (slot < 0) {
                    int got = -1;
                    if (lane_id() == 0)
                        for (int j = 0; j < kTailSlots && got < 0; j++) {
                            uint32_t z = 0u;
                            if (__hip_atomic_compare_exchange_strong(&tb.owner[j], &z, (uint32_t)wave + 1u,
                                                                     __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_WORKGROUP))
                                got = j;
                        }
                    slot = __builtin_amdgcn_readfirstlane(got);
                    if (slot >= 0) epoch = lds_load_acq(&tb.ticket[slot]) >> 8;
                }
                if (slot >= 0) {
                    const int j = slot;
                    const int nu = (int)min((uint32_t)S.tail_jobs, helpers);
                    if (lane_id() < 32) {
                        tb.ray[j][lane_id()][0] = make_float4(ro.x, ro.y, ro.z, 0.0f);
                        tb.ray[j][lane_id()][1] = make_float4(rd.x, rd.y, rd.z, 0.0f);
                        tb.key[j][lane_id()] = ~0ull;
                    }
                    epoch = (epoch + 1u) & 0xffffffu;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane_id() == 0) {
                        __hip_atomic_store(&tb.done[j], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&tb.ticket[j], epoch << 8 | (uint32_t)nu << 4, __ATOMIC_RELEASE,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    // the helpers serve the units; each claimed unit finishes
                    // without waiting on anything
                    while ((uint32_t)__builtin_amdgcn_readfirstlane((int)lds_load_acq(&tb.done[j])) < (uint32_t)nu)
                        __builtin_amdgcn_s_sleep(1);
                    if (lane_id() < 32) {
                        const unsigned long long k = tb.key[j][lane_id()];
                        if (k != ~0ull) {
                            best = __uint_as_float((uint32_t)(k >> 32));
                            bi = (int)(uint32_t)k;
                        }
                    }
                    swept = true;
                }
            }
        }
        // a ray outside the filter's range (wave-uniform): the drain's code
        if (!swept && !sweep_k5_res<S>(p, rs.rec, ro, rd, best, bi, bestK, dg, upper))
            coop_each(act, ro, rd, p, best, bi);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    const RenderParams& p = kargs<RenderParams>();
    flush_counters(L, p);
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
        }
}

}  // namespace
