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

// The MFMA A-operand fragments of both 32-ray blocks from each lane's own 16
// k-slots s[0..15] (lane l = ray l): block R's lane l holds ray 32R + (l & 31),
// k-slots 8 (l >> 5) .. +7 — what the fragment rows' ds_read_b128 gave.
// v_permlane32_swap(x, y) swaps x's lanes 32..63 with y's lanes 0..31, so with
// x = slots 0..7 and y = slots 8..15: x becomes block 0's fragment (lanes
// 0..31 their own slots 0..7, lanes 32..63 the slots 8..15 of rays 0..31) and
// y block 1's.
__device__ __forceinline__ void frag_pair(const _Float16* s, h8 out[2]) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const u4 lo = __builtin_bit_cast(u4, h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]});
    const u4 hi = __builtin_bit_cast(u4, h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]});
    u4 r0, r1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const auto r = __builtin_amdgcn_permlane32_swap(lo[k], hi[k], false, false);
        r0[k] = r[0];
        r1[k] = r[1];
    }
    out[0] = __builtin_bit_cast(h8, r0);
    out[1] = __builtin_bit_cast(h8, r1);
}

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
    const int ng = (p.n_tris + 31) >> 5;
    const h8* tb = rec + lane;
    h8 nb[4];
    auto fetch = [&]() {
        nb[0] = tb[0];
        nb[1] = tb[64];
        nb[2] = tb[128];
        nb[3] = tb[192];
        tb += 4 * 64;
    };
    if constexpr (S.prefetch) fetch();
    for (int G = 0; G < ng; G++) {
        if constexpr (!S.prefetch) fetch();
        const h8 b0 = nb[0], b2 = nb[1], b4 = nb[2], b6 = nb[3];
        if constexpr (S.prefetch)
            if (G + 1 < ng) fetch();
        const unsigned long long M = k5_cthr_group<S>(thr, a0, y1, b0, b2, b4, b6, upper, 0);
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
            if (__ballot(bestK != bk0)) build_y(bestK);
        }
    }
    return true;
}

// render_mfma's segment loop (free-running waves: no barrier after the
// records have landed) around sweep_k5_res.  The launcher takes it only for
// scenes of at most S.res_groups groups (rt2_render).
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_k5r(RenderParams p_arg) {
    static_assert(S.res_groups > 0 && !S.lockstep, "records resident in LDS; free-running waves");
    constexpr int NW = S.block / 64;
    __shared__ K5Resident<S.res_groups> rs;
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
    for (;;) {
        const RenderParams& p = kargs<RenderParams>();
        advance(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        if (!act) break;
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
        // a ray outside the filter's range (wave-uniform): the drain's code
        if (!sweep_k5_res<S>(p, rs.rec, ro, rd, best, bi, bestK, dg, upper)) coop_each(act, ro, rd, p, best, bi);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    const RenderParams& p = kargs<RenderParams>();
    flush_counters(L, p);
    if constexpr (S.diag)
        if (lane_id() == 0) {
            atomicAdd(p.seg_counter + 1, dg.groups);  // (wave, triangle group) sweeps
            atomicAdd(p.seg_counter + 2, dg.hot);     // ... with a passing pair
            atomicAdd(p.seg_counter + 3, dg.exact);   // (wave, triangle) exact tests
        }
}

}  // namespace
