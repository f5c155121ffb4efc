// The small-scene matrix kernel (render_mfma, the 5-product form without -tn
// at 4 waves per SIMD) with the workgroup's rays packed into 32-ray blocks
// once they thin out.  Included by rt2_render.hip only.
//
// Why: a wave sweeps its rays in 32-ray blocks (v_mfma_f32_32x32x16_f16 rows),
// whatever number of them is live: compaction (MfmaSpec::compact) skips the
// second block at <= 32 live rays, but a wave with 5 live rays still pays a
// whole block.  At the end of a launch — when the item pool is dry, every
// lane finishes its last pixel and the waves empty out — that is most of the
// matrix work ("Next": about 13 % of config B's launch, and most
// of a 1/8 rank slab).
//
// What: at every segment the workgroup's waves vote with their live-ray
// counts (one LDS word per wave, the lockstep barrier that was already
// there).  When packing the workgroup's rays into blocks saves a block, and
// they are at most 128, the segment is pooled: every live ray writes its
// (o, d) to a workgroup LDS array in wave order (one barrier), wave w sweeps
// packed rays 32w..32w+31 as one block (sweep_k16: the same products,
// threshold and exact phase), writes each ray's (best, index) back (a second
// barrier), and the owners read their rays' results and shade.  The path
// state never moves: only a segment's ray and its closest hit travel, so the
// result of every segment is the unpooled sweep's bit for bit (a ray's
// closest hit does not depend on the block it is swept in).
//
// LDS: 80-B fragment rows (MfmaSpec::rows80: the main fragment's first K-half
// and the Y slots) free 1 KiB per wave for the pool (128 rays x 32 B: o, d,
// closest hit) within the 4-workgroups-per-CU budget.
#pragma once

namespace {

constexpr int kPoolRays = 128;
struct RayPool {
    float od[kPoolRays][6];  // o.xyz, d.xyz of packed ray j
    float best[kPoolRays];
    int bi[kPoolRays];
};

template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma_pool(RenderParams p_arg) {
    static_assert(S.wg_pool && S.rows80 && S.k5 && S.no_tn && S.k16 && S.lane_lds == 2 && S.lockstep && S.compact,
                  "the 4-wave small-scene build");
    constexpr int NW = S.block / 64;
    static_assert(NW * 32 == kPoolRays, "one 32-ray block per wave when pooled");
    __shared__ MfmaK5nLds wl[NW];
    __shared__ RayPool pool;
    __shared__ BlockVote<NW> vote;
    uint32_t vote_parity = 0;
    MfmaK5nLds& sh = wl[threadIdx.x >> 6];
    const int wave = (int)(threadIdx.x >> 6);
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    for (;;) {
        const RenderParams& p = kargs<RenderParams>();
        advance(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        const uint32_t n_live = (uint32_t)__popcll(act);
        // the vote: this wave's live rays (one LDS word per wave; the lockstep
        // barrier render_mfma has anyway)
        if (lane_id() == 0) vote.v[vote_parity][wave] = n_live;
        __syncthreads();
        uint32_t total = 0, blocks = 0, base = 0;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            const uint32_t c = vote.v[vote_parity][k];
            total += c;
            blocks += (c + 31u) >> 5;
            if (k < wave) base += c;
        }
        vote_parity ^= 1u;
        // wave-uniform (LDS reads land in VGPRs): scalar registers
        total = __builtin_amdgcn_readfirstlane(total);
        blocks = __builtin_amdgcn_readfirstlane(blocks);
        base = __builtin_amdgcn_readfirstlane(base);
        if (total == 0) break;  // workgroup-uniform: every wave leaves together
        const bool mine = L.st == ST_TRACE;
        // pooled when packing saves a block (the cooperative drain then has
        // nothing to do: every live ray of the workgroup is in the pool)
        const bool pooled = total <= (uint32_t)kPoolRays && ((total + 31u) >> 5) < blocks;
        const uint32_t l = lane_id();
        uint32_t slot = 0, nb = 0, nblk = 1, nrange = 1, res = 0;
        int G0 = 0, G1 = -1;
        bool sweeping, upper = true;
        if (pooled) {
            slot = base + lanes_below(act);
            if (mine) {
                float* od = pool.od[slot];
                od[0] = L.o.x;
                od[1] = L.o.y;
                od[2] = L.o.z;
                od[3] = L.d.x;
                od[4] = L.d.y;
                od[5] = L.d.z;
            }
            __syncthreads();  // the pool is complete
            // wave w sweeps block b = w mod nblk (packed rays 32b .. 32b+31;
            // lanes 32..63 and the lanes past the last ray carry a copy of the
            // block's first ray); MfmaSpec::wg_split: with fewer blocks than
            // waves, the NW / nblk waves of a block split its triangle groups
            // into ranges (q = w / nblk) and the owners take the lexicographic
            // (distance, index) minimum over the ranges — the sequential scan's
            // result, as in coop_closest
            nblk = (total + 31u) >> 5;
            nrange = S.wg_split ? (uint32_t)NW / nblk : 1u;
            const uint32_t b = (uint32_t)wave % nblk, q = (uint32_t)wave / nblk;
            const uint32_t j0 = 32u * b;
            sweeping = q < nrange;
            upper = false;
            if (sweeping) {
                const int ng = (p.n_tris + 31) >> 5;
                G0 = (int)((uint32_t)ng * q / nrange);
                G1 = (int)((uint32_t)ng * (q + 1u) / nrange);
                res = q * 32u * nblk + j0;
                nb = min(32u, total - j0);
                const uint32_t j = j0 + (l < nb ? l : 0u);
                L.o = mk(pool.od[j][0], pool.od[j][1], pool.od[j][2]);
                L.d = mk(pool.od[j][3], pool.od[j][4], pool.od[j][5]);
            }
        } else {
            if (!act) continue;
            if (n_live <= (uint32_t)S.tail_lanes && __any(L.st == ST_DONE)) {
                // the cooperative drain (render_mfma's)
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
            if (n_live <= 32) {
                if (act >> 32) {
                    const bool live = (act >> l) & 1ull;
                    const int to = 4 * (int)(live ? lanes_below(act) : n_live + lanes_below(~act));
                    lane_permute(L, to);
                    act = __ballot(L.st == ST_TRACE);
                }
                upper = false;
            }
            // lanes without a ray carry the first live lane's (ST_DONE lanes
            // never read their o, d again)
            const int j0 = __builtin_ctzll(act);
            const f3 o = mk(__shfl(L.o.x, j0), __shfl(L.o.y, j0), __shfl(L.o.z, j0));
            const f3 dd = mk(__shfl(L.d.x, j0), __shfl(L.d.y, j0), __shfl(L.d.z, j0));
            if (L.st != ST_TRACE) {
                L.o = o;
                L.d = dd;
            }
            sweeping = true;
        }
        // one sweep call site for both forms: the wave's rays (its own, or its
        // block of the pool) are L.o, L.d
        float best = 1e38f;
        int bi = -1;
        if (sweeping) {
            const f3 ro = L.o, rd = L.d;
            float bestK = 1e38f * 1.0009765625f;
            lane_stash_packed(L, sh.lane, (int)l);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            const bool swept = sweep_k16<S>(p, sh, ro, rd, best, bi, bestK, dg, upper, G0, G1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            lane_unstash_packed(L, sh.lane, (int)l);
            L.o = ro;
            L.d = rd;
            if (!swept) coop_each(pooled ? (1ull << nb) - 1ull : __ballot(L.st == ST_TRACE), ro, rd, p, best, bi);
        }
        if (pooled) {
            if (sweeping && l < nb) {
                pool.best[res + l] = best;
                pool.bi[res + l] = bi;
            }
            __syncthreads();  // every block's results are in the pool
            if (mine) {
                // the ray travelled through the pool; the lane's own o, d come back from it
                L.o = mk(pool.od[slot][0], pool.od[slot][1], pool.od[slot][2]);
                L.d = mk(pool.od[slot][3], pool.od[slot][4], pool.od[slot][5]);
                best = pool.best[slot];
                bi = pool.bi[slot];
                for (uint32_t q = 1; q < nrange; q++) {
                    const float ob = pool.best[q * 32u * nblk + slot];
                    const int oi = pool.bi[q * 32u * nblk + slot];
                    if (ob < best || (ob == best && oi >= 0 && (bi < 0 || oi < bi))) {
                        best = ob;
                        bi = oi;
                    }
                }
            }
        }
        if (L.st == ST_TRACE) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    const RenderParams& p = kargs<RenderParams>();
    flush_counters(L, p);
}

}  // namespace
