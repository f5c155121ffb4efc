// Brute-force render kernel for launches with few items per lane (the rank
// slabs of a multi-GPU render): idle waves sweep triangle chunks, or whole
// rays, of the busy waves' segments through LDS jobs.  Same closest hit as
// the sequential scan, bit for bit (see below).
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

// ASSIST: waves that have run out of items help the busy waves of their own
// workgroup.  A busy wave ("owner") posts its segment — its 64 rays — to LDS
// as a job of units that any wave of the workgroup may claim:
//   - chunk jobs (many live rays): unit = a contiguous chunk of the triangle
//     array, swept for all 64 rays with the scalar-path filtered test; each
//     lane's result is folded into the job's per-lane 64-bit key (dst bits <<
//     32 | index) by an LDS atomic min — dst > 1e-6 is positive, so the key
//     order is the lexicographic (dst, index) order, the sequential strict
//     `dst < best` scan's result bit for bit;
//   - ray jobs (few live rays): unit = one live ray, whose closest hit the
//     claiming wave computes with all 64 lanes (coop_closest: lane l tests
//     triangles l, l+64, ..., then a lexicographic wave reduction).
// Units are claimed with a compare-and-swap on the job's ticket
// (seq:7 | ray job:1 | units:12 | next unit:12).  The owner serves units (its
// own job's first, then other jobs') until its own job is complete, reads its
// lanes' keys and shades; a helper serves units until no wave of its
// workgroup is busy.  Without helpers an owner sweeps alone (or serves its
// own ray job: SMEM's cooperative drain).  Waves at index >= assist_cap never
// take items: a launch with few items per lane keeps helpers beside every
// owner (split-wave speed per ray without replicated shading), and every
// wave that runs out of items joins them.  No workgroup barrier after the
// first: a busy wave leaves only after its last job is complete, and a
// helper only once no wave is busy, so every wave reaches the exit.
struct AssistSpec {
    int waves_per_block;  // NW: waves per workgroup (helpers serve their own workgroup)
    int group;
    Filter filter;
    int waves;       // minimum waves per SIMD the register allocation must allow
    int coop_rays;   // with helpers: ray jobs for at most this many live rays (chunk jobs above)
    bool mfma = false;    // sweeps and chunk units through the matrix filter (rt2_mfma.h sweep_mfma)
    bool minred = false;  // its one-compare-per-group form
};

template <AssistSpec S>
constexpr MfmaSpec assist_mfma_spec() {
    return MfmaSpec{.block = 64 * S.waves_per_block, .waves = S.waves, .tail_lanes = 16, .imax = true,
                    .minred = S.minred};
}

template <int NW, bool M = false>
struct AssistLds {
    float ray[NW][6][64];            // posted rays, [wave][o.xyz d.xyz][lane]
    unsigned long long res[NW][64];  // per-lane closest-hit key of the job
    uint8_t list[NW][64];            // ray jobs: lane of the u-th live ray
    uint32_t ticket[NW];             // seq:7 | ray job:1 | units:12 | next unit:12
    uint32_t done[NW];               // units finished
    int busy;                        // waves that may still post jobs
    int helpers;                     // waves in the helper loop
    MfmaWaveLds mw[M ? NW : 0];      // matrix filter: each wave's ray-fragment staging
};

__device__ __forceinline__ unsigned long long hit_key(float best, int bi) {
    return bi >= 0 ? (unsigned long long)__float_as_uint(best) << 32 | (uint32_t)bi : ~0ull;
}

// Claims the next unit of job `s`: returns the ticket it advanced (lane-uniform),
// or 0xffffffff when the job has no unit left.  The loop is wave-uniform: lane
// 0 alone issues the compare-and-swap and its result is broadcast under the
// full mask before any branch.
__device__ __forceinline__ uint32_t assist_claim(uint32_t* ticket) {
    uint32_t t = __builtin_amdgcn_readfirstlane(__hip_atomic_load(ticket, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
    for (;;) {
        if ((t & 0xfffu) >= ((t >> 12) & 0xfffu)) return 0xffffffffu;
        uint32_t old = t;
        if (lane_id() == 0) {
            uint32_t e = t;
            __hip_atomic_compare_exchange_strong(ticket, &e, t + 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_WORKGROUP);
            old = e;  // the value found: == t iff the swap happened
        }
        old = __builtin_amdgcn_readfirstlane(old);
        if (old == t) return t;
        t = old;
    }
}

// Runs one claimed unit (ticket value t) of job `s`.
template <AssistSpec S, int NW>
__device__ __forceinline__ void assist_unit(const RenderParams& p, AssistLds<NW, S.mfma>& sh, int w, int s, uint32_t t) {
    const int lane = (int)lane_id();
    const int u = (int)(t & 0xfffu);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (t & 0x1000000u) {
        // ray job: the u-th live ray, all lanes
        const int j = sh.list[s][u];
        const float* r = &sh.ray[s][0][j];
        float b;
        int bidx;
        coop_closest(mk(r[0], r[64], r[128]), mk(r[192], r[256], r[320]), p.tri, p.n_tris, b, bidx);
        if (lane == 0) sh.res[s][j] = hit_key(b, bidx);
    } else {
        const float* r = &sh.ray[s][0][lane];
        const int lo = u * p.assist_chunk, hi = min(lo + p.assist_chunk, p.n_tris);
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        const f3 ro = mk(r[0], r[64], r[128]), rd = mk(r[192], r[256], r[320]);
        bool done = false;
        MfmaDiag dg;  // unused (assist specs count nothing)
        if constexpr (S.mfma)  // chunks are whole 16-triangle groups; posted idle lanes carry a live ray
            done = sweep_mfma<assist_mfma_spec<S>()>(p, sh.mw[w], ro, rd, best, bi, bestK, dg, lo >> 4, (hi + 15) >> 4);
        if (!done)
            sweep_masked<S.group, true, S.filter>(ro, rd, nullptr, (const float*)p.tri + 12 * (size_t)lo, hi - lo, lo,
                                                  best, bi, bestK);
        if (bi >= 0) atomicMin(&sh.res[s][lane], hit_key(best, bi));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (lane == 0) __hip_atomic_fetch_add(&sh.done[s], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Serves units of this workgroup's jobs (own job first).  own >= 0: until
// job `own` (of `units` units) is complete; own < 0: until no wave is busy.
template <AssistSpec S, int NW>
__device__ __forceinline__ void assist_work(const RenderParams& p, AssistLds<NW, S.mfma>& sh, int w, int own,
                                            uint32_t units) {
    constexpr int WG = __HIP_MEMORY_SCOPE_WORKGROUP;
    for (;;) {
        bool any = false;
#pragma unroll 1
        for (int k = 0; k < NW && !any; k++) {
            const int s = (w + k) % NW;
            const uint32_t t = assist_claim(&sh.ticket[s]);
            if (t != 0xffffffffu) {
                assist_unit<S, NW>(p, sh, w, s, t);
                any = true;
            }
        }
        if (own >= 0) {
            if ((uint32_t)__builtin_amdgcn_readfirstlane(__hip_atomic_load(&sh.done[own], __ATOMIC_RELAXED, WG)) >=
                units)
                break;
        } else if (!any && __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sh.busy, __ATOMIC_RELAXED, WG)) == 0) {
            break;
        }
        if (!any) __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

template <AssistSpec S>
__global__ __launch_bounds__(64 * S.waves_per_block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_assist(
    RenderParams p) {
    constexpr int NW = S.waves_per_block;
    constexpr int WG = __HIP_MEMORY_SCOPE_WORKGROUP;
    __shared__ AssistLds<NW, S.mfma> sh;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = (int)(threadIdx.x & 63);
    const int cap = min(max(p.assist_cap, 1), NW);
    if (threadIdx.x == 0) {
        sh.busy = cap;
        sh.helpers = 0;
    }
    if (threadIdx.x < NW) {
        sh.ticket[threadIdx.x] = 0;  // no open job: no units
        sh.done[threadIdx.x] = 0;
    }
    __syncthreads();
    Lane L;
    lane_init(L);
    uint32_t seq = 0;
    unsigned long long t_start = 0, t_dry = 0;  // wave_log diagnostic
    if (p.wave_log) t_start = __builtin_amdgcn_s_memrealtime();
    if (w < cap) {
        for (;;) {
            advance(L, p);
            const unsigned long long act = __ballot(L.st == ST_TRACE);
            if (p.wave_log && !t_dry && __any(L.st == ST_DONE)) t_dry = __builtin_amdgcn_s_memrealtime();
            if (!act) break;
            const uint32_t live = (uint32_t)__popcll(act);
            const bool helped = __builtin_amdgcn_readfirstlane(__hip_atomic_load(&sh.helpers, __ATOMIC_RELAXED, WG)) > 0;
            // without helpers: SMEM's cooperative drain (<= 32 live rays, pool dry)
            const bool ray_job = helped ? live <= (uint32_t)S.coop_rays : live <= 32u && __any(L.st == ST_DONE);
            const bool chunk_job = !ray_job && helped && p.assist_nchunks > 1;
            float best = 1e38f, bestK = 1e38f * 1.0009765625f;
            int bi = -1;
            // matrix filter: lanes without a ray carry the first live lane's
            // (in range, so the wave keeps the matrix filter; their passes add
            // no triangle and their results are not read)
            f3 po = L.o, pd = L.d;
            if constexpr (S.mfma) {
                const int j0 = __builtin_ctzll(act);
                if (L.st != ST_TRACE) {
                    po = mk(__shfl(L.o.x, j0), __shfl(L.o.y, j0), __shfl(L.o.z, j0));
                    pd = mk(__shfl(L.d.x, j0), __shfl(L.d.y, j0), __shfl(L.d.z, j0));
                } else {
                    (void)__shfl(L.o.x, j0), (void)__shfl(L.o.y, j0), (void)__shfl(L.o.z, j0);
                    (void)__shfl(L.d.x, j0), (void)__shfl(L.d.y, j0), (void)__shfl(L.d.z, j0);
                }
            }
            if (ray_job || chunk_job) {
                float* r = &sh.ray[w][0][lane];
                r[0] = po.x;
                r[64] = po.y;
                r[128] = po.z;
                r[192] = pd.x;
                r[256] = pd.y;
                r[320] = pd.z;
                sh.res[w][lane] = ~0ull;
                if (L.st == ST_TRACE) sh.list[w][lanes_below(act)] = (uint8_t)lane;
                const uint32_t units = ray_job ? live : (uint32_t)p.assist_nchunks;
                if (lane == 0) sh.done[w] = 0;
                seq = (seq + 1u) & 0x7fu;
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0)
                    __hip_atomic_store(&sh.ticket[w], seq << 25 | (ray_job ? 0x1000000u : 0u) | units << 12,
                                       __ATOMIC_RELAXED, WG);
                assist_work<S, NW>(p, sh, w, w, units);
                const unsigned long long key = sh.res[w][lane];
                if (key != ~0ull) {
                    best = __uint_as_float((uint32_t)(key >> 32));
                    bi = (int)(uint32_t)key;
                }
            } else if constexpr (S.mfma) {
                MfmaDiag dg;
                if (!sweep_mfma<assist_mfma_spec<S>()>(p, sh.mw[w], po, pd, best, bi, bestK, dg) && L.st == ST_TRACE)
                    sweep_masked<S.group, true, S.filter>(L.o, L.d, nullptr, (const float*)p.tri, p.n_tris, 0, best,
                                                          bi, bestK);
            } else if (L.st == ST_TRACE) {
                sweep_masked<S.group, true, S.filter>(L.o, L.d, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi,
                                                      bestK);
            }
            if (L.st == ST_TRACE) {
                L.bounce += 1;
                L.segs += 1;
                shade(L, p, best, bi);
            }
        }
        if (lane == 0) __hip_atomic_fetch_add(&sh.busy, -1, __ATOMIC_RELAXED, WG);
    }
    // helper: serve this workgroup's jobs until no wave is busy
    if (lane == 0) __hip_atomic_fetch_add(&sh.helpers, 1, __ATOMIC_RELAXED, WG);
    assist_work<S, NW>(p, sh, w, -1, 0);
    flush_counters(L, p);
    if (p.wave_log) {
        const uint32_t gw = blockIdx.x * NW + (uint32_t)w;
        unsigned long long sg = L.segs;
        for (int off = 32; off > 0; off >>= 1) sg += __shfl_xor(sg, off);
        if (lane == 0 && gw < p.wave_log_n) {
            unsigned long long* e = p.wave_log + 4 * (size_t)gw;
            e[0] = t_start;
            e[1] = t_dry;
            e[2] = __builtin_amdgcn_s_memrealtime();
            e[3] = sg;
        }
    }
}

}  // namespace
