// Kernel parameters, per-lane helpers and the closest-hit sweeps of the brute
// path: Möller–Trumbore (compute.glsl:302-340) behind an exact filter, the
// scalar-cache / LDS sweeps, the cooperative drain and the named kernel specs.
// Included by rt2_render.hip only (one translation unit; internal linkage).
#pragma once

namespace {

// Division-free filter evaluated before the reference arithmetic (DESIGN.md,
// "Exactness of the filter"); every form only skips tests the reference
// would reject, so all give the same bits.
enum class Filter : int {
    Five = 0,  // mt_pass: five compares and an and-chain
    Max3 = 1,  // mt_pass3: two v_max3_f32 and one compare (default)
    Plk = 2,   // per-ray precomputed records (sweep_plk; experiment builds)
};

// What a wave does when the item pool is empty and few of its lanes still trace.
enum class Tail : int {
    None = 0,  // every lane sweeps its own ray
    Coop = 1,  // the whole wave computes each live ray's closest hit (coop_closest)
    Team = 2,  // k = 64 / 2^ceil(log2 live) lanes per live ray (team_closest)
};

struct RenderParams {
    const float4* tri;  // 3 float4 per triangle: {ax ay az e0x} {e0y e0z e1x e1y} {e1z nx ny nz}
    const int* tri_mtl;
    const rt2_material* mats;
    int n_tris;
    int n_mats;
    int W, H;
    int maxBounce, R, envLight;
    float cam[3], vpRight[3], vpUp[3], vpFront[3], pixR[3], pixU[3], defR[3], defU[3];
    uint32_t frame_begin, frame_count;
    int tile_rows, rank, nranks;
    unsigned long long n_items;  // work items: pixels, or frames x pixels when frame_split
    unsigned long long n_pix;    // pixels of the shard
    int frame_split;             // 1: item = (frame, pixel), frame-major; colours -> frame_buf
    const uint32_t* order;       // nullable: run rank -> run of 64 pixels (most expensive first)
    uint32_t n_runs;             // full 64-pixel runs covered by `order` (the partial last run keeps its place)
    uint32_t* cost_out;          // nullable: per-pixel item cost (shader clocks) for the next launch's order
    float4* frame_buf;           // frame_split: [frame_count][n_pix] per-frame colours
    float4* accum;
    uint4* accum8;
    unsigned long long* item_counter;
    unsigned long long* region_ctr;  // nullable: 8 item-region counters, 128 B apart (XCD-group regions)
    unsigned long long* seg_counter;
    int tile_tris;  // TILED: triangles per LDS tile
    const rt2_node* nodes;  // BVH traversal
    int stack_slots;        // BVH: per-lane stack entries (tree depth + 2)
    int basicShadow;        // traceBasic: basicShadingShadow
    float light[3];         // traceBasic: basicShadingLightPosition.xyz
    const float4* bvh_recs; // BVH v2: child-pair records (4 float4 each)
    int bvh_root;           // BVH v2: stack entry of node 0
    int recs_ok;            // BVH v3: every record coordinate in {0} U [2^-37, 2^59]
    const rt2_triangle* raw;     // as uploaded (texture coordinates)
    const uchar4* texels;        // all textures, RGBA8 after GL unpack + swizzle
    const int4* tex_desc;        // per texture {width, height, offset lo, offset hi}
    int n_tex;                   // textures uploaded
    int num_textures;            // uniforms.numTextures
    const float4* plk;           // nullable: per-ray-precomputed filter records (sweep_plk), 4 float4 each
    float plk_A;                 // max |a_i| over the scene's triangles (sweep_plk error bound)
    int assist_cap;              // ASSIST: waves per workgroup that take items (the others start as helpers)
    int assist_chunk;            // ASSIST: triangles per chunk of a posted sweep (a multiple of the group)
    int assist_nchunks;          // ASSIST: chunks per sweep (< 4096)
    const void* mfma_frag;       // MFMA: f16 filter records [group][quantity][lane][8] (rt2_mfma.h)
    const float* mfma_tau;       // MFMA: per-triangle record scale
    float mfma_A;                // MFMA: max |a_i| over the in-range triangles
    const void* mfma_k16_frag;   // MFMA k16: f16 filter records [32-group][op][lane][8] (sweep_k16)
    const float* mfma_k16_tau;   // MFMA k16: per-triangle record scale
    const float2* mfma_k16_bnd;  // MFMA k16: per-triangle bounds of the m.z residual slots (k5 form)
    const void* mfma_kt_frag;    // MFMA kthr: f16 records [32-group][4 ops][lane][8], threshold in the K-slots
    unsigned long long* wave_log;  // nullable diagnostic: per wave {start, pool dry, end, segments} (ASSIST)
    uint32_t wave_log_n;           // waves the log holds
};

enum : int { ST_NEED_ITEM = 0, ST_NEW_FRAME = 1, ST_NEW_RAY = 2, ST_TRACE = 3, ST_DONE = 4 };

__device__ __forceinline__ f3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 xyz4(const rt2_vec4& v) { return mk(v.x, v.y, v.z); }

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// x as a value the compiler cannot treat as loop-invariant (an empty asm in
// the loop): what is derived from it — the reciprocal sequence of an integer
// division by a kernel argument — is recomputed where it is used, instead of
// being hoisted out of a persistent loop and held in VGPRs across the sweep
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    asm volatile("" : "+s"(x));
    return x;
}

// The kernel's first argument in the kernarg segment, through a pointer the
// compiler cannot treat as loop-invariant: its fields are loaded (s_load from
// the constant address space) where they are used.
template <class T>
__device__ __forceinline__ const T& kargs() {
    typedef const __attribute__((address_space(4))) T CT;
    CT* k = (CT*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(k));
    return *(const T*)k;
}

// __syncthreads_or for a workgroup of NW waves: one vote word per wave in LDS,
// one barrier (HIP's version reduces over a linear thread id that needs
// threadIdx.y/z in registers for the whole kernel, and takes three barriers).
// The votes are double-buffered by `parity` (wave-uniform, flipped per call):
// a wave writes the other buffer next time, and it can only get there after
// every wave has passed the next barrier, i.e. has read this one.
template <int NW>
struct BlockVote {
    uint32_t v[2][NW];
};
template <int NW>
__device__ __forceinline__ bool block_any(bool pred, BlockVote<NW>& bv, uint32_t& parity) {
    const uint32_t mine = __ballot(pred) != 0ull;
    if (lane_id() == 0) bv.v[parity][threadIdx.x >> 6] = mine;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll
    for (int w = 0; w < NW; w++) r |= bv.v[parity][w];
    parity ^= 1u;
    return r != 0;
}

__device__ __forceinline__ int shard_row(int local_row, int tile_rows, int rank, int nranks) {
    tile_rows = (int)opaque((uint32_t)tile_rows);
    int t = local_row / tile_rows;
    return (t * nranks + rank) * tile_rows + local_row % tile_rows;
}

// Survivor counters of the brute sweeps (diagnostic variants only): tests a
// wave evaluated, tests where some lane passed the filter, lane survivors.
struct FiltStats {
    unsigned long long tests = 0, wave_any = 0, lanes = 0;
    __device__ __forceinline__ void add(bool f) {
        const unsigned long long act = __ballot(true), m = __ballot(f);
        if (lane_id() == (uint32_t)__builtin_ctzll(act)) {  // once per wave-test
            tests += 1;
            wave_any += m != 0;
        }
        lanes += f;
    }
    __device__ __forceinline__ void flush(unsigned long long* c) {
        unsigned long long t = tests, w = wave_any, l = lanes;
        for (int off = 32; off > 0; off >>= 1) {
            t += __shfl_xor(t, off);
            w += __shfl_xor(w, off);
            l += __shfl_xor(l, off);
        }
        if (lane_id() == 0) {
            atomicAdd(c + 0, t);
            atomicAdd(c + 1, w);
            atomicAdd(c + 2, l);
        }
    }
};

// Exact intermediates of one test (phase 1 output, reused by phase 2).
struct MtQ {
    float det, tnum, U, V;
};
__device__ __forceinline__ MtQ mt_quantities(const f3& o, const f3& d, float4 t0, float4 t1, float4 t2) {
    const f3 a = mk(t0.x, t0.y, t0.z);
    const f3 e0 = mk(t0.w, t1.x, t1.y);
    const f3 e1 = mk(t1.z, t1.w, t2.x);
    const f3 n = mk(t2.y, t2.z, t2.w);
    MtQ r;
    r.det = -dot(d, n);
    const f3 ao = sub(o, a);
    r.tnum = dot(ao, n);
    const f3 q = cross(d, ao);
    r.U = dot(e1, q);
    r.V = dot(e0, q);
    return r;
}
__device__ __forceinline__ bool mt_pass(const MtQ& q, float bestK) {
    const float B = q.det * 0x1p-60f;
    return (q.tnum > 0.0f) & (q.U <= B) & (q.V >= -B) & ((q.V - q.U) <= q.det * 1.0009765625f) &
           (q.tnum <= q.det * bestK);
}
// mt_pass in 6 VALU instead of 9 and one compare (two v_max3_f32; one lane
// mask, no SALU and-chain): with B = det*2^-60 it passes iff
//   max(U, -V, RN(V-U) - det*(1+2^-10), -tnum, tnum - det*bestK) <= B,
// the two fused differences rounded once (their sign is exact).  Each term
// above B rejects only what mt_pass's proof rejects ("Exactness of
// the filter"): U > B and -V > B as before; RN(V-U) > det*(1+2^-10) exactly is
// the w test with a tighter right side; -tnum > B >= 0 gives dst < 0;
// tnum > det*bestK + B exactly gives dst >= best.  For det <= 0 (B <= 0) every
// outcome is rejected by the exact test anyway.  A NaN term is ignored by
// fmaxf (maxNum), which can only pass more.  (A constant 2^-100 in place of B
// saves the multiply but measured 0.6 % slower.)
__device__ __forceinline__ bool mt_pass3(const MtQ& q, float bestK) {
    const float B = q.det * 0x1p-60f;
    const float X = __builtin_fmaf(-q.det, 1.0009765625f, q.V - q.U);
    const float Y = __builtin_fmaf(-q.det, bestK, q.tnum);
    return fmaxf(fmaxf(fmaxf(fmaxf(q.U, -q.V), X), -q.tnum), Y) <= B;
}
template <Filter FILT>
__device__ __forceinline__ bool mt_pass_f(const MtQ& q, float bestK) {
    if constexpr (FILT == Filter::Max3)
        return mt_pass3(q, bestK);
    else
        return mt_pass(q, bestK);
}

// Scalar-path record delivery: a triangle record is wave-uniform, so it is read
// with scalar loads (constant address space -> s_load_dwordx4 into SGPRs,
// through the scalar data cache) and fed to the VALU as SGPR operands.
typedef const __attribute__((address_space(4))) float cfloat;
__device__ __forceinline__ float4 ldc4(cfloat* p) { return make_float4(p[0], p[1], p[2], p[3]); }

// compute.glsl:312-327 on the phase-1 intermediates (exactly the reference arithmetic).
__device__ __forceinline__ void mt_exact(const MtQ& q, int idx, float& best, int& bi, float& bestK) {
    if (!((q.det < 1e-10f && q.det > -1e-10f) || q.det < 0.0f)) {
        const float inv = 1.0f / q.det;
        const float dst = q.tnum * inv;
        const float u = -q.U * inv;
        const float v = q.V * inv;
        if (!(dst <= 1e-6f) && !(u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f) && dst < best) {
            best = dst;
            bi = idx;
            bestK = best * 1.0009765625f;
        }
    }
}

// Masked two-phase sweep: phase 1 computes the intermediates and the filter of
// G triangles (the G predicates stay wave lane-masks in SGPR pairs, no
// per-lane bit packing); phase 2 runs mt_exact under each mask in index order
// (skipped by a scalar branch when the mask is empty).  SMEM selects the
// scalar-load path for the triangle records instead of LDS.
template <int G, bool SMEM, Filter FILT = Filter::Five, bool STATS = false>
__device__ __forceinline__ void sweep_masked(const f3& o, const f3& d, const float4* lds, const float* gtri,
                                             int count, int base, float& best, int& bi, float& bestK,
                                             FiltStats* fs = nullptr) {
    int i = 0;
    for (; i + G <= count; i += G) {
        MtQ q[G];
        bool f[G];
#pragma unroll
        for (int k = 0; k < G; k++) {
            float4 t0, t1, t2;
            if constexpr (SMEM) {
                cfloat* t = (cfloat*)gtri + 12 * (i + k);
                t0 = ldc4(t);
                t1 = ldc4(t + 4);
                t2 = ldc4(t + 8);
            } else {
                const float4* t = lds + 3 * (i + k);
                t0 = t[0];
                t1 = t[1];
                t2 = t[2];
            }
            q[k] = mt_quantities(o, d, t0, t1, t2);
            f[k] = mt_pass_f<FILT>(q[k], bestK);
            if constexpr (STATS) fs->add(f[k]);
        }
#pragma unroll
        for (int k = 0; k < G; k++)
            if (f[k]) mt_exact(q[k], base + i + k, best, bi, bestK);
    }
    for (; i < count; i++) {
        float4 t0, t1, t2;
        if constexpr (SMEM) {
            cfloat* t = (cfloat*)gtri + 12 * i;
            t0 = ldc4(t);
            t1 = ldc4(t + 4);
            t2 = ldc4(t + 8);
        } else {
            const float4* t = lds + 3 * i;
            t0 = t[0];
            t1 = t[1];
            t2 = t[2];
        }
        const MtQ q = mt_quantities(o, d, t0, t1, t2);
        if (mt_pass_f<FILT>(q, bestK)) mt_exact(q, base + i, best, bi, bestK);
    }
}

// Per-ray precomputed filter ("plk" records).  The reference intermediates
// are U = e1·(d×(o−a)), V = e0·(d×(o−a)), tnum = (o−a)·n.  By the triple
// product identity they equal
//     U = e1·m − d·p1,  V = e0·m − d·p0,  tnum = o·n − a·n,
// with m = d×o once per segment and p0 = a×e0, p1 = a×e1, a·n once per
// triangle (host-side in binary64).  That is 18 VALU for the four
// quantities instead of 21, and the filter needs no per-test origin shift.
// They are approximations U', V', tnum' of the reference's rounded values;
// the filter compares against a threshold T that covers the error of both
// ("The per-ray filter"):
//   |U' − s·U_ref|, |V' − s·V_ref|, |tnum' − s·tnum_ref| <= 2^-16 (|o|∞ + A)
//   T = 2^-13 (|o|∞ + A) + 2^-40                  (A = scene max |a|∞)
// where s = 2^k is the triangle's record scale (s·max(|e0|,|e1|,|n|) in
// [1,2)), so one threshold per segment serves every triangle.  The record
// is valid only in the range the bound was derived for: the host checks it
// per triangle (prep_plk: outside it a triangle's record always passes), the
// kernel per segment (|o|∞ <= 2^20, |d|∞ <= 1.0001 — every direction the path
// makes is unit length to a few ulps; otherwise the wave takes sweep_masked).  dn = d·n_s = −det_s;
// bkf = bestK while it is <= 2^60, +inf before (or without) a near hit.
// Pass iff max(U', −V', RN(V'−U') + c·dn, −tnum', tnum' + bkf·dn) <= T.
// Survivors run the reference arithmetic (mt_quantities + mt_exact) on the
// triangle's own record: the closest hit is bit-identical by construction.
// Record (4 float4): {n_s, −a·n_s} {e0_s, −p0_s.x} {−p0_s.yz, e1_s.xy} {e1_s.z, −p1_s}.
__device__ __forceinline__ bool plk_pass(const f3& o, const f3& d, const f3& m, float T, float bkf, cfloat* r) {
    const float dn = __builtin_fmaf(d.z, r[2], __builtin_fmaf(d.y, r[1], d.x * r[0]));
    const float tn = __builtin_fmaf(o.z, r[2], __builtin_fmaf(o.y, r[1], __builtin_fmaf(o.x, r[0], r[3])));
    float V = __builtin_fmaf(r[6], m.z, __builtin_fmaf(r[5], m.y, r[4] * m.x));
    V = __builtin_fmaf(d.z, r[9], __builtin_fmaf(d.y, r[8], __builtin_fmaf(d.x, r[7], V)));
    float U = __builtin_fmaf(r[12], m.z, __builtin_fmaf(r[11], m.y, r[10] * m.x));
    U = __builtin_fmaf(d.z, r[15], __builtin_fmaf(d.y, r[14], __builtin_fmaf(d.x, r[13], U)));
    const float X = __builtin_fmaf(dn, 1.0009765625f, V - U);
    const float Y = __builtin_fmaf(dn, bkf, tn);
    return fmaxf(fmaxf(fmaxf(fmaxf(U, -V), X), -tn), Y) <= T;  // two v_max3_f32
}
template <int G, bool STATS = false>
__device__ __forceinline__ void sweep_plk(const f3& o, const f3& d, const float* plk, const float* gtri, int count,
                                          float A, float& best, int& bi, float& bestK, FiltStats* fs = nullptr) {
    const f3 m = cross(d, o);
    const float O = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float T = __builtin_fmaf(0x1p-13f, O + A, 0x1p-40f);
    float bkf = bestK <= 0x1p60f ? bestK : __builtin_inff();
    int i = 0;
    for (; i + G <= count; i += G) {
        bool f[G];
#pragma unroll
        for (int k = 0; k < G; k++) {
            f[k] = plk_pass(o, d, m, T, bkf, (cfloat*)plk + 16 * (i + k));
            if constexpr (STATS) fs->add(f[k]);
        }
#pragma unroll
        for (int k = 0; k < G; k++) {
            if (f[k]) {
                cfloat* t = (cfloat*)gtri + 12 * (i + k);
                mt_exact(mt_quantities(o, d, ldc4(t), ldc4(t + 4), ldc4(t + 8)), i + k, best, bi, bestK);
                bkf = bestK <= 0x1p60f ? bestK : __builtin_inff();
            }
        }
    }
    for (; i < count; i++) {
        if (plk_pass(o, d, m, T, bkf, (cfloat*)plk + 16 * i)) {
            cfloat* t = (cfloat*)gtri + 12 * i;
            mt_exact(mt_quantities(o, d, ldc4(t), ldc4(t + 4), ldc4(t + 8)), i, best, bi, bestK);
            bkf = bestK <= 0x1p60f ? bestK : __builtin_inff();
        }
    }
}
// The segment's rays are inside the range sweep_plk's bound covers.
__device__ __forceinline__ bool plk_lane_ok(const f3& o, const f3& d) {
    const float O = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float D = fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z));
    return O <= 0x1p20f && D <= 1.0001f;  // false for NaN and inf
}

// Cooperative closest hit for the drain phase: all 64 lanes sweep ONE ray
// (lane l tests triangles l, l+64, ... in increasing order with its own
// running best) and the wave reduces (dst, index) lexicographically.  The
// result equals the sequential strict-< scan: the minimum distance, and among
// exact ties the lowest index.  Triangle records are read from `tris`
// (LDS or global) with per-lane addresses.
__device__ __forceinline__ void coop_closest(const f3& o, const f3& d, const float4* tris, int n, float& best_out,
                                             int& bi_out) {
    const int lane = (int)lane_id();
    float best = 1e38f, bestK = 1e38f * 1.0009765625f;
    int bi = -1;
    for (int i = lane; i < n; i += 64) {
        const float4* t = tris + 3 * i;
        const MtQ q = mt_quantities(o, d, t[0], t[1], t[2]);
        if (mt_pass3(q, bestK)) mt_exact(q, i, best, bi, bestK);
    }
    for (int off = 32; off > 0; off >>= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        const bool take = (ob < best) || (ob == best && oi >= 0 && (bi < 0 || oi < bi));
        if (take) {
            best = ob;
            bi = oi;
        }
    }
    best_out = best;
    bi_out = bi;
}

// Team sweep (tail mode): the n live rays of a wave each get a team of
// k = 64 / 2^ceil(log2 n) lanes; member j of a team tests triangles j, j+k,
// j+2k, ... of its ray (vector loads: the k members read k consecutive
// records, every team the same ones), then the team reduces (dst, index)
// lexicographically — the sequential strict `dst < best` scan's result.  A
// segment of every live ray costs N/k tests per lane instead of N, so the
// last rays of a launch (and small per-GPU slabs) finish up to k times sooner.
// Returns the closest hit of the calling lane's own ray (live lanes).
__device__ __forceinline__ void team_closest(const f3& lo, const f3& ld, const float4* tris, int n_tris,
                                             unsigned long long act, float& best_out, int& bi_out) {
    const int n = __popcll(act);
    const int lg = n <= 1 ? 0 : 32 - __builtin_clz((unsigned)(n - 1));
    const int k = 64 >> lg;
    const int me = (int)lane_id();
    const int t = me / k, j = me - t * k;
    // the t-th live lane of the wave: the lane whose live-rank is t
    int leader = 0;
    {
        unsigned long long m = act;
        for (int r = 0; r < t && m; r++) m &= m - 1;
        leader = m ? __builtin_ctzll(m) : 0;
    }
    const bool member = t < n;
    const f3 o = mk(__shfl(lo.x, leader), __shfl(lo.y, leader), __shfl(lo.z, leader));
    const f3 d = mk(__shfl(ld.x, leader), __shfl(ld.y, leader), __shfl(ld.z, leader));
    float best = 1e38f, bestK = 1e38f * 1.0009765625f;
    int bi = -1;
    if (member) {
        for (int i = j; i < n_tris; i += k) {
            const float4* tp = tris + 3 * i;
            const MtQ q = mt_quantities(o, d, tp[0], tp[1], tp[2]);
            if (mt_pass(q, bestK)) mt_exact(q, i, best, bi, bestK);
        }
    }
    for (int off = 1; off < k; off <<= 1) {
        const float ob = __shfl_xor(best, off);
        const int oi = __shfl_xor(bi, off);
        const bool take = (ob < best) || (ob == best && oi >= 0 && (bi < 0 || oi < bi));
        if (take) {
            best = ob;
            bi = oi;
        }
    }
    // each live lane reads its team's result (team index = its live rank)
    const int src = (int)lanes_below(act) * k;
    best_out = __shfl(best, src);
    bi_out = __shfl(bi, src);
}

}  // namespace
