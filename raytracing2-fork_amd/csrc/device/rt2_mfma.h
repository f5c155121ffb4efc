// Brute-force render kernel whose triangle filter runs on the matrix cores.
// Included by rt2_render.hip only (one translation unit; internal linkage).
//
// The filter quantities of a ray-triangle test are linear in the ray once
// m = d×o is formed per segment (the triple-product form of sweep_plk):
//     U = E1·m − d·P1,  −V = −E0·m + d·P0,  X = V − U + c·dn = (E0−E1)·m + d·(P1−P0+cN),
//     −tn = −o·N + AN,  dn = d·N = −det
// (E0, E1, N = s·e0, s·e1, s·n; P0, P1 = s·(a×e0), s·(a×e1); AN = s·(a·n);
// c = 1 + 2^-10; s = 2^k with s·max(|e0|,|e1|,|n|)∞ in [1,2)).  So for 16
// rays × 16 triangles each quantity is one 16×16 matrix product over the ray
// vector (d, m, o, 1): v_mfma_f32_16x16x32_f16 with every value split into two
// f16 halves (x ≈ hi + lo; hi·hi + hi·lo + lo·hi in 3 of the 32 k-slots), an
// approximation to ~2^-18 of the terms' magnitude at 16× the f32 VALU rate.
// The distance term Y = s (tnum − bk·det) is the −tn record times a second
// ray fragment (−(o + bk·d), −1), rebuilt when a lane's bound improves (with
// no usable bound: (−Bmax·d, 0), the det > 0 test) — MfmaSpec::ymma, the
// default; the older form computes dn = d·N and forms Y with one FMA per pair.
// The VALU then only takes the max of the five terms.
// Like the division-free filter it only decides which tests to skip: a term
// above the threshold T implies the reference rejects ("The matrix
// filter"), and every (wave, triangle) with a passing pair runs the exact
// phase (mt_pass3 + mt_exact: the reference arithmetic) for all 64 rays in
// index order — the sequential strict `dst < best` scan's result bit for bit.
//
// Layout (MFMA f16 16x16x32 operand maps): A = rays, lane l holds ray
// 16R + (l&15), k-slots 8(l>>4)..+7; B = triangles, lane l holds triangle
// 16G + (l&15), the same k-slots; D: lane l holds rays 16R + 4(l>>4) + i
// (i = 0..3) × triangle l&15.  Records: [group][quantity][lane][8 f16] (5 KiB
// per 16 triangles) plus a per-triangle scale tau (power of two that puts the
// triangle's largest coefficient in [2^13, 2^14)).
#pragma once

namespace {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));

constexpr int kMfmaQ = 5;                   // quantities per triangle: U, -V, X, -tn, dn
constexpr float kMfmaC = 1.0009765625f;     // c = 1 + 2^-10 (the w test's slack, as in F)
constexpr float kMfmaE = 0x1p-14f;          // dn bias: > the bound on |dn' - dn| in s-units
constexpr float kMfmaTs = 0x1p-10f;         // T = 2^-10 (Omax + A + 1)
constexpr float kMfmaB = 2.0f;              // distance test active while bestK <= 2 (Omax + A + 1)

struct MfmaSpec {
    int block;
    int waves;       // minimum waves per SIMD the register allocation must allow
    int tail_lanes;  // cooperative drain at <= this many live rays (pool dry)
    bool imax = false;      // max of the five terms on their bit patterns (no NaN quieting; see sweep_mfma)
    bool prefetch = false;  // the next group's records are requested before this group's products
    bool minred = false;    // imax + one compare per group: min over the lane's 16 pairs (all one triangle)
    bool lockstep = true;   // the workgroup's waves start every segment together (one barrier per segment)
    bool diag = false;      // count groups / groups with survivors / exact tests (experiment variants only)
    bool ymma = false;      // Y = tn - bk det by a matrix product too (-tn record x ray fragment (-w, -1)): no FMA per pair
    int tshift = 10;        // T = 2^-tshift (Omax + A + 1); 12 for the ymma product variants
    int lds_pad = 0;        // extra static LDS per workgroup (bytes): caps the resident workgroups (experiments)
    bool k16 = false;       // sweep_k16: v_mfma_f32_32x32x16_f16 on 32-triangle groups, 8 products per 32 rays
    bool afrag_lds = false; // k16: the ray fragments are re-read from LDS every group (fewer VGPRs)
    bool rsplit = false;    // k16: scheduling fence between the two 32-ray blocks (one block's terms live at a time)
    int lane_lds = 0;       // k16: the lane's path state (all but o, d) waits in LDS during the sweep (fewer VGPRs);
                            // 2 = packed into 16 words with 96-B fragment rows (10 KiB of LDS per wave: 4 waves/SIMD)
    bool lateload = false;  // k16 (serial 1/3/4): the next group's records are requested into the operand registers
                            // right after this group's last product is issued (no extra VGPRs)
    bool compact = false;   // k16: <= 32 live rays move to lanes 0..31 and the second 32-ray block is skipped
    bool k5 = false;        // k16: U, -V, X from the first K-half only (5 products per 32-ray block instead of 8);
                            // the two m.z slots left out are bounded per (wave, triangle) and added to the threshold
    bool no_tn = false;     // k5 experiment: no -tn term (4 products per block; the filter stays conservative,
                            // it only passes more pairs to the exact phase)
    int serial = 0;         // k16: scheduling fences per 32-ray block: 1 = U V X products | their max | -tn Y
                            // products | the rest (48 accumulator VGPRs live); 2 = all 8 products | the reduction;
                            // 3 = 1 without the fence between the blocks; 4 = 3 without the fence at the group end
    bool pipe = false;      // (removed: the software-pipelined k16 sweep, DESIGN.md "Tried and measured")
    int tile_groups = 0;    // k5 (render_mfma_k5t, rt2_k5_tiles.h): 32-triangle groups per LDS record tile
    bool dpp = false;       // the per-segment wave maxima by DPP lane moves (wave_max_dpp) instead of ds_bpermute
    bool rows80 = false;    // no_tn: 80-B fragment rows, main slots 0..15 (the first K-half) + the Y slots at 16..31
    int tile_bufs = 2;      // render_mfma_k5t: record tile buffers (3: tile t+2 in flight while t is swept)
    int ylds = 0;           // cthr: each block's Y fragment (1), or its main and Y fragments (2), read from LDS right
                            // before its products
    bool cthr = false;      // k5 no_tn: the threshold rides in the products' accumulator operand (one matrix
                            // product per group, mfma_thr_frag), and the reduction is a sign-bit AND / OR
                            // (2 v_bitop3_b32 per pair instead of 2.5 min / max)
    bool perm_frag = false; // render_mfma_k5t: fragments built in registers by v_permlane32_swap (no LDS rows)
    bool thr_hoist = false;  // k5_cthr_group: the threshold fragment built once per sweep, not once per group
    bool fair_prio = false;  // render_mfma_k5r: issue priority (s_setprio) by the rays the wave's slowest lane has
                             // left, quartiles of the rays per pixel (fair share among a SIMD's waves)
    int res_groups = 0;     // render_mfma_k5r (rt2_k5_resident.h): every group's records resident in the
                            // workgroup's LDS for the whole launch (scenes of <= res_groups 32-triangle groups)
    bool exact_pf = false;  // render_mfma_k5r: the exact phase requests the next triangle before testing this one
    bool kt_lane_w = false; // kthr: the B_q slot's ray factor W per ray (its own mw_y + mw_z), not the wave's maximum
    bool lean = false;      // render_mfma_k5r: x, y recomputed from the item, segments counted per wave (fewer
                            // VGPRs live across the sweep)
    int kthr = 0;           // the threshold in the K-slots (round 6, DESIGN.md "The threshold in the K-slots"):
                            // U, -V, X drop the m.y and m.z cross slots and carry -tau x Tw' and -B x W' in slots
                            // 14, 15; Y carries -tau x Tw' in slot 29: 8 products per group with a zero
                            // accumulator, no TT product.  Schedule per 32-ray block: 1 = the four products, then
                            // the 32 sign-bit VALU; 2 = U V X | their AND | Y | the fold (cthr's order); 3 = no
                            // fences (the compiler's order)
    bool res_l2 = false;    // render_mfma_k5r + kthr: groups beyond res_groups are read from L2 (global loads per
                            // wave) after the resident ones: scenes of up to 256 groups
    int phase_prio = 0;      // render_mfma_k5r: issue priority by phase (1 products high, 2 exact phase high,
                             // 3 shading high; rt2_k5_resident.h phase_prio)
    bool flow_prio = false;  // tile_flow: issue priority by the wave's finishing rank in the last tile
    bool tile_flow = false;  // render_mfma_k5t + kthr: the tiles as a stream with LDS counters, no barrier per tile;
                             // every wave issues and publishes its share of each tile (rt2_k5_tiles.h sweep_kt_flow)
    int sol = 0;            // speed-of-light probes (WRONG images; diag clocks only): 1 = every group reads group
                            // 0's records, 2 = no exact phase, 3 = 2 + only the U term is reduced; marginal-cost
                            // probes (same image): 4 = exact phase twice, 5 = products and reduction twice,
                            // 6 = the reduction's VALU twice, 7 = the products twice
};

// per-wave diagnostic counts of sweep_mfma (wave-uniform; MfmaSpec::diag)
struct MfmaDiag {
    unsigned long long groups = 0, hot = 0, exact = 0;
    // shader clocks (s_memtime) of the loop's phases, per wave: item refill +
    // ray generation (advance), the closest-hit sweep, shading, the
    // cooperative drain
    unsigned long long t_advance = 0, t_sweep = 0, t_shade = 0, t_tail = 0;
    // sweep_kt_flow: waiting for a tile, the products (with the records' LDS
    // reads), the exact phase (with the Y rebuilds), the whole sweep; the
    // wave's whole life in the kernel
    unsigned long long t_wait = 0, t_filt = 0, t_exact = 0, t_swp = 0, t_all = 0;
    // ... and of that: issuing the wave's tile shares, waiting for them to land; shares issued
    unsigned long long t_issue = 0, t_pub = 0, claims = 0;
};

// per wave: the ray fragments' staging rows (80-B stride: conflict-free
// 16-B reads) and the rays' distance-test bounds
struct MfmaWaveLds {
    _Float16 ray[64][40];
    float bk[64];
};

// Filter coefficients of padded triangle i (binary64, from the pre-transformed
// f32 triangle) and its record scale tau (a power of two that puts the largest
// coefficient in [2^13, 2^14)).  A triangle outside the validated range (as
// sweep_plk's: |a_i| <= 2^20, e0/e1/n components 0 or in [2^-100, 2^20], max
// >= 2^-30; non-finite) gets all-zero coefficients, which always pass (the
// exact test decides); padding triangles get -tn = +2^13, which never passes
// in the forms that evaluate -tn.  The forms without it (MfmaSpec::no_tn:
// variants 231/233/243/252) let padding pairs through (U = V = X = 0, Y <= 0);
// their exact phase stops at idx >= n_tris before any triangle is read, so a
// padding slot is never tested (tests/test_gpu_mfma.py test_range_edges: 1, 37
// and 302 triangles, bit-exact on every variant).
// flags[0] += out-of-range triangles, flags[1] = max |a_i| (float bits).
// Shared by both record layouts (prep_mfma, prep_mfma_k16).
struct MfmaCoef {
    double c[kMfmaQ][10];  // quantity x ray slot (d.xyz, m.xyz, o.xyz, 1)
    double tau;
};
__device__ __forceinline__ void mfma_coefs(const float4* tri, int i, int n, MfmaCoef& k, uint32_t* flags) {
    for (int q = 0; q < kMfmaQ; q++)
        for (int c = 0; c < 10; c++) k.c[q][c] = 0.0;
    k.tau = 1.0;
    if (i >= n) {
        k.c[3][9] = 0x1p13;  // padding: -tn' = 2^13 sigma > T
        return;
    }
    const float4 t0 = tri[3 * i], t1 = tri[3 * i + 1], t2 = tri[3 * i + 2];
    const float a[3] = {t0.x, t0.y, t0.z}, e0[3] = {t0.w, t1.x, t1.y}, e1[3] = {t1.z, t1.w, t2.x},
                nn[3] = {t2.y, t2.z, t2.w};
    bool ok = true;
    float A = 0.0f, M = 0.0f;
    for (int j = 0; j < 3; j++) {
        ok = ok && fabsf(a[j]) <= 0x1p20f;
        A = fmaxf(A, fabsf(a[j]));
        for (float x : {e0[j], e1[j], nn[j]}) {
            const float ax = fabsf(x);
            ok = ok && (x == 0.0f || (ax >= 0x1p-100f && ax <= 0x1p20f));
            M = fmaxf(M, ax);
        }
    }
    ok = ok && M >= 0x1p-30f;
    if (!ok) {
        atomicAdd(&flags[0], 1u);
        return;
    }
    int ex;
    (void)frexpf(M, &ex);
    const double s = ldexp(1.0, 1 - ex);
    double E0[3], E1[3], N[3], P0[3], P1[3], A0[3];
    for (int j = 0; j < 3; j++) {
        E0[j] = s * e0[j];
        E1[j] = s * e1[j];
        N[j] = s * nn[j];
        A0[j] = a[j];
    }
    P0[0] = A0[1] * E0[2] - A0[2] * E0[1];
    P0[1] = A0[2] * E0[0] - A0[0] * E0[2];
    P0[2] = A0[0] * E0[1] - A0[1] * E0[0];
    P1[0] = A0[1] * E1[2] - A0[2] * E1[1];
    P1[1] = A0[2] * E1[0] - A0[0] * E1[2];
    P1[2] = A0[0] * E1[1] - A0[1] * E1[0];
    const double AN = A0[0] * N[0] + A0[1] * N[1] + A0[2] * N[2];
    for (int j = 0; j < 3; j++) {
        k.c[0][j] = -P1[j];                                // U: d
        k.c[0][3 + j] = E1[j];                             //    m
        k.c[1][j] = P0[j];                                 // -V: d
        k.c[1][3 + j] = -E0[j];                            //     m
        k.c[2][j] = P1[j] - P0[j] + (double)kMfmaC * N[j];  // X: d
        k.c[2][3 + j] = E0[j] - E1[j];                     //    m
        k.c[3][6 + j] = -N[j];                             // -tn: o
        k.c[4][j] = N[j];                                  // dn: d
    }
    k.c[3][9] = AN;  // -tn: 1
    double mx = 0.0;
    for (int q = 0; q < kMfmaQ; q++)
        for (int c = 0; c < 10; c++) mx = fmax(mx, fabs(k.c[q][c]));
    int e2;
    (void)frexp(mx, &e2);  // mx in [2^(e2-1), 2^e2)
    k.tau = ldexp(1.0, 14 - e2);
    atomicMax(&flags[1], __float_as_uint(A));
}

// The 32 k-slots of one quantity's record: coefficient c < 9 as (hi, hi, lo)
// against the ray's (hi, lo, hi) in slots 3c..3c+2 (hi*hi + hi*lo + lo*hi),
// the constant as (hi, lo) against (sigma, sigma) in slots 27, 28.
__device__ __forceinline__ void mfma_slots(const double* coef, double tau, _Float16 slot[32]) {
    for (int k = 0; k < 32; k++) slot[k] = (_Float16)0.0f;
    for (int c = 0; c < 10; c++) {
        const double v = coef[c] * tau;
        const _Float16 hi = (_Float16)(float)v;
        const _Float16 lo = (_Float16)(float)(v - (double)(float)hi);
        if (c < 9) {
            slot[3 * c] = hi;      // x hi * ray hi
            slot[3 * c + 1] = hi;  // x hi * ray lo
            slot[3 * c + 2] = lo;  // x lo * ray hi
        } else {
            slot[27] = hi;  // * sigma
            slot[28] = lo;  // * sigma
        }
    }
}

// Records in the v_mfma_f32_16x16x32_f16 B-operand order (one thread per
// padded triangle): [16-group][quantity][lane][8 f16] (5 KiB per 16 triangles).
__global__ void prep_mfma(const float4* tri, int n, int n_pad, _Float16* out, float* tau_out, uint32_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    MfmaCoef k;
    mfma_coefs(tri, i, n, k, flags);
    const int G = i >> 4, t = i & 15;
    for (int q = 0; q < kMfmaQ; q++) {
        _Float16 slot[32];
        mfma_slots(k.c[q], k.tau, slot);
        for (int s = 0; s < 32; s++) out[((size_t)(G * kMfmaQ + q) * 64 + 16 * (s >> 3) + t) * 8 + (s & 7)] = slot[s];
    }
    tau_out[i] = (float)k.tau;
}

__device__ __forceinline__ float wave_max(float x) {
    for (int off = 32; off > 0; off >>= 1) x = fmaxf(x, __shfl_xor(x, off));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
// The same maximum through DPP lane moves (no LDS crossbar round trips):
// quad swaps, half-row and row mirrors leave every lane of a 16-lane row with
// the row's maximum; row_bcast:15 / :31 fold rows 0-1 and 2-3 and then the
// halves into row 3, whose lane 63 is read.  Exact (a maximum of the same
// values in another order); x must not be NaN (the callers' values are
// finite, or range-checked before).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_max_step(float x) {
    // rows outside ROW_MASK keep `old` = x: max(x, x) = x
    const int y = __builtin_amdgcn_update_dpp(__float_as_int(x), __float_as_int(x), CTRL, ROW_MASK, 0xf, false);
    return fmaxf(x, __int_as_float(y));
}
__device__ __forceinline__ float wave_max_dpp(float x) {
    x = dpp_max_step<0xB1, 0xf>(x);   // quad_perm [1,0,3,2]
    x = dpp_max_step<0x4E, 0xf>(x);   // quad_perm [2,3,0,1]
    x = dpp_max_step<0x141, 0xf>(x);  // row_half_mirror
    x = dpp_max_step<0x140, 0xf>(x);  // row_mirror
    x = dpp_max_step<0x142, 0xa>(x);  // row_bcast:15 into rows 1, 3
    x = dpp_max_step<0x143, 0xc>(x);  // row_bcast:31 into rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
template <MfmaSpec S>
__device__ __forceinline__ float wave_max_s(float x) {
    if constexpr (S.dpp)
        return wave_max_dpp(x);
    else
        return wave_max(x);
}

__device__ __forceinline__ float abs_max3(const f3& v) { return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fabsf(v.z)); }

// Per-wave, per-segment scales of the matrix filter (shared by every sweep
// layout and by the filter probe): sigma puts the rays' largest |o|, |m| (and,
// ymma, |o + bk d| for every usable bound) in [2^13, 2^14); Tw = sigma * T
// with T = 2^-tshift (Omax + A + 1); Bmax = the largest usable distance bound.
// False (wave-uniform) when a ray is outside the filter's range: the caller
// sweeps with the scalar-path filter.
struct MfmaScale {
    float sigma, Tw, Bmax;
};
template <MfmaSpec S>
__device__ __forceinline__ bool mfma_scale(float mfma_A, const f3& o, const f3& d, const f3& m, MfmaScale& sc) {
    if (__ballot(!(abs_max3(o) <= 0x1p20f && abs_max3(d) <= 1.0001f))) return false;  // NaN fails too
    const float Omax = wave_max_s<S>(abs_max3(o));
    const float R0 = Omax + mfma_A + 1.0f;
    float mx = fmaxf(fmaxf(Omax, wave_max_s<S>(abs_max3(m))), 1.0f);
    if constexpr (S.ymma) mx = fmaxf(mx, __builtin_fmaf(2.25f, R0, Omax));  // |o + bk d| for every bk <= Bmax
    int ex;
    (void)frexpf(mx, &ex);
    sc.sigma = ldexpf(1.0f, 14 - ex);  // sigma * mx in [2^13, 2^14)
    sc.Tw = sc.sigma * (ldexpf(kMfmaTs, 10 - S.tshift) * R0);
    sc.Bmax = kMfmaB * R0;
    return true;
}

// This lane's ray vector (sigma-scaled d, m, o, 1) as the 32 f16 k-slots
// (hi, lo, hi per component against the records' hi, hi, lo), stored as four
// 16-byte pieces at `row`.
__device__ __forceinline__ void mfma_main_row(_Float16* row, const f3& d, const f3& m, const f3& o, float sigma) {
    const float comp[9] = {d.x, d.y, d.z, m.x, m.y, m.z, o.x, o.y, o.z};
    _Float16 s[32];
#pragma unroll
    for (int c = 0; c < 9; c++) {
        const float v = comp[c] * sigma;
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        s[3 * c] = hi;
        s[3 * c + 1] = lo;
        s[3 * c + 2] = hi;
    }
    s[27] = s[28] = (_Float16)sigma;
    s[29] = s[30] = s[31] = (_Float16)0.0f;
    h8* r = reinterpret_cast<h8*>(row);
#pragma unroll
    for (int k = 0; k < 4; k++)
        r[k] = h8{s[8 * k], s[8 * k + 1], s[8 * k + 2], s[8 * k + 3], s[8 * k + 4], s[8 * k + 5], s[8 * k + 6],
                  s[8 * k + 7]};
}

// mfma_main_row's first K-half only (slots 0..15: d, m.x, m.y, m.z hi), the
// whole main fragment the forms without -tn read (MfmaSpec::rows80)
__device__ __forceinline__ void mfma_main_half_slots(_Float16 s[18], const f3& d, const f3& m, float sigma) {
    const float comp[6] = {d.x, d.y, d.z, m.x, m.y, m.z};
#pragma unroll
    for (int c = 0; c < 6; c++) {
        const float v = comp[c] * sigma;
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        s[3 * c] = hi;
        s[3 * c + 1] = lo;
        s[3 * c + 2] = hi;
    }
}
__device__ __forceinline__ void mfma_main_row_half(_Float16* row, const f3& d, const f3& m, float sigma) {
    _Float16 s[18];
    mfma_main_half_slots(s, d, m, sigma);
    h8* r = reinterpret_cast<h8*>(row);
    r[0] = h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
    r[1] = h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]};
}

// The Y fragment's k-slots 16..31 for this lane's distance bound bkv: w = o +
// bkv d (bkv <= Bmax) with the constant slot -sigma, so that the -tn record
// gives Y = w.N - AN = s (tnum - bkv det); or, with no usable bound, w = Bmax d
// and constant 0: Y = -s Bmax det (the det > 0 test).  -w sigma as f16 hi/lo
// in the o slots (18..26, hi lo hi like the main fragment); slots 0..15 are 0.
__device__ __forceinline__ void mfma_y_chunk(_Float16 s[16], const f3& d, const f3& o, float bkv, float sigma,
                                             float Bmax) {
    const bool fin = bkv <= Bmax;
    const float wx = fin ? __builtin_fmaf(bkv, d.x, o.x) : Bmax * d.x;
    const float wy = fin ? __builtin_fmaf(bkv, d.y, o.y) : Bmax * d.y;
    const float wz = fin ? __builtin_fmaf(bkv, d.z, o.z) : Bmax * d.z;
    const float wc[3] = {wx, wy, wz};
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const float v = -wc[c] * sigma;
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        s[2 + 3 * c] = hi;
        s[3 + 3 * c] = lo;
        s[4 + 3 * c] = hi;
    }
    s[0] = s[1] = (_Float16)0.0f;  // slots 16, 17: m.z (zero here)
    s[11] = s[12] = (_Float16)(fin ? -sigma : 0.0f);
    s[13] = s[14] = s[15] = (_Float16)0.0f;
}

// Closest hit of every lane's ray (o, d) over the 16-triangle groups [G0, G1)
// (all of them by default); the whole wave calls it (lanes without a ray of
// their own carry a copy of a live one).  Returns false (nothing done) when a
// ray is outside the bound's range.
template <MfmaSpec S>
__device__ __forceinline__ bool sweep_mfma(const RenderParams& p, MfmaWaveLds& sh, const f3& o, const f3& d, float& best,
                                           int& bi, float& bestK, MfmaDiag& dg, int G0 = 0, int G1 = -1) {
    const int lane = (int)lane_id();
    const f3 m = cross(d, o);
    MfmaScale sc;
    if (!mfma_scale<S>(p.mfma_A, o, d, m, sc)) return false;
    const float sigma = sc.sigma, Tw = sc.Tw, Bmax = sc.Bmax;
    const float Cw = -kMfmaE * sigma;

    // this lane's ray vector (sigma-scaled d, m, o, 1) as f16 slots -> LDS row `lane`
    mfma_main_row(&sh.ray[lane][0], d, m, o, sigma);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    h8 ra[4];
#pragma unroll
    for (int R = 0; R < 4; R++) ra[R] = *reinterpret_cast<const h8*>(&sh.ray[16 * R + (lane & 15)][8 * (lane >> 4)]);
    f4v bk[4];
    h8 ya[4];  // ymma: the Y fragment (-w, -1) / (-Bmax d, 0), built in the same LDS rows
    // Y fragment of this lane's ray for its distance bound bkv (mfma_y_chunk),
    // built in the same LDS rows (slots 0..15 zero)
    auto build_y = [&](float bkv) {
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bkv, sigma, Bmax);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // every lane has read the rows' previous contents
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        h8* row = reinterpret_cast<h8*>(&sh.ray[lane][0]);
        row[0] = h8{};
        row[1] = h8{};
        row[2] = h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
        row[3] = h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]};
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int R = 0; R < 4; R++) ya[R] = *reinterpret_cast<const h8*>(&sh.ray[16 * R + (lane & 15)][8 * (lane >> 4)]);
    };
    if constexpr (S.ymma) {
        build_y(bestK);
    } else {
#pragma unroll
        for (int R = 0; R < 4; R++) bk[R] = f4v{__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
    }

    const h8* frag = reinterpret_cast<const h8*>(p.mfma_frag);
    const int ng = G1 < 0 ? (p.n_tris + 15) >> 4 : G1;
    h8 b0, b1, b2, b3, b4;
    float tau;
    // per-lane record pointers advanced in VGPRs (no per-group reload of the
    // spilled base addresses)
    const h8* fg = frag + (size_t)G0 * (kMfmaQ * 64) + lane;
    const float* tg = p.mfma_tau + 16 * G0 + (lane & 15);
    auto fetch = [&]() {
        b0 = fg[0], b1 = fg[64], b2 = fg[128], b3 = fg[192];
        if constexpr (!S.ymma) b4 = fg[256];
        tau = *tg;
        fg += kMfmaQ * 64;
        tg += 16;
    };
    if constexpr (S.prefetch) fetch();
    for (int G = G0; G < ng; G++) {
        if constexpr (!S.prefetch) fetch();
        const h8 c0 = b0, c1 = b1, c2 = b2, c3 = b3, c4 = S.ymma ? b3 : b4;
        const float ct = tau;
        if constexpr (S.prefetch)
            if (G + 1 < ng) fetch();  // in flight during this group's products
        const float Tl = ct * Tw;
        const float cd = ct * Cw;
        const f4v zero = {0.0f, 0.0f, 0.0f, 0.0f};
        const f4v cdn = {cd, cd, cd, cd};
        unsigned long long M = 0;
        int tmin = 0x7fffffff;  // minred: min over this lane's pairs of the max term
#pragma unroll
        for (int R = 0; R < 4; R++) {
            const f4v qU = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[R], c0, zero, 0, 0, 0);
            const f4v qV = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[R], c1, zero, 0, 0, 0);
            const f4v qX = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[R], c2, zero, 0, 0, 0);
            const f4v qT = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[R], c3, zero, 0, 0, 0);
            f4v qD;
            if constexpr (S.ymma)
                qD = __builtin_amdgcn_mfma_f32_16x16x32_f16(ya[R], c3, zero, 0, 0, 0);  // Y itself
            else
                qD = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra[R], c4, cdn, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const float Y = S.ymma ? qD[i] : __builtin_fmaf(bk[R][i], qD[i], -qT[i]);
                if constexpr (S.imax) {
                    // t <= Tl (Tl > 0) on the bit patterns as signed integers:
                    // negative floats are negative integers, positive floats
                    // order like their patterns, so max_int(terms) <= int(Tl)
                    // iff every term <= Tl.  A NaN term (Y = inf * 0 when
                    // qD = 0, i.e. det < 0, which the reference rejects) may
                    // pass or fail; no other term can be NaN (finite products).
                    const int t3 = max(max(__float_as_int(qU[i]), __float_as_int(qV[i])), __float_as_int(qX[i]));
                    const int t = max(max(t3, __float_as_int(qT[i])), __float_as_int(Y));  // two v_max3_i32
                    if constexpr (S.minred)
                        tmin = min(tmin, t);  // every pair of a lane is triangle 16G + (lane & 15)
                    else
                        M |= __ballot(t <= __float_as_int(Tl));
                } else {
                    const float t = fmaxf(fmaxf(fmaxf(qU[i], qV[i]), fmaxf(qX[i], qT[i])), Y);
                    M |= __ballot(t <= Tl);
                }
            }
        }
        if constexpr (S.minred) M = __ballot(tmin <= __float_as_int(Tl));
        if constexpr (S.diag) dg.groups += 1;
        if (M) {
            if constexpr (S.diag) dg.hot += 1;
            // triangles of the group with a passing pair: the exact phase, in index order
            uint32_t m16 = (uint32_t)((M | M >> 16 | M >> 32 | M >> 48) & 0xffffull);
            const float bk0 = bestK;
            while (m16) {
                const int t = __builtin_ctz(m16);
                m16 &= m16 - 1;
                const int idx = 16 * G + t;
                if (idx >= p.n_tris) break;
                if constexpr (S.diag) dg.exact += 1;
                cfloat* tp = (cfloat*)p.tri + 12 * idx;
                const MtQ q = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                if (mt_pass3(q, bestK)) mt_exact(q, idx, best, bi, bestK);
            }
            if constexpr (S.ymma) {
                if (__ballot(bestK != bk0)) build_y(bestK);
            } else if (__ballot(bestK != bk0)) {
                sh.bk[lane] = bestK <= Bmax ? bestK : __builtin_inff();
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int R = 0; R < 4; R++) bk[R] = *reinterpret_cast<const f4v*>(&sh.bk[16 * R + 4 * (lane >> 4)]);
            }
        }
    }
    return true;
}


// ---------------------------------------------------------------------------
// The k16 sweep (MfmaSpec::k16): the same filter on v_mfma_f32_32x32x16_f16.
// A 32x32 product with K = 16 yields 1,024 terms per 32 matrix cycles, twice
// the terms per cycle of the 16x16x32 form whenever a quantity fits 16 k-slots.
// The ray vector's 32 slots are two K-halves: [d (9), m.x m.y m.z-hi (7)] and
// [m.z lo/hi (2), o (9), constant (2), 0 (3)].  U, -V and X use d and m (18
// slots): two chained products each; -tn uses o and the constant (second half
// only) and Y the second half of its own fragment: one product each.  So a
// 32-ray x 32-triangle block takes 8 MFMAs — 256 matrix cycles and 64 cycles
// of MFMA issue on the VALU port per 1,024 pairs, against 320 and 160 for 20
// v_mfma_f32_16x16x32_f16 — and the same 2 v_max3_i32 + 1/2 v_min3 per pair.
// Operand maps (32x32x16, K = 16): lane l holds A[row l&31][k 8(l>>5)+j] and
// B[k 8(l>>5)+j][col l&31]; D: column l&31 in all 16 registers (rows
// 8(i>>2) + 4(l>>5) + (i&3)), so every term a lane holds belongs to triangle
// 32G + (l&31): min over them, one ballot, lanes l and l+32 share a triangle.
// Records: [32-group][op][lane][8 f16], ops U0 U1 V0 V1 X0 X1 T1 (7 KiB per 32
// triangles); tau per triangle.  The arithmetic of every product — the same
// f16 hi/lo slots, the same scales — is the 16x16x32 form's, so its error
// budget applies unchanged ("The matrix filter"); the probe
// (mfma_probe_kernel) measures both forms on the hardware.
constexpr int kK16Ops = 7;
typedef float f16v __attribute__((ext_vector_type(16)));

struct MfmaK16Lds {
    // slots 0..31: the main fragment; 32..47: the Y fragment's slots 16..31
    // (112-B rows: 16-B reads of 16 consecutive rows hit distinct banks)
    _Float16 ray[64][56];
};
// MfmaSpec::lane_lds: the path state a lane does not need during the sweep,
// field-major (one 256-B row per field: conflict-free)
constexpr int kLaneStash = 20;
struct MfmaK16LaneLds : MfmaK16Lds {
    uint32_t lane[kLaneStash][64];
};
__device__ __forceinline__ void lane_stash(const Lane& L, uint32_t (*st)[64], int l) {
    const uint32_t v[kLaneStash] = {(uint32_t)L.st, L.item, (uint32_t)L.x, (uint32_t)L.y, L.frame, L.seed,
                                    (uint32_t)L.ray, (uint32_t)L.bounce, (uint32_t)L.inside,
                                    __float_as_uint(L.rayColor.x), __float_as_uint(L.rayColor.y),
                                    __float_as_uint(L.rayColor.z), __float_as_uint(L.incoming.x),
                                    __float_as_uint(L.incoming.y), __float_as_uint(L.incoming.z),
                                    __float_as_uint(L.colorCum.x), __float_as_uint(L.colorCum.y),
                                    __float_as_uint(L.colorCum.z), L.segs, 0u};
#pragma unroll
    for (int f = 0; f < kLaneStash; f++) st[f][l] = v[f];
}
// ds_permute of a lane's whole path state to lane to/4 (push; a permutation)
__device__ __forceinline__ int perm_i(int to, int v) { return __builtin_amdgcn_ds_permute(to, v); }
__device__ __forceinline__ float perm_f(int to, float v) { return __int_as_float(__builtin_amdgcn_ds_permute(to, __float_as_int(v))); }
__device__ __forceinline__ f3 perm_f3(int to, const f3& v) { return mk(perm_f(to, v.x), perm_f(to, v.y), perm_f(to, v.z)); }
// XY = false: the caller does not keep x, y (advance<S, false>); SEGS = false:
// nor the per-lane segment count (MfmaSpec::lean)
template <bool XY = true, bool SEGS = true>
__device__ __forceinline__ void lane_permute(Lane& L, int to) {
    L.st = perm_i(to, L.st);
    L.item = (uint32_t)perm_i(to, (int)L.item);
    if constexpr (XY) {
        L.x = perm_i(to, L.x);
        L.y = perm_i(to, L.y);
    }
    L.frame = (uint32_t)perm_i(to, (int)L.frame);
    L.seed = (uint32_t)perm_i(to, (int)L.seed);
    L.ray = perm_i(to, L.ray);
    L.bounce = perm_i(to, L.bounce);
    L.inside = perm_i(to, (int)L.inside) != 0;
    L.o = perm_f3(to, L.o);
    L.d = perm_f3(to, L.d);
    L.rayColor = perm_f3(to, L.rayColor);
    L.incoming = perm_f3(to, L.incoming);
    L.colorCum = perm_f3(to, L.colorCum);
    if constexpr (SEGS) L.segs = (uint32_t)perm_i(to, (int)L.segs);
}
// lane_lds = 2: 15 words (st:3 inside:1 bounce:12 ray:16 | item | x:16 y:16 |
// frame | seed | colours | segs); the launcher uses it
// only when bounce <= 4095, rays per pixel <= 65535 and the image fits 16-bit
// coordinates
struct MfmaK16PackedLds {
    _Float16 ray[64][48];  // 96-B rows (two-way bank conflicts on the per-segment fragment reads)
    uint32_t lane[15][64];
};
// the same with 80-B rows (MfmaSpec::rows80, the forms without -tn): slots
// 0..15 the main fragment's first K-half, 16..31 the Y fragment's second half
struct MfmaK5nLds {
    _Float16 ray[64][40];
    uint32_t lane[15][64];
};
// ... without the path-state stash (the path state stays in VGPRs)
struct MfmaK5rLds {
    _Float16 ray[64][40];
};
__device__ __forceinline__ void lane_stash_packed(const Lane& L, uint32_t (*st)[64], int l) {
    const uint32_t v[15] = {(uint32_t)L.st | (uint32_t)L.inside << 3 | (uint32_t)L.bounce << 4 | (uint32_t)L.ray << 16,
                            L.item, (uint32_t)L.x | (uint32_t)L.y << 16, L.frame, L.seed,
                            __float_as_uint(L.rayColor.x), __float_as_uint(L.rayColor.y),
                            __float_as_uint(L.rayColor.z), __float_as_uint(L.incoming.x),
                            __float_as_uint(L.incoming.y), __float_as_uint(L.incoming.z),
                            __float_as_uint(L.colorCum.x), __float_as_uint(L.colorCum.y),
                            __float_as_uint(L.colorCum.z), L.segs};
#pragma unroll
    for (int f = 0; f < 15; f++) st[f][l] = v[f];
}
__device__ __forceinline__ void lane_unstash_packed(Lane& L, const uint32_t (*st)[64], int l) {
    const uint32_t w = st[0][l], xy = st[2][l];
    L.st = (int)(w & 7u);
    L.inside = ((w >> 3) & 1u) != 0;
    L.bounce = (int)((w >> 4) & 0xfffu);
    L.ray = (int)(w >> 16);
    L.item = st[1][l];
    L.x = (int)(xy & 0xffffu);
    L.y = (int)(xy >> 16);
    L.frame = st[3][l];
    L.seed = st[4][l];
    L.rayColor = mk(__uint_as_float(st[5][l]), __uint_as_float(st[6][l]), __uint_as_float(st[7][l]));
    L.incoming = mk(__uint_as_float(st[8][l]), __uint_as_float(st[9][l]), __uint_as_float(st[10][l]));
    L.colorCum = mk(__uint_as_float(st[11][l]), __uint_as_float(st[12][l]), __uint_as_float(st[13][l]));
    L.segs = st[14][l];
}
__device__ __forceinline__ void lane_unstash(Lane& L, const uint32_t (*st)[64], int l) {
    L.st = (int)st[0][l];
    L.item = st[1][l];
    L.x = (int)st[2][l];
    L.y = (int)st[3][l];
    L.frame = st[4][l];
    L.seed = st[5][l];
    L.ray = (int)st[6][l];
    L.bounce = (int)st[7][l];
    L.inside = st[8][l] != 0;
    L.rayColor = mk(__uint_as_float(st[9][l]), __uint_as_float(st[10][l]), __uint_as_float(st[11][l]));
    L.incoming = mk(__uint_as_float(st[12][l]), __uint_as_float(st[13][l]), __uint_as_float(st[14][l]));
    L.colorCum = mk(__uint_as_float(st[15][l]), __uint_as_float(st[16][l]), __uint_as_float(st[17][l]));
    L.segs = st[18][l];
}

// bnd_out (the 5-product form, MfmaSpec::k5): per triangle, the largest
// |slot 16| and |slot 17| over U, -V, X — the m.z products hi x ray-lo and
// lo x ray-hi that the form leaves out (sweep_k16 adds their bound to the
// threshold)
__global__ void prep_mfma_k16(const float4* tri, int n, int n_pad, _Float16* out, float* tau_out, float2* bnd_out,
                              uint32_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    MfmaCoef k;
    mfma_coefs(tri, i, n, k, flags);
    const int G = i >> 5, t = i & 31;
    float ch = 0.0f, cl = 0.0f;
    for (int op = 0; op < kK16Ops; op++) {
        const int q = op < 6 ? op >> 1 : 3, h = op < 6 ? (op & 1) : 1;
        _Float16 slot[32];
        mfma_slots(k.c[q], k.tau, slot);
        if (op == 6) {
            // the threshold slots 29..31 of the -tn record (zero in every ray
            // fragment but mfma_thr_frag): -tau, -CH, -CL, all exact in f16
            // (tau a power of two in [2^-9, 2^13]; CH, CL f16 magnitudes)
            slot[29] = (_Float16)(float)-k.tau;
            slot[30] = (_Float16)-ch;
            slot[31] = (_Float16)-cl;
        }
        for (int j = 0; j < 16; j++)
            out[((size_t)(G * kK16Ops + op) * 64 + t + 32 * (j >> 3)) * 8 + (j & 7)] = slot[16 * h + j];
        if (op < 6) {
            ch = fmaxf(ch, fabsf((float)slot[16]));
            cl = fmaxf(cl, fabsf((float)slot[17]));
        }
    }
    tau_out[i] = (float)k.tau;
    if (bnd_out) bnd_out[i] = make_float2(ch, cl);
}

// f16 of v > 0 rounded up (the threshold may only grow)
__device__ __forceinline__ _Float16 f16_up(float v) {
    _Float16 h = (_Float16)v;
    if ((float)h < v) h = __builtin_bit_cast(_Float16, (uint16_t)(__builtin_bit_cast(uint16_t, h) + 1u));
    return h;
}
// MfmaSpec::cthr: the A fragment whose product with the -tn record's second
// K-half is -Tl'' in every row, Tl'' = tau Tw + CH ML + CL MH with the wave's
// factors padded by 2^-8 and rounded up to f16 (slots 29..31 against the
// record's -tau, -CH, -CL; every other slot 0).  The three products are exact
// in f32 and of one sign, so the sum's rounding (2^-23) is inside the pad:
// Tl'' > Tl' = tau Tw + (CH ML + CL MH)(1 + 2^-10), sweep_k16's threshold.
// Added as the accumulator operand, it turns "term <= Tl'" into "term' < 0";
// DESIGN.md, "The threshold in the accumulator".  The factors are wave-uniform
// and kept as two scalar words (elements 4, 5 = 0, Tw; 6, 7 = ML, MH of the
// upper lanes' 8 slots); the fragment is rebuilt from them every group (two
// v_cndmask), so its 4 VGPRs are not live across the sweep.
struct ThrBits {
    uint32_t w2, w3;
};
__device__ __forceinline__ ThrBits mfma_thr_bits(float Tw, float zlo, float zhi) {
    constexpr float pad = 1.00390625f;  // 1 + 2^-8
    const uint32_t t = __builtin_bit_cast(uint16_t, f16_up(Tw * pad));
    const uint32_t a = __builtin_bit_cast(uint16_t, f16_up(zlo * pad));
    const uint32_t b = __builtin_bit_cast(uint16_t, f16_up(zhi * pad));
    return ThrBits{(uint32_t)__builtin_amdgcn_readfirstlane(t << 16), (uint32_t)__builtin_amdgcn_readfirstlane(a | b << 16)};
}
__device__ __forceinline__ h8 mfma_thr_frag(ThrBits tb) {
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    const bool up = lane_id() >= 32;  // slots 8..15 of the K-half: 29, 30, 31 are elements 5, 6, 7
    // opaque() outside the selects: an asm value inside a ?: compiled to two
    // exec-masked branches per group instead of two v_cndmask
    const uint32_t w2 = opaque(tb.w2), w3 = opaque(tb.w3);
    const u4 v = {0u, 0u, up ? w2 : 0u, up ? w3 : 0u};
    return __builtin_bit_cast(h8, v);
}

// MfmaSpec::perm_frag / render_mfma_k5r: the MFMA A-operand fragments of both 32-ray blocks from each lane's own 16
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

// The five terms of 32 rays (fragments a0/a1 = the main fragment's two
// K-halves, y1 = the Y fragment's second half) x 32 triangles (records b[7]).
struct K16Terms {
    f16v U, V, X, T, Y;
};
__device__ __forceinline__ K16Terms k16_terms(const h8& a0, const h8& a1, const h8& y1, const h8* b) {
    const f16v zero = {};
    K16Terms r;
    r.U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[0], zero, 0, 0, 0);
    r.V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[2], zero, 0, 0, 0);
    r.X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[4], zero, 0, 0, 0);
    r.U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b[1], r.U, 0, 0, 0);
    r.V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b[3], r.V, 0, 0, 0);
    r.X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b[5], r.X, 0, 0, 0);
    r.T = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, b[6], zero, 0, 0, 0);
    r.Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1, b[6], zero, 0, 0, 0);
    return r;
}

// MfmaSpec::cthr: one group's filter for the wave's one or two 32-ray blocks.
// TT = -Tl'' in every row (mfma_thr_frag x the -tn record); each term is
// computed as its sum plus TT, so a pair passes iff all four shifted terms
// are negative: the sign bit of U & V & X & Y (two v_bitop3_b32), ORed over
// the lane's 16 pairs (all one triangle).  The accumulation error of the 17
// summands is inside the 31 x 2^-24 budget of the 30-product form.
// MfmaSpec::ylds: a block's fragments are read from the wave's LDS rows right
// before its products (no fragment live across the group: 4-wave budget).
template <MfmaSpec S, class SH>
__device__ __forceinline__ unsigned long long k5_cthr_group(ThrBits tb, const h8* a0, const h8* y1, const h8& b0,
                                                            const h8& b2, const h8& b4, const h8& b6, bool upper,
                                                            const SH& sh, const h8& tfh = h8{}) {
    static_assert(S.k5 && S.no_tn && S.sol == 0, "the 4-product form");
    [[maybe_unused]] constexpr int YO = S.rows80 ? 16 : 32;
    [[maybe_unused]] const int r32 = (int)lane_id() & 31, hl = (int)lane_id() >> 5;
    const f16v zero = {};
    const f16v TT = __builtin_amdgcn_mfma_f32_32x32x16_f16(S.thr_hoist ? tfh : mfma_thr_frag(tb), b6, zero, 0, 0, 0);
    int acc = 0;
#pragma unroll
    for (int R = 0; R < 2; R++) {
        if (R == 1 && !upper) break;
        h8 aR;
        if constexpr (S.ylds == 2)
            aR = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][8 * hl]);
        else
            aR = a0[R];
        const f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(aR, b0, TT, 0, 0, 0);
        const f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(aR, b2, TT, 0, 0, 0);
        const f16v X = __builtin_amdgcn_mfma_f32_32x32x16_f16(aR, b4, TT, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        int t3[16];
#pragma unroll
        for (int i = 0; i < 16; i++)  // U & V & X (LUT index 4 S0 + 2 S1 + S2)
            t3[i] = __builtin_amdgcn_bitop3_b32(__float_as_int(U[i]), __float_as_int(V[i]), __float_as_int(X[i]), 0x80);
        __builtin_amdgcn_sched_barrier(0);
        h8 yR;
        if constexpr (S.ylds != 0)
            yR = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][YO + 8 * hl]);
        else
            yR = y1[R];
        const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(yR, b6, TT, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 16; i++)  // (t3 & Y) | acc: one chain, no OR tree (which costs 0.5 more per pair)
            acc = __builtin_amdgcn_bitop3_b32(t3[i], __float_as_int(Y[i]), acc, 0xEA);
        if (R == 1) __builtin_amdgcn_sched_barrier(0);
    }
    return __ballot(acc < 0);
}

// ---------------------------------------------------------------------------
// MfmaSpec::kthr — the threshold in the K-slots (round 6; DESIGN.md "The
// threshold in the K-slots").  The cthr form spends a tenth matrix product per
// group on TT = -Tl'' and holds its 16 VGPRs live as the accumulator operand of
// every other product, which also chains U, -V, X and Y behind it.  Here the
// threshold is two more k-slots of the products themselves:
//   - U, -V, X keep d (9 slots), m.x (3) and the hi x hi products of m.y and
//     m.z; the four cross slots of m.y and m.z (coefficient hi x ray lo,
//     coefficient lo x ray hi) are left out and bounded, per component c, by
//     2^-10 CT_c mw_c with CT_c = max(|c_hi|, 2^11 |c_lo|) (triangle) and
//     mw_c = max(|r_hi|, 2^11 |r_lo|) (ray): |c_hi r_lo| <= CT 2^-11 mw and
//     |c_lo r_hi| <= 2^-11 CT mw.  Summed over y and z, <= B_q W with
//     B_q = 2^-10 max(CT_y, CT_z) of the quantity's own coefficients and
//     W = max over the wave of (mw_y + mw_z);
//   - slot 14 carries -tau against Tw' = Tw (1 + 2^-8) rounded up to f16, and
//     slot 15 -B_q (rounded up in magnitude) against W' = W (1 + 2^-8) rounded
//     up, so each product comes out as its kept sum minus (tau Tw' + B_q W');
//   - Y's fragment carries Tw' in slot 29 against the -tn record's -tau.
// A pair passes iff all four terms are negative (the sign-bit AND of the cthr
// form); the 8 products per group take a zero accumulator and are independent.
// Records: [32-group][4: U, -V, X (first K-half), T1 (-tn second half)][64][8].
constexpr int kKtOps = 4;
__global__ void prep_mfma_kt(const float4* tri, int n, int n_pad, _Float16* out, uint32_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    MfmaCoef k;
    mfma_coefs(tri, i, n, k, flags);
    const int G = i >> 5, t = i & 31;
    for (int op = 0; op < kKtOps; op++) {
        _Float16 slot[32], h[16];
        if (op < 3) {
            mfma_slots(k.c[op], k.tau, slot);
            // slots 12, 13, 14: m.y (hi, hi, lo); 15, 16, 17: m.z (hi, hi, lo)
            const float ct = fmaxf(fmaxf(fabsf((float)slot[12]), 2048.0f * fabsf((float)slot[14])),
                                   fmaxf(fabsf((float)slot[15]), 2048.0f * fabsf((float)slot[17])));
            for (int j = 0; j < 13; j++) h[j] = slot[j];  // d (0..8), m.x (9..11), m.y hi x hi (12)
            h[13] = slot[15];                             // m.z hi x hi
            h[14] = (_Float16)(float)-k.tau;              // a power of two in [2^-9, 2^13]: exact
            h[15] = -f16_up(ct * 0x1p-10f);               // B_q, rounded up in magnitude
        } else {
            mfma_slots(k.c[3], k.tau, slot);
            for (int j = 0; j < 16; j++) h[j] = slot[16 + j];  // o (18..26), the constant (27, 28)
            h[13] = (_Float16)(float)-k.tau;                    // slot 29 against Y's Tw'
            h[14] = h[15] = (_Float16)0.0f;
        }
        for (int j = 0; j < 16; j++) out[((size_t)(G * kKtOps + op) * 64 + t + 32 * (j >> 3)) * 8 + (j & 7)] = h[j];
    }
}

// This lane's first K-half of the kthr main fragment: d and m.x as (hi, lo,
// hi), m.y hi, m.z hi; slots 14, 15 (Tw', W') are wave-uniform and filled by
// the caller.  Returns the lane's mw_y + mw_z.
__device__ __forceinline__ float kt_main_slots(_Float16 s[16], const f3& d, const f3& m, float sigma) {
    const float comp[4] = {d.x, d.y, d.z, m.x};
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const float v = comp[c] * sigma;
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        s[3 * c] = hi;
        s[3 * c + 1] = lo;
        s[3 * c + 2] = hi;
    }
    float W = 0.0f;
    const float yz[2] = {m.y, m.z};
#pragma unroll
    for (int c = 0; c < 2; c++) {
        const float v = yz[c] * sigma;
        const _Float16 hi = (_Float16)v;
        const _Float16 lo = (_Float16)(v - (float)hi);
        s[12 + c] = hi;
        W += fmaxf(fabsf((float)hi), 2048.0f * fabsf((float)lo));
    }
    return W;
}

// The wave's kthr fragments: a0 (both 32-ray blocks' first K-half with the
// threshold factors) and y1 via frag_pair; tw16 keeps Tw' for the Y rebuilds.
template <MfmaSpec S>
__device__ __forceinline__ void kt_frags(const f3& d, const f3& m, const MfmaScale& sc, h8 a0[2], _Float16& tw16) {
    constexpr float pad = 1.00390625f;  // 1 + 2^-8 (the f32 sum mw_y + mw_z and the scale product round)
    _Float16 s[16];
    // MfmaSpec::kt_lane_w: each ray's fragment carries its own mw_y + mw_z
    // (the bound is per (ray, triangle) product: no wave maximum needed)
    const float Wl = kt_main_slots(s, d, m, sc.sigma);
    const float W = S.kt_lane_w ? Wl : wave_max_s<S>(Wl);
    tw16 = f16_up(sc.Tw * pad);
    s[14] = tw16;
    s[15] = f16_up(W * pad);
    frag_pair(s, a0);
}
__device__ __forceinline__ void kt_y(const f3& d, const f3& o, float bkv, const MfmaScale& sc, _Float16 tw16,
                                     h8 y1[2]) {
    _Float16 s[16];
    mfma_y_chunk(s, d, o, bkv, sc.sigma, sc.Bmax);
    s[13] = tw16;  // slot 29: Tw' against the record's -tau
    frag_pair(s, y1);
}

// One group's filter for the wave's one or two 32-ray blocks (records bu, bv,
// bx: U, -V, X; bt: the -tn record's second K-half).  Returns the ballot of
// lanes whose triangle has a passing pair.
template <MfmaSpec S>
__device__ __forceinline__ unsigned long long kt_group(const h8* a0, const h8* y1, const h8& bu, const h8& bv,
                                                       const h8& bx, const h8& bt, bool upper) {
    static_assert(S.kthr >= 1 && S.kthr <= 5, "kthr schedule");
    const f16v zero = {};
    int acc = 0;
    if constexpr (S.kthr == 4 || S.kthr == 5) {
        // kthr 4: the two blocks interleaved so that each wave's own products
        // run beside its own reduction VALU, at cthr's register peak (48
        // product VGPRs): [U0 V0 X0] [AND0] [Y0 U1] [fold0] [V1 X1] [AND1]
        // [Y1] [fold1] (scheduling groups; one basic block per form)
        auto andv = [](const f16v& U, const f16v& V, const f16v& X, int* t3) {
#pragma unroll
            for (int i = 0; i < 16; i++)
                t3[i] = __builtin_amdgcn_bitop3_b32(__float_as_int(U[i]), __float_as_int(V[i]), __float_as_int(X[i]), 0x80);
        };
        // kthr 5: the fold as two interleaved chains (even / odd pairs), ORed
        // at the group's end: half the dependent-VALU latency, one VALU more
        int acc2 = 0;
        auto fold = [&](const int* t3, const f16v& Y, int a) {
            if constexpr (S.kthr == 5) {
#pragma unroll
                for (int i = 0; i < 16; i += 2) {
                    a = __builtin_amdgcn_bitop3_b32(t3[i], __float_as_int(Y[i]), a, 0xEA);
                    acc2 = __builtin_amdgcn_bitop3_b32(t3[i + 1], __float_as_int(Y[i + 1]), acc2, 0xEA);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 16; i++) a = __builtin_amdgcn_bitop3_b32(t3[i], __float_as_int(Y[i]), a, 0xEA);
            }
            return a;
        };
        if (upper) {
            int t0[16], t1[16];
            const f16v U0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bu, zero, 0, 0, 0);
            const f16v V0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bv, zero, 0, 0, 0);
            const f16v X0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bx, zero, 0, 0, 0);
            andv(U0, V0, X0, t0);
            const f16v Y0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[0], bt, zero, 0, 0, 0);
            const f16v U1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[1], bu, zero, 0, 0, 0);
            acc = fold(t0, Y0, acc);
            const f16v V1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[1], bv, zero, 0, 0, 0);
            const f16v X1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[1], bx, zero, 0, 0, 0);
            andv(U1, V1, X1, t1);
            const f16v Y1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[1], bt, zero, 0, 0, 0);
            acc = fold(t1, Y1, acc);
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
        } else {
            int t0[16];
            const f16v U0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bu, zero, 0, 0, 0);
            const f16v V0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bv, zero, 0, 0, 0);
            const f16v X0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[0], bx, zero, 0, 0, 0);
            andv(U0, V0, X0, t0);
            const f16v Y0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[0], bt, zero, 0, 0, 0);
            acc = fold(t0, Y0, acc);
        }
        if constexpr (S.kthr == 5) acc |= acc2;
        return __ballot(acc < 0);
    }
#pragma unroll
    for (int R = 0; R < 2; R++) {
        if (R == 1 && !upper) break;
        const f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], bu, zero, 0, 0, 0);
        const f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], bv, zero, 0, 0, 0);
        const f16v X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], bx, zero, 0, 0, 0);
        if constexpr (S.kthr == 1) {
            // the four products first, then the 32 sign-bit VALU (scheduling
            // groups: a plain sched_barrier between them does not hold, the
            // products are pure and the DAG places Y after the AND)
            const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], bt, zero, 0, 0, 0);
            int t3[16];
#pragma unroll
            for (int i = 0; i < 16; i++)
                t3[i] = __builtin_amdgcn_bitop3_b32(__float_as_int(U[i]), __float_as_int(V[i]), __float_as_int(X[i]), 0x80);
#pragma unroll
            for (int i = 0; i < 16; i++) acc = __builtin_amdgcn_bitop3_b32(t3[i], __float_as_int(Y[i]), acc, 0xEA);
            __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 32, 0);  // VALU
            __builtin_amdgcn_sched_barrier(0);
        } else {
            if constexpr (S.kthr == 2) __builtin_amdgcn_sched_barrier(0);
            int t3[16];
#pragma unroll
            for (int i = 0; i < 16; i++)
                t3[i] = __builtin_amdgcn_bitop3_b32(__float_as_int(U[i]), __float_as_int(V[i]), __float_as_int(X[i]), 0x80);
            if constexpr (S.kthr == 2) __builtin_amdgcn_sched_barrier(0);
            const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], bt, zero, 0, 0, 0);
            if constexpr (S.kthr == 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; i++) acc = __builtin_amdgcn_bitop3_b32(t3[i], __float_as_int(Y[i]), acc, 0xEA);
            if constexpr (S.kthr == 2)
                if (R == 1) __builtin_amdgcn_sched_barrier(0);
        }
    }
    return __ballot(acc < 0);
}

__device__ __forceinline__ f16v Y_unused_init() { return f16v{}; }
template <MfmaSpec S, class SH>
__device__ __forceinline__ bool sweep_k16(const RenderParams& p, SH& sh, const f3& o, const f3& d, float& best,
                                          int& bi, float& bestK, MfmaDiag& dg, bool upper = true, int G0 = 0,
                                          int G1 = -1) {
    // [G0, G1): the 32-triangle groups to sweep (all of them by default; a
    // range when several waves split one block's sweep: render_mfma_pool)
    // upper = false: lanes 32..63 carry no ray of their own (MfmaSpec::compact moved the live rays to the
    // low half), so the second 32-ray block's products and reduction are skipped
    static_assert(S.ymma && S.imax && S.minred, "the k16 sweep implements the ymma / imax / minred form");
    static_assert(!S.k5 || (!S.prefetch && !S.lateload && !S.afrag_lds && (S.serial == 1 || S.serial == 3 || S.serial == 4)),
                  "the 5-product form is built on the serialised sweep");
    const int lane = (int)lane_id();
    const int r32 = lane & 31, hl = lane >> 5;
    const f3 m = cross(d, o);
    MfmaScale sc;
    if (!mfma_scale<S>(p.mfma_A, o, d, m, sc)) return false;
    static_assert(!S.rows80 || (S.k5 && S.no_tn), "80-B rows hold the first K-half of the main fragment only");
    constexpr int YO = S.rows80 ? 16 : 32;  // the Y slots' offset in a row
    if constexpr (S.rows80)
        mfma_main_row_half(&sh.ray[lane][0], d, m, sc.sigma);
    else
        mfma_main_row(&sh.ray[lane][0], d, m, o, sc.sigma);
    // k5: the wave's largest |ray lo| and |ray hi| of m.z (slots 16 and 17 of
    // the main fragment, the same arithmetic as mfma_main_row): with the
    // records' per-triangle |hi|, |lo| of the m.z coefficients they bound the
    // two products the 5-product form leaves out of U, -V and X
    [[maybe_unused]] float zlo = 0.0f, zhi = 0.0f;
    if constexpr (S.k5) {
        const float vz = m.z * sc.sigma;
        const _Float16 hz = (_Float16)vz;
        const _Float16 lz = (_Float16)(vz - (float)hz);
        zhi = wave_max_s<S>(fabsf((float)hz));
        zlo = wave_max_s<S>(fabsf((float)lz));
    }
    auto write_y = [&](float bkv) {
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bkv, sc.sigma, sc.Bmax);
        h8* row = reinterpret_cast<h8*>(&sh.ray[lane][YO]);
        row[0] = h8{s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]};
        row[1] = h8{s[8], s[9], s[10], s[11], s[12], s[13], s[14], s[15]};
    };
    write_y(bestK);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    h8 a0[2], a1[2], y1[2];
    auto read_a = [&]() {
#pragma unroll
        for (int R = 0; R < 2; R++) {
            a0[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][8 * hl]);
            if constexpr (!S.rows80) a1[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][16 + 8 * hl]);
        }
    };
    auto read_y = [&]() {
#pragma unroll
        for (int R = 0; R < 2; R++) y1[R] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][YO + 8 * hl]);
    };
    if constexpr (!S.afrag_lds && S.ylds < 2) read_a();
    if constexpr (!S.ylds) read_y();
    [[maybe_unused]] ThrBits thr = {};
    if constexpr (S.cthr) thr = mfma_thr_bits(sc.Tw, zlo, zhi);

    const int ng = G1 < 0 ? (p.n_tris + 31) >> 5 : G1;
    const h8* fg = reinterpret_cast<const h8*>(p.mfma_k16_frag) + (size_t)G0 * (kK16Ops * 64) + lane;
    const float* tg = p.mfma_k16_tau + 32 * G0 + r32;
    h8 b[kK16Ops], nb[kK16Ops];
    float tau = 0.0f, ntau = 0.0f;
    [[maybe_unused]] float2 bnd = make_float2(0.0f, 0.0f);
    [[maybe_unused]] const float2* bg = p.mfma_k16_bnd + 32 * G0 + r32;
    auto fetch = [&](h8* dst, float& t) {
#pragma unroll
        for (int op = 0; op < kK16Ops; op++)
            if (!S.k5 || !(op & 1) || op == 6) dst[op] = fg[64 * op];  // k5: the second K-halves of U V X unused
        if constexpr (!S.cthr) {  // cthr: the -tn record carries the threshold
            t = *tg;
            if constexpr (S.k5) {
                bnd = *bg;
                bg += 32;
            }
        }
        fg += kK16Ops * 64;
        tg += 32;
    };
    if constexpr (S.prefetch) fetch(nb, ntau);
    if constexpr (S.lateload) fetch(b, tau);
    for (int G = G0; G < ng; G++) {
        if constexpr (S.lateload) {
            // b, tau arrived during the previous group (requested right after
            // its last product was issued)
        } else if constexpr (S.prefetch) {
            // this group's records arrived during the previous group's
            // products; the next group's are requested before this group's
#pragma unroll
            for (int op = 0; op < kK16Ops; op++) b[op] = nb[op];
            tau = ntau;
            if (G + 1 < ng) fetch(nb, ntau);
        } else if constexpr (S.sol == 1) {
            if (G == 0) fetch(b, tau);
        } else {
            fetch(b, tau);
        }
        if constexpr (S.afrag_lds) read_a();
        unsigned long long M;
        if constexpr (S.cthr) {
            M = k5_cthr_group<S>(thr, a0, y1, b[0], b[2], b[4], b[6], upper, sh);
        } else {
        float Tl = tau * sc.Tw;
        // k5: + |c_hi| max|ray lo| + |c_lo| max|ray hi| of the left-out m.z
        // slots, padded by 2^-10 for its own rounding ("The
        // 5-product form")
        if constexpr (S.k5) Tl += (bnd.x * zlo + bnd.y * zhi) * 1.0009765625f;
        int tmin = 0x7fffffff;
        [[maybe_unused]] int u3[16], tmin6 = 0;
        [[maybe_unused]] f16v ex = {};
        if constexpr (S.sol == 7) ex[0] = p.mfma_A * 0.0f;
#pragma unroll
        for (int R = 0; R < 2; R++) {
            if (R == 1 && !upper) break;
            if constexpr (S.serial == 1 || S.serial == 3 || S.serial == 4) {
                const f16v zero = {};
                f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[0], zero, 0, 0, 0);
                f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[2], zero, 0, 0, 0);
                f16v X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[4], zero, 0, 0, 0);
                if constexpr (!S.k5) {
                    U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[1], U, 0, 0, 0);
                    V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[3], V, 0, 0, 0);
                    X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[5], X, 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                int t3[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    t3[i] = max(max(__float_as_int(U[i]), __float_as_int(V[i])), __float_as_int(X[i]));
                if constexpr (S.sol == 6) {
                    // marginal-cost probe: the reduction's VALU once more (min/max swapped: no CSE)
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        u3[i] = min(min(__float_as_int(U[i]), __float_as_int(V[i])), __float_as_int(X[i]));
                }
                __builtin_amdgcn_sched_barrier(0);
                f16v T = Y_unused_init();
                if constexpr (!S.no_tn) T = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[6], zero, 0, 0, 0);
                const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], b[6], zero, 0, 0, 0);
                if constexpr (S.sol == 7) {
                    // marginal-cost probe: the block's 8 products once more, one chain (sunk per group)
#pragma unroll
                    for (int k = 0; k < 8; k++)
                        ex = __builtin_amdgcn_mfma_f32_32x32x16_f16(k < 3 ? a0[R] : a1[R], b[k < 7 ? k : 6], ex, 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                if constexpr (S.lateload) {
                    // the group's last product is issued: its operand registers
                    // take the next group's records, whose latency the rest of
                    // this group (reduction, ballot, exact phase) covers
                    if (R == 1 || !upper) {
                        if (G + 1 < ng) fetch(b, tau);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                }
#pragma unroll
                for (int i = 0; i < 16; i++) {
                    if constexpr (S.no_tn)
                        tmin = min(tmin, max(t3[i], __float_as_int(Y[i])));
                    else
                        tmin = min(tmin, max(max(t3[i], __float_as_int(T[i])), __float_as_int(Y[i])));
                }
                if constexpr (S.sol == 6) {
#pragma unroll
                    for (int i = 0; i < 16; i++)
                        tmin6 = max(tmin6, min(min(u3[i], __float_as_int(T[i])), __float_as_int(Y[i])));
                }
                // serial 3: block R's last reduction may overlap block R+1's products;
                // serial 4: and the next group's record loads may move up
                if constexpr (S.serial == 1) __builtin_amdgcn_sched_barrier(0);
                if constexpr (S.serial == 3) {
                    if (R == 1) __builtin_amdgcn_sched_barrier(0);
                }
                continue;
            }
            const K16Terms q = k16_terms(a0[R], a1[R], y1[R], b);
            if constexpr (S.serial == 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                // max of the five terms on their bit patterns (see sweep_mfma)
                if constexpr (S.sol == 3) {
                    tmin = min(tmin, __float_as_int(q.U[i]));
                } else {
                    const int t3 = max(max(__float_as_int(q.U[i]), __float_as_int(q.V[i])), __float_as_int(q.X[i]));
                    const int t = max(max(t3, __float_as_int(q.T[i])), __float_as_int(q.Y[i]));
                    tmin = min(tmin, t);
                }
            }
            if constexpr (S.rsplit || S.serial == 2) __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (S.sol == 5) {
            // marginal-cost probe: the products and the reduction once more (a
            // runtime-zero accumulator keeps the compiler from reusing them)
            f16v ez = {};
            ez[0] = p.mfma_A * 0.0f;
            int tmin2 = 0x7fffffff;
#pragma unroll
            for (int R = 0; R < 2; R++) {
                f16v U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[0], ez, 0, 0, 0);
                f16v V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[2], ez, 0, 0, 0);
                f16v X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[4], ez, 0, 0, 0);
                U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[1], U, 0, 0, 0);
                V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[3], V, 0, 0, 0);
                X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[5], X, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                int t3[16];
#pragma unroll
                for (int i = 0; i < 16; i++)
                    t3[i] = max(max(__float_as_int(U[i]), __float_as_int(V[i])), __float_as_int(X[i]));
                __builtin_amdgcn_sched_barrier(0);
                const f16v T = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1[R], b[6], ez, 0, 0, 0);
                const f16v Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], b[6], ez, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int i = 0; i < 16; i++)
                    tmin2 = min(tmin2, max(max(t3[i], __float_as_int(T[i])), __float_as_int(Y[i])));
                __builtin_amdgcn_sched_barrier(0);
            }
            if (tmin2 == 0x12345677) best = -best;  // never (a sink)
        }
        if constexpr (S.sol == 6)
            if (tmin6 == 0x12345677) best = -best;  // never (a sink)
        if constexpr (S.sol == 7)
            if (ex[0] == 1.2345e-30f) best = -best;  // never (a sink)
        M = (S.sol == 2 || S.sol == 3) ? (unsigned long long)(tmin == 0x7ffffffe)
                                       : __ballot(tmin <= __float_as_int(Tl));
        }
        if constexpr (S.diag) dg.groups += 1;
        if (M) {
            if constexpr (S.diag) dg.hot += 1;
            // triangles of the group with a passing pair: the exact phase, in index order
            uint32_t m32 = (uint32_t)(M | M >> 32);
            const float bk0 = bestK;
            if constexpr (S.sol == 4) {
                // marginal-cost probe: the exact phase once more, on copies
                uint32_t mm = m32;
                float best2 = best, bestK2 = bestK;
                int bi2 = bi;
                while (mm) {
                    const int t = __builtin_ctz(mm);
                    mm &= mm - 1;
                    const int idx = 32 * G + t;
                    if (idx >= p.n_tris) break;
                    cfloat* tp = (cfloat*)p.tri + 12 * idx;
                    const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                    if (mt_pass3(qq, bestK2)) mt_exact(qq, idx, best2, bi2, bestK2);
                }
                if (bi2 == -12345) best = -best;  // never (a sink)
            }
            while (m32) {
                const int t = __builtin_ctz(m32);
                m32 &= m32 - 1;
                const int idx = 32 * G + t;
                if (idx >= p.n_tris) break;
                if constexpr (S.diag) dg.exact += 1;
                cfloat* tp = (cfloat*)p.tri + 12 * idx;
                const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
            }
            if (__ballot(bestK != bk0)) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // every lane has read the rows' previous Y slots
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                write_y(bestK);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                if constexpr (!S.ylds) read_y();
            }
        }
    }
    return true;
}

// ---------------------------------------------------------------------------
// Filter probe (test hook rt2_mfma_probe, not part of the render): the five
// filter terms of every (ray, triangle) pair exactly as a product sweep
// computes them — the same scales (mfma_scale), fragments (mfma_main_row,
// mfma_y_chunk, through the same LDS rows), records and MFMA instructions —
// written out instead of reduced, with the operand fragments and the
// reference's own accept decision (mt_quantities + mt_exact against the ray's
// bound), so the host can measure the products' error against a binary64
// evaluation of the same operands and check the filter's conservativeness on
// the hardware.  One wave per 64 rays (n_rays a multiple of 64).
//   rays:   per ray {o.x, o.y, o.z, best} {d.x, d.y, d.z, 0}
//   terms:  [ray][tri][5] (U, -V, X, -tn, Y; tri < n_pad)
//   frags:  [ray][48] f16: main slots 0..31, Y slots 16..31
//   rinfo:  [ray][8]: in range, sigma, Tw, Bmax, m.x, m.y, m.z, bestK
//   accept: [ray][tri] (tri < n_tris): the reference accepts the pair
template <MfmaSpec S>
__global__ __launch_bounds__(64) void mfma_probe_kernel(RenderParams p, const float4* rays, int n_pad, float* terms,
                                                        _Float16* frags, float* rinfo, uint8_t* accept) {
    __shared__ MfmaK16Lds sh;
    const int lane = (int)threadIdx.x;
    const size_t ray = (size_t)blockIdx.x * 64 + lane;
    const float4 r0 = rays[2 * ray], r1 = rays[2 * ray + 1];
    const f3 o = mk(r0.x, r0.y, r0.z), d = mk(r1.x, r1.y, r1.z);
    const float best = r0.w, bestK = best * 1.0009765625f;
    for (int t = 0; t < p.n_tris; t++) {
        cfloat* tp = (cfloat*)p.tri + 12 * t;
        float b = best, bk = bestK;
        int bi = -1;
        mt_exact(mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8)), t, b, bi, bk);
        accept[ray * p.n_tris + t] = bi == t;
    }
    const f3 m = cross(d, o);
    MfmaScale sc{0.0f, 0.0f, 0.0f};
    const bool ok = mfma_scale<S>(p.mfma_A, o, d, m, sc);
    float* ri = rinfo + ray * 8;
    ri[0] = ok ? 1.0f : 0.0f;
    ri[1] = sc.sigma;
    ri[2] = sc.Tw;
    ri[3] = sc.Bmax;
    ri[4] = m.x;
    ri[5] = m.y;
    ri[6] = m.z;
    ri[7] = bestK;
    if (!ok) return;  // wave-uniform
    mfma_main_row(&sh.ray[lane][0], d, m, o, sc.sigma);
    {
        _Float16 s[16];
        mfma_y_chunk(s, d, o, bestK, sc.sigma, sc.Bmax);
        for (int j = 0; j < 16; j++) sh.ray[lane][32 + j] = s[j];
    }
    __syncthreads();
    for (int j = 0; j < 48; j++) frags[ray * 80 + j] = sh.ray[lane][j];
    const size_t ray0 = (size_t)blockIdx.x * 64;
    if constexpr (S.perm_frag) {
        // the shipping kernels' operand path (282 / 293 / 298 and the kthr
        // kernels): fragments built in registers by frag_pair, not read from
        // LDS rows.  frags[ray][48..63] receives the main fragment and
        // [64..79] the Y fragment as the MFMA A operand holds them (block R,
        // lane l: ray 32R + (l & 31), k-slots 8 (l >> 5) .. +7), so the host
        // can check the permutation against the rows above.
        const int r32 = lane & 31, hl = lane >> 5;
        h8 a0[2], y1[2];
        [[maybe_unused]] ThrBits tb = {};
        [[maybe_unused]] _Float16 tw16 = (_Float16)0.0f;
        if constexpr (S.kthr) {
            kt_frags<S>(d, m, sc, a0, tw16);
            kt_y(d, o, bestK, sc, tw16, y1);
        } else {
            _Float16 s[18];
            mfma_main_half_slots(s, d, m, sc.sigma);
            frag_pair(s, a0);
            _Float16 t[16];
            mfma_y_chunk(t, d, o, bestK, sc.sigma, sc.Bmax);
            frag_pair(t, y1);
            const float vz = m.z * sc.sigma;
            const _Float16 hz = (_Float16)vz;
            const _Float16 lz = (_Float16)(vz - (float)hz);
            tb = mfma_thr_bits(sc.Tw, wave_max(fabsf((float)lz)), wave_max(fabsf((float)hz)));
        }
        for (int R = 0; R < 2; R++)
            for (int j = 0; j < 8; j++) {
                frags[(ray0 + 32 * R + r32) * 80 + 48 + 8 * hl + j] = a0[R][j];
                frags[(ray0 + 32 * R + r32) * 80 + 64 + 8 * hl + j] = y1[R][j];
            }
        const h8* fg = reinterpret_cast<const h8*>(S.kthr ? p.mfma_kt_frag : p.mfma_k16_frag) + lane;
        const int nops = S.kthr ? kKtOps : kK16Ops;
        const f16v zero = {};
        for (int G = 0; G < n_pad / 32; G++) {
            h8 b[kK16Ops];
            for (int op = 0; op < nops; op++) b[op] = fg[(size_t)G * nops * 64 + 64 * op];
            for (int R = 0; R < 2; R++) {
                K16Terms q;
                if constexpr (S.kthr) {
                    q.U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[0], zero, 0, 0, 0);
                    q.V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[1], zero, 0, 0, 0);
                    q.X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[2], zero, 0, 0, 0);
                    q.T = zero;
                    q.Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], b[3], zero, 0, 0, 0);
                } else {
                    const f16v c = __builtin_amdgcn_mfma_f32_32x32x16_f16(mfma_thr_frag(tb), b[6], zero, 0, 0, 0);
                    q.U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[0], c, 0, 0, 0);
                    q.V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[2], c, 0, 0, 0);
                    q.X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0[R], b[4], c, 0, 0, 0);
                    q.T = c;
                    q.Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1[R], b[6], c, 0, 0, 0);
                }
                for (int i = 0; i < 16; i++) {
                    const size_t rr = ray0 + 32 * R + 8 * (i >> 2) + 4 * hl + (i & 3);
                    float* tt = terms + (rr * n_pad + 32 * G + r32) * 5;
                    tt[0] = q.U[i];
                    tt[1] = q.V[i];
                    tt[2] = q.X[i];
                    tt[3] = q.T[i];
                    tt[4] = q.Y[i];
                }
            }
        }
    } else if constexpr (S.k16) {
        const int r32 = lane & 31, hl = lane >> 5;
        // MfmaSpec::cthr: the sweep's threshold factors (the wave's m.z halves)
        [[maybe_unused]] ThrBits tb = {};
        if constexpr (S.cthr) {
            const float vz = m.z * sc.sigma;
            const _Float16 hz = (_Float16)vz;
            const _Float16 lz = (_Float16)(vz - (float)hz);
            tb = mfma_thr_bits(sc.Tw, wave_max(fabsf((float)lz)), wave_max(fabsf((float)hz)));
        }
        const h8* fg = reinterpret_cast<const h8*>(p.mfma_k16_frag) + lane;
        for (int G = 0; G < n_pad / 32; G++) {
            h8 b[kK16Ops];
            for (int op = 0; op < kK16Ops; op++) b[op] = fg[(size_t)G * kK16Ops * 64 + 64 * op];
            for (int R = 0; R < 2; R++) {
                const h8 a0 = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][8 * hl]);
                const h8 a1 = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][16 + 8 * hl]);
                const h8 y1 = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][32 + 8 * hl]);
                K16Terms q = k16_terms(a0, a1, y1, b);
                if constexpr (S.k5) {
                    // the 5-product form: U, -V, X from the first K-half only;
                    // cthr: all four with the threshold product TT as the
                    // accumulator (k5_cthr_group), TT itself in the -tn slot
                    const f16v zero = {};
                    f16v c = zero;
                    if constexpr (S.cthr) c = __builtin_amdgcn_mfma_f32_32x32x16_f16(mfma_thr_frag(tb), b[6], zero, 0, 0, 0);
                    q.U = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[0], c, 0, 0, 0);
                    q.V = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[2], c, 0, 0, 0);
                    q.X = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, b[4], c, 0, 0, 0);
                    if constexpr (S.cthr) {
                        q.T = c;
                        q.Y = __builtin_amdgcn_mfma_f32_32x32x16_f16(y1, b[6], c, 0, 0, 0);
                    }
                }
                for (int i = 0; i < 16; i++) {
                    const size_t rr = ray0 + 32 * R + 8 * (i >> 2) + 4 * hl + (i & 3);
                    float* tt = terms + (rr * n_pad + 32 * G + r32) * 5;
                    tt[0] = q.U[i];
                    tt[1] = q.V[i];
                    tt[2] = q.X[i];
                    tt[3] = q.T[i];
                    tt[4] = q.Y[i];
                }
            }
        }
    } else {
        // the 16x16x32 form (sweep_mfma, ymma): A rows in the main/Y LDS rows,
        // the Y fragment as sweep_mfma builds it (slots 0..15 zero)
        const h8* fg = reinterpret_cast<const h8*>(p.mfma_frag) + lane;
        const f4v zero = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int G = 0; G < n_pad / 16; G++) {
            const h8 c0 = fg[(size_t)G * kMfmaQ * 64], c1 = fg[(size_t)G * kMfmaQ * 64 + 64],
                     c2 = fg[(size_t)G * kMfmaQ * 64 + 128], c3 = fg[(size_t)G * kMfmaQ * 64 + 192];
            for (int R = 0; R < 4; R++) {
                const int row = 16 * R + (lane & 15), k0 = 8 * (lane >> 4);
                const h8 ra = *reinterpret_cast<const h8*>(&sh.ray[row][k0]);
                h8 ya = h8{};
                if (k0 >= 16) ya = *reinterpret_cast<const h8*>(&sh.ray[row][32 + k0 - 16]);
                const f4v qU = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra, c0, zero, 0, 0, 0);
                const f4v qV = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra, c1, zero, 0, 0, 0);
                const f4v qX = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra, c2, zero, 0, 0, 0);
                const f4v qT = __builtin_amdgcn_mfma_f32_16x16x32_f16(ra, c3, zero, 0, 0, 0);
                const f4v qY = __builtin_amdgcn_mfma_f32_16x16x32_f16(ya, c3, zero, 0, 0, 0);
                for (int i = 0; i < 4; i++) {
                    const size_t rr = ray0 + 16 * R + 4 * (lane >> 4) + i;
                    float* tt = terms + (rr * n_pad + 16 * G + (lane & 15)) * 5;
                    tt[0] = qU[i];
                    tt[1] = qV[i];
                    tt[2] = qX[i];
                    tt[3] = qT[i];
                    tt[4] = qY[i];
                }
            }
        }
    }
}

// Closest hit of every ray of `act` (lane j's o, d), one ray at a time by the
// whole wave (coop_closest: the sequential strict-< scan's result); lane j
// receives its own ray's (best, bi), lanes outside `act` keep theirs.
__device__ __forceinline__ void coop_each(unsigned long long act, const f3& o, const f3& d, const RenderParams& p,
                                          float& best, int& bi) {
    while (act) {
        const int j = __builtin_ctzll(act);
        act &= act - 1;
        const f3 oj = mk(__shfl(o.x, j), __shfl(o.y, j), __shfl(o.z, j));
        const f3 dj = mk(__shfl(d.x, j), __shfl(d.y, j), __shfl(d.z, j));
        float b;
        int bidx;
        coop_closest(oj, dj, p.tri, p.n_tris, b, bidx);
        if ((int)lane_id() == j) {
            best = b;
            bi = bidx;
        }
    }
}

// MFMA: render_smem's lockstep segment loop and cooperative drain with the
// matrix-core filter (sweep_mfma) as the closest-hit sweep; a wave whose
// rays leave the filter's range computes them with the cooperative drain's
// code instead (coop_each).
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma(RenderParams p_arg) {
    const RenderParams& p = p_arg;
    using WL = std::conditional_t<
        S.k16, std::conditional_t<S.lane_lds == 2, MfmaK16PackedLds, std::conditional_t<S.lane_lds == 1, MfmaK16LaneLds, MfmaK16Lds>>,
        MfmaWaveLds>;
    __shared__ WL wl[S.block / 64];
    WL& sh = wl[threadIdx.x >> 6];
    __shared__ BlockVote<S.block / 64> vote;  // lockstep: block_any
    uint32_t vote_parity = 0;
    if constexpr (S.lds_pad > 0) {
        __shared__ uint32_t pad[S.lds_pad / 4];
        if (p.n_items == 0) pad[threadIdx.x] = 0;  // never taken at launch; keeps the allocation
    }
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    unsigned long long tc = 0;  // diag: s_memtime at the current phase's start
    if constexpr (S.diag) tc = __builtin_amdgcn_s_memtime();
    // diag wave timeline (p.wave_log, 10 words per wave): start, first lane out
    // of items, end (s_memrealtime, 100 MHz), segment rounds with two 32-ray
    // blocks, with one, idle (lockstep: the wave had no ray), cooperative drain,
    // the wave's place (HW_ID | XCC_ID << 32), and shader clocks (s_memtime) at
    // start and end: their ratio to the real-time ticks is the in-kernel clock
    unsigned long long wl_t0 = 0, wl_c0 = 0, wl_dry = 0, wl_r2 = 0, wl_r1 = 0, wl_idle = 0, wl_coop = 0;
    if constexpr (S.diag)
        if (p.wave_log) {
            wl_t0 = __builtin_amdgcn_s_memrealtime();
            wl_c0 = __builtin_amdgcn_s_memtime();
        }
    auto stamp = [&](unsigned long long& acc) {
        if constexpr (S.diag) {
            const unsigned long long t = __builtin_amdgcn_s_memtime();
            acc += t - tc;
            tc = t;
        }
    };
    for (;;) {
        // the kernel arguments are re-read from the kernarg segment (scalar
        // loads) in every segment instead of being held in SGPRs across the
        // sweep (whose register pressure then spills them to VGPR lanes)
        const RenderParams& p = kargs<RenderParams>();
        advance(L, p);
        unsigned long long act = __ballot(L.st == ST_TRACE);
        stamp(dg.t_advance);
        if constexpr (S.diag)
            if (p.wave_log && !wl_dry && __any(L.st == ST_DONE)) wl_dry = __builtin_amdgcn_s_memrealtime();
        if constexpr (S.lockstep) {
            if (!block_any<S.block / 64>(act != 0, vote, vote_parity)) break;
            if (!act) {
                if constexpr (S.diag) wl_idle++;
                continue;
            }
        } else if (!act) {
            break;
        }
        if constexpr (S.diag) {
            if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE))
                wl_coop++;
            else if (S.compact && __popcll(act) <= 32)
                wl_r1++;
            else
                wl_r2++;
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
            stamp(dg.t_tail);
            continue;
        }
        bool upper = true;
        if constexpr (S.compact) {
            // at most 32 live rays: move them to lanes 0..31 (every lane's path
            // state travels with it; lanes are interchangeable), so that the
            // sweep runs the first 32-ray block only
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
        // lanes without a ray carry the first live lane's (their passes add no
        // triangle; such a lane is ST_DONE and never reads its o, d again)
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
        if constexpr (S.k16 && S.lane_lds) {
            // the path state waits in LDS (its registers are free during the sweep)
            if constexpr (S.lane_lds == 2) {
                lane_stash_packed(L, sh.lane, (int)lane_id());
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                swept = sweep_k16<S>(p, sh, ro, rd, best, bi, bestK, dg, upper);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                lane_unstash_packed(L, sh.lane, (int)lane_id());
                L.o = ro;  // (the same values: the stash does not hold o, d)
                L.d = rd;
            } else {
                lane_stash(L, sh.lane, (int)lane_id());
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                swept = sweep_k16<S>(p, sh, ro, rd, best, bi, bestK, dg, upper);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const f3 lo = L.o, ld = L.d;
                lane_unstash(L, sh.lane, (int)lane_id());
                L.o = lo;
                L.d = ld;
            }
        } else if constexpr (S.k16)
            swept = sweep_k16<S>(p, sh, ro, rd, best, bi, bestK, dg, upper);
        else
            swept = sweep_mfma<S>(p, sh, ro, rd, best, bi, bestK, dg);
        // a ray outside the filter's range (wave-uniform): the wave computes each
        // live ray's closest hit together (the drain's code, vector loads: no
        // SGPR block of records competing with the sweep's registers)
        if (!swept) coop_each(act, ro, rd, p, best, bi);
        stamp(dg.t_sweep);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
        stamp(dg.t_shade);
    }
    flush_counters(L, p);
    if constexpr (S.diag)
        if (p.wave_log) {
            const uint32_t gw = blockIdx.x * (S.block / 64) + (threadIdx.x >> 6);
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
                e[5] = wl_idle;
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
            atomicAdd(p.seg_counter + 8, dg.t_advance);
            atomicAdd(p.seg_counter + 9, dg.t_sweep);
            atomicAdd(p.seg_counter + 10, dg.t_shade);
            atomicAdd(p.seg_counter + 11, dg.t_tail);
        }
}

}  // namespace
