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
};

// per-wave diagnostic counts of sweep_mfma (wave-uniform; MfmaSpec::diag)
struct MfmaDiag {
    unsigned long long groups = 0, hot = 0, exact = 0;
};

// per wave: the ray fragments' staging rows (80-B stride: conflict-free
// 16-B reads) and the rays' distance-test bounds
struct MfmaWaveLds {
    _Float16 ray[64][40];
    float bk[64];
};

// Triangle records (one thread per padded triangle), in binary64 from the
// pre-transformed f32 triangle.  A triangle outside the validated range (as
// sweep_plk's: |a_i| <= 2^20, e0/e1/n components 0 or in [2^-100, 2^20],
// max >= 2^-30; non-finite) gets all-zero coefficients, which always pass
// (the exact test decides); padding triangles get -tn = +2^13, which never
// passes.  flags[0] += out-of-range triangles, flags[1] = max |a_i| (float bits).
__global__ void prep_mfma(const float4* tri, int n, int n_pad, _Float16* out, float* tau_out, uint32_t* flags) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_pad) return;
    double coef[kMfmaQ][10];
    for (int q = 0; q < kMfmaQ; q++)
        for (int c = 0; c < 10; c++) coef[q][c] = 0.0;
    double tau = 1.0;
    if (i >= n) {
        coef[3][9] = 0x1p13;  // padding: -tn' = 2^13 sigma > T
    } else {
        const float4 t0 = tri[3 * i], t1 = tri[3 * i + 1], t2 = tri[3 * i + 2];
        const float a[3] = {t0.x, t0.y, t0.z}, e0[3] = {t0.w, t1.x, t1.y}, e1[3] = {t1.z, t1.w, t2.x},
                    nn[3] = {t2.y, t2.z, t2.w};
        bool ok = true;
        float A = 0.0f, M = 0.0f;
        for (int k = 0; k < 3; k++) {
            ok = ok && fabsf(a[k]) <= 0x1p20f;
            A = fmaxf(A, fabsf(a[k]));
            for (float x : {e0[k], e1[k], nn[k]}) {
                const float ax = fabsf(x);
                ok = ok && (x == 0.0f || (ax >= 0x1p-100f && ax <= 0x1p20f));
                M = fmaxf(M, ax);
            }
        }
        ok = ok && M >= 0x1p-30f;
        if (ok) {
            int ex;
            (void)frexpf(M, &ex);
            const double s = ldexp(1.0, 1 - ex);
            double E0[3], E1[3], N[3], P0[3], P1[3], A0[3];
            for (int k = 0; k < 3; k++) {
                E0[k] = s * e0[k];
                E1[k] = s * e1[k];
                N[k] = s * nn[k];
                A0[k] = a[k];
            }
            P0[0] = A0[1] * E0[2] - A0[2] * E0[1];
            P0[1] = A0[2] * E0[0] - A0[0] * E0[2];
            P0[2] = A0[0] * E0[1] - A0[1] * E0[0];
            P1[0] = A0[1] * E1[2] - A0[2] * E1[1];
            P1[1] = A0[2] * E1[0] - A0[0] * E1[2];
            P1[2] = A0[0] * E1[1] - A0[1] * E1[0];
            const double AN = A0[0] * N[0] + A0[1] * N[1] + A0[2] * N[2];
            for (int k = 0; k < 3; k++) {
                coef[0][k] = -P1[k];                               // U: d
                coef[0][3 + k] = E1[k];                            //    m
                coef[1][k] = P0[k];                                // -V: d
                coef[1][3 + k] = -E0[k];                           //     m
                coef[2][k] = P1[k] - P0[k] + (double)kMfmaC * N[k];  // X: d
                coef[2][3 + k] = E0[k] - E1[k];                    //    m
                coef[3][6 + k] = -N[k];                            // -tn: o
                coef[4][k] = N[k];                                 // dn: d
            }
            coef[3][9] = AN;  // -tn: 1
            double mx = 0.0;
            for (int q = 0; q < kMfmaQ; q++)
                for (int c = 0; c < 10; c++) mx = fmax(mx, fabs(coef[q][c]));
            int e2;
            (void)frexp(mx, &e2);  // mx in [2^(e2-1), 2^e2)
            tau = ldexp(1.0, 14 - e2);
            atomicMax(&flags[1], __float_as_uint(A));
        } else {
            atomicAdd(&flags[0], 1u);
        }
    }
    const int G = i >> 4, t = i & 15;
    for (int q = 0; q < kMfmaQ; q++) {
        _Float16 slot[32];
        for (int k = 0; k < 32; k++) slot[k] = (_Float16)0.0f;
        for (int c = 0; c < 10; c++) {
            const double v = coef[q][c] * tau;
            const _Float16 hi = (_Float16)(float)v;
            const _Float16 lo = (_Float16)(float)(v - (double)(float)hi);
            if (c < 9) {
                slot[3 * c] = hi;  // x hi * ray hi
                slot[3 * c + 1] = hi;  // x hi * ray lo
                slot[3 * c + 2] = lo;  // x lo * ray hi
            } else {
                slot[27] = hi;  // * sigma
                slot[28] = lo;  // * sigma
            }
        }
        for (int k = 0; k < 32; k++) out[((size_t)(G * kMfmaQ + q) * 64 + 16 * (k >> 3) + t) * 8 + (k & 7)] = slot[k];
    }
    tau_out[i] = (float)tau;
}

__device__ __forceinline__ float wave_max(float x) {
    for (int off = 32; off > 0; off >>= 1) x = fmaxf(x, __shfl_xor(x, off));
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

__device__ __forceinline__ float abs_max3(const f3& v) { return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fabsf(v.z)); }

// Closest hit of every lane's ray (o, d) over the 16-triangle groups [G0, G1)
// (all of them by default); the whole wave calls it (lanes without a ray of
// their own carry a copy of a live one).  Returns false (nothing done) when a
// ray is outside the bound's range.
template <MfmaSpec S>
__device__ __forceinline__ bool sweep_mfma(const RenderParams& p, MfmaWaveLds& sh, const f3& o, const f3& d, float& best,
                                           int& bi, float& bestK, MfmaDiag& dg, int G0 = 0, int G1 = -1) {
    const int lane = (int)lane_id();
    const f3 m = cross(d, o);
    if (__ballot(!(abs_max3(o) <= 0x1p20f && abs_max3(d) <= 1.0001f))) return false;  // NaN fails too
    const float Omax = wave_max(abs_max3(o));
    const float R0 = Omax + p.mfma_A + 1.0f;
    float mx = fmaxf(fmaxf(Omax, wave_max(abs_max3(m))), 1.0f);
    if constexpr (S.ymma) mx = fmaxf(mx, __builtin_fmaf(2.25f, R0, Omax));  // |o + bk d| for every bk <= Bmax
    int ex;
    (void)frexpf(mx, &ex);
    const float sigma = ldexpf(1.0f, 14 - ex);  // sigma * mx in [2^13, 2^14)
    const float Tw = sigma * (ldexpf(kMfmaTs, 10 - S.tshift) * R0);
    const float Cw = -kMfmaE * sigma;
    const float Bmax = kMfmaB * R0;

    // this lane's ray vector (sigma-scaled d, m, o, 1) as f16 slots -> LDS row `lane`
    {
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
        h8* row = reinterpret_cast<h8*>(&sh.ray[lane][0]);
#pragma unroll
        for (int k = 0; k < 4; k++) row[k] = h8{s[8 * k], s[8 * k + 1], s[8 * k + 2], s[8 * k + 3], s[8 * k + 4],
                                                s[8 * k + 5], s[8 * k + 6], s[8 * k + 7]};
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    h8 ra[4];
#pragma unroll
    for (int R = 0; R < 4; R++) ra[R] = *reinterpret_cast<const h8*>(&sh.ray[16 * R + (lane & 15)][8 * (lane >> 4)]);
    f4v bk[4];
    h8 ya[4];  // ymma: the Y fragment (-w, -1) / (-Bmax d, 0), built in the same LDS rows
    // Y fragment of this lane's ray for its distance bound bkv: w = o + bkv d
    // (bkv <= Bmax) with the constant slot -sigma, so that the -tn record gives
    // Y = w.N - AN = s (tnum - bkv det); or, with no usable bound, w = Bmax d
    // and constant 0: Y = -s Bmax det (the det > 0 test).  -w sigma as f16
    // hi/lo in the o slots (18..26, hi lo hi like the main fragment).
    auto build_y = [&](float bkv) {
        const bool fin = bkv <= Bmax;
        const float wx = fin ? __builtin_fmaf(bkv, d.x, o.x) : Bmax * d.x;
        const float wy = fin ? __builtin_fmaf(bkv, d.y, o.y) : Bmax * d.y;
        const float wz = fin ? __builtin_fmaf(bkv, d.z, o.z) : Bmax * d.z;
        const float wc[3] = {wx, wy, wz};
        _Float16 s[16];
#pragma unroll
        for (int c = 0; c < 3; c++) {
            const float v = -wc[c] * sigma;
            const _Float16 hi = (_Float16)v;
            const _Float16 lo = (_Float16)(v - (float)hi);
            s[2 + 3 * c] = hi;
            s[3 + 3 * c] = lo;
            s[4 + 3 * c] = hi;
        }
        s[0] = s[1] = (_Float16)0.0f;  // slots 16, 17: d.z (zero here)
        s[11] = s[12] = (_Float16)(fin ? -sigma : 0.0f);
        s[13] = s[14] = s[15] = (_Float16)0.0f;
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

// MFMA: render_smem's lockstep segment loop and cooperative drain with the
// matrix-core filter (sweep_mfma) as the closest-hit sweep; a wave whose
// rays leave the filter's range sweeps with the scalar-path filter instead.
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma(RenderParams p) {
    __shared__ MfmaWaveLds wl[S.block / 64];
    MfmaWaveLds& sh = wl[threadIdx.x >> 6];
    if constexpr (S.lds_pad > 0) {
        __shared__ uint32_t pad[S.lds_pad / 4];
        if (p.n_items == 0) pad[threadIdx.x] = 0;  // never taken at launch; keeps the allocation
    }
    Lane L;
    lane_init(L);
    MfmaDiag dg;
    for (;;) {
        advance(L, p);
        const unsigned long long act = __ballot(L.st == ST_TRACE);
        if constexpr (S.lockstep) {
            if (!__syncthreads_or(act != 0)) break;
            if (!act) continue;
        } else if (!act) {
            break;
        }
        if (__popcll(act) <= (unsigned)S.tail_lanes && __any(L.st == ST_DONE)) {
            float mybest = 1e38f;
            int mybi = -1;
            unsigned long long mm = act;
            while (mm) {
                const int j = __builtin_ctzll(mm);
                mm &= mm - 1;
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
        // lanes without a ray carry the first live lane's (their passes add no triangle)
        const int j0 = __builtin_ctzll(act);
        const bool mine = L.st == ST_TRACE;
        const f3 o = mk(__shfl(L.o.x, j0), __shfl(L.o.y, j0), __shfl(L.o.z, j0));
        const f3 dd = mk(__shfl(L.d.x, j0), __shfl(L.d.y, j0), __shfl(L.d.z, j0));
        const f3 ro = mine ? L.o : o, rd = mine ? L.d : dd;
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        if (!sweep_mfma<S>(p, sh, ro, rd, best, bi, bestK, dg) && mine)
            sweep_masked<8, true, Filter::Max3>(ro, rd, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
    if constexpr (S.diag)
        if (lane_id() == 0) {
            atomicAdd(p.seg_counter + 1, dg.groups);  // (wave, 16-triangle group) sweeps
            atomicAdd(p.seg_counter + 2, dg.hot);     // ... with a passing pair
            atomicAdd(p.seg_counter + 3, dg.exact);   // (wave, triangle) exact tests
        }
}

}  // namespace
