// Experiment (RT2_EXPERIMENTS only): the matrix-filter sweep of rt2_mfma.h
// (ymma form, one compare per group) on v_mfma_f32_32x32x16_f16 — 32 rays ×
// 32 triangles per product, K = 16 slots, so each quantity takes two products
// (slots 0..15 and 16..31) and a 1,024-pair block issues 10 MFMAs instead of
// 20 (half the MFMA issue holds on the VALU port, the same matrix cycles).
// Operand maps (cdna_hip_programming.md): lane l holds A[row l&31][k 8(l>>5)+j]
// and B[k 8(l>>5)+j][col l&31]; D: column l&31, rows in the 16 registers — so
// every value a lane holds belongs to one triangle, and the min over them plus
// one ballot gives the group's triangles with a passing pair.  B fragments are
// read straight from prep_mfma's 16-triangle record layout (triangle t of a
// 32-group = 16-group 2G + (t>>4), lane t&15; slot octet 2h + (l>>5)).
// Included by rt2_render.hip after rt2_mfma.h.
#pragma once

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));

template <MfmaSpec S>
__device__ __forceinline__ bool sweep_mfma32(const RenderParams& p, MfmaWaveLds& sh, const f3& o, const f3& d,
                                             float& best, int& bi, float& bestK) {
    const int lane = (int)lane_id();
    const f3 m = cross(d, o);
    if (__ballot(!(abs_max3(o) <= 0x1p20f && abs_max3(d) <= 1.0001f))) return false;  // NaN fails too
    const float Omax = wave_max(abs_max3(o));
    const float R0 = Omax + p.mfma_A + 1.0f;
    float mx = fmaxf(fmaxf(Omax, wave_max(abs_max3(m))), 1.0f);
    mx = fmaxf(mx, __builtin_fmaf(2.25f, R0, Omax));  // |o + bk d| for every bk <= Bmax
    int ex;
    (void)frexpf(mx, &ex);
    const float sigma = ldexpf(1.0f, 14 - ex);
    const float Tw = sigma * (ldexpf(kMfmaTs, 10 - S.tshift) * R0);
    const float Bmax = kMfmaB * R0;
    const int r32 = lane & 31, hl = lane >> 5;

    {  // main fragment (sigma-scaled d, m, o, 1) -> LDS row `lane`, as in sweep_mfma
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
    h8 ra[2][2], ya[2][2];  // [ray block R][k half h]
#pragma unroll
    for (int R = 0; R < 2; R++)
#pragma unroll
        for (int h = 0; h < 2; h++) ra[R][h] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][16 * h + 8 * hl]);
    auto build_y = [&](float bkv) {  // as sweep_mfma's build_y
        const bool fin = bkv <= Bmax;
        const float wc[3] = {fin ? __builtin_fmaf(bkv, d.x, o.x) : Bmax * d.x,
                             fin ? __builtin_fmaf(bkv, d.y, o.y) : Bmax * d.y,
                             fin ? __builtin_fmaf(bkv, d.z, o.z) : Bmax * d.z};
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
        s[0] = s[1] = (_Float16)0.0f;
        s[11] = s[12] = (_Float16)(fin ? -sigma : 0.0f);
        s[13] = s[14] = s[15] = (_Float16)0.0f;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
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
        for (int R = 0; R < 2; R++)
#pragma unroll
            for (int h = 0; h < 2; h++)
                ya[R][h] = *reinterpret_cast<const h8*>(&sh.ray[32 * R + r32][16 * h + 8 * hl]);
    };
    build_y(bestK);

    const h8* frag = reinterpret_cast<const h8*>(p.mfma_frag);
    const int ng16 = (p.n_tris + 15) >> 4;
    const int ng = (ng16 + 1) >> 1;
    const int half = r32 >> 4;  // which 16-group of the 32-group this lane's triangle is in
    for (int G = 0; G < ng; G++) {
        const int g16 = 2 * G + half;
        const bool have = g16 < ng16;  // the last 32-group may have one 16-group only
        const int gl = have ? g16 : ng16 - 1;
        const h8* fg = frag + (size_t)gl * (kMfmaQ * 64) + (lane & 15);
        h8 b[4][2];
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int h = 0; h < 2; h++) b[q][h] = fg[q * 64 + 16 * (2 * h + hl)];
        const float tau = p.mfma_tau[16 * gl + (lane & 15)];
        const float Tl = tau * Tw;
        const f16v zero = {};
        int tmin = 0x7fffffff;
#pragma unroll
        for (int R = 0; R < 2; R++) {
            f16v q[5];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                q[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[R][0], b[k][0], zero, 0, 0, 0);
                q[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ra[R][1], b[k][1], q[k], 0, 0, 0);
            }
            q[4] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ya[R][0], b[3][0], zero, 0, 0, 0);  // Y
            q[4] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ya[R][1], b[3][1], q[4], 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) {
                const int t3 = max(max(__float_as_int(q[0][i]), __float_as_int(q[1][i])), __float_as_int(q[2][i]));
                const int t = max(max(t3, __float_as_int(q[3][i])), __float_as_int(q[4][i]));
                tmin = min(tmin, t);
            }
        }
        const unsigned long long M = __ballot(have && tmin <= __float_as_int(Tl));
        if (M) {
            uint32_t m32 = (uint32_t)((M | M >> 32) & 0xffffffffull);
            const float bk0 = bestK;
            while (m32) {
                const int t = __builtin_ctz(m32);
                m32 &= m32 - 1;
                const int idx = 32 * G + t;
                if (idx >= p.n_tris) break;
                cfloat* tp = (cfloat*)p.tri + 12 * idx;
                const MtQ qq = mt_quantities(o, d, ldc4(tp), ldc4(tp + 4), ldc4(tp + 8));
                if (mt_pass3(qq, bestK)) mt_exact(qq, idx, best, bi, bestK);
            }
            if (__ballot(bestK != bk0)) build_y(bestK);
        }
    }
    return true;
}

// render_mfma with the 32x32x16 sweep (lockstep segments, cooperative drain)
template <MfmaSpec S>
__global__ __launch_bounds__(S.block) __attribute__((amdgpu_waves_per_eu(S.waves))) void render_mfma32(RenderParams p) {
    __shared__ MfmaWaveLds wl[S.block / 64];
    MfmaWaveLds& sh = wl[threadIdx.x >> 6];
    Lane L;
    lane_init(L);
    for (;;) {
        advance(L, p);
        const unsigned long long act = __ballot(L.st == ST_TRACE);
        if (!__syncthreads_or(act != 0)) break;
        if (!act) continue;
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
        const int j0 = __builtin_ctzll(act);
        const bool mine = L.st == ST_TRACE;
        const f3 o = mk(__shfl(L.o.x, j0), __shfl(L.o.y, j0), __shfl(L.o.z, j0));
        const f3 dd = mk(__shfl(L.d.x, j0), __shfl(L.d.y, j0), __shfl(L.d.z, j0));
        const f3 ro = mine ? L.o : o, rd = mine ? L.d : dd;
        float best = 1e38f, bestK = 1e38f * 1.0009765625f;
        int bi = -1;
        if (!sweep_mfma32<S>(p, sh, ro, rd, best, bi, bestK) && mine)
            sweep_masked<8, true, Filter::Max3>(ro, rd, nullptr, (const float*)p.tri, p.n_tris, 0, best, bi, bestK);
        if (mine) {
            L.bounce += 1;
            L.segs += 1;
            shade(L, p, best, bi);
        }
    }
    flush_counters(L, p);
}

}  // namespace
