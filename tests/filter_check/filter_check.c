/* Conservativeness check of the brute-force kernel's division-free filters
 * (rt2_sweep.h mt_pass and mt_pass3) against the reference's Möller–Trumbore
 * update decision (compute.glsl:302-340 + the strict `dst < best` of :432).
 *
 * A filter may pass pairs the exact test rejects (they just take the exact
 * path) but must never reject a pair the exact test would accept.  The
 * arithmetic restates the device forms in binary32 with explicit fmaf (built
 * with -ffp-contract=off), over random and adversarial rays: rays through
 * triangle edges and vertices nudged by a few ulps, grazing rays around the
 * det = 1e-10 cut, `best` at and around the hit distance, coordinates over
 * six decades.  The per-ray precomputed filter (sweep_plk, plk_pass) is
 * checked the same way on its own record (built as prep_plk does, binary64
 * then one rounding) with extra draws of small triangles far from the origin
 * (the cancellation case of o·n − a·n).
 *
 *   filter_check <pairs> <seed>
 *     -> "pairs accepts violations_old violations_new pass_old pass_new violations_plk pass_plk"
 * (pass_old / pass_new over the draws at ordinary scales, 1e-2 .. 1e2: the
 * constant threshold of pass_new is absolute, so on microscopic coordinates it
 * passes more — still conservative, checked on every draw)
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef struct { float x, y, z; } f3;
static f3 mk(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static f3 sub(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static float dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static f3 cross(f3 a, f3 b) {
    return mk(fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)), fmaf(a.x, b.y, -(a.y * b.x)));
}

static uint64_t s_rng;
static uint64_t next64(void) {
    s_rng ^= s_rng << 13;
    s_rng ^= s_rng >> 7;
    s_rng ^= s_rng << 17;
    return s_rng;
}
static float uni(void) { return (float)((next64() >> 40) * (1.0 / 16777216.0)); }  /* [0,1) */
static float sym(void) { return 2.0f * uni() - 1.0f; }
static float nudge(float x, int k) {
    for (; k > 0; k--) x = nextafterf(x, INFINITY);
    for (; k < 0; k++) x = nextafterf(x, -INFINITY);
    return x;
}
static int ik(int span) { return (int)(next64() % (uint64_t)(2 * span + 1)) - span; }
static f3 normalize(f3 v) {
    const float l = sqrtf(dot(v, v));
    return mk(v.x / l, v.y / l, v.z / l);
}

typedef struct { float det, tnum, U, V; } Q;

static Q quantities(f3 o, f3 d, f3 a, f3 e0, f3 e1, f3 n) {
    Q q;
    q.det = -dot(d, n);
    const f3 ao = sub(o, a);
    q.tnum = dot(ao, n);
    const f3 c = cross(d, ao);
    q.U = dot(e1, c);
    q.V = dot(e0, c);
    return q;
}
static int exact_updates(Q q, float best) {
    if ((q.det < 1e-10f && q.det > -1e-10f) || q.det < 0.0f) return 0;
    const float inv = 1.0f / q.det;
    const float dst = q.tnum * inv;
    const float u = -q.U * inv;
    const float v = q.V * inv;
    return !(dst <= 1e-6f) && !(u < 0.0f || v < 0.0f || 1.0f - u - v < 0.0f) && dst < best;
}
static int pass_old(Q q, float bestK) {
    const float B = q.det * 0x1p-60f;
    return (q.tnum > 0.0f) & (q.U <= B) & (q.V >= -B) & ((q.V - q.U) <= q.det * 1.0009765625f) &
           (q.tnum <= q.det * bestK);
}
static int pass_new(Q q, float bestK) {
    const float B = q.det * 0x1p-60f;
    const float X = fmaf(-q.det, 1.0009765625f, q.V - q.U);
    const float Y = fmaf(-q.det, bestK, q.tnum);
    return fmaxf(fmaxf(fmaxf(fmaxf(q.U, -q.V), X), -q.tnum), Y) <= B;
}

/* prep_plk (rt2_misc_kernels.h): record of one triangle; returns 0 when the
 * triangle is outside the validated range (the scene keeps the old filter). */
static int plk_record(f3 a, f3 e0, f3 e1, f3 n, float r[16], float* Aout) {
    const float av[3] = {a.x, a.y, a.z}, e0v[3] = {e0.x, e0.y, e0.z}, e1v[3] = {e1.x, e1.y, e1.z},
                nv[3] = {n.x, n.y, n.z};
    float A = 0.0f, M = 0.0f;
    int ok = 1;
    for (int k = 0; k < 3; k++) {
        ok = ok && fabsf(av[k]) <= 0x1p20f;
        A = fmaxf(A, fabsf(av[k]));
        const float xs[3] = {e0v[k], e1v[k], nv[k]};
        for (int j = 0; j < 3; j++) {
            const float ax = fabsf(xs[j]);
            ok = ok && (xs[j] == 0.0f || (ax >= 0x1p-100f && ax <= 0x1p20f));
            M = fmaxf(M, ax);
        }
    }
    for (int k = 0; k < 16; k++) r[k] = 0.0f;  /* all-zero record: always passes */
    *Aout = A;
    if (!ok || !(M >= 0x1p-30f)) return 0;
    int ex;
    (void)frexpf(M, &ex);
    const double s = ldexp(1.0, 1 - ex);
    const double p0[3] = {(double)a.y * e0.z - (double)a.z * e0.y, (double)a.z * e0.x - (double)a.x * e0.z,
                          (double)a.x * e0.y - (double)a.y * e0.x};
    const double p1[3] = {(double)a.y * e1.z - (double)a.z * e1.y, (double)a.z * e1.x - (double)a.x * e1.z,
                          (double)a.x * e1.y - (double)a.y * e1.x};
    const double an = (double)a.x * n.x + (double)a.y * n.y + (double)a.z * n.z;
    r[0] = (float)(n.x * s); r[1] = (float)(n.y * s); r[2] = (float)(n.z * s); r[3] = (float)(-an * s);
    r[4] = (float)(e0.x * s); r[5] = (float)(e0.y * s); r[6] = (float)(e0.z * s); r[7] = (float)(-p0[0] * s);
    r[8] = (float)(-p0[1] * s); r[9] = (float)(-p0[2] * s); r[10] = (float)(e1.x * s); r[11] = (float)(e1.y * s);
    r[12] = (float)(e1.z * s); r[13] = (float)(-p1[0] * s); r[14] = (float)(-p1[1] * s); r[15] = (float)(-p1[2] * s);
    return 1;
}
/* sweep_plk's segment constants and plk_pass */
static int pass_plk(f3 o, f3 d, const float* r, float A, float bestK) {
    const f3 m = cross(d, o);
    const float O = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float T = fmaf(0x1p-13f, O + A, 0x1p-40f);
    const float bkf = bestK <= 0x1p60f ? bestK : INFINITY;
    const float dn = fmaf(d.z, r[2], fmaf(d.y, r[1], d.x * r[0]));
    const float tn = fmaf(o.z, r[2], fmaf(o.y, r[1], fmaf(o.x, r[0], r[3])));
    float V = fmaf(r[6], m.z, fmaf(r[5], m.y, r[4] * m.x));
    V = fmaf(d.z, r[9], fmaf(d.y, r[8], fmaf(d.x, r[7], V)));
    float U = fmaf(r[12], m.z, fmaf(r[11], m.y, r[10] * m.x));
    U = fmaf(d.z, r[15], fmaf(d.y, r[14], fmaf(d.x, r[13], U)));
    const float X = fmaf(dn, 1.0009765625f, V - U);
    const float Y = fmaf(dn, bkf, tn);
    return fmaxf(fmaxf(fmaxf(fmaxf(U, -V), X), -tn), Y) <= T;
}

/* ---- the matrix-core filter (rt2_mfma.h prep_mfma / sweep_mfma) ----------
 * binary16 rounding (RNE, subnormals down to 2^-24, as the f32->f16 convert) */
static double to_f16(double x) {
    const double ax = fabs(x);
    if (ax == 0.0 || isnan(x)) return x;
    if (ax >= 65520.0) return x > 0 ? INFINITY : -INFINITY;
    int e;
    (void)frexp(ax, &e);                                  /* ax in [2^(e-1), 2^e) */
    const double quantum = ax < 0x1p-14 ? 0x1p-24 : ldexp(1.0, e - 11);
    return rint(x / quantum) * quantum;
}
enum { MQ = 5 };
/* prep_mfma: one triangle's 5 x 32 f16 slots and its scale tau; 0 = out of range */
static int mfma_record(f3 a, f3 e0, f3 e1, f3 n, double slot[MQ][32], double* tau_out, float* Aout) {
    const float av[3] = {a.x, a.y, a.z}, e0v[3] = {e0.x, e0.y, e0.z}, e1v[3] = {e1.x, e1.y, e1.z},
                nv[3] = {n.x, n.y, n.z};
    double coef[MQ][10] = {{0}};
    double tau = 1.0;
    float A = 0.0f, M = 0.0f;
    int ok = 1;
    for (int k = 0; k < 3; k++) {
        ok = ok && fabsf(av[k]) <= 0x1p20f;
        A = fmaxf(A, fabsf(av[k]));
        const float xs[3] = {e0v[k], e1v[k], nv[k]};
        for (int j = 0; j < 3; j++) {
            const float ax = fabsf(xs[j]);
            ok = ok && (xs[j] == 0.0f || (ax >= 0x1p-100f && ax <= 0x1p20f));
            M = fmaxf(M, ax);
        }
    }
    ok = ok && M >= 0x1p-30f;
    *Aout = A;
    if (ok) {
        int ex;
        (void)frexpf(M, &ex);
        const double s = ldexp(1.0, 1 - ex);
        double E0[3], E1[3], N[3], P0[3], P1[3];
        for (int k = 0; k < 3; k++) E0[k] = s * e0v[k], E1[k] = s * e1v[k], N[k] = s * nv[k];
        P0[0] = (double)av[1] * E0[2] - (double)av[2] * E0[1];
        P0[1] = (double)av[2] * E0[0] - (double)av[0] * E0[2];
        P0[2] = (double)av[0] * E0[1] - (double)av[1] * E0[0];
        P1[0] = (double)av[1] * E1[2] - (double)av[2] * E1[1];
        P1[1] = (double)av[2] * E1[0] - (double)av[0] * E1[2];
        P1[2] = (double)av[0] * E1[1] - (double)av[1] * E1[0];
        const double AN = (double)av[0] * N[0] + (double)av[1] * N[1] + (double)av[2] * N[2];
        for (int k = 0; k < 3; k++) {
            coef[0][k] = -P1[k];
            coef[0][3 + k] = E1[k];
            coef[1][k] = P0[k];
            coef[1][3 + k] = -E0[k];
            coef[2][k] = P1[k] - P0[k] + 1.0009765625 * N[k];
            coef[2][3 + k] = E0[k] - E1[k];
            coef[3][6 + k] = -N[k];
            coef[4][k] = N[k];
        }
        coef[3][9] = AN;
        double mx = 0.0;
        for (int q = 0; q < MQ; q++)
            for (int c = 0; c < 10; c++) mx = fmax(mx, fabs(coef[q][c]));
        int e2;
        (void)frexp(mx, &e2);
        tau = ldexp(1.0, 14 - e2);
    }
    for (int q = 0; q < MQ; q++) {
        for (int k = 0; k < 32; k++) slot[q][k] = 0.0;
        for (int c = 0; c < 10; c++) {
            const double v = coef[q][c] * tau;
            const double hi = to_f16((float)v);
            const double lo = to_f16((float)(v - (double)(float)hi));
            if (c < 9) slot[q][3 * c] = hi, slot[q][3 * c + 1] = hi, slot[q][3 * c + 2] = lo;
            else slot[q][27] = hi, slot[q][28] = lo;
        }
    }
    *tau_out = tau;
    return ok;
}
/* sweep_mfma's decision for one (ray, triangle) pair in a wave whose other
 * rays raise max|o| to Ow and max(|o|,|m|) to Mw, in a scene whose max |a| is
 * As.  The accumulation of the 32 exact f16 products (+ C) in f32 is replaced
 * by the exact sum moved by the worst-case f32 summation error (31 u Σ|p|)
 * toward rejection: a pass here is a pass for any summation order. */
/* the threshold of the Y-by-matrix-product form (rt2_mfma.h MfmaSpec::tshift
 * of the product variants), T = YMMA_TS (Omax + A + 1) */
#ifndef YMMA_TS
#define YMMA_TS 0x1p-12f
#endif
/* k5 (rt2_mfma.h MfmaSpec::k5, with ymma): U, -V, X leave out their m.z
 * slots 16 and 17 (coefficient hi x ray lo, coefficient lo x ray hi) and the
 * threshold grows by the bound CH max|ray lo| + CL max|ray hi| (CH, CL: the
 * record's largest |slot 16|, |slot 17| over U, -V, X), padded by 2^-10.  The
 * wave's maxima are at least this ray's own values; the check uses exactly
 * those (the smallest bound a wave can have). */
/* f16 of v > 0 rounded up (rt2_mfma.h f16_up) */
static double f16_up(float v) {
    double h = to_f16(v);
    if (h < v) {
        int e;
        (void)frexp(h, &e);
        h += h < 0x1p-14 ? 0x1p-24 : ldexp(1.0, e - 12);  /* h in [2^(e-1), 2^e): quantum 2^(e-11) */
    }
    return h;
}
/* k5 = 2 (MfmaSpec::cthr): the same 4-term form with the threshold in the
 * accumulator: TT = -(tau Tw'' + CH ML'' + CL MH'') from the -tn record's
 * slots 29..31 (-tau, -CH, -CL) times mfma_thr_frag's f16 factors (padded by
 * 2^-8, rounded up), its 3-term sum moved toward zero by 2^-12 (the matrix
 * core's measured worst is 2^-18.6, tests/test_gpu_filter_probe.py); each term is
 * its products plus TT, moved by 31 u (sum |p| + |TT|) toward rejection, and
 * passes iff negative (the sign-bit AND). */
static int pass_mfma(f3 o, f3 d, double slot[MQ][32], double tau, float As, float Ow, float Mw, float bestK,
                     int ymma, float ts, int k5) {
    const f3 m = cross(d, o);
    const float ao = fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    const float am = fmaxf(fmaxf(fabsf(m.x), fabsf(m.y)), fabsf(m.z));
    const float Omax = fmaxf(ao, Ow);
    const float R0 = Omax + As + 1.0f;
    float mx = fmaxf(fmaxf(Omax, fmaxf(am, Mw)), 1.0f);
    if (ymma) mx = fmaxf(mx, fmaf(2.25f, R0, Omax));  /* |o + bk d| for any bk <= Bmax */
    int ex;
    (void)frexpf(mx, &ex);
    const float sigma = ldexpf(1.0f, 14 - ex);
    const float Tw = sigma * (ts * R0);
    const float Cw = -0x1p-14f * sigma;
    const float Bmax = 2.0f * R0;
    const float comp[9] = {d.x, d.y, d.z, m.x, m.y, m.z, o.x, o.y, o.z};
    double ray[32];
    for (int c = 0; c < 9; c++) {
        const float v = comp[c] * sigma;
        const double hi = to_f16(v);
        const double lo = to_f16(v - (float)hi);
        ray[3 * c] = hi, ray[3 * c + 1] = lo, ray[3 * c + 2] = hi;
    }
    ray[27] = ray[28] = sigma;
    ray[29] = ray[30] = ray[31] = 0.0;
    float Tl = (float)tau * Tw;
    double TT = 0.0;
    if (k5 == 2) {
        float ch = 0.0f, cl = 0.0f;
        for (int q = 0; q < 3; q++) ch = fmaxf(ch, (float)fabs(slot[q][16])), cl = fmaxf(cl, (float)fabs(slot[q][17]));
        const float pad = 1.00390625f;
        const double s3 = (double)(float)tau * f16_up(Tw * pad) + (double)ch * f16_up((float)fabs(ray[16]) * pad) +
                          (double)cl * f16_up((float)fabs(ray[17]) * pad);
        TT = -s3 * (1.0 - 0x1p-12);
    } else if (k5) {
        float ch = 0.0f, cl = 0.0f;
        for (int q = 0; q < 3; q++) ch = fmaxf(ch, (float)fabs(slot[q][16])), cl = fmaxf(cl, (float)fabs(slot[q][17]));
        Tl += (ch * (float)fabs(ray[16]) + cl * (float)fabs(ray[17])) * 1.0009765625f;
    }
    /* k5 = 4 (MfmaSpec::kthr, the threshold in the K-slots): U, -V, X keep
     * slots 0..12 and 15 (d, m.x, the hi x hi products of m.y and m.z); the
     * cross slots 13, 14 (m.y) and 16, 17 (m.z) are left out, and two slots
     * carry -tau x Tw' and -B_q x W': Tw' = Tw (1 + 2^-8) and W' = W (1 + 2^-8)
     * rounded up to f16, W = mw_y + mw_z with mw_c = max(|ray hi|, 2^11 |ray
     * lo|) (this ray's own: the smallest a wave's maximum can be), B_q =
     * 2^-10 max over y, z of max(|coef hi|, 2^11 |coef lo|) rounded up.  Y
     * carries -tau x Tw' (slot 29).  Each term is its 16 products moved by
     * 31 u sum|p| toward rejection and passes iff negative. */
    double kt_thr[3] = {0.0, 0.0, 0.0}, kt_y = 0.0;
    if (k5 == 4) {
        const float pad = 1.00390625f;
        const double tw = f16_up(Tw * pad);
        const float W = fmaxf((float)fabs(ray[12]), 2048.0f * (float)fabs(ray[13])) +
                        fmaxf((float)fabs(ray[15]), 2048.0f * (float)fabs(ray[16]));
        const double w16 = f16_up(W * pad);
        for (int q = 0; q < 3; q++) {
            const float ct = fmaxf(fmaxf((float)fabs(slot[q][12]), 2048.0f * (float)fabs(slot[q][14])),
                                   fmaxf((float)fabs(slot[q][15]), 2048.0f * (float)fabs(slot[q][17])));
            kt_thr[q] = -(tau * tw + f16_up(ct * 0x1p-10f) * w16);
        }
        kt_y = -tau * tw;
    }
    const float cd = (float)tau * Cw;
    float qv[MQ], qe[MQ];
    for (int q = 0; q < MQ; q++) {
        double s = q == 4 ? cd : TT, sa = q == 4 ? fabs(cd) : fabs(TT);
        if (k5 == 4 && q < 3) s = kt_thr[q], sa = fabs(kt_thr[q]);
        for (int k = 0; k < 32; k++) {
            if (k5 == 4 && q < 3 && (k == 13 || k == 14)) continue;  /* kthr: m.y's cross slots left out too */
            if (k5 && q < 3 && (k == 16 || k == 17)) continue;  /* the products the 5-product form leaves out */
            const double p = ray[k] * slot[q][k];
            s += p;
            sa += fabs(p);
        }
        qv[q] = (float)s;
        qe[q] = (float)(31.0 * 0x1p-24 * sa) + 0x1p-149f;
    }
    float Y;
    if (ymma) {
        /* sweep_mfma<ymma>: Y is the -tn record (slot row 3) times the ray
         * fragment (-w, -1) with w = o + bk d (bk finite), or (-Bmax d, 0)
         * (bk = inf: Y = Bmax d.N = -s Bmax det, the sign test) */
        const int fin = bestK <= Bmax;
        const float w[3] = {fin ? fmaf(bestK, d.x, o.x) : Bmax * d.x, fin ? fmaf(bestK, d.y, o.y) : Bmax * d.y,
                            fin ? fmaf(bestK, d.z, o.z) : Bmax * d.z};
        double yr[32];
        for (int k = 0; k < 32; k++) yr[k] = 0.0;
        for (int c = 0; c < 3; c++) {
            const float v = -w[c] * sigma;
            const double hi = to_f16(v);
            const double lo = to_f16(v - (float)hi);
            yr[18 + 3 * c] = hi, yr[19 + 3 * c] = lo, yr[20 + 3 * c] = hi;
        }
        yr[27] = yr[28] = fin ? -sigma : 0.0f;
        double sy = k5 == 4 ? kt_y : TT, sa = k5 == 4 ? fabs(kt_y) : fabs(TT);
        for (int k = 0; k < 29; k++) {  /* slots 29..31 (the cthr threshold) are 0 in this fragment */
            const double p = yr[k] * slot[3][k];
            sy += p;
            sa += fabs(p);
        }
        Y = (float)sy + ((float)(31.0 * 0x1p-24 * sa) + 0x1p-149f);
    } else {
        const float bk = bestK <= Bmax ? bestK : INFINITY;
        Y = fmaf(bk, qv[4] + qe[4], -(qv[3] - qe[3]));
    }
    if (k5 == 2 || k5 == 4)  /* no -tn term; all four shifted terms negative */
        return qv[0] + qe[0] < 0.0f && qv[1] + qe[1] < 0.0f && qv[2] + qe[2] < 0.0f && Y < 0.0f;
    /* k5 = 3: the 5-product form without its -tn term (MfmaSpec::no_tn) */
    const float tn = k5 == 3 ? -INFINITY : qv[3] + qe[3];
    const float t = fmaxf(fmaxf(fmaxf(qv[0] + qe[0], qv[1] + qe[1]), fmaxf(qv[2] + qe[2], tn)), Y);
    return t <= Tl;
}

int main(int argc, char** argv) {
    const long long n = argc > 1 ? atoll(argv[1]) : 1000000;
    s_rng = argc > 2 ? strtoull(argv[2], 0, 10) * 0x9E3779B97F4A7C15ull + 1 : 88172645463325252ull;
    long long accepts = 0, bad_old = 0, bad_new = 0, p_old = 0, p_new = 0, bad_plk = 0, p_plk = 0, p_plk_near = 0, p_old_near = 0;
    long long bad_mfma = 0, p_mfma = 0, n_mfma = 0, p_mfma_near = 0, n_mfma_near = 0;
    long long bad_y = 0, p_y = 0, p_y_near = 0;
    long long bad_k5 = 0, p_k5 = 0, p_k5_near = 0, bad_ct = 0, p_ct = 0, p_ct_near = 0, p_kn = 0, p_kn_near = 0;
    long long bad_kt = 0, p_kt = 0, p_kt_near = 0;
    for (long long it = 0; it < n; it++) {
        const int kind = (int)(next64() % 6);
        const int far = (next64() % 4) == 0;  /* small triangle far from the origin */
        const int wide = (next64() % 8) == 0;  /* coordinates over 1e-12 .. 1e15 (det up to ~1e30) */
        const float scale = wide ? powf(10.0f, 27.0f * uni() - 12.0f) : powf(10.0f, 4.0f * uni() - 2.0f);
        const float tsz = scale * powf(10.0f, -3.0f * uni());
        const float off = far ? powf(10.0f, 5.0f * uni()) * scale : 0.0f;
        const f3 c0 = mk(off * sym() + scale * sym(), off * sym() + scale * sym(), off * sym() + scale * sym());
        const f3 a = c0;
        const f3 b = mk(c0.x + tsz * sym(), c0.y + tsz * sym(), c0.z + tsz * sym());
        const f3 c = mk(c0.x + tsz * sym(), c0.y + tsz * sym(), c0.z + tsz * sym());
        const f3 e0 = sub(b, a), e1 = sub(c, a), nrm = cross(e0, e1);
        /* aim point: inside, on an edge, at a vertex */
        float wu = uni(), wv = uni();
        if (wu + wv > 1.0f) { wu = 1.0f - wu; wv = 1.0f - wv; }
        if (kind == 1) wu = 0.0f;
        if (kind == 2) wv = 0.0f;
        if (kind == 3) wv = 1.0f - wu;
        if (kind == 4) { wu = (float)(next64() & 1); wv = wu > 0.0f ? 0.0f : (float)(next64() & 1); }
        const f3 p = mk(a.x + wu * e0.x + wv * e1.x, a.y + wu * e0.y + wv * e1.y, a.z + wu * e0.z + wv * e1.z);
        f3 o = mk(c0.x + 2.0f * scale * sym(), c0.y + 2.0f * scale * sym(), c0.z + 2.0f * scale * sym());
        if (far && (next64() & 1)) o = mk(2.0f * scale * sym(), 2.0f * scale * sym(), 2.0f * scale * sym());
        f3 d;
        if (kind == 5) {
            /* grazing: direction (nearly) in the triangle's plane */
            const f3 t = normalize(e0);
            const f3 nn = normalize(nrm);
            const float eps = powf(10.0f, -12.0f * uni()) * (float)(next64() & 1 ? 1 : -1);
            d = normalize(mk(t.x + eps * nn.x, t.y + eps * nn.y, t.z + eps * nn.z));
            o = mk(p.x - 3.0f * scale * d.x, p.y - 3.0f * scale * d.y, p.z - 3.0f * scale * d.z);
        } else {
            d = normalize(sub(p, o));
        }
        d = mk(nudge(d.x, ik(2)), nudge(d.y, ik(2)), nudge(d.z, ik(2)));
        o = mk(nudge(o.x, ik(3)), nudge(o.y, ik(3)), nudge(o.z, ik(3)));
        const Q q = quantities(o, d, a, e0, e1, nrm);
        float best;
        const int bk = (int)(next64() % 4);
        if (bk == 0) {
            best = 1e38f;
        } else {
            const float dst = q.det != 0.0f ? q.tnum * (1.0f / q.det) : 1.0f;
            best = bk == 1 ? nudge(fabsf(dst), ik(4)) : fabsf(dst) * (0.5f + uni());
            if (!(best > 0.0f) || isinf(best) || isnan(best)) best = 1e38f;
        }
        const float bestK = best * 1.0009765625f;
        const int ex = exact_updates(q, best);
        const int fo = pass_old(q, bestK), fn = pass_new(q, bestK);
        float rec[16], A;
        /* an out-of-range triangle keeps its all-zero record (always passes);
         * the scene's A is at least this triangle's |a| */
        (void)plk_record(a, e0, e1, nrm, rec, &A);
        if (fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) <= 0x1p20f) {
            const int fp = pass_plk(o, d, rec, A, bestK);
            p_plk += fp;
            if (ex && !fp) bad_plk++;
            if (!far) p_plk_near += fp, p_old_near += fo;
        }
        /* matrix filter: rays in its range (|o| <= 2^20, |d| <= 1.0001); the
         * wave's other rays and the scene's other triangles may be larger */
        if (fmaxf(fmaxf(fabsf(o.x), fabsf(o.y)), fabsf(o.z)) <= 0x1p20f &&
            fmaxf(fmaxf(fabsf(d.x), fabsf(d.y)), fabsf(d.z)) <= 1.0001f) {
            double slot[MQ][32], tau;
            float Am;
            const int inr = mfma_record(a, e0, e1, nrm, slot, &tau, &Am);
            const int wk = (int)(next64() % 4);
            const float Ow = wk == 1 ? 0x1p20f * uni() : wk == 2 ? 2.0f * scale * uni() : 0.0f;
            const float Mw = wk == 3 ? 0x1p20f * uni() : 0.0f;
            const float As = inr ? fmaxf(Am, (next64() % 3) == 0 ? 0x1p20f * uni() : 0.0f) : 0x1p20f;
            const int fm = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 0, 0x1p-10f, 0);
            const int fy = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 1, YMMA_TS, 0);
            const int f5 = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 1, YMMA_TS, 1);
            p_k5 += f5;
            if (ex && !f5) bad_k5++;
            if (!far && !wide && wk == 0 && inr) p_k5_near += f5;
            const int fc = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 1, YMMA_TS, 2);
            const int fk = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 1, YMMA_TS, 3);
            p_kn += fk;
            if (!far && !wide && wk == 0 && inr) p_kn_near += fk;
            p_ct += fc;
            if (ex && !fc) bad_ct++;
            const int ft = pass_mfma(o, d, slot, tau, As, Ow, Mw, bestK, 1, YMMA_TS, 4);
            p_kt += ft;
            if (ex && !ft) bad_kt++;
            if (!far && !wide && wk == 0 && inr) p_kt_near += ft;
            if (!far && !wide && wk == 0 && inr) p_ct_near += fc;
            n_mfma++;
            p_mfma += fm;
            p_y += fy;
            if (!far && !wide && wk == 0 && inr) n_mfma_near++, p_mfma_near += fm, p_y_near += fy;
            if (ex && !fm) bad_mfma++;
            if (ex && !fy) bad_y++;
        }
        accepts += ex;
        if (!wide) {  /* pass counts (filter efficiency) at ordinary scales only */
            p_old += fo;
            p_new += fn;
        }
        if (ex && !fo) bad_old++;
        if (ex && !fn) bad_new++;
    }
    printf("%lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld"
           " %lld %lld %lld\n",
           n, accepts, bad_old, bad_new, p_old, p_new, bad_plk, p_plk, bad_mfma, p_mfma, n_mfma, p_mfma_near,
           n_mfma_near, bad_y, p_y, p_y_near, bad_k5, p_k5, p_k5_near, bad_ct, p_ct, p_ct_near, p_kn, p_kn_near,
           bad_kt, p_kt, p_kt_near);
    fprintf(stderr, "near-origin draws: pass_old %lld pass_plk %lld\n", p_old_near, p_plk_near);
    return 0;
}
