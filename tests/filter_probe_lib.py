"""Host half of the matrix-filter probe (rt2_mfma_probe): adversarial scenes and
rays, and the binary64 evaluation the hardware's filter terms are measured
against.  Used by tests/test_gpu_filter_probe.py (needs the GPU) and, for the
pure-numpy parts, by tests/test_filter_exactness.py.

What is measured, per (ray, triangle) pair and filter term q (U, -V, X, -tn, Y):
  hw      the term v_mfma_f32_16x16x32_f16 / v_mfma_f32_32x32x16_f16 returned,
          from the exact operand fragments the product sweeps build;
  exact   sum over the 32 k-slots of a_k * b_k of those same f16 operands, in
          binary64 (each product exact; 29 products summed to ~2^-48 relative);
  ideal   the filter quantity itself, sum over the 10 coefficients (binary64,
          as prep_mfma computes them) times the f32 ray vector (d, m, o, 1)
          scaled by sigma * tau: what hi/lo f16 splitting approximates.
The DESIGN.md error budget ("The matrix filter") assumes
  |hw - exact| <= 31 * 2^-24 * sum_k |a_k b_k|      (f32 accumulation, any order)
and a total |hw - ideal| (representation + accumulation) of about 0.31 T.  The
end-to-end property is conservativeness: every pair the reference accepts
(mt_exact: compute.glsl:302-340 with the ray's bound) has all five terms <= T.
"""
import numpy as np

Q_NAMES = ("U", "-V", "X", "-tn", "Y")
KMFMA_C = np.float64(1.0009765625)


def coefs(tri12):
    """(n, 12) pre-transformed triangles -> coef (n, 5, 10) and tau (n,), the
    binary64 arithmetic of mfma_coefs (rt2_mfma.h); out-of-range triangles get
    zeros (always pass), as on the device."""
    t = tri12.astype(np.float32)
    a, e0, e1, nn = t[:, 0:3], t[:, 3:6], t[:, 6:9], t[:, 9:12]
    edges = np.concatenate([e0, e1, nn], axis=1)
    ax = np.abs(edges)
    ok = (np.abs(a) <= 2.0 ** 20).all(1) & ((edges == 0) | ((ax >= 2.0 ** -100) & (ax <= 2.0 ** 20))).all(1)
    M = ax.max(1)
    ok &= M >= 2.0 ** -30
    _, ex = np.frexp(np.where(M > 0, M, 1.0).astype(np.float32))
    s = np.ldexp(1.0, 1 - ex.astype(np.int64))[:, None]
    E0, E1, N = s * e0.astype(np.float64), s * e1.astype(np.float64), s * nn.astype(np.float64)
    A = a.astype(np.float64)

    def cross(x, y):
        return np.stack([x[:, 1] * y[:, 2] - x[:, 2] * y[:, 1], x[:, 2] * y[:, 0] - x[:, 0] * y[:, 2],
                         x[:, 0] * y[:, 1] - x[:, 1] * y[:, 0]], 1)

    P0, P1 = cross(A, E0), cross(A, E1)
    AN = A[:, 0] * N[:, 0] + A[:, 1] * N[:, 1] + A[:, 2] * N[:, 2]
    c = np.zeros((len(t), 5, 10))
    c[:, 0, 0:3], c[:, 0, 3:6] = -P1, E1
    c[:, 1, 0:3], c[:, 1, 3:6] = P0, -E0
    c[:, 2, 0:3], c[:, 2, 3:6] = P1 - P0 + KMFMA_C * N, E0 - E1
    c[:, 3, 6:9], c[:, 3, 9] = -N, AN
    c[:, 4, 0:3] = N
    mx = np.abs(c).reshape(len(t), -1).max(1)
    _, e2 = np.frexp(np.where(mx > 0, mx, 1.0))
    tau = np.ldexp(1.0, 14 - e2.astype(np.int64))
    c[~ok] = 0.0
    tau[~ok] = 1.0
    return c, tau, ok


def records_16x16(rec, n_tris):
    """render_mfma records ([16-group][5][64][8] f16) -> B slots (n_tris, 5, 32)."""
    r = rec.view(np.float16).reshape(-1, 5, 4, 16, 8)        # [G, q, s>>3, t, s&7]
    return r.transpose(0, 3, 1, 2, 4).reshape(-1, 5, 32)[:n_tris].astype(np.float64)


def records_k16(rec, n_tris):
    """sweep_k16 records ([32-group][7 ops][64][8] f16) -> B slots (n_tris, 5, 32)
    (quantity 4, the FMA form's dn, is not stored: zeros)."""
    r = rec.view(np.float16).reshape(-1, 7, 2, 32, 8)        # [G, op, k8, t, j]
    ops = r.transpose(0, 3, 1, 2, 4).reshape(-1, 7, 16)[:n_tris].astype(np.float64)
    B = np.zeros((len(ops), 5, 32))
    for q in range(3):
        B[:, q, :16], B[:, q, 16:] = ops[:, 2 * q], ops[:, 2 * q + 1]
    B[:, 3, 16:] = ops[:, 6]
    return B


def fma32(x, y, z):
    """fmaf for float32 arrays via binary64 (x*y exact; one rounding of the sum,
    exact except in double-rounding corner cases)."""
    return (x.astype(np.float64) * y.astype(np.float64) + z.astype(np.float64)).astype(np.float32)


def k5_bounds(B):
    """The k5 form's per-triangle bounds (prep_mfma_k16 bnd_out): the largest
    |slot 16| and |slot 17| of U, -V, X (float32)."""
    return (np.abs(B[:, :3, 16]).max(1).astype(np.float32), np.abs(B[:, :3, 17]).max(1).astype(np.float32))


def analyse(terms, frags, rinfo, accept, B, coef, tau, rays, T_tau, bnd=None):
    """Measures one probe run.  Returns a dict of statistics and the arrays of
    violations (empty when the filter is conservative).  bnd = (CH, CL) per
    triangle: the 5-product form (k5), whose U, -V, X leave out slots 16/17 and
    whose threshold grows by (CH max|ray slot 16| + CL max|ray slot 17|)(1 +
    2^-10), the maxima over the ray's wave of 64 (sweep_k16)."""
    n_tris = accept.shape[1]
    live = rinfo[:, 0] == 1.0
    hw = terms[live][:, :n_tris, :].astype(np.float64)          # (R, T, 5)
    if bnd is not None:
        B = B.copy()
        B[:, :3, 16:18] = 0.0  # the products the k5 form leaves out
        fw = np.abs(frags.astype(np.float32)).reshape(-1, 64, 48)
        zlo = np.repeat(fw[:, :, 16].max(1), 64)[live]
        zhi = np.repeat(fw[:, :, 17].max(1), 64)[live]
        ch, cl = bnd[0][:n_tris], bnd[1][:n_tris]
        Bk = ((ch[None, :] * zlo[:, None] + cl[None, :] * zhi[:, None]) * np.float32(1.0009765625)).astype(np.float32)
    fr = frags[live].astype(np.float64)
    A_main = fr[:, :32]
    A_y = np.concatenate([np.zeros((len(fr), 16)), fr[:, 32:48]], 1)
    exact = np.empty_like(hw)
    sabs = np.empty_like(hw)
    for q in range(4):
        exact[..., q] = A_main @ B[:, q, :].T
        sabs[..., q] = np.abs(A_main) @ np.abs(B[:, q, :]).T
    exact[..., 4] = A_y @ B[:, 3, :].T
    sabs[..., 4] = np.abs(A_y) @ np.abs(B[:, 3, :]).T
    ulp = 2.0 ** -24 * sabs
    acc_err = np.abs(hw - exact)
    acc_ratio = np.where(ulp > 0, acc_err / np.where(ulp > 0, ulp, 1.0), np.where(acc_err > 0, np.inf, 0.0))
    rn_match = float((hw == exact.astype(np.float32).astype(np.float64)).mean())

    # ideal terms: coefficients x sigma-scaled f32 ray vector (d, m, o, 1); Y
    # with w = fma(bk, d, o) (bk <= Bmax) or Bmax * d and constant -1 / 0
    r = rays[live].astype(np.float32)
    o, d = r[:, 0:3], r[:, 4:7]
    sigma, Tw, Bmax = rinfo[live, 1], rinfo[live, 2], rinfo[live, 3]
    m = rinfo[live, 4:7].astype(np.float64)
    bk = rinfo[live, 7]
    v = np.concatenate([d.astype(np.float64), m, o.astype(np.float64), np.ones((len(r), 1))], 1)
    v *= sigma[:, None].astype(np.float64)
    ct = coef * tau[:, None, None]                              # (T, 5, 10)
    ideal = np.einsum("rc,tqc->rtq", v, ct[:, :4, :])
    fin = bk <= Bmax
    w = np.where(fin[:, None], fma32(np.broadcast_to(bk[:, None], d.shape), d, o),
                 (Bmax[:, None] * d).astype(np.float32)).astype(np.float64)
    vy = np.concatenate([np.zeros((len(r), 6)), -w, np.where(fin, -1.0, 0.0)[:, None]], 1) * sigma[:, None]
    ideal_y = vy @ ct[:, 3, :].T
    ideal = np.concatenate([ideal, ideal_y[..., None]], 2)
    Tl = (T_tau[None, :n_tris].astype(np.float32) * Tw[:, None].astype(np.float32)).astype(np.float32)
    dev = np.abs(hw - ideal)
    if bnd is not None:
        dev[..., :3] = np.maximum(dev[..., :3] - Bk[..., None].astype(np.float64), 0.0)  # beyond the k5 bound
    tot_ratio = dev / Tl[..., None].astype(np.float64)
    T0 = Tl
    if bnd is not None:
        Tl = (Tl + Bk).astype(np.float32)  # sweep_k16: Tl += (bnd.x zlo + bnd.y zhi) (1 + 2^-10)

    # conservativeness: accepted => every term <= Tl (the kernels' integer max)
    bits = hw.astype(np.float32).view(np.int32).max(-1)
    passes = bits <= Tl.view(np.int32)
    acc = accept[live]
    violations = np.argwhere(acc & ~passes)
    near = acc & (np.abs(ideal).min(-1) < Tl)                    # accepted within T of a boundary
    out = {
        "rays_in_range": int(live.sum()), "pairs": int(acc.size), "accepted_pairs": int(acc.sum()),
        "accepted_within_T_of_a_boundary": int(near.sum()),
        "filter_pass_frac": float(passes.mean()),
        "acc_err_max_in_2^-24_sum_abs": float(acc_ratio.max()),
        "acc_err_bound_assumed": 31.0,
        "hw_equals_rn_of_exact_frac": rn_match,
        "total_err_max_over_T": float(tot_ratio.max()),
        "total_err_by_term_max_over_T": {Q_NAMES[q]: float(tot_ratio[..., q].max()) for q in range(5)},
        "violations": int(len(violations)),
    }
    if bnd is not None:
        g = (Bk / T0).astype(np.float64)
        out["k5_bound_over_T"] = {"max": float(g.max()), "mean": float(g.mean()), "p99": float(np.percentile(g, 99))}
    return out, violations


def f16_up(v):
    """f16 of v > 0 rounded up, as float64 (rt2_mfma.h f16_up)."""
    v = np.asarray(v, dtype=np.float32)
    h = v.astype(np.float16)
    h = np.where(h.astype(np.float32) < v, np.nextafter(h, np.float16(np.inf)), h)
    return h.astype(np.float64)


def analyse_cthr(terms, frags, rinfo, accept, B, tau, T_tau, bnd):
    """One probe run of MfmaSpec::cthr (layout 3): terms [..., 0:3] and 4 are
    U, -V, X, Y with TT = -Tl'' as their accumulator, terms[..., 3] is TT.
    Checks TT against its construction (the wave's factors padded by 2^-8 and
    rounded up to f16, times the record's -tau, -CH, -CL) and against the
    5-product threshold Tl' it must exceed; the shifted terms' accumulation
    error against the exact sum of their f16 products plus TT; and that every
    reference-accepted pair passes (all four shifted terms negative: the sign
    bit of U & V & X & Y)."""
    n_tris = accept.shape[1]
    live = rinfo[:, 0] == 1.0
    hw = terms[live][:, :n_tris, :].astype(np.float64)
    B = B.copy()
    B[:, :3, 16:18] = 0.0
    fw = np.abs(frags.astype(np.float32)).reshape(-1, 64, 48)
    zlo = np.repeat(fw[:, :, 16].max(1), 64)[live].astype(np.float64)
    zhi = np.repeat(fw[:, :, 17].max(1), 64)[live].astype(np.float64)
    ch, cl = bnd[0][:n_tris].astype(np.float64), bnd[1][:n_tris].astype(np.float64)
    Tw = rinfo[live, 2]
    pad = np.float32(1.00390625)
    tt = T_tau[:n_tris].astype(np.float64)
    Tl2 = (tt[None, :] * f16_up(Tw * pad)[:, None] + ch[None, :] * f16_up(zlo.astype(np.float32) * pad)[:, None]
           + cl[None, :] * f16_up(zhi.astype(np.float32) * pad)[:, None])
    Tl1 = (T_tau[None, :n_tris].astype(np.float32) * Tw[:, None].astype(np.float32)).astype(np.float64) + \
        (ch[None, :] * zlo[:, None] + cl[None, :] * zhi[:, None]) * (1 + 2.0 ** -10)
    TT = hw[..., 3]
    tt_err = np.abs(TT + Tl2) / Tl2
    w = np.unravel_index(np.argmax(tt_err), tt_err.shape)
    r_, t_ = int(w[0]), int(w[1])
    worst = {"TT": float(TT[w]), "Tl2": float(Tl2[w]), "Tl1": float(Tl1[w]),
             "tau": float(tt[t_]), "Tw": float(Tw[r_]), "zlo": float(zlo[r_]), "zhi": float(zhi[r_]),
             "ch": float(ch[t_]), "cl": float(cl[t_]),
             "Tw16": float(f16_up(Tw[r_] * pad)), "zlo16": float(f16_up(np.float32(zlo[r_]) * pad)),
             "zhi16": float(f16_up(np.float32(zhi[r_]) * pad))}
    fr = frags[live].astype(np.float64)
    A_main = fr[:, :32]
    A_y = np.concatenate([np.zeros((len(fr), 16)), fr[:, 32:48]], 1)
    exact = np.empty(hw.shape[:2] + (4,))
    sabs = np.empty_like(exact)
    for j, q in enumerate((0, 1, 2)):
        exact[..., j] = A_main @ B[:, q, :].T
        sabs[..., j] = np.abs(A_main) @ np.abs(B[:, q, :]).T
    exact[..., 3] = A_y @ B[:, 3, :].T
    sabs[..., 3] = np.abs(A_y) @ np.abs(B[:, 3, :]).T
    sh = hw[..., [0, 1, 2, 4]]
    acc_err = np.abs(sh - (exact + TT[..., None]))
    ulp = 2.0 ** -24 * (sabs + np.abs(TT)[..., None])
    acc_ratio = acc_err / np.where(ulp > 0, ulp, 1.0)
    sign = sh.astype(np.float32).view(np.int32) < 0
    passes = sign.all(-1)
    acc = accept[live]
    violations = np.argwhere(acc & ~passes)
    out = {
        "rays_in_range": int(live.sum()), "pairs": int(acc.size), "accepted_pairs": int(acc.sum()),
        "filter_pass_frac": float(passes.mean()),
        "tt_rel_err_max": float(tt_err.max()),
        "tt_worst": worst,
        "tt_over_Tl_min": float((-TT / Tl1).min()),
        "acc_err_max_in_2^-24_sum_abs": float(acc_ratio.max()),
        "acc_err_bound_assumed": 31.0,
        "violations": int(len(violations)),
    }
    return out, violations


def records_kt(rec, n_tris):
    """kthr records ([32-group][4 ops][64][8] f16: U, -V, X first K-half, the
    -tn record's second half) -> slots (n_tris, 4, 16)."""
    r = rec.view(np.float16).reshape(-1, 4, 2, 32, 8)        # [G, op, k8, t, j]
    return r.transpose(0, 3, 1, 2, 4).reshape(-1, 4, 16)[:n_tris].astype(np.float64)


def perm_fragments_match(frags, live):
    """Layouts 4 / 5 write the LDS-row slots (0..47) and the fragments the MFMA
    read after frag_pair (48..79).  For the cthr layout the register main
    fragment must equal the row's first K-half and the Y fragment the row's Y
    slots; returns the mismatching (ray, slot) count."""
    fr = frags[live].astype(np.float32)
    a = fr[:, 48:64] != fr[:, 0:16]
    y = fr[:, 64:80] != fr[:, 32:48]
    return int(a.sum() + y.sum())


def kt_expected_fragments(frags, rinfo, lane_w=False):
    """The kthr fragments (kt_frags / kt_y) recomputed on the host from the LDS
    row slots of the same rays: main K-half = d, m.x (hi lo hi), m.y hi, m.z
    hi, Tw', W'; Y = the row's Y slots with Tw' at slot 29.  Tw' = f16_up(Tw (1
    + 2^-8)); W' = f16_up(W (1 + 2^-8)), W = the wave's largest mw_y + mw_z
    (lane_w: the ray's own), mw_c = max(|hi|, 2^11 |lo|) (float32 arithmetic as
    on the device)."""
    row = frags[:, :48].astype(np.float32)
    pad = np.float32(1.00390625)
    tw = f16_up(rinfo[:, 2].astype(np.float32) * pad)
    mw = (np.maximum(np.abs(row[:, 12]), np.float32(2048.0) * np.abs(row[:, 13])) +
          np.maximum(np.abs(row[:, 15]), np.float32(2048.0) * np.abs(row[:, 16]))).astype(np.float32)
    W = mw if lane_w else np.repeat(mw.reshape(-1, 64).max(1), 64)
    w16 = f16_up(W * pad)
    A = np.concatenate([row[:, 0:13], row[:, 15:16], tw[:, None], w16[:, None]], 1).astype(np.float64)
    Ay = row[:, 32:48].astype(np.float64).copy()
    Ay[:, 13] = tw
    return A, Ay, tw, w16


def analyse_kt(terms, frags, rinfo, accept, Bkt, B16, T_tau, lane_w=False):
    """One probe run of MfmaSpec::kthr (layout 5).  Checks: the records are the
    k16 records' slots with the threshold slots as specified (-tau; -B_q =
    -f16_up(2^-10 max over m.y, m.z of max(|hi|, 2^11 |lo|))); the register
    fragments the MFMA read equal the host's recomputation; the terms equal
    the exact sum of their 16 f16 products within the assumed accumulation
    bound; and every reference-accepted pair has all four terms negative."""
    n_tris = accept.shape[1]
    live = rinfo[:, 0] == 1.0
    tau = T_tau[:n_tris].astype(np.float64)
    rec_bad = 0
    for q in range(3):
        c = B16[:, q, :]
        ct = np.maximum(np.maximum(np.abs(c[:, 12]), 2048.0 * np.abs(c[:, 14])),
                        np.maximum(np.abs(c[:, 15]), 2048.0 * np.abs(c[:, 17]))).astype(np.float32)
        want = np.concatenate([c[:, 0:13], c[:, 15:16], -tau[:, None], -f16_up(ct * np.float32(2.0 ** -10))[:, None]], 1)
        rec_bad += int((Bkt[:, q, :] != want).sum())
    want_t = B16[:, 3, 16:32].copy()
    want_t[:, 13], want_t[:, 14], want_t[:, 15] = -tau, 0.0, 0.0
    rec_bad += int((Bkt[:, 3, :] != want_t).sum())
    A_exp, Ay_exp, tw, w16 = kt_expected_fragments(frags, rinfo, lane_w)
    fr = frags.astype(np.float64)
    frag_bad = int((fr[live, 48:64] != A_exp[live]).sum() + (fr[live, 64:80] != Ay_exp[live]).sum())
    hw = terms[live][:, :n_tris, :].astype(np.float64)
    A, Ay = fr[live, 48:64], fr[live, 64:80]
    exact = np.empty(hw.shape[:2] + (4,))
    sabs = np.empty_like(exact)
    for q in range(3):
        exact[..., q] = A @ Bkt[:, q, :].T
        sabs[..., q] = np.abs(A) @ np.abs(Bkt[:, q, :]).T
    exact[..., 3] = Ay @ Bkt[:, 3, :].T
    sabs[..., 3] = np.abs(Ay) @ np.abs(Bkt[:, 3, :]).T
    sh = hw[..., [0, 1, 2, 4]]
    acc_err = np.abs(sh - exact)
    ulp = 2.0 ** -24 * sabs
    acc_ratio = acc_err / np.where(ulp > 0, ulp, 1.0)
    passes = (sh.astype(np.float32).view(np.int32) < 0).all(-1)
    acc = accept[live]
    violations = np.argwhere(acc & ~passes)
    # how far the K-slot threshold reaches beyond the base threshold tau Tw
    base = tau[None, :] * rinfo[live, 2].astype(np.float64)[:, None]
    thr = -(A[:, None, None, 14] * Bkt[None, :, :3, 14] + A[:, None, None, 15] * Bkt[None, :, :3, 15])  # (R, T, q)
    grow = thr.max(-1) / base
    out = {
        "rays_in_range": int(live.sum()), "pairs": int(acc.size), "accepted_pairs": int(acc.sum()),
        "filter_pass_frac": float(passes.mean()),
        "record_slot_mismatches": rec_bad,
        "fragment_slot_mismatches": frag_bad,
        "acc_err_max_in_2^-24_sum_abs": float(acc_ratio.max()),
        "acc_err_bound_assumed": 31.0,
        "threshold_over_tauTw": {"min": float(grow.min()), "mean": float(grow.mean()),
                                 "p99": float(np.percentile(grow, 99)), "max": float(grow.max())},
        "violations": int(len(violations)),
    }
    return out, violations


def _unit(v):
    return v / np.linalg.norm(v, axis=-1, keepdims=True)


def scene_and_rays(kind, rng, n_tris=448, n_rays=512):
    """Adversarial cases: returns triangle vertices (n, 3, 3) float32 and rays
    (n_rays, 8) float32 {o, best, d, 0}.
      unit  triangles of size 0.1..3 in an 8-unit box;
      far   coordinates near 2^19..2^20 (A and |o| at the filter's range limit);
      tiny  edges of 2^-24..2^-14 (lo halves and products near the f16
            subnormal floor at the largest sigma/tau);
      mixed skinny triangles (one edge 1e-6 of the other) among unit ones.
    Rays aim at points within +-{0, 1e-7, 1e-5, 1e-3} (barycentric) of an edge,
    a vertex or the w = 0 edge of a random triangle, from distances 1e-6..1e2
    of the triangle's scale, a third of them grazing (det down to ~1e-10), with
    bounds best = hit distance x (1 +- {1e-7, 1e-5, 1e-3}) or none."""
    scale = {"unit": 1.0, "far": 64.0, "tiny": 2.0 ** -18, "mixed": 1.0}[kind]
    base = {"unit": 0.0, "far": 2.0 ** 19.5, "tiny": 3.0, "mixed": 0.0}[kind]
    a = rng.uniform(-4, 4, (n_tris, 3)) * (1.0 if kind != "far" else 8.0)
    if kind == "far":
        a += base * rng.choice([-1.0, 1.0], (n_tris, 3)) * rng.uniform(0.5, 0.999, (n_tris, 3)) ** 0.01
    elif kind == "tiny":
        a += base
    e0 = rng.normal(size=(n_tris, 3)) * scale * rng.uniform(0.1, 3, (n_tris, 1))
    e1 = rng.normal(size=(n_tris, 3)) * scale * rng.uniform(0.1, 3, (n_tris, 1))
    if kind == "mixed":
        sk = rng.random(n_tris) < 0.5
        e1[sk] = e0[sk] * (1 + 1e-6 * rng.normal(size=(sk.sum(), 1))) + 1e-6 * rng.normal(size=(sk.sum(), 3))
    V = np.stack([a, a + e0, a + e1], 1).astype(np.float32)
    Vd = V.astype(np.float64)
    t = rng.integers(0, n_tris, n_rays)
    va, vb, vc = Vd[t, 0], Vd[t, 1], Vd[t, 2]
    eps = rng.choice([0.0, 1e-7, -1e-7, 1e-5, -1e-5, 1e-3, -1e-3], n_rays)
    r = rng.random(n_rays)
    where = rng.integers(0, 4, n_rays)                  # edge u=0, edge v=0, edge w=0, vertex
    u = np.where(where == 0, eps, np.where(where == 1, r, np.where(where == 2, r, eps)))
    vv = np.where(where == 0, r, np.where(where == 1, eps, np.where(where == 2, 1 - r + eps, eps)))
    P = va + u[:, None] * (vb - va) + vv[:, None] * (vc - va)
    n = _unit(np.cross(vb - va, vc - va))
    d = _unit(rng.normal(size=(n_rays, 3)))
    d = np.where((np.sum(d * n, 1) > 0)[:, None], -d, d)            # front-facing (det > 0) mostly
    graze = rng.random(n_rays) < 0.33
    tang = _unit(np.cross(n, rng.normal(size=(n_rays, 3))))
    eta = rng.choice([1e-3, 1e-5, 1e-7, 1e-9, -1e-9, -1e-7], n_rays)
    d = np.where(graze[:, None], _unit(tang - eta[:, None] * n), d)
    dist = np.exp(rng.uniform(np.log(1e-6), np.log(1e2), n_rays)) * max(scale, 1e-3)
    o = P - dist[:, None] * d
    if kind == "far":
        o = np.clip(o, -(2.0 ** 20), 2.0 ** 20)
    rel = rng.choice([1e-7, -1e-7, 1e-5, -1e-5, 1e-3, -1e-3], n_rays)
    best = np.where(rng.random(n_rays) < 0.35, 1e38, dist * (1 + rel))
    rays = np.zeros((n_rays, 8), dtype=np.float32)
    rays[:, 0:3], rays[:, 3], rays[:, 4:7] = o, best, d
    return V, rays
