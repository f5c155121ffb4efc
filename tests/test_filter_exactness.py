"""The brute-force kernel's division-free filters never reject a pair the
reference's Möller–Trumbore test accepts (CPU restatement of rt2_sweep.h
mt_pass / mt_pass3 and the per-ray precomputed plk_pass in binary32, and of
the matrix-core filter of rt2_mfma.h: f16 hi/lo slots, exact products, the
f32 accumulation moved by its worst-case error toward rejection; proofs in
DESIGN.md, "Exactness of the filter", "The per-ray filter" and "The matrix
filter").  tests/filter_check/filter_check.c draws random and adversarial
rays (edges, vertices, grazing, best at the hit distance); a tightened
filter mutant shows violations, so the harness is sensitive."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "filter_check", "filter_check.c")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("fc") / "filter_check")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, SRC, "-lm"], check=True)
    return exe


def _run(exe, n, seed):
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    v = list(map(int, out.split()))
    return tuple(v[:8])


def _run_mfma(exe, n, seed):
    """(violations, passes, in-range draws, passes and draws at ordinary scales)
    of the matrix-core filter (rt2_mfma.h)."""
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    return tuple(map(int, out.split()))[8:13]


def _run_mfma_y(exe, n, seed):
    """(violations, passes, passes at ordinary scales) of the matrix-core filter
    whose Y term is a matrix product too (MfmaSpec::ymma), and the same three
    figures for the FMA form, on the same draws."""
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    v = tuple(map(int, out.split()))
    return v[13:16], (v[8], v[9], v[11])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_filters_conservative(checker, seed):
    pairs, accepts, bad_old, bad_new, p_old, p_new, bad_plk, p_plk = _run(checker, 3_000_000, seed)
    assert accepts > pairs // 20          # the adversarial draws do reach the accept region
    assert bad_old == 0 and bad_new == 0  # no accepted pair is filtered out
    assert bad_plk == 0
    assert p_new <= p_old * 1.01          # and the new form filters as much as the old one
    assert p_plk < pairs                  # the per-ray filter does reject (its margin is not everything)


def test_harness_detects_a_wrong_filter(tmp_path):
    src = open(SRC).read()
    old = "return fmaxf(fmaxf(fmaxf(fmaxf(q.U, -q.V), X), -q.tnum), Y) <= B;"
    assert old in src
    mutant = src.replace(old, "return fmaxf(fmaxf(fmaxf(fmaxf(q.U, -q.V), fmaf(-q.det, 1.0f, q.V - q.U)), "
                              "-q.tnum), fmaf(-q.det, best_plain(bestK), q.tnum)) <= 0.0f;")
    mutant = mutant.replace("static int pass_new(", "static float best_plain(float k) { return k / 1.0009765625f; }\n"
                                                    "static int pass_new(")
    p = tmp_path / "mut.c"
    p.write_text(mutant)
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    _, _, bad_old, bad_new, _, _, _, _ = _run(exe, 3_000_000, 1)
    assert bad_old == 0 and bad_new > 0


def test_harness_detects_a_plk_threshold_without_margin(tmp_path):
    """plk_pass with T = 0 (no error margin) filters out accepted pairs."""
    src = open(SRC).read()
    old = "const float T = fmaf(0x1p-13f, O + A, 0x1p-40f);"
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, "const float T = 0.0f;"))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    _, _, _, _, _, _, bad_plk, _ = _run(exe, 3_000_000, 1)
    assert bad_plk > 0


@pytest.mark.parametrize("seed", [4, 5])
def test_matrix_filter_conservative(checker, seed):
    """sweep_mfma's skip decision, for rays inside its range in waves whose
    other rays (and scenes whose other triangles) are up to 2^20 large."""
    bad, passes, draws, p_near, n_near = _run_mfma(checker, 2_000_000, seed)
    assert draws > 1_500_000 and n_near > 100_000
    assert bad == 0
    assert p_near < 0.8 * n_near  # it does reject on ordinary scales (adversarial draws aim at the triangles)


@pytest.mark.parametrize("old,new", [
    ("const float Tw = sigma * (ts * R0);", "const float Tw = sigma * (ts * 0x1p-10f * R0);"),  # margin too thin
    ("const float Cw = -0x1p-14f * sigma;", "const float Cw = 0x1p-14f * sigma;"),  # det bias the wrong way
])
def test_harness_detects_a_wrong_matrix_filter(tmp_path, old, new):
    src = open(SRC).read()
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, new))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    bad, _, _, _, _ = _run_mfma(exe, 1_000_000, 1)
    assert bad > 0


@pytest.mark.parametrize("seed", [6, 7])
def test_matrix_filter_ymma_conservative(checker, seed):
    """sweep_mfma<ymma>: Y = tn - bk det from the -tn record and the ray
    fragment (-(o + bk d), -1), or -Bmax det with no usable bound; no accepted
    pair is skipped, and it skips about as much as the FMA form."""
    (bad, passes, p_near), (bad_fma, passes_fma, p_near_fma) = _run_mfma_y(checker, 2_000_000, seed)
    assert bad == 0 and bad_fma == 0
    assert passes <= passes_fma * 1.05 and p_near <= p_near_fma * 1.05


@pytest.mark.parametrize("old,new", [
    # the distance-bound fragment without its constant slot (Y = o.N + bk d.N, AN dropped)
    ("yr[27] = yr[28] = fin ? -sigma : 0.0f;", "yr[27] = yr[28] = 0.0f;"),
    # the sign test with the wrong sign (Y = +s Bmax det)
    ("fin ? fmaf(bestK, d.x, o.x) : Bmax * d.x", "fin ? fmaf(bestK, d.x, o.x) : -Bmax * d.x"),
])
def test_harness_detects_a_wrong_ymma_filter(tmp_path, old, new):
    src = open(SRC).read()
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, new))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    (bad, _, _), _ = _run_mfma_y(exe, 1_000_000, 1)
    assert bad > 0


def _run_k5(exe, n, seed):
    """(violations, passes, passes at ordinary scales) of the 5-product form
    (MfmaSpec::k5) and the same three figures of the 8-product ymma form, on
    the same draws."""
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    v = tuple(map(int, out.split()))
    return v[16:19], v[13:16]


@pytest.mark.parametrize("seed", [8, 9])
def test_matrix_filter_k5_conservative(checker, seed):
    """The 5-product form: U, -V, X without their m.z slots 16/17, the
    threshold raised by the per-(wave, triangle) bound of what is left out.
    No accepted pair is skipped, and it passes at most a few percent more
    pairs than the 8-product form on the same draws."""
    (bad, passes, p_near), (bad_y, passes_y, p_near_y) = _run_k5(checker, 2_000_000, seed)
    assert bad == 0 and bad_y == 0
    assert passes_y <= passes <= passes_y * 1.03 and p_near <= p_near_y * 1.03


def _run_cthr(exe, n, seed):
    """(violations, passes, passes at ordinary scales) of the threshold-in-
    the-accumulator form (MfmaSpec::cthr) and (violations of the 5-product
    form, passes and passes at ordinary scales of that form without its -tn
    term, the one cthr restates), on the same draws."""
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    v = tuple(map(int, out.split()))
    return v[19:22], (v[16], v[22], v[23])


@pytest.mark.parametrize("seed", [10, 11])
def test_matrix_filter_cthr_conservative(checker, seed):
    """MfmaSpec::cthr: the threshold enters every term through the
    accumulator (TT = -(tau Tw + CH ML + CL MH), its factors padded and
    rounded up to f16) and a pair passes iff all four shifted terms are
    negative.  No accepted pair is skipped, and it passes no more than a
    percent beyond the 5-product form it restates (the pad)."""
    (bad, passes, p_near), (bad5, passes5, p_near5) = _run_cthr(checker, 2_000_000, seed)
    assert bad == 0 and bad5 == 0
    assert passes5 <= passes <= passes5 * 1.01 and p_near <= p_near5 * 1.01


def test_harness_detects_cthr_without_its_threshold(tmp_path):
    """With TT = 0 (no threshold in the accumulator) the sign test skips
    accepted pairs: the harness sees it."""
    src = open(SRC).read()
    old = "        TT = -s3 * (1.0 - 0x1p-12);"
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, "        TT = 0.0 * s3;"))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    (bad, _, _), _ = _run_cthr(exe, 1_000_000, 1)
    assert bad > 0


def test_harness_detects_k5_without_its_bound(tmp_path):
    """Leaving out the m.z slots without raising the threshold skips accepted
    pairs: the bound is necessary, and the harness sees its absence."""
    src = open(SRC).read()
    old = "    } else if (k5) {\n        float ch"
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, "    } else if (0) {\n        float ch"))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    (bad, _, _), _ = _run_k5(exe, 1_000_000, 1)
    assert bad > 0


def _run_kt(exe, n, seed):
    """(violations, passes, passes at ordinary scales) of the threshold-in-the-
    K-slots form (MfmaSpec::kthr) and the same three of the cthr form, on the
    same draws."""
    out = subprocess.run([exe, str(n), str(seed)], check=True, capture_output=True, text=True).stdout
    v = tuple(map(int, out.split()))
    return v[24:27], v[19:22]


@pytest.mark.parametrize("seed", [12, 13])
def test_matrix_filter_kthr_conservative(checker, seed):
    """MfmaSpec::kthr: U, -V, X drop the m.y and m.z cross slots, and two
    k-slots carry -tau Tw' and -B_q W' (the bound of what is dropped); Y
    carries -tau Tw'.  No accepted pair is skipped, and it passes at most a
    few percent more pairs than the cthr form (measured: ~1 %)."""
    (bad, passes, p_near), (bad_c, passes_c, p_near_c) = _run_kt(checker, 2_000_000, seed)
    assert bad == 0 and bad_c == 0
    assert passes <= passes_c * 1.03 and p_near <= p_near_c * 1.03


@pytest.mark.parametrize("old,new", [
    # the bound of the dropped m.y / m.z cross products left out of the threshold
    ("kt_thr[q] = -(tau * tw + f16_up(ct * 0x1p-10f) * w16);", "kt_thr[q] = -(tau * tw + 0.0 * ct * w16);"),
    # Y without its threshold slot
    ("kt_y = -tau * tw;", "kt_y = 0.0 * tw;"),
])
def test_harness_detects_kthr_without_its_bounds(tmp_path, old, new):
    src = open(SRC).read()
    assert old in src
    p = tmp_path / "mut.c"
    p.write_text(src.replace(old, new))
    exe = str(tmp_path / "mut")
    subprocess.run(["gcc", "-O2", "-std=c11", "-ffp-contract=off", "-o", exe, str(p), "-lm"], check=True)
    (bad, _, _), _ = _run_kt(exe, 1_000_000, 1)
    assert bad > 0
