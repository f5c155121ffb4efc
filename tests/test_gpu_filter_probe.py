"""The matrix filter's exactness argument, measured on the hardware it depends on.

render_mfma skips the reference's Moller-Trumbore test (compute.glsl:302-340)
for every (ray, triangle) pair whose filter term exceeds T (rt2_mfma.h); the
safety argument ("The matrix filter") assumes f16 x f16 products and
an f32 accumulation within 31 * 2^-24 * sum|p| in any order.  Here the real
v_mfma_f32_16x16x32_f16 (render_mfma's 16x16 form) and v_mfma_f32_32x32x16_f16
(the k16 form) run on the exact operand fragments the product sweeps build
(rt2_mfma_probe: same scales, LDS rows, records and instructions) over
adversarial rays and triangles (tests/filter_probe_lib.py), and the terms are
compared with a binary64 evaluation on the host:
  - accumulation error vs the exact sum of the same f16 operands <= the
    assumed bound (and the observed worst case is recorded);
  - total error vs the ideal filter quantity well inside T;
  - conservativeness end to end: every pair the reference accepts (the device's
    mt_exact, bit-identical to the oracle) passes the filter.
RT2_PROBE_OUT=<file> writes the measured statistics as JSON
(profiles/r03_filter_probe.json).  Then a near-threshold scene (shared edges
hit dead on, coplanar near-duplicate triangles, stacked planes 2e-6 apart so
hits land near dst = 1e-6, grazing views) is rendered by every product
matrix-filter variant and compared with the oracle bit for bit.
"""
import json
import os

import numpy as np
import pytest

import filter_probe_lib as fpl
from conftest import EXPERIMENTS, require_variant
from test_gpu_parity import assert_exact, oracle_mean

pytestmark = pytest.mark.gpu

KINDS = ["unit", "far", "tiny", "mixed"]
_results = {}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return torch


def _tri_array(rt2mod, V):
    t = np.zeros(len(V), dtype=rt2mod.TRI_DTYPE)
    t["a"][:, :3], t["b"][:, :3], t["c"][:, :3] = V[:, 0], V[:, 1], V[:, 2]
    return t


def _materials(rt2mod):
    sd = rt2mod.SceneData()
    sd.add_material(rt2mod.Material.diffuse((0.8, 0.8, 0.8)))
    return sd.materials()


@pytest.mark.parametrize("layout", [0, 1, 2], ids=["f16x32", "k16", "k5"])
@pytest.mark.parametrize("kind", KINDS)
def test_filter_terms_on_hardware(rt2mod, torch_cuda, kind, layout):
    rng = np.random.default_rng(100 + KINDS.index(kind))
    V, rays = fpl.scene_and_rays(kind, rng)
    scene = rt2mod.Scene(triangles=_tri_array(rt2mod, V), materials=_materials(rt2mod))
    tri = scene.export(0, np.float32).reshape(-1, 12)[:len(V)]
    coef, tau, ok = fpl.coefs(tri)
    if layout == 0:
        B = fpl.records_16x16(scene.export(1, np.uint16), len(V))
        T_tau = scene.export(2, np.float32)
    else:
        B = fpl.records_k16(scene.export(3, np.uint16), len(V))
        T_tau = scene.export(4, np.float32)
    bnd = None
    if layout == 2:
        # the device's k5 bounds are the records' largest |slot 16|, |slot 17| of U, -V, X
        dev = scene.export(5, np.float32).reshape(-1, 2)[:len(V)]
        bnd = fpl.k5_bounds(B)
        np.testing.assert_array_equal(dev[:, 0], bnd[0])
        np.testing.assert_array_equal(dev[:, 1], bnd[1])
    # the device's records are the host's coefficients split into f16 hi/lo slots
    np.testing.assert_array_equal(T_tau[:len(V)], tau.astype(np.float32))
    hi = (coef * tau[:, None, None]).astype(np.float32).astype(np.float16).astype(np.float64)
    np.testing.assert_array_equal(B[:, :4, 0:27:3], hi[:, :4, :9])
    terms, frags, rinfo, accept = scene.mfma_probe(layout, rays)
    st, viol = fpl.analyse(terms, frags, rinfo, accept, B, coef, tau, rays, T_tau, bnd)
    st["triangles_in_range"] = int(ok.sum())
    _results[f"{kind}/{['f16x32', 'k16', 'k5'][layout]}"] = st
    assert st["rays_in_range"] >= len(rays) // 2
    assert st["accepted_pairs"] > 0
    assert st["violations"] == 0, f"reference-accepted pairs rejected by the filter: {viol[:10]}"
    assert st["acc_err_max_in_2^-24_sum_abs"] <= st["acc_err_bound_assumed"], st
    assert st["total_err_max_over_T"] < 0.5, st
    # padding triangles never pass
    n_pad = terms.shape[1]
    if n_pad > len(V):
        pad_bits = terms[rinfo[:, 0] == 1.0, len(V):, :].view(np.int32).max(-1)
        Tl = (T_tau[None, len(V):] * rinfo[rinfo[:, 0] == 1.0, 2][:, None]).astype(np.float32)
        assert (pad_bits > Tl.view(np.int32)).all()


@pytest.mark.parametrize("kind", KINDS)
def test_filter_cthr_on_hardware(rt2mod, torch_cuda, kind):
    """MfmaSpec::cthr on the hardware: the threshold product TT is -Tl'' as
    constructed (within 2^-12 of the exact sum of its three exact products)
    and beyond the 5-product threshold Tl'; the shifted terms are their f16
    products' exact sum plus TT within the assumed accumulation bound; every
    pair the reference accepts has all four shifted terms negative."""
    rng = np.random.default_rng(200 + KINDS.index(kind))
    V, rays = fpl.scene_and_rays(kind, rng)
    scene = rt2mod.Scene(triangles=_tri_array(rt2mod, V), materials=_materials(rt2mod))
    B = fpl.records_k16(scene.export(3, np.uint16), len(V))
    T_tau = scene.export(4, np.float32)
    dev = scene.export(5, np.float32).reshape(-1, 2)[:len(V)]
    bnd = fpl.k5_bounds(B)
    np.testing.assert_array_equal(dev[:, 0], bnd[0])
    # the -tn record's threshold slots: -tau, -CH, -CL
    np.testing.assert_array_equal(B[:, 3, 29], -T_tau[:len(V)].astype(np.float64))
    np.testing.assert_array_equal(B[:, 3, 30], -bnd[0].astype(np.float64))
    np.testing.assert_array_equal(B[:, 3, 31], -bnd[1].astype(np.float64))
    terms, frags, rinfo, accept = scene.mfma_probe(3, rays)
    st, viol = fpl.analyse_cthr(terms, frags, rinfo, accept, B, None, T_tau, bnd)
    _results[f"{kind}/cthr"] = st
    print(json.dumps(st, indent=1))
    assert st["rays_in_range"] >= len(rays) // 2
    assert st["accepted_pairs"] > 0
    assert st["violations"] == 0, f"reference-accepted pairs rejected by the cthr filter: {viol[:10]}"
    assert st["tt_over_Tl_min"] > 1.0, st
    assert st["acc_err_max_in_2^-24_sum_abs"] <= st["acc_err_bound_assumed"], st
    # the matrix core's sum of the three threshold products: up to 2^-18.6 below
    # the exact sum on this data (measured; smaller products lose low bits in
    # the alignment), which the 2^-8 pad covers many times over
    assert st["tt_rel_err_max"] <= 2.0 ** -12, st


@pytest.mark.parametrize("kind", KINDS)
def test_filter_cthr_perm_on_hardware(rt2mod, torch_cuda, kind):
    """The operand path the cthr kernels (round 5's 293 / 282 / 298) use: the
    fragments built in registers by frag_pair (v_permlane32_swap), not read
    from LDS rows.  The MFMA must see exactly the row's slots, and the layout-3
    checks (TT, accumulation, conservativeness) must hold on those terms."""
    rng = np.random.default_rng(200 + KINDS.index(kind))
    V, rays = fpl.scene_and_rays(kind, rng)
    scene = rt2mod.Scene(triangles=_tri_array(rt2mod, V), materials=_materials(rt2mod))
    B = fpl.records_k16(scene.export(3, np.uint16), len(V))
    T_tau = scene.export(4, np.float32)
    bnd = fpl.k5_bounds(B)
    terms, frags, rinfo, accept = scene.mfma_probe(4, rays)
    live = rinfo[:, 0] == 1.0
    mism = fpl.perm_fragments_match(frags, live)
    st, viol = fpl.analyse_cthr(terms, np.ascontiguousarray(frags[:, :48]), rinfo, accept, B, None, T_tau, bnd)
    st["fragment_slot_mismatches"] = mism
    _results[f"{kind}/cthr_perm"] = st
    print(json.dumps(st, indent=1))
    assert mism == 0
    assert st["rays_in_range"] >= len(rays) // 2 and st["accepted_pairs"] > 0
    assert st["violations"] == 0, f"reference-accepted pairs rejected: {viol[:10]}"
    assert st["tt_over_Tl_min"] > 1.0, st
    assert st["acc_err_max_in_2^-24_sum_abs"] <= st["acc_err_bound_assumed"], st


@pytest.mark.parametrize("layout", [5, 6], ids=["wave_w", "lane_w"])
@pytest.mark.parametrize("kind", KINDS)
def test_filter_kthr_on_hardware(rt2mod, torch_cuda, kind, layout):
    """MfmaSpec::kthr (the threshold in the K-slots) on the hardware, with the
    shipping frag_pair operand path, the B slot's ray factor W the wave's
    maximum (layout 5) or each ray's own (layout 6, kt_lane_w): the kt records and register fragments are
    as specified, the terms are their 16 f16 products' exact sum within the
    assumed accumulation bound, and every reference-accepted pair passes."""
    rng = np.random.default_rng(300 + KINDS.index(kind))
    V, rays = fpl.scene_and_rays(kind, rng)
    scene = rt2mod.Scene(triangles=_tri_array(rt2mod, V), materials=_materials(rt2mod))
    B16 = fpl.records_k16(scene.export(3, np.uint16), len(V))
    Bkt = fpl.records_kt(scene.export(6, np.uint16), len(V))
    T_tau = scene.export(4, np.float32)
    terms, frags, rinfo, accept = scene.mfma_probe(layout, rays)
    st, viol = fpl.analyse_kt(terms, frags, rinfo, accept, Bkt, B16, T_tau, lane_w=layout == 6)
    _results[f"{kind}/kthr" + ("_lane_w" if layout == 6 else "")] = st
    print(json.dumps(st, indent=1))
    assert st["record_slot_mismatches"] == 0 and st["fragment_slot_mismatches"] == 0, st
    assert st["rays_in_range"] >= len(rays) // 2 and st["accepted_pairs"] > 0
    assert st["violations"] == 0, f"reference-accepted pairs rejected by the kthr filter: {viol[:10]}"
    assert st["acc_err_max_in_2^-24_sum_abs"] <= st["acc_err_bound_assumed"], st


def test_write_probe_summary():
    out = os.environ.get("RT2_PROBE_OUT")
    if not out or not _results:
        pytest.skip("RT2_PROBE_OUT not set")
    summary = {
        "what": "matrix-filter terms on gfx950 vs binary64 (tests/test_gpu_filter_probe.py)",
        "T": "2^-12 (Omax + A + 1) sigma tau (MfmaSpec::tshift = 12)",
        "worst": {
            "acc_err_max_in_2^-24_sum_abs": max(v["acc_err_max_in_2^-24_sum_abs"] for v in _results.values()),
            "total_err_max_over_T": max(v.get("total_err_max_over_T", 0.0) for v in _results.values()),
            "violations": sum(v["violations"] for v in _results.values()),
            "accepted_pairs": sum(v["accepted_pairs"] for v in _results.values()),
            "accepted_within_T_of_a_boundary": sum(v.get("accepted_within_T_of_a_boundary", 0) for v in _results.values()),
            "cthr_tt_rel_err_max": max((v["tt_rel_err_max"] for v in _results.values() if "tt_rel_err_max" in v),
                                       default=None),
            "cthr_tt_over_Tl_min": min((v["tt_over_Tl_min"] for v in _results.values() if "tt_over_Tl_min" in v),
                                       default=None),
        },
        "cases": _results,
    }
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        json.dump(summary, f, indent=1)


def near_threshold_scene(rt2mod):
    """Grazing and edge-on geometry around a light: a tessellated floor whose
    shared edges and vertices fall on pixel rays, its coplanar near-duplicate
    (1e-6 perturbed) copy, a stack of parallel plates 2e-6 apart (hits near
    the dst <= 1e-6 cut after a bounce), and a wall seen almost edge-on."""
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    diff = sd.add_material(M.diffuse((0.8, 0.75, 0.7)))
    light = sd.add_material(M.light((1, 1, 1), 6.0))
    mirror = sd.add_material(M.specular((0.9, 0.9, 0.9), (1, 1, 1), 1.0, 1.0))
    rng = np.random.default_rng(7)
    tris = []
    step = 0.5
    for i in range(-6, 6):
        for j in range(-6, 6):
            x0, z0 = i * step, -4.0 + j * step
            p = [(x0, 0.0, z0), (x0 + step, 0.0, z0), (x0 + step, 0.0, z0 + step), (x0, 0.0, z0 + step)]
            tris.append((p[0], p[2], p[1], diff))
            tris.append((p[0], p[3], p[2], diff))
    dup = [(tuple(np.float32(np.array(a) + rng.normal(0, 1e-6, 3))), b, c, mirror) for a, b, c, _ in tris[::3]]
    tris += dup
    for k in range(4):  # stacked plates, 2e-6 apart
        y = 1.0 + 2e-6 * k
        tris.append(((-1.0, y, -3.0), (1.0, y, -3.0), (1.0, y, -1.0), diff if k % 2 else mirror))
        tris.append(((-1.0, y, -3.0), (1.0, y, -1.0), (-1.0, y, -1.0), diff))
    tris.append(((3.0, -1.0, -8.0), (3.0 + 1e-4, 6.0, -8.0), (3.0 + 2e-4, -1.0, 2.0), diff))  # wall almost edge-on
    tris.append(((-2.0, 4.0, -5.0), (2.0, 4.0, -5.0), (0.0, 4.0, -2.0), light))
    tris.append(((-2.0, 4.0, -5.0), (0.0, 4.0, -2.0), (2.0, 4.0, -5.0), light))
    for a, b, c, m in tris:
        sd.add_triangle(a, b, c, m)
    return sd


# the product's matrix-filter kernels, and in an experiment build its A/B variants too
NEAR_THRESHOLD_VARIANTS = [227, 380, 353, 354, 355, 356] + (
    [351, 370, 293, 342, 344, 345, 346, 228, 231, 233, 212, 213, 217, 260, 261, 262, 263, 243, 250, 252, 280, 282, 298, 320,
     321, 322, 323, 325, 326, 329, 330, 332, 336, 337, 340, 347, 348, 349, 350, 352, 368, 369, 381, 382, 387, 388, 389, 391] if EXPERIMENTS else [])


@pytest.mark.parametrize("variant", NEAR_THRESHOLD_VARIANTS)
def test_near_threshold_scene_bit_exact(rt2mod, oraclemod, torch_cuda, variant):
    require_variant(rt2mod, variant)
    sd = near_threshold_scene(rt2mod)
    u = rt2mod.offline_uniforms(64, 48, 8, 4, sd.num_triangles)
    u.cameraPos.x, u.cameraPos.y, u.cameraPos.z = 0.0, 0.5, 4.0  # low over the floor: grazing rays
    scene = rt2mod.Scene(sd, 0)
    scene.set_variant(variant)
    img = scene.render_host(u, 0, 2)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(48), 0, 2)
    assert_exact(img, ref, f"near-threshold scene, variant {variant}")
