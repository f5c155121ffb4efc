"""Parity of the A/B kernel variants of the experiment build (make
EXPERIMENTS=1; collected only with RT2_LIB=exp, see conftest.py): the per-ray
precomputed filter (plk) and the team tail mode.  Same bar as the product
kernels: bit-exact against the CPU oracle."""
import numpy as np
import pytest

from conftest import require_variant
from test_gpu_parity import assert_exact, oracle_mean, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

PLK_VARIANTS = [74, 76, 79, 80]


def plk_info(rt2mod, scene):
    import ctypes as C
    ok, A, n_out = C.c_int(), C.c_float(), C.c_int()
    assert rt2mod.lib().rt2_scene_plk_info(scene._p, C.byref(ok), C.byref(A), C.byref(n_out)) == 0
    return ok.value, A.value, n_out.value


@pytest.mark.parametrize("variant", PLK_VARIANTS)
def test_plk_filter_diverse_materials(rt2mod, oraclemod, torch_cuda, variant):
    """Per-ray precomputed filter (sweep_plk) on glass/mirror/checker/glossy
    paths: every direction a path makes passes the per-segment range check."""
    require_variant(rt2mod, variant)
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    red = sd.add_material(M.diffuse((1, 0, 0)))
    green = sd.add_material(M.diffuse((0, 1, 0)))
    white = sd.add_material(M.diffuse((1, 1, 1)))
    light = sd.add_material(M.light((1, 1, 1), 15.0))
    glass = sd.add_material(M.glass((0.9, 0.95, 1.0), 1.5))
    mirror = sd.add_material(M.specular((1, 1, 1), (1, 1, 1), 1.0, 1.0))
    checker = sd.add_material(M.checker(8.0))
    metal = sd.add_material(M.specular((0.8, 0.6, 0.3), (1, 1, 1), 0.7, 0.4))
    sd.create_diverse_cornell_box(10.0, red, green, white, light, glass, mirror, checker, metal)
    sd.add_cube((0.0, -2.0, 0.0), (1.0, 1.0, 1.0), (0.3, 0.2, 0.1), 7)
    W, H = 96, 64
    u = rt2mod.offline_uniforms(W, H, 12, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    ok, A, n_out = plk_info(rt2mod, scene)
    assert ok == 1 and n_out == 0 and A > 0
    scene.set_variant(variant)
    img = scene.render_host(u, 0, 2)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 2)
    assert_exact(img, ref, f"plk variant {variant} diverse")
    assert scene.stats().segments == segs


def _with_extra_triangles(sd, extra):
    tris = np.concatenate([sd.triangles(), np.zeros(len(extra), dtype=sd.triangles().dtype)])
    for k, (a, b, c) in enumerate(extra):
        t = tris[len(tris) - len(extra) + k]
        t["a"][:3], t["b"][:3], t["c"][:3] = a, b, c
        t["materialIndex"] = 0
    return tris


def test_plk_out_of_range_triangles(rt2mod, oraclemod, config_scene, torch_cuda):
    """Triangles outside the filter's validated range (|a| > 2^20, edges
    < 2^-30, a component below 2^-100, degenerate) get always-pass records and
    are decided by the exact test; with more than 1/64 of them the scene keeps
    the exact-intermediate filter.  Both renders match the oracle bit for bit."""
    require_variant(rt2mod, 76)
    sd, spec = config_scene("B")
    extra = [((3e6, 0, -3e6), (3e6, 1, -3e6), (3e6, 0, -3e6 + 1)),        # |a| > 2^20
             ((0.1, 2.0, 3.0), (0.1 + 1e-10, 2.0, 3.0), (0.1, 2.0 + 1e-10, 3.0)),  # microscopic
             ((-2, 1e-32, 1), (2, 1e-32, 1), (2, 2e-32, 1)),              # e1.y = 1e-32 < 2^-100
             ((1, 1, 1), (1, 1, 1), (1, 1, 1)),                             # degenerate
             ((-4, 9.5, -4), (4, 9.5, -4), (0, 9.5, 4))]                   # ordinary, hit by the sky-bound rays
    W, H, R = 64, 36, 3
    for n_copies, want_ok in ((1, 1), (60, 0)):
        tris = _with_extra_triangles(sd, extra * n_copies)
        u = rt2mod.offline_uniforms(W, H, spec.bounces, R, len(tris))
        scene = rt2mod.Scene(triangles=tris, materials=sd.materials())
        ok, A, n_out = plk_info(rt2mod, scene)
        assert ok == want_ok and n_out == 4 * n_copies
        scene.set_variant(76)
        img = scene.render_host(u, 0, 2)
        ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 2, tris=tris)
        assert_exact(img, ref, f"plk out-of-range x{n_copies}")


@pytest.mark.parametrize("variant", [64, 66])
def test_team_tail_small_slab(rt2mod, oraclemod, config_scene, torch_cuda, variant):
    """A slab smaller than the number of lanes (rank 5 of 8, tiles of 3 rows):
    the team mode runs from the first segment."""
    require_variant(rt2mod, variant)
    sd, spec = config_scene("B")
    W, H = 160, 90
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 8, sd.num_triangles)
    sh = rt2mod.shard(3, 5, 8)
    scene = rt2mod.Scene(sd, 0)
    scene.set_variant(variant)
    img = scene.render_host(u, 0, 1, sh)
    rows = rt2mod.shard_row_ids(H, sh)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 0, 1)
    assert_exact(img, ref, f"team variant {variant} slab")
