"""GPU BVH traversal (§8f row 1) vs the oracle's reference-faithful BVH mode
(calculateRayCollisionBVH, compute.glsl:410-460): bit-exact, including the
visiting-order tie behaviour, and equal leaf-test counts."""
import numpy as np
import pytest

from conftest import EXPERIMENTS, require_variant

from test_gpu_parity import assert_exact, oracle_mean

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return torch


def bvh_scene(rt2mod, sd):
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal("bvh")
    return scene


@pytest.mark.parametrize("cfg,W,H,R", [("A", 256, 256, 4), ("B", 192, 108, 8)])
def test_bvh_matches_oracle_bvh(rt2mod, oraclemod, config_scene, torch_cuda, cfg, W, H, R):
    sd, spec = config_scene(cfg)
    u = rt2mod.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    img = scene.render_host(u, 0, 2)
    st = scene.stats(reset=True)
    acc, _, segs, tests = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(H), 0, 2, "bvh",
                                           nodes=sd.nodes())
    assert_exact(img, acc[..., :3] / np.float32(2), f"bvh {cfg}")
    assert st.segments == segs
    assert st.tests == tests


def test_bvh_full_size_config_B_rows(rt2mod, oraclemod, config_scene, torch_cuda):
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    img = scene.render_host(u, 0, spec.frames)
    rows = np.arange(3, 1080, 36, dtype=np.int32)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 0, spec.frames, "bvh")
    assert_exact(img[rows], ref, "bvh config B")
    # and the brute-force kernel agrees except on exact distance ties
    brute = rt2mod.Scene(sd, 0).render_host(u, 0, spec.frames)
    d = np.abs(brute[..., :3] - img[..., :3])
    assert (d.max(-1) == 0).mean() > 0.999 and np.sqrt((d ** 2).mean()) < 1e-4


def test_bvh_large_mesh_config_C(rt2mod, oraclemod, config_scene, torch_cuda):
    sd, spec = config_scene("C")
    u = rt2mod.offline_uniforms(64, 36, spec.bounces, 4, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(36), 0, 1, "bvh")
    assert_exact(img, ref, "bvh config C")


def test_bvh_diverse_materials(rt2mod, oraclemod, torch_cuda):
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    ids = [sd.add_material(m) for m in (M.diffuse((1, 0, 0)), M.diffuse((0, 1, 0)), M.diffuse((1, 1, 1)),
                                        M.light((1, 1, 1), 15.0), M.glass((0.9, 0.95, 1.0), 1.5),
                                        M.specular((1, 1, 1), (1, 1, 1), 1.0, 1.0), M.checker(8.0),
                                        M.specular((0.8, 0.6, 0.3), (1, 1, 1), 0.7, 0.4))]
    sd.create_diverse_cornell_box(10.0, *ids)
    sd.build_bvh()
    u = rt2mod.offline_uniforms(80, 60, 12, 3, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    img = scene.render_host(u, 0, 2)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(60), 0, 2, "bvh")
    assert_exact(img, ref, "bvh diverse")


def test_bvh_requires_nodes_and_validates(rt2mod, torch_cuda):
    sd = rt2mod.SceneData()
    sd.add_material(rt2mod.Material.default())
    sd.add_triangle((0, 0, 0), (1, 0, 0), (0, 1, 0), 0)
    scene = rt2mod.Scene(sd, 0)  # no BVH built: no nodes
    with pytest.raises(rt2mod.RT2Error, match="node array"):
        scene.set_traversal("bvh")
    sd.build_bvh()
    nodes = sd.nodes()
    nodes["childIndex"][0] = 99
    with pytest.raises(rt2mod.RT2Error, match="out of range"):
        rt2mod.Scene(triangles=sd.triangles(), materials=sd.materials(), nodes=nodes)


# render_bvh2 (child-pair records, Markstein slabs, while-while),
# render_bvh3 (+ wave-uniform fast slab path, fused interior/leaf sub-steps) and
# render_bvh4 (+ the next entry in a register, depth-sized LDS stack)
# (109 = the product kernel; the others are experiment-build variants)
BVH2_VARIANTS = [109] + ([40, 41, 43, 45, 46, 47, 48, 50, 53, 54, 55] if EXPERIMENTS else [])
BVH_SPOT = (109, 53, 40, 46, 50, 55)


@pytest.mark.parametrize("mode", [0, 1])
def test_exact_slab_division(rt2mod, torch_cuda, mode):
    """div_mk (mode 0) / div64 (mode 1) == IEEE n/d on 2^32 random pairs of the
    ranges the BVH kernels use them on."""
    import ctypes as C
    bad = C.c_ulonglong(0)
    first = C.c_uint32(0)
    for seed in (1, 2, 3, 4):
        assert rt2mod.lib().rt2_device_div_check(seed, 1 << 30, mode, C.byref(bad), C.byref(first)) == 0
        assert bad.value == 0, f"mode {mode} seed {seed}: {bad.value} mismatches, first index {first.value}"


@pytest.mark.parametrize("variant", BVH2_VARIANTS)
def test_bvh2_matches_oracle_bvh(rt2mod, oraclemod, config_scene, torch_cuda, variant):
    require_variant(rt2mod, variant)
    sd, spec = config_scene("B")
    W, H, R = 192, 108, 8
    u = rt2mod.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    scene.set_variant(variant)
    img = scene.render_host(u, 0, 2)
    st = scene.stats(reset=True)
    acc, _, segs, tests = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(H), 0, 2, "bvh",
                                           nodes=sd.nodes())
    assert_exact(img, acc[..., :3] / np.float32(2), f"bvh2 variant {variant}")
    assert st.segments == segs
    assert st.tests == tests


def test_bvh2_large_mesh_and_diverse(rt2mod, oraclemod, config_scene, torch_cuda):
    sd, spec = config_scene("C")
    u = rt2mod.offline_uniforms(96, 54, spec.bounces, 4, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    for v in [v for v in BVH_SPOT if rt2mod.has_variant(v)]:
        scene.set_variant(v)
        img = scene.render_host(u, 0, 1)
        ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(54), 0, 1, "bvh")
        assert_exact(img, ref, f"variant {v} config C")
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    ids = [sd.add_material(m) for m in (M.diffuse((1, 0, 0)), M.diffuse((0, 1, 0)), M.diffuse((1, 1, 1)),
                                        M.light((1, 1, 1), 15.0), M.glass((0.9, 0.95, 1.0), 1.5),
                                        M.specular((1, 1, 1), (1, 1, 1), 1.0, 1.0), M.checker(8.0),
                                        M.specular((0.8, 0.6, 0.3), (1, 1, 1), 0.7, 0.4))]
    sd.create_diverse_cornell_box(10.0, *ids)
    sd.build_bvh()
    u = rt2mod.offline_uniforms(80, 60, 12, 3, sd.num_triangles)
    scene = bvh_scene(rt2mod, sd)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(60), 0, 2, "bvh")
    for v in [v for v in BVH_SPOT if rt2mod.has_variant(v)]:
        scene.set_variant(v)
        img = scene.render_host(u, 0, 2)
        assert_exact(img, ref, f"variant {v} diverse")


def test_bvh2_big_leaves_and_single_node(rt2mod, oraclemod, torch_cuda):
    """Leaves of > 30 triangles take the node-array lookup; a one-node BVH is a leaf root."""
    M = rt2mod.Material
    rng = np.random.default_rng(5)
    for n_tris, tiny in ((1, False), (40, False), (300, False), (300, True)):
        sd = rt2mod.SceneData()
        sd.add_material(M.diffuse((0.8, 0.8, 0.8)))
        sd.add_material(M.light((1, 1, 1), 5.0))
        a = rng.uniform(-3, 3, (n_tris, 3)).astype(np.float32) + np.float32([0, 5, -5])
        for i in range(n_tris):
            sd.add_triangle(tuple(a[i]), tuple(a[i] + rng.uniform(-1, 1, 3)), tuple(a[i] + rng.uniform(-1, 1, 3)),
                            i % 2)
        if tiny:  # a box coordinate of 1e-30 disables bvh3's fast slab path (IEEE slabs)
            sd.add_triangle((1e-30, 4.0, -5.0), (1.0, 4.0, -5.0), (0.5, 5.0, -5.0), 0)
            n_tris += 1
        sd.build_bvh()
        nodes = sd.nodes().copy()
        # one flat leaf over everything: exercises the count-31 escape and a leaf root
        flat = nodes[:1].copy()
        flat["childIndex"][0] = -1
        flat["triangleIndex"][0] = 0
        flat["triangleCount"][0] = n_tris
        for nd in (nodes, flat):
            scene = rt2mod.Scene(triangles=sd.triangles(), materials=sd.materials(), nodes=nd)
            scene.set_traversal("bvh")
            u = rt2mod.offline_uniforms(48, 32, 6, 2, n_tris)
            acc, _, _, _ = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(32), 0, 1, "bvh", nodes=nd)
            for v in [v for v in BVH_SPOT if rt2mod.has_variant(v)]:
                scene.set_variant(v)
                img = scene.render_host(u, 0, 1)
                assert_exact(img, acc[..., :3], f"variant {v} n={n_tris} nodes={len(nd)}")


@pytest.mark.parametrize("traversal", ["brute", "bvh"])
@pytest.mark.parametrize("brute_variant", [0, 86], ids=["auto-k5", "tiled"])
def test_config_E_million_triangles(rt2mod, oraclemod, config_scene, torch_cuda, traversal, brute_variant):
    """Config E (1,000,014 triangles, mirror box, 16 bounces) at a small image:
    both traversals bit-exact against the oracle; brute force by the automatic
    choice (the 5-product k16 matrix kernel, variant 227) and the scalar LDS-tiled kernel."""
    if traversal == "bvh" and brute_variant:
        pytest.skip("the brute-force variant does not apply to the BVH traversal")
    sd, spec = config_scene("E")
    W, H = (12, 8) if traversal == "brute" else (48, 32)
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal(traversal)
    if brute_variant:
        scene.set_variant(brute_variant)
    img = scene.render_host(u, 0, 1)
    st = scene.stats(reset=True)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 1, traversal)
    assert_exact(img, ref, f"config E {traversal}")
    assert st.segments == segs
