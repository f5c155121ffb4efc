"""GPU parity: the HIP render path (through the C-ABI) against the CPU oracle.

Bar: bit-exact.  Both sides evaluate the pinned arithmetic of DESIGN.md
§Numerics (IEEE f32, explicit fma in dot/cross, pinned transcendentals), so a
pixel either matches in every bit or the implementation has a bug.  The
north-star tolerance (per-pixel RMSE < 1e-4) is asserted as well, as the
outer bound.
"""
import os

import numpy as np
import pytest

from conftest import EXPERIMENTS, require_variant

pytestmark = pytest.mark.gpu

RMSE_TOL = 1e-4


@pytest.fixture(scope="module")
def torch_cuda():
    import torch  # loads torch's HIP runtime first: librt2 then shares it
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return torch


def oracle_mean(oraclemod, sd, u, rows, fb, fc, mode="brute", tris=None, mats=None):
    acc, acc8, segs, tests = oraclemod.render(sd.triangles() if tris is None else tris,
                                              sd.materials() if mats is None else mats, u, rows, fb, fc, mode,
                                              nodes=sd.nodes() if mode == "bvh" else None, with_acc8=True)
    return acc[..., :3] / np.float32(fc), acc8, segs


def assert_exact(gpu, ref, what=""):
    d = np.abs(gpu[..., :3].astype(np.float64) - ref[..., :3].astype(np.float64))
    rmse = float(np.sqrt((d ** 2).mean())) if d.size else 0.0
    assert rmse < RMSE_TOL, f"{what}: rmse {rmse}"
    bad = (d.max(-1) > 0)
    assert not bad.any(), f"{what}: {bad.sum()} of {bad.size} pixels differ, max {d.max():.3e}, rmse {rmse:.3e}"


def test_device_numerics(rt2mod, oraclemod, torch_cuda):
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(-20, 20, 3000), rng.uniform(-1, 1, 1000),
                        np.exp(rng.uniform(-80, 80, 1000)) * rng.choice([-1, 1], 1000)]).astype(np.float32)
    n = len(x)
    out = rt2mod.device_selftest(x)
    y = x[(np.arange(n) * 7 + 3) % n]
    with np.errstate(all="ignore"):
        assert np.array_equal(out[:, 0], x / y, equal_nan=True)
        assert np.array_equal(out[:, 1], np.sqrt(np.abs(x)))
        assert np.array_equal(out[:, 9], np.float32(1.0) / x)
        fma = (x.astype(np.float64) * y.astype(np.float64) + x.astype(np.float64)).astype(np.float32)
    # float64 product+sum then one rounding == fma except double-rounding corner cases
    assert (out[:, 2] == fma).mean() > 0.999
    for col, k, arg in ((3, 0, x), (4, 1, np.abs(x)), (5, 2, np.clip(y, -1, 1)), (6, 3, x), (7, 4, x)):
        host = np.array([oraclemod.pinned(k, float(v)) for v in arg], np.float32)
        assert np.array_equal(out[:, col], host, equal_nan=True), (col, k)


def test_config_A_full_frame_exact(rt2mod, oraclemod, config_scene, torch_cuda):
    sd, spec = config_scene("A")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, spec.frames)
    st = scene.stats(reset=True)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(spec.height), 0, spec.frames)
    assert_exact(img, ref, "config A")
    assert st.segments == segs
    assert st.samples == spec.width * spec.height * spec.rays * spec.frames


def test_config_B_full_size_rows_exact(rt2mod, oraclemod, config_scene, torch_cuda):
    """Config B at its full size (1920x1080, 64 rays, 8 bounces); strided rows vs the oracle."""
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, spec.frames)
    assert img.shape == (1080, 1920, 4)
    assert np.all(img[..., 3] == 1.0)
    assert np.isfinite(img).all() and (img[..., :3] >= 0).all() and (img[..., :3] <= 1).all()
    rows = np.array([0, 1, 539, 540, 1078, 1079], np.int32)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 0, spec.frames, "brute")
    assert_exact(img[rows], ref, "config B brute rows")
    rows = np.arange(5, 1080, 45, dtype=np.int32)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 0, spec.frames, "bvh")
    # BVH traversal equals brute force except on exact distance ties
    d = np.abs(img[rows][..., :3] - ref)
    assert (d.max(-1) == 0).mean() > 0.999
    assert np.sqrt((d ** 2).mean()) < RMSE_TOL


@pytest.mark.parametrize("cfg,W,H", [("B", 1920, 1080), ("C", 480, 270), ("E", 240, 135)],
                         ids=["B-full", "C-480x270", "E-240x135"])
def test_full_frame_every_pixel(rt2mod, oraclemod, config_scene, torch_cuda, cfg, W, H):
    """Every pixel of a whole frame, by a traversal cross-check: the GPU BVH
    image equals the oracle's BVH image bit for bit at every pixel; the GPU
    brute-force image (the automatic matrix kernel) equals it too except where
    the two traversals may legitimately differ (exact distance ties), and at
    each such pixel, plus 96 random ones, it equals the oracle's brute force.
    (The oracle's brute force over a whole config C frame would take hours;
    its BVH mode takes seconds.)"""
    sd, spec = config_scene(cfg)
    u = rt2mod.offline_uniforms(W, H, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == (AUTO_RES if cfg == "B" else AUTO_TILES)
    st = scene.stats(reset=True)
    assert st.samples == W * H * spec.rays
    scene.set_traversal("bvh")
    img_bvh = scene.render_host(u, 0, 1)
    ref_bvh, _, _ = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 1, "bvh")
    assert_exact(img_bvh, ref_bvh, f"config {cfg} GPU BVH, whole frame")
    diff = np.argwhere((img[..., :3] != ref_bvh).any(-1))
    assert len(diff) <= max(W * H // 10000, 8), f"{len(diff)} pixels where brute force and BVH differ"
    rng = np.random.default_rng(7)
    pick = np.concatenate([diff, np.stack([rng.integers(0, H, 96), rng.integers(0, W, 96)], 1)])
    acc, _, _, _ = oraclemod.render_pixels(sd.triangles(), sd.materials(), u, pick[:, 1], pick[:, 0], 0, 1, "brute")
    assert_exact(img[pick[:, 0], pick[:, 1]], acc[:, :3], f"config {cfg} brute force at {len(diff)} + 96 pixels")


def _last_variant(rt2mod, scene):
    import ctypes as C
    c = (C.c_ulonglong * 8)()
    lv = C.c_int(-1)
    assert rt2mod.lib().rt2_scene_diag(scene._p, c, C.byref(lv)) == 0
    return rt2mod.lib().rt2_variant_name(lv.value).decode()


AUTO_TILES = "mfmat5/1024/kt4/tile19/coop0/w4/cmp/regs/perm/lw/flowp/lean"  # variant 380: > 8,192 triangles, LDS record tiles
AUTO_RES = "mfmar/1024/kt4/res38/coop4/w4/cmp/dpp/lean/lw/pp4"  # 353: <= 38 groups (1,216 triangles), records resident in LDS
AUTO_RES_SLAB = "mfmar/1024/kt4/res38/coop4/w4/cmp/fair/dpp/lean/lw"  # 354: the same, < 6 items per lane (rank slabs)
AUTO_RES_L2 = "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/dpp/lean/lw/pp4"  # 355: 39..256 groups, the rest from L2
AUTO_RES_L2_SLAB = "mfmarl2/1024/kt4/res38l2/coop4/w4/cmp/fair/dpp/lean/lw"  # 356: its rank slabs


def test_auto_variant_large_scene(rt2mod, oraclemod, config_scene, torch_cuda):
    """Scenes whose matrix-filter records outgrow an XCD's L2 (config C: 100k
    triangles, 12.8 MB of k5 records) run the LDS-tiled 5-product form (one
    12-wave workgroup per CU sharing each record tile), even on this small
    image; its path state stays in registers, so a bounce limit the small-scene
    kernel's packed state cannot hold takes it too — bit-exact either way."""
    sd, spec = config_scene("C")
    u = rt2mod.offline_uniforms(64, 36, spec.bounces, 1, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_TILES
    u.maxBounceCount = 5000
    img2 = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_TILES
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(0, 36, 5), 0, 1)
    assert_exact(img2[::5], ref, "config C, 5000 bounces")


def _scene_between_res_and_tiles(rt2mod, config_scene):
    """Config B's scene plus 800 small triangles behind the camera (at z 11-14;
    it sits at z = 10 looking down -z): 2,008
    triangles, above the LDS-resident kernel's 38 groups and below the tiled
    kernel's 8,192 (the range of the resident kernel's L2 continuation)."""
    _, spec = config_scene("B")
    sd, _ = rt2mod.build_config_scene("B")  # a fresh copy (config_scene's is shared)
    rng = np.random.default_rng(3)
    for i in range(800):
        c = (float(rng.uniform(-4, 4)), 5.0 + float(rng.uniform(-4, 4)), 11.0 + float(rng.uniform(0, 3)))
        sd.add_triangle(c, (c[0] + 0.1, c[1], c[2]), (c[0], c[1] + 0.1, c[2]), 0)
    return sd, spec


@pytest.mark.parametrize("extra,want", [(8, "res"), (9, "l2")], ids=["1216-tris", "1217-tris"])
def test_auto_variant_resident_boundary(rt2mod, oraclemod, torch_cuda, extra, want):
    """The LDS holds the records of 38 groups (1,216 triangles): config B's
    1,208 triangles plus 8 take the all-resident kernel, plus 9 (a 39th group
    of one triangle) its L2 continuation — bit-exact either way, the last
    group's padding included (a small image: the rank-slab builds)."""
    sd, spec = rt2mod.build_config_scene("B")
    for i in range(extra):  # small triangles behind the camera (z = 10, looking down -z)
        x = -3.0 + 0.7 * i
        sd.add_triangle((x, 4.0, 12.0), (x + 0.3, 4.0, 12.0), (x, 4.3, 12.0), 0)
    assert sd.num_triangles == 1208 + extra
    u = rt2mod.offline_uniforms(64, 36, spec.bounces, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == (AUTO_RES_SLAB if want == "res" else AUTO_RES_L2_SLAB)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(36), 0, 1)
    assert_exact(img, ref, f"{sd.num_triangles} triangles")


def test_auto_variant_l2_continuation(rt2mod, oraclemod, config_scene, torch_cuda):
    """Scenes between 38 and 256 groups run the resident kernel's L2
    continuation, whose path state stays in registers: a bounce limit of 5000
    (beyond the 12-bit packed fields of round 4-5's 263) takes the same kernel
    — same image as the oracle either way; a whole image takes the build
    without fair-share priority."""
    sd, spec = _scene_between_res_and_tiles(rt2mod, config_scene)
    assert 38 * 32 < sd.num_triangles <= 8192
    u = rt2mod.offline_uniforms(40, 24, spec.bounces, 3, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_RES_L2_SLAB
    u.maxBounceCount = 5000
    img2 = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_RES_L2_SLAB
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(24), 0, 1)
    assert_exact(img2, ref, "5000 bounces")
    u.maxBounceCount = spec.bounces
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(24), 0, 1)
    assert_exact(img, ref, "L2 continuation")
    uw = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, 1, sd.num_triangles)
    scene.render_host(uw, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_RES_L2


def test_auto_variant_by_items_per_lane(rt2mod, config_scene, torch_cuda):
    """The launcher picks the LDS-resident matrix-filter kernel for the full
    config B image and its fair-share build for the 1/2, 1/4 and 1/8 slabs
    (fewer than 6 items per lane; DESIGN.md "Fair-share issue priority"; the
    assist kernel serves slabs of scenes outside the matrix filter's range),
    and every slab is bit-identical to the same rows of the full image."""
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    full = scene.render_host(u, 0, 1)
    assert _last_variant(rt2mod, scene) == AUTO_RES
    for n, want in ((2, AUTO_RES_SLAB), (4, AUTO_RES_SLAB), (8, AUTO_RES_SLAB)):
        sh = rt2mod.shard(1, n - 1, n)
        img = scene.render_host(u, 0, 1, sh)
        assert _last_variant(rt2mod, scene) == want
        rows = rt2mod.shard_row_ids(spec.height, sh)
        assert np.array_equal(img, full[rows]), f"1/{n} slab differs from the full image"


def test_frames_split_across_calls_bit_identical(rt2mod, config_scene, torch_cuda):
    torch = torch_cuda
    sd, spec = config_scene("A")
    W, H = 64, 40
    u = rt2mod.offline_uniforms(W, H, 4, 3, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    sh = rt2mod.shard()
    a = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
    b = torch.zeros_like(a)
    a8 = torch.zeros((H, W, 4), dtype=torch.int32, device="cuda")
    b8 = torch.zeros_like(a8)
    scene.render(u, 5, 4, sh, a.data_ptr(), a8.data_ptr())
    for fb, fc in ((5, 1), (6, 2), (8, 1)):
        scene.render(u, fb, fc, sh, b.data_ptr(), b8.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(a, b) and torch.equal(a8, b8)


def test_shards_assemble_to_full_image(rt2mod, config_scene, torch_cuda):
    sd, spec = config_scene("A")
    W, H = 96, 61
    u = rt2mod.offline_uniforms(W, H, 4, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    full = scene.render_host(u, 0, 2)
    for tile, n in ((1, 2), (8, 3), (4, 8)):
        img = np.zeros_like(full)
        for r in range(n):
            sh = rt2mod.shard(tile, r, n)
            slab = scene.render_host(u, 0, 2, sh)
            img[rt2mod.shard_row_ids(H, sh)] = slab
        assert np.array_equal(img, full), (tile, n)


def test_rgb8_reference_path(rt2mod, oraclemod, config_scene, torch_cuda):
    sd, spec = config_scene("A")
    W, H, F = 80, 50, 3
    u = rt2mod.offline_uniforms(W, H, 4, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img, rgb8 = scene.render_host(u, 0, F, rgb8=True)
    ref, acc8, _ = oracle_mean(oraclemod, sd, u, np.arange(H), 0, F)
    assert_exact(img, ref)
    expect = np.minimum(255.0, acc8[..., :3].astype(np.float32) / np.float32(F)).astype(np.uint8)
    assert np.array_equal(rgb8, expect)


@pytest.mark.parametrize("W,H,R,B", [(37, 13, 1, 8), (17, 9, 3, 0), (33, 7, 2, 1), (1, 1, 5, 20)])
def test_odd_sizes_and_bounce_limits(rt2mod, oraclemod, config_scene, torch_cuda, W, H, R, B):
    sd, spec = config_scene("A")
    u = rt2mod.offline_uniforms(W, H, B, R, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 3, 2)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(H), 3, 2)
    assert_exact(img, ref, f"{W}x{H} R{R} B{B}")
    assert scene.stats().segments == segs
    if B == 0:
        assert np.all(img[..., :3] == 0)


def test_diverse_materials_exact(rt2mod, oraclemod, torch_cuda):
    """Glass, checker, mirror and glossy-specular materials (compute.glsl:499-546)."""
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
    edge = M.diffuse((0.5, 0.5, 0.9))
    edge.isEdgeHighlight = 1
    sd.add_material(edge)
    sd.create_diverse_cornell_box(10.0, red, green, white, light, glass, mirror, checker, metal)
    sd.add_cube((0.0, -2.0, 0.0), (1.0, 1.0, 1.0), (0.3, 0.2, 0.1), 8)
    sd.build_bvh()
    W, H = 96, 64
    u = rt2mod.offline_uniforms(W, H, 12, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 2)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 2)
    assert_exact(img, ref, "diverse")
    assert scene.stats().segments == segs


def test_defocus_and_frame_wrap(rt2mod, oraclemod, config_scene, torch_cuda):
    """Non-zero defocus exercises cos/sin of randomDirection2D; frame indices near
    2^32 exercise the uint32 seed wrap (compute.glsl:668)."""
    sd, spec = config_scene("A")
    cam = rt2mod.default_camera(48, 32)
    cam.defocus_angle = 0.05
    u = rt2mod.offline_uniforms(48, 32, 6, 3, sd.num_triangles)
    rt2mod.camera_uniforms(cam, u)
    assert u.defocusDiskRight.x != 0
    scene = rt2mod.Scene(sd, 0)
    fb = 2**32 - 2
    img = scene.render_host(u, fb, 3)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(32), fb, 3)
    assert_exact(img, ref, "defocus + wrap")


def test_tiled_kernel_exact(rt2mod, oraclemod, config_scene, torch_cuda):
    """The scalar-path LDS-tiled sweep (variant 86: the automatic choice above
    131,072 triangles for scenes outside the matrix filter's range), forced on
    config B and on config C's 100k triangles."""
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(96, 54, 8, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    scene.set_variant(86)
    img = scene.render_host(u, 0, 1)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(54), 0, 1)
    assert_exact(img, ref, "tiled B")
    assert scene.stats().segments == segs
    sdc, specc = config_scene("C")
    assert sdc.num_triangles == 100016
    u = rt2mod.offline_uniforms(24, 14, 8, 2, sdc.num_triangles)
    ref, _, _ = oracle_mean(oraclemod, sdc, u, np.arange(14), 0, 1, "bvh")
    out = {}
    for v in (86, 0):  # forced scalar-path LDS tiles; automatic (the matrix filter's tiled kernel at 100k triangles)
        scene = rt2mod.Scene(sdc, 0)
        scene.set_variant(v)
        out[v] = scene.render_host(u, 0, 1)
        d = np.abs(out[v][..., :3] - ref)
        assert (d.max(-1) == 0).mean() > 0.99 and np.sqrt((d ** 2).mean()) < RMSE_TOL
    assert np.array_equal(out[86], out[0])  # both brute force: identical bits


def test_empty_and_single_triangle_scenes(rt2mod, oraclemod, torch_cuda):
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    sd.add_material(M.diffuse((0.7, 0.7, 0.7)))
    u = rt2mod.offline_uniforms(20, 10, 4, 2, 0)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(10), 0, 1)
    assert_exact(img, ref, "empty scene (sky only)")
    sd.add_triangle((-3, 0, -2), (3, 0, -2), (0, 8, -2), 0)
    u = rt2mod.offline_uniforms(20, 10, 4, 2, 1)
    scene = rt2mod.Scene(sd, 0)
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(10), 0, 1)
    assert_exact(img, ref, "one triangle")


def test_bad_material_index_rejected(rt2mod, torch_cuda):
    sd = rt2mod.SceneData()
    sd.add_material(rt2mod.Material.default())
    sd.add_triangle((0, 0, 0), (1, 0, 0), (0, 1, 0), 5)
    with pytest.raises(rt2mod.RT2Error, match="material index"):
        rt2mod.Scene(sd, 0)


@pytest.mark.parametrize("traversal", ["brute", "bvh"])
def test_frame_split_identical(rt2mod, oraclemod, config_scene, torch_cuda, traversal):
    """(frame, pixel) work items + frame_accumulate give the same bits as whole-pixel items."""
    sd, spec = config_scene("B")
    W, H, R, F = 96, 54, 4, 3
    u = rt2mod.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    out = {}
    for split in (False, True):
        scene = rt2mod.Scene(sd, 0)
        scene.set_traversal(traversal)
        scene.set_frame_split(split)
        out[split] = scene.render_host(u, 2, F, rgb8=True)
        st = scene.stats(reset=True)
        assert st.samples == W * H * R * F
    assert np.array_equal(out[False][0], out[True][0])
    assert np.array_equal(out[False][1], out[True][1])
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(H), 2, F, traversal)
    assert_exact(out[True][0], ref, f"split {traversal}")


# brute-force kernel variants that change the schedule, not the arithmetic:
# the product variants (0 = automatic, 86, 92, 227 = the matrix filter, 380 = its LDS-tiled form, 353/354 = its
# LDS-resident forms and 355/356 their L2 continuation, 136 = the scalar path forced) and, in an experiment build, the A/B
# variants (masked/plk filters, resident LDS, cooperative and team tail modes,
# split waves, the round-1 slab kernels, occupancy hints)
BRUTE_VARIANTS = [0, 86, 92, 227, 380, 353, 354, 355, 356, 136] + (
    [217, 262, 263, 282, 298, 213, 231, 243, 252, 260, 261, 212, 246, 228, 233, 250, 280, 320, 321, 322, 323, 325, 326,
     327, 328, 329, 336, 337, 338, 340, 343, 351, 369, 370, 67, 85, 106, 64, 66, 74, 76, 79, 80] if EXPERIMENTS else [])


@pytest.mark.parametrize("variant", BRUTE_VARIANTS)
def test_brute_variants_bit_exact(rt2mod, oraclemod, config_scene, torch_cuda, variant):
    require_variant(rt2mod, variant)
    sd, spec = config_scene("B")
    W, H, R = 96, 54, 4
    u = rt2mod.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    scene.set_variant(variant)
    img = scene.render_host(u, 0, 2)
    st = scene.stats(reset=True)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(H), 0, 2)
    assert_exact(img, ref, f"variant {variant}")
    assert st.segments == segs


@pytest.mark.parametrize("variant", [92] + ([85] if EXPERIMENTS else []))
@pytest.mark.parametrize("split_frames", [False, True])
def test_split_waves_outputs(rt2mod, oraclemod, config_scene, torch_cuda, variant, split_frames):
    """Kernels whose waves share rays — split mode (S waves per 64 rays, one
    writer wave) and the assist kernel (helpers sweep chunks or whole rays of
    an owner's segment): the float and 8-bit accumulators, the per-frame planes
    and the counters see each pixel-frame once — identical to the default
    kernel on a shard slab with 3 frames."""
    require_variant(rt2mod, variant)
    sd, spec = config_scene("B")
    W, H, R, F = 80, 45, 4, 3
    u = rt2mod.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    sh = rt2mod.shard(2, 1, 3)
    out = {}
    for v in (0, variant):
        scene = rt2mod.Scene(sd, 0)
        scene.set_variant(v)
        scene.set_frame_split(split_frames)
        out[v] = scene.render_host(u, 1, F, sh, rgb8=True)
        st = scene.stats(reset=True)
        out[v] += (st.segments, st.tests)
    assert np.array_equal(out[0][0], out[variant][0])
    assert np.array_equal(out[0][1], out[variant][1])
    assert out[0][2:] == out[variant][2:]
    rows = rt2mod.shard_row_ids(H, sh)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 1, F)
    assert_exact(out[variant][0], ref, f"split-wave variant {variant}")


@pytest.mark.parametrize("traversal,frames", [("brute", 1), ("bvh", 1), ("brute", 3), ("bvh", 2)])
def test_cost_ordered_renders_identical(rt2mod, oraclemod, config_scene, torch_cuda, traversal, frames):
    """Renders after the first hand out pixels most-expensive-first (the previous
    render's cost map): same bits, every pixel exactly once."""
    sd, spec = config_scene("B")
    W, H = 120, 66
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal(traversal)
    scene.set_cost_order(True)
    # frame-major launches too write the map (frame 0's item of each pixel
    # measures: ADVICE r5), so a sequence of them is cost-ordered from the
    # second render on without a whole-pixel launch first
    imgs = [scene.render_host(u, 0, frames, rgb8=True) for _ in range(3)]
    cm = scene.cost_map()
    assert cm is not None and len(cm) == W * H and (cm > 0).mean() > 0.99
    st = scene.stats(reset=True)
    assert st.samples == 3 * W * H * 4 * frames
    for img, img8 in imgs[1:]:
        assert np.array_equal(img, imgs[0][0]) and np.array_equal(img8, imgs[0][1])
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(H), 0, frames, traversal)
    assert_exact(imgs[2][0], ref, f"cost-ordered {traversal} F={frames}")
    # a different slab invalidates the map (no stale order is applied)
    sh = rt2mod.shard(2, 1, 3)
    img = scene.render_host(u, 0, frames, sh)
    rows = rt2mod.shard_row_ids(H, sh)
    assert np.array_equal(img, imgs[0][0][rows])


def test_frame_chunks_identical(rt2mod, config_scene, torch_cuda):
    """Per-frame planes beyond the scratch cap: the frames render in chunks,
    accumulated in order — the same bits as one launch."""
    import ctypes as C
    sd, spec = config_scene("B")
    W, H, F = 64, 40, 5
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 2, sd.num_triangles)
    a = rt2mod.Scene(sd, 0)
    ref = a.render_host(u, 1, F, rgb8=True)
    b = rt2mod.Scene(sd, 0)
    L = rt2mod.lib()
    L.rt2_scene_set_frame_scratch_cap.argtypes = [C.c_void_p, C.c_ulonglong]
    assert L.rt2_scene_set_frame_scratch_cap(b._p, W * H * 16 * 2) == 0  # two frames per chunk
    got = b.render_host(u, 1, F, rgb8=True)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert b.stats().samples == W * H * 2 * F
