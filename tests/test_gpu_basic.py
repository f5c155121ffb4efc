"""traceBasic preview (§8f row 4; compute.glsl:565-645 and main's basicShading
branch, :672-678) on the GPU vs the oracle: bit-exact, both traversals, with
and without the shadow ray, over every material type."""
import numpy as np
import pytest

from test_gpu_parity import assert_exact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return torch


def basic_uniforms(rt2mod, W, H, bounces, n_tris, shadow, light=(0.0, 9.0, 0.0)):
    u = rt2mod.offline_uniforms(W, H, bounces, 1, n_tris)
    u.basicShading = 1
    u.basicShadingShadow = int(shadow)
    u.basicShadingLightPosition = rt2mod.Vec4(light[0], light[1], light[2], 1.0)
    return u


def diverse_scene(rt2mod):
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    ids = [sd.add_material(m) for m in (M.diffuse((1, 0, 0)), M.diffuse((0, 1, 0)), M.diffuse((1, 1, 1)),
                                        M.light((2, 1.5, 1), 15.0), M.glass((0.9, 0.95, 1.0), 1.5),
                                        M.specular((1, 1, 1), (1, 1, 1), 1.0, 1.0), M.checker(8.0),
                                        M.specular((0.8, 0.6, 0.3), (1, 1, 1), 0.7, 0.4))]
    sd.create_diverse_cornell_box(10.0, *ids)
    sd.build_bvh()
    return sd


def render_both(rt2mod, oraclemod, sd, u, traversal, frames=2):
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal(traversal)
    img = scene.render_host(u, 0, frames)
    st = scene.stats(reset=True)
    H = u.height
    acc, _, segs, tests = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(H), 0, frames, traversal,
                                           nodes=sd.nodes() if traversal == "bvh" else None)
    return img, acc[..., :3] / np.float32(frames), st, segs, tests


@pytest.mark.parametrize("traversal", ["brute", "bvh"])
@pytest.mark.parametrize("shadow", [False, True])
def test_basic_diverse(rt2mod, oraclemod, torch_cuda, traversal, shadow):
    sd = diverse_scene(rt2mod)
    u = basic_uniforms(rt2mod, 96, 72, 12, sd.num_triangles, shadow)
    img, ref, st, segs, tests = render_both(rt2mod, oraclemod, sd, u, traversal)
    assert_exact(img, ref, f"basic {traversal} shadow={shadow}")
    assert st.segments == segs
    assert st.tests == tests
    # the preview is deterministic: two frames average to the one-frame colour
    assert np.isfinite(img).all()


@pytest.mark.parametrize("traversal", ["brute", "bvh"])
def test_basic_config_B(rt2mod, oraclemod, config_scene, torch_cuda, traversal):
    sd, spec = config_scene("B")
    u = basic_uniforms(rt2mod, 160, 90, spec.bounces, sd.num_triangles, True, light=(0.0, 8.0, 2.0))
    img, ref, st, segs, _ = render_both(rt2mod, oraclemod, sd, u, traversal, frames=1)
    assert_exact(img, ref, f"basic config B {traversal}")
    assert st.segments == segs


def test_basic_accumulates_and_8bit(rt2mod, oraclemod, torch_cuda):
    sd = diverse_scene(rt2mod)
    u = basic_uniforms(rt2mod, 40, 30, 6, sd.num_triangles, True)
    scene = rt2mod.Scene(sd, 0)
    img, img8 = scene.render_host(u, 3, 5, rgb8=True)
    acc, acc8, _, _ = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(30), 3, 5, "brute",
                                       with_acc8=True)
    assert_exact(img, acc[..., :3] / np.float32(5), "basic 5 frames")
    ref8 = np.minimum(255.0, acc8[..., :3].astype(np.float32) / np.float32(5)).astype(np.uint8)
    assert np.array_equal(img8, ref8)
