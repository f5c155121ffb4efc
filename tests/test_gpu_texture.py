"""TEXTURE materials on the GPU (§8f row 3): getTriangleTextureColor
(compute.glsl:342-368) with GL_LINEAR + GL_REPEAT sampling of textures
uploaded with GL's unpack rules, bit-exact against the oracle — both
traversals, trace() and traceBasic(), 1/2/3/4-channel textures, a row length
that is not a multiple of 4, UVs outside [0, 1], and the index rules (-1 and
>= numTextures: black; 5: magenta)."""
import os

import numpy as np
import pytest

from test_gpu_parity import assert_exact

pytestmark = pytest.mark.gpu
IMAGES = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "images")
FILES = ["rgb8.png", "gray2_trns.png", "rgba8.png", "gray8.png", "rgb8_wide_odd.png"]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return torch


def textured_scene(rt2mod):
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    red, green, white = (sd.add_material(M.diffuse(c)) for c in ((0.8, 0.1, 0.1), (0.1, 0.8, 0.1), (0.8, 0.8, 0.8)))
    light = sd.add_material(M.light((1.0, 0.9, 0.8), 12.0))
    sd.create_classic_cornell_box(10.0, red, green, white, light)
    tex_ids = [0, 1, 2, 3, 4, 5, -1, 7]
    mats = [sd.add_material(M.texture(i)) for i in tex_ids]
    tris = np.zeros(2 * len(mats), dtype=rt2mod.TRI_DTYPE)
    for k, mi in enumerate(mats):
        x0, x1 = -4.2 + k * 1.05, -4.2 + k * 1.05 + 0.95
        y0, y1 = 1.0 + (k % 2) * 0.5, 7.5 - (k % 3) * 0.7
        z = -2.0 - 0.3 * k
        u0, u1, v0, v1 = -0.7 + 0.1 * k, 1.9 - 0.05 * k, -0.35, 2.6
        quad = [((x0, y0), (u0, v0)), ((x1, y0), (u1, v0)), ((x1, y1), (u1, v1)), ((x0, y1), (u0, v1))]
        for j, (a, b, c) in enumerate(((0, 1, 2), (0, 2, 3))):
            t = tris[2 * k + j]
            for name, vi in zip(("a", "b", "c"), (a, b, c)):
                (px, py), uv = quad[vi]
                t[name][:3] = (px, py, z)
            t["aTex"], t["bTex"], t["cTex"] = quad[a][1], quad[b][1], quad[c][1]
            t["materialIndex"] = mi
    sd.add_triangles(tris)
    sd.build_bvh()
    images = [rt2mod.load_image(os.path.join(IMAGES, f)) for f in FILES]
    return sd, images


def render_pair(rt2mod, oraclemod, sd, images, u, traversal, frames):
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal(traversal)
    scene.set_textures(images)
    img = scene.render_host(u, 0, frames)
    oraclemod.set_textures(images)
    try:
        acc, _, _, _ = oraclemod.render(sd.triangles(), sd.materials(), u, np.arange(u.height), 0, frames, traversal,
                                        nodes=sd.nodes() if traversal == "bvh" else None)
    finally:
        oraclemod.set_textures([])
    return img, acc[..., :3] / np.float32(frames)


@pytest.mark.parametrize("traversal", ["brute", "bvh"])
def test_textured_render_matches_oracle(rt2mod, oraclemod, torch_cuda, traversal):
    sd, images = textured_scene(rt2mod)
    u = rt2mod.offline_uniforms(96, 72, 6, 4, sd.num_triangles, num_textures=6)
    img, ref = render_pair(rt2mod, oraclemod, sd, images, u, traversal, 2)
    assert_exact(img, ref, f"textured {traversal}")
    # the textures are really sampled: without them the image changes
    u0 = rt2mod.offline_uniforms(96, 72, 6, 4, sd.num_triangles, num_textures=0)
    scene = rt2mod.Scene(sd, 0)
    scene.set_traversal(traversal)
    assert not np.array_equal(scene.render_host(u0, 0, 2), img)


@pytest.mark.parametrize("shadow", [False, True])
def test_textured_basic_preview(rt2mod, oraclemod, torch_cuda, shadow):
    sd, images = textured_scene(rt2mod)
    u = rt2mod.offline_uniforms(128, 96, 8, 1, sd.num_triangles, num_textures=6)
    u.basicShading = 1
    u.basicShadingShadow = int(shadow)
    u.basicShadingLightPosition = rt2mod.Vec4(0.0, 9.0, 2.0, 1.0)
    img, ref = render_pair(rt2mod, oraclemod, sd, images, u, "bvh", 1)
    assert_exact(img, ref, "textured traceBasic")
    # magenta quad (index 5 >= the five samplers) and black quads are visible
    px = img[..., :3].reshape(-1, 3)
    assert ((px[:, 0] == 1) & (px[:, 1] == 0) & (px[:, 2] == 1)).any()


def test_texture_upload_errors(rt2mod, torch_cuda):
    sd, images = textured_scene(rt2mod)
    scene = rt2mod.Scene(sd, 0)
    with pytest.raises(rt2mod.RT2Error, match="channels"):
        scene.set_textures([np.zeros((4, 4, 5), np.uint8)])
    scene.set_textures([])
    scene.set_textures(images)
