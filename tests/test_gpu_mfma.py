"""The matrix-core filter kernel (render_mfma, rt2_mfma.h) against the oracle:
bit-exact on the benchmark scenes, on scenes that exercise the filter's range
checks (out-of-range triangles get always-pass records; rays far outside the
scene make the wave take the scalar-path filter), on triangle counts that are
not a multiple of the 16-triangle group and on the cooperative drain."""
import numpy as np
import pytest

from conftest import EXPERIMENTS, require_variant

from test_gpu_parity import assert_exact, oracle_mean

pytestmark = pytest.mark.gpu

MFMA = 227
# every matrix-filter variant of the loaded library runs each case: the
# product build's automatic kernels (227, the resident 353 / 354 and their L2
# continuation 355 / 356, the LDS-tiled 380); the experiment build adds its A/B variants
# (other drain thresholds, wave counts, record tiles, the kthr forms 320-325)


def _mfma_variants():
    """Every matrix-filter variant the loaded library carries (ids 130-399:
    the product defaults 353-356 / 380 included)."""
    import rt2
    out = []
    for v in range(130, 400):
        name = rt2.lib().rt2_variant_name(v)
        # (speed-of-light probes, "/sol", skip the exact phase: wrong images by design)
        if name and name.decode().startswith(("mfma", "massist")) and "/sol" not in name.decode():
            out.append(v)
    return out


VARIANTS = _mfma_variants()


@pytest.fixture(params=VARIANTS, ids=lambda v: f"v{v}")
def mfma_variant(request):
    return request.param


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    return torch


RES_MAX_TRIS = 38 * 32  # render_mfma_k5r ("mfmar"): records resident in LDS, scenes of <= 38 groups
RESL2_MAX_TRIS = 256 * 32  # ... "mfmarl2": 38 groups resident, the rest from L2, scenes of <= 256 groups


def mfma_scene(rt2mod, sd=None, variant=MFMA, **kw):
    require_variant(rt2mod, variant)
    n = sd.num_triangles if sd is not None else len(kw["triangles"])
    name = rt2mod.lib().rt2_variant_name(variant).decode()
    if name.startswith("mfmar/") and n > RES_MAX_TRIS:
        pytest.skip(f"variant {variant} holds scenes of <= {RES_MAX_TRIS} triangles")
    if name.startswith("mfmarl2/") and n > RESL2_MAX_TRIS:
        pytest.skip(f"variant {variant} holds scenes of <= {RESL2_MAX_TRIS} triangles")
    scene = rt2mod.Scene(sd, 0) if sd is not None else rt2mod.Scene(**kw)
    scene.set_variant(variant)
    return scene


def test_config_A_full_frame(rt2mod, oraclemod, config_scene, torch_cuda, mfma_variant):
    sd, spec = config_scene("A")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = mfma_scene(rt2mod, sd, mfma_variant)
    img = scene.render_host(u, 0, spec.frames)
    st = scene.stats(reset=True)
    ref, _, segs = oracle_mean(oraclemod, sd, u, np.arange(spec.height), 0, spec.frames)
    assert_exact(img, ref, "mfma config A")
    assert st.segments == segs


def test_config_B_full_size_rows(rt2mod, oraclemod, config_scene, torch_cuda, mfma_variant):
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = mfma_scene(rt2mod, sd, mfma_variant)
    img = scene.render_host(u, 0, spec.frames)
    rows = np.arange(2, 1080, 67, dtype=np.int32)
    ref, _, _ = oracle_mean(oraclemod, sd, u, rows, 0, spec.frames)
    assert_exact(img[rows], ref, "mfma config B rows")


def test_config_C_small_image(rt2mod, oraclemod, config_scene, torch_cuda, mfma_variant):
    sd, spec = config_scene("C")
    u = rt2mod.offline_uniforms(48, 27, spec.bounces, 2, sd.num_triangles)
    scene = mfma_scene(rt2mod, sd, mfma_variant)
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(27), 0, 1)
    assert_exact(img, ref, "mfma config C")


@pytest.mark.parametrize("cfg", ["W", "K"])
def test_mid_size_models(rt2mod, oraclemod, config_scene, torch_cuda, mfma_variant, cfg):
    """Configs W and K (windmill, cat + the Cornell box: 57 and 89 groups,
    beyond the 38 the LDS holds): every variant that can hold them, the L2
    continuation of the resident kernel (mfmarl2) included, bit-exact on a
    small whole image."""
    sd, spec = config_scene(cfg)
    u = rt2mod.offline_uniforms(64, 36, spec.bounces, 4, sd.num_triangles)
    scene = mfma_scene(rt2mod, sd, mfma_variant)
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(36), 0, 1)
    assert_exact(img, ref, f"config {cfg}")


def test_diverse_materials(rt2mod, oraclemod, torch_cuda, mfma_variant):
    M = rt2mod.Material
    sd = rt2mod.SceneData()
    ids = [sd.add_material(m) for m in (M.diffuse((1, 0, 0)), M.diffuse((0, 1, 0)), M.diffuse((1, 1, 1)),
                                        M.light((1, 1, 1), 15.0), M.glass((0.9, 0.95, 1.0), 1.5),
                                        M.specular((1, 1, 1), (1, 1, 1), 1.0, 1.0), M.checker(8.0),
                                        M.specular((0.8, 0.6, 0.3), (1, 1, 1), 0.7, 0.4))]
    sd.create_diverse_cornell_box(10.0, *ids)
    u = rt2mod.offline_uniforms(80, 60, 12, 3, sd.num_triangles)
    img = mfma_scene(rt2mod, sd, mfma_variant).render_host(u, 0, 2)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(60), 0, 2)
    assert_exact(img, ref, "mfma diverse")


@pytest.mark.parametrize("case", ["ragged", "tiny_and_huge", "far_camera", "one"])
def test_range_edges(rt2mod, oraclemod, torch_cuda, case, mfma_variant):
    """Random triangle soups around a light: 1, 37 and 300 triangles (ragged
    last group); triangles with 1e-30 / 3e6 coordinates (out of the validated
    range: always-pass records); a camera 2^21 away (rays out of range: the
    scalar-path fallback)."""
    M = rt2mod.Material
    rng = np.random.default_rng({"ragged": 1, "tiny_and_huge": 2, "far_camera": 3, "one": 4}[case])
    n = {"ragged": 37, "tiny_and_huge": 300, "far_camera": 300, "one": 1}[case]
    sd = rt2mod.SceneData()
    sd.add_material(M.diffuse((0.8, 0.7, 0.6)))
    sd.add_material(M.light((1, 1, 1), 4.0))
    sd.add_material(M.specular((0.9, 0.9, 0.9), (1, 1, 1), 0.8, 0.3))
    a = rng.uniform(-3, 3, (n, 3)).astype(np.float32) + np.float32([0, 0, -6])
    for i in range(n):
        sd.add_triangle(tuple(a[i]), tuple(a[i] + rng.uniform(-1.5, 1.5, 3)), tuple(a[i] + rng.uniform(-1.5, 1.5, 3)),
                        i % 3)
    if case == "tiny_and_huge":
        sd.add_triangle((1e-30, 0.0, -4.0), (1.0, 0.0, -4.0), (0.5, 1.0, -4.0), 0)
        sd.add_triangle((3e6, -1.0, -5.0), (-3e6, -1.0, -5.0), (0.0, -1.0, 3e6), 1)
        n += 2
    u = rt2mod.offline_uniforms(40, 30, 6, 3, n)
    if case == "far_camera":
        u.cameraPos.z = float(2 ** 21)
    scene = mfma_scene(rt2mod, variant=mfma_variant, triangles=sd.triangles(), materials=sd.materials())
    img = scene.render_host(u, 0, 1)
    ref, _, _ = oracle_mean(oraclemod, sd, u, np.arange(30), 0, 1)
    assert_exact(img, ref, f"mfma {case}")
