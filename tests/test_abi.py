"""The drop-in boundary: librt2.so loads and exports exactly what include/rt2.h
declares, with the reference's struct layouts (mesh.h / BVH.h / camera.h)."""
import ctypes as C
import os
import re

from conftest import ROOT


def header_functions():
    text = open(os.path.join(ROOT, "include", "rt2.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt2_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_exported(rt2mod):
    L = C.CDLL(rt2mod.LIB_PATH)
    names = header_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(rt2mod.EXPORTED) == names


def test_struct_layouts(rt2mod):
    assert C.sizeof(rt2mod.Triangle) == 80
    assert C.sizeof(rt2mod.Material) == 96
    assert C.sizeof(rt2mod.Node) == 48
    assert C.sizeof(rt2mod.Uniforms) == 192
    # std430 offsets read by compute.glsl:46-56 / std140 GlobalUniformsBlock :119-146
    assert rt2mod.Triangle.materialIndex.offset == 72
    assert rt2mod.Triangle.aTex.offset == 48
    assert rt2mod.Material.materialType.offset == 72
    assert rt2mod.Material.isEdgeHighlight.offset == 80
    assert rt2mod.Uniforms.environmentalLight.offset == 48
    assert rt2mod.Uniforms.frameIndex.offset == 60
    assert rt2mod.Uniforms.cameraPos.offset == 64
    assert rt2mod.Uniforms.defocusDiskUp.offset == 176


def test_abi_version_and_errors(rt2mod):
    L = rt2mod.lib()
    assert L.rt2_abi_version() == 4 == rt2mod.ABI_VERSION
    sd = rt2mod.SceneData()
    try:
        sd.load_obj_folder("/nonexistent/folder")
        raise AssertionError("expected failure")
    except rt2mod.RT2Error as e:
        assert "OBJ file not found" in str(e)
    # no-GPU safe: argument validation happens before any device call
    p = C.c_void_p()
    assert L.rt2_scene_create(None, 0, None, 0, None, 0, 0, C.byref(p)) < 0
    assert b"bad argument" in L.rt2_last_error()


def test_shard_rows(rt2mod):
    for H in (1, 7, 1080, 2160):
        for n in (1, 2, 3, 8):
            for tile in (1, 4, 8):
                rows = []
                for r in range(n):
                    ids = rt2mod.shard_row_ids(H, rt2mod.shard(tile, r, n))
                    assert list(ids) == sorted(ids)
                    rows.extend(ids)
                assert sorted(rows) == list(range(H))


def test_comm_argument_validation(rt2mod):
    """Multi-GPU ABI: argument errors are reported before any HIP/RCCL call
    (no GPU needed)."""
    L = rt2mod.lib()
    p = C.c_void_p()
    uid = (C.c_uint8 * rt2mod.COMM_ID_BYTES)()
    assert L.rt2_comm_init(uid, 2, 2, 0, C.byref(p)) < 0  # rank outside [0, nranks)
    assert b"bad argument" in L.rt2_last_error()
    assert L.rt2_comm_init(None, 1, 0, 0, C.byref(p)) < 0
    assert L.rt2_comm_wrap(None, 0, C.byref(p)) < 0
    assert L.rt2_comm_check(None) < 0
    assert L.rt2_comm_wait(None, None) < 0
    assert L.rt2_gather_slabs(None, None, 8, 8, rt2mod.shard(), 0, None, None) < 0
    # max_rows smaller than the largest slab of the layout
    assert L.rt2_unshard_slabs(C.c_void_p(16), 1, 8, 8, rt2mod.shard(1, 0, 2), C.c_void_p(16), None) < 0
    assert b"bad argument" in L.rt2_last_error()
    L.rt2_comm_destroy(None)  # no-op


def test_experiment_variants_not_in_product_build(rt2mod):
    """The product library carries only the automatically chosen kernels
    (DESIGN.md §Kernels); A/B variants live in the EXPERIMENTS=1 build."""
    if os.environ.get("RT2_LIB") == "exp":
        return
    for v in (0, 86, 92, 109, 136, 227, 353, 354, 355, 356, 380):
        assert rt2mod.has_variant(v)
    for v in (213, 217, 231, 243, 252, 260, 261, 262, 263, 282, 298, 130, 131, 132, 133, 134, 135, 137, 138, 139, 143,
              144, 145, 146, 150, 152, 200, 206, 228, 233, 245, 250, 251, 1, 22, 28, 40, 46, 53, 64, 67, 74, 84, 85, 87,
              90, 280, 287, 288, 320, 321, 322, 323, 324, 325, 329, 336, 337, 338, 339, 340, 341, 343):
        assert not rt2mod.has_variant(v)
