"""rt2 — Python mirror of the reference's render-path surface over the rt2 C-ABI.

The reference drives its renderer from C++ (RayTracing/src/rayTracing.cpp):
getTrianglesData_ -> material appends -> a Cornell builder -> BVH -> Camera ->
SSBO/UBO upload -> glDispatchCompute per frame -> readback/accumulate -> PNG.
This module exposes the same steps, with the same names and argument meaning,
over ``librt2.so`` (include/rt2.h):

    sd = SceneData()                          # rtxTriangles/bvhTriangles/materials
    sd.load_obj_folder(path)                  # getTrianglesData_   mesh.h:279
    red = sd.add_material(Material.diffuse((1, 0, 0)))
    sd.add_cornell_box(0.17, 0.3, light, True)  # addCornellBox    rayTracing.cpp:453
    sd.build_bvh()                            # BVH(bvh, rtx)       BVH.h:150
    u = offline_uniforms(W, H, bounces, rays, sd.num_triangles)
    scene = Scene(sd, device=0)               # SSBO uploads        rayTracing.cpp:1323
    img = scene.render_host(u, 0, frames)     # dispatch x frames + resolve

The render itself runs only on the HIP path: if librt2.so is missing or no
GPU is present the calls raise — there is no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT2_LIB=exp selects the experiment build (make EXPERIMENTS=1: the product
# kernels plus the A/B variants of DESIGN.md "Tried and measured").
LIB_PATH = os.path.join(_HERE, "librt2_exp.so" if os.environ.get("RT2_LIB") == "exp" else "librt2.so")

DIFFUSE, SPECULAR, LIGHT, CHECKER, GLASS, TEXTURE, GLASS_HIGHLIGHT = range(7)


class Vec4(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("z", C.c_float), ("w", C.c_float)]


class Vec2(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float)]


class Triangle(C.Structure):  # RTXTriangle, mesh.h:112-139
    _fields_ = [("a", Vec4), ("b", Vec4), ("c", Vec4), ("aTex", Vec2), ("bTex", Vec2), ("cTex", Vec2),
                ("materialIndex", C.c_int32), ("pad", C.c_float)]


class Material(C.Structure):  # Material, mesh.h:26-103
    _fields_ = [("color", Vec4), ("specularColor", Vec4), ("emissionColor", Vec4),
                ("textureIndex", C.c_int32), ("emissionStrength", C.c_float), ("smoothness", C.c_float),
                ("specularProbability", C.c_float), ("checkerScale", C.c_float), ("refractiveIndex", C.c_float),
                ("materialType", C.c_int32), ("index", C.c_int32), ("isEdgeHighlight", C.c_int32),
                ("pad1", C.c_int32), ("pad2", C.c_int32), ("pad3", C.c_int32)]

    @staticmethod
    def default() -> "Material":
        m = Material()
        lib().rt2_material_default(C.byref(m))
        return m

    @staticmethod
    def diffuse(col) -> "Material":  # makeDiffusive, mesh.h:49-53
        m = Material.default()
        lib().rt2_material_make_diffuse(C.byref(m), *map(float, col))
        return m

    @staticmethod
    def light(col, strength: float) -> "Material":  # makeLight, mesh.h:72-77
        m = Material.default()
        lib().rt2_material_make_light(C.byref(m), *map(float, col), float(strength))
        return m

    @staticmethod
    def specular(col, spec_col, smooth: float, prob: float) -> "Material":  # makeSpecular, mesh.h:63-70
        m = Material.default()
        lib().rt2_material_make_specular(C.byref(m), *map(float, col), *map(float, spec_col), float(smooth),
                                         float(prob))
        return m

    @staticmethod
    def texture(index: int, col=(1.0, 1.0, 1.0)) -> "Material":  # map_Kd in an MTL, mesh.h:430-450
        m = Material.diffuse(col)
        m.materialType = 5
        m.textureIndex = int(index)
        return m

    @staticmethod
    def checker(scale: float) -> "Material":  # makeChecker, mesh.h:79-83
        m = Material.default()
        lib().rt2_material_make_checker(C.byref(m), float(scale))
        return m

    @staticmethod
    def glass(col, ior: float) -> "Material":  # makeGlass, mesh.h:85-90
        m = Material.default()
        lib().rt2_material_make_glass(C.byref(m), *map(float, col), float(ior))
        return m


class Node(C.Structure):  # Node, BVH.h:54-65
    _fields_ = [("bmin", C.c_float * 3), ("pad0", C.c_float), ("bmax", C.c_float * 3), ("pad1", C.c_float),
                ("triangleIndex", C.c_int32), ("triangleCount", C.c_int32), ("childIndex", C.c_int32),
                ("pad", C.c_int32)]


class Uniforms(C.Structure):  # GlobalUniforms, camera.h:10-36
    _fields_ = [("pad", C.c_int32), ("numTextures", C.c_int32), ("width", C.c_uint32), ("height", C.c_uint32),
                ("numSpheres", C.c_int32), ("numTriangles", C.c_int32), ("basicShading", C.c_int32),
                ("basicShadingShadow", C.c_int32), ("basicShadingLightPosition", Vec4),
                ("environmentalLight", C.c_int32), ("maxBounceCount", C.c_int32), ("numRaysPerPixel", C.c_int32),
                ("frameIndex", C.c_uint32), ("cameraPos", Vec4), ("viewportRight", Vec4), ("viewportUp", Vec4),
                ("viewportFront", Vec4), ("pixelRight", Vec4), ("pixelUp", Vec4), ("defocusDiskRight", Vec4),
                ("defocusDiskUp", Vec4)]


class Shard(C.Structure):
    _fields_ = [("tile_rows", C.c_int32), ("rank", C.c_int32), ("nranks", C.c_int32)]


ABI_VERSION = 4  # include/rt2.h RT2_ABI_VERSION
COMM_ID_BYTES = 128  # RT2_COMM_ID_BYTES


class Image(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("channels", C.c_int32),
                ("pixels", C.POINTER(C.c_uint8))]


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("segments", C.c_uint64), ("tests", C.c_uint64),
                ("node_visits", C.c_uint64)]


class CameraDesc(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("position", C.c_float * 3), ("hfov", C.c_float),
                ("pitch", C.c_float), ("yaw", C.c_float), ("focus_distance", C.c_float),
                ("defocus_angle", C.c_float), ("zoom", C.c_float)]


assert C.sizeof(Triangle) == 80 and C.sizeof(Material) == 96
assert C.sizeof(Node) == 48 and C.sizeof(Uniforms) == 192

TRI_DTYPE = np.dtype([("a", "<f4", 4), ("b", "<f4", 4), ("c", "<f4", 4), ("aTex", "<f4", 2), ("bTex", "<f4", 2),
                      ("cTex", "<f4", 2), ("materialIndex", "<i4"), ("pad", "<f4")])
MAT_DTYPE = np.dtype([("color", "<f4", 4), ("specularColor", "<f4", 4), ("emissionColor", "<f4", 4),
                      ("textureIndex", "<i4"), ("emissionStrength", "<f4"), ("smoothness", "<f4"),
                      ("specularProbability", "<f4"), ("checkerScale", "<f4"), ("refractiveIndex", "<f4"),
                      ("materialType", "<i4"), ("index", "<i4"), ("isEdgeHighlight", "<i4"), ("pad1", "<i4"),
                      ("pad2", "<i4"), ("pad3", "<i4")])
NODE_DTYPE = np.dtype([("bmin", "<f4", 3), ("pad0", "<f4"), ("bmax", "<f4", 3), ("pad1", "<f4"),
                       ("triangleIndex", "<i4"), ("triangleCount", "<i4"), ("childIndex", "<i4"), ("pad", "<i4")])
assert TRI_DTYPE.itemsize == 80 and MAT_DTYPE.itemsize == 96 and NODE_DTYPE.itemsize == 48

# Every symbol include/rt2.h declares (tests check the library exports them all).
EXPORTED = [
    "rt2_last_error", "rt2_abi_version", "rt2_scene_create", "rt2_scene_destroy", "rt2_shard_rows",
    "rt2_shard_row", "rt2_render", "rt2_render_host", "rt2_resolve_rgba32f", "rt2_resolve_rgb8_reference",
    "rt2_scene_stats", "rt2_scene_set_variant", "rt2_scene_set_traversal", "rt2_scene_set_frame_split", "rt2_scene_set_cost_order", "rt2_sd_create", "rt2_sd_destroy", "rt2_sd_load_obj_folder",
    "rt2_sd_add_material", "rt2_sd_add_triangle", "rt2_sd_add_triangles", "rt2_sd_add_cornell_box", "rt2_sd_add_mirror_cornell_box",
    "rt2_sd_add_side_lit_cornell_box", "rt2_sd_add_sky_light_plane", "rt2_sd_add_cube",
    "rt2_sd_create_classic_cornell_box", "rt2_sd_create_diverse_cornell_box", "rt2_sd_build_bvh",
    "rt2_sd_num_triangles", "rt2_sd_num_materials", "rt2_sd_num_nodes", "rt2_sd_num_textures",
    "rt2_sd_triangles", "rt2_sd_materials", "rt2_sd_nodes", "rt2_sd_bvh_triangles", "rt2_sd_texture_name",
    "rt2_material_default", "rt2_material_make_diffuse", "rt2_material_make_light", "rt2_material_make_specular",
    "rt2_material_make_checker", "rt2_material_make_glass", "rt2_camera_default", "rt2_camera_uniforms",
    "rt2_uniforms_offline", "rt2_write_png", "rt2_image_load", "rt2_image_free", "rt2_sd_texture",
    "rt2_scene_set_textures", "rt2_comm_unique_id", "rt2_comm_init", "rt2_comm_wrap", "rt2_comm_destroy",
    "rt2_comm_size", "rt2_comm_check", "rt2_gather_slabs", "rt2_unshard_slabs", "rt2_render_host_gather",
    "rt2_comm_wait",
]

_lib: Optional[C.CDLL] = None


class RT2Error(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load librt2.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RT2Error(f"{LIB_PATH} is missing: build it with `make -C raytracing2-fork_amd` "
                       "(or __graft_entry__.build()); the render path has no CPU fallback")
    # One HIP runtime per process.  torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7, but its libs NEED the file name "libamdhip64.so"): if
    # librt2 loaded /opt/rocm's runtime first, importing torch afterwards would
    # bring a second runtime and the two would fight over the device.  Loading
    # torch first makes librt2's NEEDED libamdhip64.so.7 bind to torch's copy,
    # so torch tensors and rt2 kernels share one runtime (and one context).
    if os.environ.get("RT2_NO_TORCH", "0") != "1":
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = C.CDLL(LIB_PATH)
    P, I32, U32, I64, F = C.c_void_p, C.c_int32, C.c_uint32, C.c_int64, C.c_float
    sig = {
        "rt2_last_error": (C.c_char_p, []),
        "rt2_abi_version": (C.c_int, []),
        "rt2_scene_create": (C.c_int, [P, I32, P, I32, P, I32, I32, C.POINTER(P)]),
        "rt2_scene_destroy": (None, [P]),
        "rt2_shard_rows": (I32, [I32, Shard]),
        "rt2_shard_row": (I32, [I32, Shard]),
        "rt2_render": (C.c_int, [P, C.POINTER(Uniforms), U32, U32, Shard, P, P, P]),
        "rt2_render_host": (C.c_int, [P, C.POINTER(Uniforms), U32, U32, Shard, P, P]),
        "rt2_resolve_rgba32f": (C.c_int, [P, I64, U32, P, P]),
        "rt2_resolve_rgb8_reference": (C.c_int, [P, I64, U32, P]),
        "rt2_scene_stats": (C.c_int, [P, C.POINTER(Stats), C.c_int]),
        "rt2_scene_set_variant": (C.c_int, [P, C.c_int]),
        "rt2_scene_set_traversal": (C.c_int, [P, C.c_int]),
        "rt2_scene_set_frame_split": (C.c_int, [P, C.c_int]),
        "rt2_scene_set_cost_order": (C.c_int, [P, C.c_int]),
        "rt2_scene_set_textures": (C.c_int, [P, C.POINTER(Image), I32]),
        "rt2_image_load": (C.c_int, [C.c_char_p, I32, C.POINTER(Image)]),
        "rt2_image_free": (None, [C.POINTER(Image)]),
        "rt2_sd_texture": (C.c_int, [P, I32, C.POINTER(Image)]),
        "rt2_sd_create": (P, []),
        "rt2_sd_destroy": (None, [P]),
        "rt2_sd_load_obj_folder": (C.c_int, [P, C.c_char_p]),
        "rt2_sd_add_material": (I32, [P, C.POINTER(Material)]),
        "rt2_sd_add_triangle": (C.c_int, [P, P, P, P, I32]),
        "rt2_sd_add_triangles": (C.c_int, [P, P, I32]),
        "rt2_sd_add_cornell_box": (C.c_int, [P, F, F, I32, I32]),
        "rt2_sd_add_mirror_cornell_box": (C.c_int, [P, F, F, I32, I32]),
        "rt2_sd_add_side_lit_cornell_box": (C.c_int, [P, F, F, I32, I32, I32]),
        "rt2_sd_add_sky_light_plane": (C.c_int, [P, I32]),
        "rt2_sd_add_cube": (C.c_int, [P, P, P, P, I32]),
        "rt2_sd_create_classic_cornell_box": (C.c_int, [P, F, I32, I32, I32, I32]),
        "rt2_sd_create_diverse_cornell_box": (C.c_int, [P, F, I32, I32, I32, I32, I32, I32, I32, I32]),
        "rt2_sd_build_bvh": (C.c_int, [P]),
        "rt2_sd_num_triangles": (I32, [P]),
        "rt2_sd_num_materials": (I32, [P]),
        "rt2_sd_num_nodes": (I32, [P]),
        "rt2_sd_num_textures": (I32, [P]),
        "rt2_sd_triangles": (P, [P]),
        "rt2_sd_materials": (P, [P]),
        "rt2_sd_nodes": (P, [P]),
        "rt2_sd_bvh_triangles": (C.c_int, [P, P]),
        "rt2_sd_texture_name": (C.c_char_p, [P, I32]),
        "rt2_material_default": (None, [C.POINTER(Material)]),
        "rt2_material_make_diffuse": (None, [C.POINTER(Material), F, F, F]),
        "rt2_material_make_light": (None, [C.POINTER(Material), F, F, F, F]),
        "rt2_material_make_specular": (None, [C.POINTER(Material), F, F, F, F, F, F, F, F]),
        "rt2_material_make_checker": (None, [C.POINTER(Material), F]),
        "rt2_material_make_glass": (None, [C.POINTER(Material), F, F, F, F]),
        "rt2_camera_default": (None, [C.POINTER(CameraDesc), I32, I32]),
        "rt2_camera_uniforms": (C.c_int, [C.POINTER(CameraDesc), C.POINTER(Uniforms)]),
        "rt2_uniforms_offline": (None, [C.POINTER(Uniforms), I32, I32, I32, I32, I32, I32]),
        "rt2_write_png": (C.c_int, [C.c_char_p, I32, I32, I32, P, I32]),
        "rt2_comm_unique_id": (C.c_int, [P]),
        "rt2_comm_init": (C.c_int, [P, I32, I32, I32, C.POINTER(P)]),
        "rt2_comm_wrap": (C.c_int, [P, I32, C.POINTER(P)]),
        "rt2_comm_destroy": (None, [P]),
        "rt2_comm_size": (C.c_int, [P, C.POINTER(I32), C.POINTER(I32)]),
        "rt2_comm_check": (C.c_int, [P]),
        "rt2_comm_wait": (C.c_int, [P, P]),
        "rt2_gather_slabs": (C.c_int, [P, P, I32, I32, Shard, I32, P, P]),
        "rt2_unshard_slabs": (C.c_int, [P, I32, I32, I32, Shard, P, P]),
        "rt2_render_host_gather": (C.c_int, [P, C.POINTER(Uniforms), U32, U32, Shard, P, I32, P, P]),
        "rt2_device_selftest": (C.c_int, [P, I32, P]),
        "rt2_device_rcp_check": (C.c_int, [U32, U32, C.c_int, C.POINTER(C.c_ulonglong), C.POINTER(U32)]),
        "rt2_device_div_check": (C.c_int, [U32, C.c_ulonglong, C.c_int, C.POINTER(C.c_ulonglong), C.POINTER(U32)]),
        "rt2_variant_name": (C.c_char_p, [C.c_int]),
        "rt2_scene_diag": (C.c_int, [P, C.POINTER(C.c_ulonglong), C.POINTER(C.c_int)]),
        "rt2_scene_plk_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_float), C.POINTER(C.c_int)]),
        "rt2_scene_export": (C.c_longlong, [P, C.c_int, P, C.c_ulonglong]),
        "rt2_mfma_probe": (C.c_int, [P, C.c_int, P, I32, P, P, P, P]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if L.rt2_abi_version() != ABI_VERSION:
        raise RT2Error(f"librt2.so ABI {L.rt2_abi_version()} != {ABI_VERSION}: rebuild (make -C raytracing2-fork_amd)")
    _lib = L
    return L


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RT2Error(f"{what}: {lib().rt2_last_error().decode()}")


def _f3(v) -> C.Array:
    return (C.c_float * 3)(*map(float, v))


class SceneData:
    """The reference's host scene arrays (rayTracing.cpp:1256-1293)."""

    def __init__(self):
        self._p = lib().rt2_sd_create()
        if not self._p:
            raise RT2Error("rt2_sd_create failed")

    def __del__(self):
        if getattr(self, "_p", None) and _lib is not None:
            try:
                _lib.rt2_sd_destroy(self._p)
            except Exception:  # interpreter shutdown
                pass
            self._p = None

    def load_obj_folder(self, folder: str) -> None:  # getTrianglesData_, mesh.h:279-613
        _check(lib().rt2_sd_load_obj_folder(self._p, folder.encode()), f"load {folder}")

    def add_material(self, m: Material) -> int:
        i = lib().rt2_sd_add_material(self._p, C.byref(m))
        if i < 0:
            _check(-1, "add_material")
        return i

    def add_triangle(self, a, b, c, material_index: int) -> None:
        _check(lib().rt2_sd_add_triangle(self._p, _f3(a), _f3(b), _f3(c), int(material_index)), "add_triangle")

    def add_triangles(self, tris: np.ndarray) -> None:
        tris = np.ascontiguousarray(tris, dtype=TRI_DTYPE)
        _check(lib().rt2_sd_add_triangles(self._p, tris.ctypes.data, len(tris)), "add_triangles")

    def add_cornell_box(self, light_size, pad, light_mtl, light_enabled=True):  # rayTracing.cpp:453
        _check(lib().rt2_sd_add_cornell_box(self._p, light_size, pad, light_mtl, int(bool(light_enabled))),
               "addCornellBox")

    def add_mirror_cornell_box(self, light_size, pad, light_mtl, mirror_mtl):  # :569
        _check(lib().rt2_sd_add_mirror_cornell_box(self._p, light_size, pad, light_mtl, mirror_mtl),
               "addMirrorCornellBox")

    def add_side_lit_cornell_box(self, light_size, pad, light_mtl, wall_mtl, rotate=False):  # :690
        _check(lib().rt2_sd_add_side_lit_cornell_box(self._p, light_size, pad, light_mtl, wall_mtl, int(rotate)),
               "addSideLitCornellBox")

    def add_sky_light_plane(self, light_mtl):  # :388
        _check(lib().rt2_sd_add_sky_light_plane(self._p, light_mtl), "addSkyLightPlane")

    def add_cube(self, center, size, rotation, mtl):  # :867
        _check(lib().rt2_sd_add_cube(self._p, _f3(center), _f3(size), _f3(rotation), mtl), "addCube")

    def create_classic_cornell_box(self, room, red, green, white, light):  # :949
        _check(lib().rt2_sd_create_classic_cornell_box(self._p, room, red, green, white, light),
               "createClassicCornellBox")

    def create_diverse_cornell_box(self, room, red, green, white, light, glass, mirror, checker, metal):  # :1071
        _check(lib().rt2_sd_create_diverse_cornell_box(self._p, room, red, green, white, light, glass, mirror,
                                                       checker, metal), "createDiverseCornellBox")

    def build_bvh(self) -> None:  # BVH.h:150-163
        _check(lib().rt2_sd_build_bvh(self._p), "BVH")

    @property
    def num_triangles(self) -> int:
        return lib().rt2_sd_num_triangles(self._p)

    @property
    def num_materials(self) -> int:
        return lib().rt2_sd_num_materials(self._p)

    @property
    def num_nodes(self) -> int:
        return lib().rt2_sd_num_nodes(self._p)

    @property
    def texture_names(self) -> list:
        return [lib().rt2_sd_texture_name(self._p, i).decode() for i in range(lib().rt2_sd_num_textures(self._p))]

    def texture(self, i: int) -> np.ndarray:
        """Decoded texture i as (height, width, channels) uint8, row 0 first (flipped on load)."""
        im = Image()
        _check(lib().rt2_sd_texture(self._p, i, C.byref(im)), "rt2_sd_texture")
        return _image_array(im)

    def textures(self) -> list:
        return [self.texture(i) for i in range(lib().rt2_sd_num_textures(self._p))]

    def _view(self, ptr, n, dtype) -> np.ndarray:
        if n == 0:
            return np.zeros(0, dtype=dtype)
        buf = (C.c_char * (n * dtype.itemsize)).from_address(ptr)
        return np.frombuffer(buf, dtype=dtype).copy()

    def triangles(self) -> np.ndarray:
        return self._view(lib().rt2_sd_triangles(self._p), self.num_triangles, TRI_DTYPE)

    def materials(self) -> np.ndarray:
        return self._view(lib().rt2_sd_materials(self._p), self.num_materials, MAT_DTYPE)

    def nodes(self) -> np.ndarray:
        return self._view(lib().rt2_sd_nodes(self._p), self.num_nodes, NODE_DTYPE)

    def bvh_triangles(self) -> np.ndarray:
        out = np.zeros((self.num_triangles, 9), dtype=np.float32)
        _check(lib().rt2_sd_bvh_triangles(self._p, out.ctypes.data), "bvh_triangles")
        return out


def default_camera(width: int, height: int) -> CameraDesc:
    cam = CameraDesc()
    lib().rt2_camera_default(C.byref(cam), width, height)
    return cam


def camera_uniforms(cam: CameraDesc, u: Optional[Uniforms] = None) -> Uniforms:
    u = u or Uniforms()
    _check(lib().rt2_camera_uniforms(C.byref(cam), C.byref(u)), "camera")
    return u


def _image_array(im: Image) -> np.ndarray:
    n = im.width * im.height * im.channels
    buf = (C.c_uint8 * n).from_address(C.addressof(im.pixels.contents))
    return np.frombuffer(buf, dtype=np.uint8).copy().reshape(im.height, im.width, im.channels)


def load_image(path: str, flip_vertically: bool = True) -> np.ndarray:
    """rt2_image_load: stbi_load(path, ..., 0) as Texture2D uses it -> (h, w, channels) uint8."""
    im = Image()
    _check(lib().rt2_image_load(path.encode(), int(bool(flip_vertically)), C.byref(im)), "rt2_image_load")
    try:
        return _image_array(im)
    finally:
        lib().rt2_image_free(C.byref(im))


def offline_uniforms(width, height, max_bounce, rays_per_pixel, num_triangles, num_textures=0) -> Uniforms:
    """screenshot() settings (rayTracing.cpp:146-153) + main()'s per-frame fields."""
    u = Uniforms()
    lib().rt2_uniforms_offline(C.byref(u), width, height, max_bounce, rays_per_pixel, num_triangles, num_textures)
    return u


def shard(tile_rows=1, rank=0, nranks=1) -> Shard:
    return Shard(tile_rows, rank, nranks)


def shard_rows(height: int, sh: Shard) -> int:
    return lib().rt2_shard_rows(height, sh)


def shard_row_ids(height: int, sh: Shard) -> np.ndarray:
    n = shard_rows(height, sh)
    return np.array([lib().rt2_shard_row(i, sh) for i in range(n)], dtype=np.int32)


class Comm:
    """RCCL communicator of the multi-GPU C-ABI (rt2_comm_*): one per rank/GPU."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_uint8 * COMM_ID_BYTES)()
        _check(lib().rt2_comm_unique_id(buf), "rt2_comm_unique_id")
        return bytes(buf)

    def __init__(self, uid: bytes, nranks: int, rank: int, device: int = 0):
        if len(uid) != COMM_ID_BYTES:
            raise RT2Error(f"communicator id must be {COMM_ID_BYTES} bytes")
        buf = (C.c_uint8 * COMM_ID_BYTES).from_buffer_copy(uid)
        p = C.c_void_p()
        _check(lib().rt2_comm_init(buf, nranks, rank, device, C.byref(p)), "rt2_comm_init")
        self._p = p
        self.nranks, self.rank, self.device = nranks, rank, device

    def close(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.rt2_comm_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def check(self) -> None:
        _check(lib().rt2_comm_check(self._p), "rt2_comm_check")

    def gather_slabs(self, slab_ptr: int, width: int, height: int, sh: Shard, root: int, image_ptr: int,
                     stream: int = 0) -> None:
        _check(lib().rt2_gather_slabs(self._p, C.c_void_p(slab_ptr), width, height, sh, root,
                                      C.c_void_p(image_ptr) if image_ptr else None,
                                      C.c_void_p(stream) if stream else None), "rt2_gather_slabs")

    def wait(self, stream: int = 0) -> None:
        """rt2_comm_wait: the stream drained under the RT2_COMM_TIMEOUT_S deadline."""
        _check(lib().rt2_comm_wait(self._p, C.c_void_p(stream) if stream else None), "rt2_comm_wait")


def unshard_slabs(gathered_ptr: int, max_rows: int, width: int, height: int, layout: Shard, image_ptr: int,
                  stream: int = 0) -> None:
    """Root-side un-interleave of [nranks][max_rows][width] 16-byte pixels (rt2_unshard_slabs)."""
    _check(lib().rt2_unshard_slabs(C.c_void_p(gathered_ptr), max_rows, width, height, layout, C.c_void_p(image_ptr),
                                   C.c_void_p(stream) if stream else None), "rt2_unshard_slabs")


class Scene:
    """Device-resident scene: the SSBO uploads of rayTracing.cpp:1323-1325."""

    def __init__(self, sd: Optional[SceneData] = None, device: int = 0, triangles=None, materials=None,
                 nodes=None):
        if sd is not None:
            triangles, materials, nodes = sd.triangles(), sd.materials(), sd.nodes()
        triangles = np.ascontiguousarray(triangles, dtype=TRI_DTYPE)
        materials = np.ascontiguousarray(materials, dtype=MAT_DTYPE)
        nodes = None if nodes is None or len(nodes) == 0 else np.ascontiguousarray(nodes, dtype=NODE_DTYPE)
        self.n_tris = len(triangles)
        self.device = device
        p = C.c_void_p()
        _check(lib().rt2_scene_create(triangles.ctypes.data, len(triangles), materials.ctypes.data, len(materials),
                                      None if nodes is None else nodes.ctypes.data,
                                      0 if nodes is None else len(nodes), device, C.byref(p)), "rt2_scene_create")
        self._p = p

    def close(self):
        if getattr(self, "_p", None) and _lib is not None:
            _lib.rt2_scene_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter shutdown
            pass

    def set_variant(self, v: int) -> int:
        """Forces kernel variant v (0 = automatic); raises if v is not in this build."""
        r = lib().rt2_scene_set_variant(self._p, v)
        if r < 0:
            _check(r, "set_variant")
        return r

    def set_traversal(self, traversal: str) -> None:
        """"brute" (north-star kernel) or "bvh" (compute.glsl:410-460 on the uploaded nodes)."""
        _check(lib().rt2_scene_set_traversal(self._p, {"brute": 0, "bvh": 1}[traversal]), "set_traversal")

    def set_frame_split(self, enable: bool) -> None:
        """(frame, pixel) work items for multi-frame renders (rt2_scene_set_frame_split)."""
        _check(lib().rt2_scene_set_frame_split(self._p, int(bool(enable))), "set_frame_split")

    def set_cost_order(self, enable: bool) -> None:
        """Most-expensive-first pixel order from the previous render (rt2_scene_set_cost_order)."""
        _check(lib().rt2_scene_set_cost_order(self._p, int(bool(enable))), "set_cost_order")

    def set_textures(self, images) -> None:
        """Uploads textures (list of (h, w, channels) uint8 arrays, stb layout) — the
        reference's texture units 0..4 (rt2_scene_set_textures)."""
        arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
        arrs = [a if a.ndim == 3 else a[..., None] for a in arrs]
        ims = (Image * max(len(arrs), 1))()
        for i, a in enumerate(arrs):
            ims[i].width, ims[i].height, ims[i].channels = a.shape[1], a.shape[0], a.shape[2]
            ims[i].pixels = a.ctypes.data_as(C.POINTER(C.c_uint8))
        _check(lib().rt2_scene_set_textures(self._p, ims, len(arrs)), "rt2_scene_set_textures")

    def render(self, u: Uniforms, frame_begin: int, frame_count: int, sh: Shard, accum_ptr: int,
               accum8_ptr: int = 0, stream: int = 0) -> None:
        """Asynchronous device render into caller-owned device accumulators (rt2_render)."""
        _check(lib().rt2_render(self._p, C.byref(u), frame_begin, frame_count, sh, C.c_void_p(accum_ptr),
                                C.c_void_p(accum8_ptr) if accum8_ptr else None,
                                C.c_void_p(stream) if stream else None), "rt2_render")

    def render_host(self, u: Uniforms, frame_begin: int, frame_count: int, sh: Optional[Shard] = None,
                    rgb8: bool = False):
        """Blocking render; returns the mean rgba32f slab (rows, W, 4) [and the 8-bit reference average]."""
        sh = sh or shard()
        rows = shard_rows(u.height, sh)
        out = np.zeros((rows, u.width, 4), dtype=np.float32)
        out8 = np.zeros((rows, u.width, 3), dtype=np.uint8) if rgb8 else None
        _check(lib().rt2_render_host(self._p, C.byref(u), frame_begin, frame_count, sh, out.ctypes.data,
                                     None if out8 is None else out8.ctypes.data), "rt2_render_host")
        return (out, out8) if rgb8 else out

    def render_host_gather(self, u: Uniforms, frame_begin: int, frame_count: int, sh: Shard, comm: "Comm",
                           root: int = 0, rgb8: bool = False):
        """rt2_render_host_gather: this rank's shard, gathered to `root`; returns the
        whole (H, W, 4) mean image [and the 8-bit average] on the root, None elsewhere."""
        is_root = comm.rank == root
        out = np.zeros((u.height, u.width, 4), dtype=np.float32) if is_root else None
        out8 = np.zeros((u.height, u.width, 3), dtype=np.uint8) if (is_root and rgb8) else None
        _check(lib().rt2_render_host_gather(self._p, C.byref(u), frame_begin, frame_count, sh, comm._p, root,
                                            None if out is None else out.ctypes.data,
                                            None if out8 is None else out8.ctypes.data), "rt2_render_host_gather")
        if not is_root:
            return None
        return (out, out8) if rgb8 else out

    def export(self, what: int, dtype) -> np.ndarray:
        """A derived device array of the scene (rt2_scene_export, test hook): 0 =
        pre-transformed triangles, 1/2 = render_mfma records/tau, 3/4 = sweep_k16 records/tau,
        5 = the k5 form's per-triangle m.z residual bounds (float32 pairs), 6 = the kthr records (threshold in
        the K-slots)."""
        n = lib().rt2_scene_export(self._p, what, None, 0)
        if n < 0:
            raise RT2Error("rt2_scene_export: bad argument")
        out = np.zeros(n // np.dtype(dtype).itemsize, dtype=dtype)
        if n and lib().rt2_scene_export(self._p, what, out.ctypes.data, n) != n:
            raise RT2Error("rt2_scene_export failed")
        return out

    def mfma_probe(self, layout: int, rays: np.ndarray):
        """The matrix filter's terms on the device (rt2_mfma_probe, test hook):
        rays (n, 8) float32 {o, best, d, 0}, n a multiple of 64; layout 0 =
        16x16x32 (render_mfma), 1 = k16, 2 = its 5-product form (k5), 3 = k5 with the threshold in the
        accumulator (cthr: U, -V, X, Y shifted by TT, TT in slot 3), 4 = layout 3 with the fragments built in
        registers (frag_pair: the operand path of the shipping kernels), 5 = the threshold in the K-slots (kthr:
        U, -V, X, Y; slot 3 zero; frag_pair fragments).  Returns (terms [n, n_pad, 5], frags [n, 48] float16
        (layouts 4, 5: [n, 80], the register fragments at 48..63 and 64..79), rinfo [n, 8], accept [n, n_tris]
        bool)."""
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = rays.shape[0]
        g = 32 if layout >= 1 else 16
        n_pad = -(-self.n_tris // g) * g
        terms = np.zeros((n, n_pad, 5), dtype=np.float32)
        frags = np.zeros((n, 80), dtype=np.uint16)
        rinfo = np.zeros((n, 8), dtype=np.float32)
        acc = np.zeros((n, self.n_tris), dtype=np.uint8)
        _check(lib().rt2_mfma_probe(self._p, layout, rays.ctypes.data, n, terms.ctypes.data, frags.ctypes.data,
                                    rinfo.ctypes.data, acc.ctypes.data), "rt2_mfma_probe")
        frags = frags.view(np.float16)
        return terms, (frags if layout >= 4 else np.ascontiguousarray(frags[:, :48])), rinfo, acc.astype(bool)

    def cost_map(self) -> np.ndarray | None:
        """The per-pixel cost map of the last cost-ordered launch (test hook
        rt2_scene_cost_map; shader clocks), or None when there is none."""
        fn = lib().rt2_scene_cost_map
        fn.restype = C.c_longlong
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_ulonglong]
        n = fn(self._p, None, 0)
        if n <= 0:
            return None
        out = np.zeros(n, dtype=np.uint32)
        if fn(self._p, out.ctypes.data, n) != n:
            raise RT2Error("rt2_scene_cost_map failed")
        return out

    def stats(self, reset: bool = False) -> Stats:
        s = Stats()
        _check(lib().rt2_scene_stats(self._p, C.byref(s), int(reset)), "stats")
        return s


def has_variant(v: int) -> bool:
    """Whether kernel variant v is compiled into the loaded library (experiment
    variants need make EXPERIMENTS=1 and RT2_LIB=exp)."""
    return v == 0 or lib().rt2_variant_name(v) is not None


def resolve_rgba32f(accum_ptr: int, n_pixels: int, frames: int, out_ptr: int, stream: int = 0) -> None:
    _check(lib().rt2_resolve_rgba32f(C.c_void_p(accum_ptr), n_pixels, frames, C.c_void_p(out_ptr),
                                     C.c_void_p(stream) if stream else None), "resolve")


def resolve_rgb8_reference(acc8: np.ndarray, frames: int) -> np.ndarray:
    acc8 = np.ascontiguousarray(acc8, dtype=np.uint32)
    n = acc8.size // 4
    out = np.zeros(acc8.shape[:-1] + (3,), dtype=np.uint8)
    _check(lib().rt2_resolve_rgb8_reference(acc8.ctypes.data, n, frames, out.ctypes.data), "resolve_rgb8")
    return out


def write_png(path: str, img: np.ndarray) -> None:
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape[:2]
    comps = 1 if img.ndim == 2 else img.shape[2]
    _check(lib().rt2_write_png(path.encode(), w, h, comps, img.ctypes.data, w * comps), "write_png")


def device_selftest(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.zeros((len(x), 10), dtype=np.float32)
    _check(lib().rt2_device_selftest(x.ctypes.data, len(x), out.ctypes.data), "device_selftest")
    return out


from .scenes import (REF_DATA_ENV, build_config_scene, config_spec, generate_torus_obj,  # noqa: E402,F401
                     CONFIGS)
