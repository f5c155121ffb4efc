"""The measurement configurations of SURVEY.md §8d, built through the host surface.

A  createClassicCornellBox(10, red, green, white, light), no OBJ      38 tris,   256x256,   R4  F1  B4
B  campfire + addCornellBox(0.17, 0.3, light, true)                  1,208,     1920x1080, R64 F1  B8
C  torus 250x200 quads (100k tris) + addCornellBox                   100,016,   1920x1080, R64 F4  B8
D  scene B                                                           1,208,     3840x2160, R64 F16 B8
E  torus 1000x500 (1M tris) + addMirrorCornellBox                    1,000,014, 1920x1080, R4  F1  B16
W  windmill + addCornellBox(0.17, 0.3, light, true)                  1,821,     1920x1080, R64 F1  B8
K  cat + addCornellBox(0.17, 0.3, light, true)                       2,848,     1920x1080, R64 F1  B8

W and K (not in SURVEY.md §8d) are config B with two of
the reference's other texture-free bundled models: scenes of 57 and 89
32-triangle groups, beyond the 38 whose records the LDS holds.

Camera = reference defaults (rayTracing.cpp:82-89), environmental light on,
seed schedule x + y*W + frame*968824447 (compute.glsl:668).

The campfire (windmill, cat) model is taken from the reference's
RayTracing/Data/<model> when that tree is present (here), else from the
loader-output fixture tests/golden/<model>_loaded.npz (the GPU box has no
reference tree); the
torus OBJ is generated deterministically and goes through the same loader.
"""
from __future__ import annotations

import math
import os
import tempfile
from dataclasses import dataclass

import numpy as np

REF_DATA_ENV = "RT2_REFERENCE_DATA"
_REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
CAMPFIRE_FIXTURE = os.path.join(_REPO, "tests", "golden", "campfire_loaded.npz")
MODEL_OF = {"B": "campfire", "D": "campfire", "W": "windmill", "K": "cat"}


@dataclass(frozen=True)
class ConfigSpec:
    name: str
    width: int
    height: int
    rays: int      # numRaysPerPixel (R)
    frames: int    # F
    bounces: int   # maxBounceCount
    description: str


CONFIGS = {
    "A": ConfigSpec("A", 256, 256, 4, 1, 4, "createClassicCornellBox(10), no OBJ, 38 tris"),
    "B": ConfigSpec("B", 1920, 1080, 64, 1, 8, "campfire (1,192 tris) + addCornellBox, 1,208 tris"),
    "C": ConfigSpec("C", 1920, 1080, 64, 4, 8, "torus 250x200 quads (100,000 tris) + addCornellBox, 100,016 tris"),
    "D": ConfigSpec("D", 3840, 2160, 64, 16, 8, "scene B at 4K, 1024 spp"),
    "E": ConfigSpec("E", 1920, 1080, 4, 1, 16, "torus 1000x500 quads (1,000,000 tris) + addMirrorCornellBox"),
    "W": ConfigSpec("W", 1920, 1080, 64, 1, 8, "windmill (1,805 tris) + addCornellBox, 1,821 tris"),
    "K": ConfigSpec("K", 1920, 1080, 64, 1, 8, "cat (2,832 tris) + addCornellBox, 2,848 tris"),
}


def config_spec(name: str) -> ConfigSpec:
    return CONFIGS[name.upper()]


def reference_data_dir() -> str | None:
    d = os.environ.get(REF_DATA_ENV, "/root/reference/RayTracing/Data")
    return d if os.path.isdir(d) else None


def generate_torus_obj(folder: str, nu: int, nv: int, major: float = 2.0, minor: float = 0.8,
                       center=(0.0, 2.0, 0.0), kd=(0.8, 0.8, 0.8)) -> str:
    """Write a deterministic triangulated torus (2*nu*nv faces, outward winding) as OBJ + MTL."""
    os.makedirs(folder, exist_ok=True)
    with open(os.path.join(folder, "torus.mtl"), "w") as f:
        f.write("newmtl torus\nKd %.6f %.6f %.6f\nKe 0.000000 0.000000 0.000000\n" % tuple(kd))
    lines = ["mtllib torus.mtl", "o torus"]
    cx, cy, cz = center
    for i in range(nu):
        u = 2.0 * math.pi * i / nu
        for j in range(nv):
            v = 2.0 * math.pi * j / nv
            rr = major + minor * math.cos(v)
            lines.append("v %.6f %.6f %.6f" % (cx + rr * math.cos(u), cy + minor * math.sin(v), cz + rr * math.sin(u)))
    lines.append("usemtl torus")

    def vid(i, j):
        return (i % nu) * nv + (j % nv) + 1

    for i in range(nu):
        for j in range(nv):
            a, b, c, d = vid(i, j), vid(i + 1, j), vid(i + 1, j + 1), vid(i, j + 1)
            # (a, d, c) / (a, c, b): normal = e0 x e1 points away from the tube axis
            lines.append("f %d %d %d" % (a, d, c))
            lines.append("f %d %d %d" % (a, c, b))
    path = os.path.join(folder, "torus.obj")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def _append_main_materials(sd, Material):
    """main() appends red, green, wall, light(15), mirror (rayTracing.cpp:1268-1283)."""
    red = sd.add_material(Material.diffuse((1.0, 0.0, 0.0)))
    green = sd.add_material(Material.diffuse((0.0, 1.0, 0.0)))
    wall = sd.add_material(Material.diffuse((1.0, 1.0, 1.0)))
    light = sd.add_material(Material.light((1.0, 1.0, 1.0), 15.0))
    mirror = sd.add_material(Material.specular((1.0, 1.0, 1.0), (1.0, 1.0, 1.0), 1.0, 1.0))
    return red, green, wall, light, mirror


def _load_model(sd, model: str = "campfire") -> None:
    d = reference_data_dir()
    if d and os.path.isdir(os.path.join(d, model)):
        sd.load_obj_folder(os.path.join(d, model))
        return
    fixture = os.path.join(_REPO, "tests", "golden", f"{model}_loaded.npz")
    if not os.path.exists(fixture):
        raise FileNotFoundError(f"neither the reference {model} model nor " + fixture)
    z = np.load(fixture, allow_pickle=False)
    from . import Material
    import ctypes as C
    for m in z["materials"]:
        mm = Material()
        C.memmove(C.addressof(mm), np.ascontiguousarray(m).tobytes(), C.sizeof(mm))
        sd.add_material(mm)
    sd.add_triangles(z["triangles"])


def build_config_scene(name: str, workdir: str | None = None):
    """Returns (SceneData with BVH built, ConfigSpec)."""
    from . import Material, SceneData
    spec = config_spec(name)
    sd = SceneData()
    if spec.name == "A":
        red, green, wall, light, mirror = _append_main_materials(sd, Material)
        sd.create_classic_cornell_box(10.0, red, green, wall, light)
    elif spec.name in ("B", "D", "W", "K"):
        _load_model(sd, MODEL_OF[spec.name])
        red, green, wall, light, mirror = _append_main_materials(sd, Material)
        sd.add_cornell_box(0.17, 0.3, light, True)
    elif spec.name in ("C", "E"):
        nu, nv = (250, 200) if spec.name == "C" else (1000, 500)
        tmp = workdir or tempfile.mkdtemp(prefix="rt2_torus_")
        folder = os.path.join(tmp, f"torus_{nu}x{nv}")
        if not os.path.exists(os.path.join(folder, "torus.obj")):
            generate_torus_obj(folder, nu, nv)
        sd.load_obj_folder(folder)
        red, green, wall, light, mirror = _append_main_materials(sd, Material)
        if spec.name == "C":
            sd.add_cornell_box(0.17, 0.3, light, True)
        else:
            sd.add_mirror_cornell_box(0.17, 0.3, light, mirror)
    else:
        raise ValueError(name)
    sd.build_bvh()
    return sd, spec
