"""Generates the committed golden fixtures of tests/golden/ (run in the build
container, where /root/reference exists).  Every fixture is data: inputs and
expected outputs produced by the reference's own host code (oracle/_ref/ref_dump,
compiled from /root/reference by `make -C oracle ref`) or by this repo's loader
from the reference's model files.

  campfire_loaded.npz   RayTracing/Data/campfire through rt2's OBJ/MTL loader
                        (triangles + materials; the GPU box has no reference tree)
  camera_<W>x<H>.bin    GlobalUniforms from Camera(...)+updateUniforms (ref_dump)
  builders_campfire.bin the scene builders of rayTracing.cpp applied to campfire (ref_dump)
  builders_empty.bin    the same with no model (classic/diverse boxes)
  bvh_campfire_cornell.bin  BVH.h node array + reordered triangles (ref_dump)
  materials.bin         mesh.h Material constructors (ref_dump)
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import rt2  # noqa: E402

REF_DUMP = os.path.join(ROOT, "oracle", "_ref", "ref_dump")
DATA = "/root/reference/RayTracing/Data"


def main():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True, stdout=subprocess.DEVNULL)
    sd = rt2.SceneData()
    sd.load_obj_folder(os.path.join(DATA, "campfire"))
    tris, mats = sd.triangles(), sd.materials()
    np.savez_compressed(os.path.join(HERE, "campfire_loaded.npz"), triangles=tris, materials=mats)

    for W, H in ((256, 256), (1920, 1080), (3840, 2160), (1000, 1000), (64, 48)):
        subprocess.run([REF_DUMP, "camera", "-", os.path.join(HERE, f"camera_{W}x{H}.bin"), str(W), str(H)],
                       check=True, stdout=subprocess.DEVNULL)
    subprocess.run([REF_DUMP, "materials", "-", os.path.join(HERE, "materials.bin")], check=True,
                   stdout=subprocess.DEVNULL)

    tmp = os.path.join(HERE, "_campfire_tris.bin")
    tris.tofile(tmp)
    subprocess.run([REF_DUMP, "builders", tmp, os.path.join(HERE, "builders_campfire.bin")], check=True,
                   stdout=subprocess.DEVNULL)
    empty = os.path.join(HERE, "_empty.bin")
    open(empty, "wb").close()
    subprocess.run([REF_DUMP, "builders", empty, os.path.join(HERE, "builders_empty.bin")], check=True,
                   stdout=subprocess.DEVNULL)

    # BVH over campfire + addCornellBox (config B's scene before the BVH)
    sd2 = rt2.SceneData()
    sd2.load_obj_folder(os.path.join(DATA, "campfire"))
    lights = [sd2.add_material(rt2.Material.diffuse((1, 0, 0))) for _ in range(3)]
    light = sd2.add_material(rt2.Material.light((1, 1, 1), 15.0))
    sd2.add_cornell_box(0.17, 0.3, light, True)
    sd2.triangles().tofile(tmp)
    subprocess.run([REF_DUMP, "bvh", tmp, os.path.join(HERE, "bvh_campfire_cornell.bin")], check=True,
                   stdout=subprocess.DEVNULL)
    # BVH over the classic box (config A)
    sd3 = rt2.SceneData()
    sd3.create_classic_cornell_box(10.0, 0, 1, 2, 3)
    sd3.triangles().tofile(tmp)
    subprocess.run([REF_DUMP, "bvh", tmp, os.path.join(HERE, "bvh_classic.bin")], check=True,
                   stdout=subprocess.DEVNULL)
    os.remove(tmp)
    os.remove(empty)
    compact_builders(len(tris))
    print("golden fixtures written to", HERE)


BUILDERS = ["cornell", "mirror", "sidelit0", "sidelit1", "sky", "classic", "diverse"]


def read_builders(path):
    raw = open(path, "rb").read()
    off, out = 0, []
    for _ in BUILDERS:
        n = int(np.frombuffer(raw, np.int32, 1, off)[0])
        off += 4
        t = np.frombuffer(raw, rt2.TRI_DTYPE, n, off).copy()
        off += 80 * n
        b = np.frombuffer(raw, np.float32, 9 * n, off).reshape(n, 9).copy()
        off += 36 * n
        out.append((t, b))
    return out


def compact_builders(base_n):
    """builders_*.bin -> builders.npz keeping only what each builder appended."""
    arrays = {}
    for tag, path, base in (("campfire", "builders_campfire.bin", base_n), ("empty", "builders_empty.bin", 0)):
        full = os.path.join(HERE, path)
        for name, (t, b) in zip(BUILDERS, read_builders(full)):
            arrays[f"{tag}_{name}_tris"] = t[base:]
            arrays[f"{tag}_{name}_btris"] = b[base:]
        os.remove(full)
    np.savez_compressed(os.path.join(HERE, "builders.npz"), **arrays)


if __name__ == "__main__":
    main()
