"""Generates the mid-size model fixtures of tests/golden/ (run in the build
container, where /root/reference exists): two texture-free bundled models of
the reference, loaded by this repo's OBJ/MTL loader (the GPU box has no
reference tree).  Data only: the loader's triangles and materials.

  windmill_loaded.npz   RayTracing/Data/windmill (1,805 triangles)
  cat_loaded.npz        RayTracing/Data/cat (2,832 triangles)

With addCornellBox they are the bench's configs W and K (raytracing2-fork_amd/
rt2/scenes.py): scenes of 57 and 89 32-triangle groups, between the 38 the
LDS holds and the 256 of the L2-resident kernels."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import rt2  # noqa: E402

DATA = "/root/reference/RayTracing/Data"

for name in ("windmill", "cat"):
    sd = rt2.SceneData()
    sd.load_obj_folder(os.path.join(DATA, name))
    np.savez_compressed(os.path.join(HERE, f"{name}_loaded.npz"), triangles=sd.triangles(), materials=sd.materials())
    print(name, sd.num_triangles)
