"""Pixel-level comparison of kernel variants against a reference variant
(debugging aid): renders a configuration with each variant and reports how
many pixels differ from the first variant's image and by how much."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402,F401
import rt2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="A")
ap.add_argument("--variants", default="282,342")
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--rays", type=int, default=0)
ap.add_argument("--frames", type=int, default=0)
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
W, H, R = a.width or spec.width, a.height or spec.height, a.rays or spec.rays
F = a.frames or spec.frames
u = rt2.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
scene = rt2.Scene(sd, 0)
ref = None
for v in [int(x) for x in a.variants.split(",")]:
    scene.set_variant(v)
    img = scene.render_host(u, 0, F)
    st = scene.stats(reset=False)
    import ctypes as C
    c = (C.c_ulonglong * 32)()
    rt2.lib().rt2_scene_diag_ex(scene._p, c, 32)
    scene.stats(reset=True)
    diag = list(c)[16:24]
    if ref is None:
        ref = img
    d = np.abs(img[..., :3] - ref[..., :3]).max(-1)
    bad = np.argwhere(d > 0)
    print(json.dumps({"variant": v, "name": rt2.lib().rt2_variant_name(v).decode(), "segments": st.segments,
                      "pixels_differing": int(len(bad)), "max_abs": float(d.max()),
                      "first": bad[:8].tolist(), "diag16_23": diag}), flush=True)
