"""Matrix-filter survivor statistics (diagnostic variants 147 / 151 = the
matrix kernels 140 / 150 (the default) plus counters; experiment build, RT2_LIB=exp): per
(wave, 16-triangle group) sweep, how often a pair passes the filter (the wave
enters the exact phase) and how many (wave, triangle) exact tests follow."""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402,F401
import rt2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--variants", default="150,151")
ap.add_argument("--width", type=int, default=1920)
ap.add_argument("--height", type=int, default=1080)
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
u = rt2.offline_uniforms(a.width, a.height, spec.bounces, spec.rays, sd.num_triangles)
scene = rt2.Scene(sd, 0)
res = {"config": a.config, "width": a.width, "height": a.height, "triangles": sd.num_triangles}
imgs = {}
for v in [int(x) for x in a.variants.split(",")]:
    scene.set_variant(v)
    scene.render_host(u, 0, 1)  # warm
    scene.stats(reset=True)
    t = time.perf_counter()
    img = scene.render_host(u, 0, 1)
    dt = time.perf_counter() - t
    st = scene.stats(reset=False)
    c = (C.c_ulonglong * 32)()
    rt2.lib().rt2_scene_diag_ex(scene._p, c, 32)
    scene.stats(reset=True)
    imgs[v] = img
    groups, hot, exact = c[2], c[3], c[4]
    res[rt2.lib().rt2_variant_name(v).decode()] = dict(
        ms=round(dt * 1e3, 1), segments=st.segments, wave_groups=groups,
        hot_group_rate=hot / max(groups, 1), exact_tests_per_group=exact / max(groups, 1),
        exact_tests_per_hot_group=exact / max(hot, 1),
        wave_triangle_exact_rate=exact / max(16 * groups, 1))
vs = list(imgs)
res["bit_identical"] = all(bool((imgs[v] == imgs[vs[0]]).all()) for v in vs[1:])
print(json.dumps(res, indent=1))
