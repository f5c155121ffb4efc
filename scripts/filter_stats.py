"""Filter survivor statistics of the brute sweeps (diagnostic variants 81/82):
per wave-test, how often some lane passes the division-free filter (and the
wave enters the exact path), and the lane-level survivor rate."""
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
ap.add_argument("--variants", default="82,81")
ap.add_argument("--width", type=int, default=480)
ap.add_argument("--height", type=int, default=270)
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
u = rt2.offline_uniforms(a.width, a.height, spec.bounces, spec.rays, sd.num_triangles)
scene = rt2.Scene(sd, 0)
ok, A, n_out = C.c_int(), C.c_float(), C.c_int()
rt2.lib().rt2_scene_plk_info(scene._p, C.byref(ok), C.byref(A), C.byref(n_out))
res = {"plk_ok": ok.value, "A": A.value, "outside": n_out.value}
for v in [int(x) for x in a.variants.split(",")]:
    scene.set_variant(v)
    scene.stats(reset=True)
    t = time.perf_counter()
    scene.render_host(u, 0, 1)
    dt = time.perf_counter() - t
    st = scene.stats(reset=False)
    c = (C.c_ulonglong * 32)()
    rt2.lib().rt2_scene_diag_ex(scene._p, c, 32)
    scene.stats(reset=True)
    tests, wave_any, lanes = c[21], c[22], c[23]
    res[rt2.lib().rt2_variant_name(v).decode()] = dict(
        ms=round(dt * 1e3, 1), segments=st.segments, wave_tests=tests, lane_tests_est=st.tests,
        wave_any_rate=wave_any / max(tests, 1), lane_rate=lanes / max(st.tests, 1))
print(json.dumps(res, indent=1))
