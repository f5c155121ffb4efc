"""Lane-utilisation breakdown of the BVH kernel (variant 58 = bvh3 with DIAG
counters): where the 64 lanes of a wave spend the traversal loop."""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402,F401
import rt2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--variant", type=int, default=58)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--rays", type=int, default=0)
ap.add_argument("--frames", type=int, default=0)
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
W, H, R, F = a.width or spec.width, a.height or spec.height, a.rays or spec.rays, a.frames or spec.frames
u = rt2.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
scene = rt2.Scene(sd, 0)
scene.set_traversal("bvh")
scene.set_variant(a.variant)
scene.stats(reset=True)
scene.render_host(u, 0, F)
st = scene.stats(reset=False)
c = (C.c_ulonglong * 32)()
L = rt2.lib()
L.rt2_scene_diag_ex.restype = C.c_int
L.rt2_scene_diag_ex.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.c_int]
L.rt2_scene_diag_ex(scene._p, c, 32)
scene.stats(reset=True)
dg = [c[8 + k] for k in range(8)]
it = max(dg[0], 1)
out = {
    "config": a.config, "W": W, "H": H, "R": R, "F": F,
    "segments": st.segments, "interior_visits": st.node_visits, "leaf_tests": st.tests,
    "inner_iterations": dg[0], "outer_iterations": dg[5],
    "interior_lanes_per_iteration": dg[1] / it,
    "interior_lanes_when_body_runs": dg[1] / max(dg[7], 1),
    "leaf_lanes_per_iteration": dg[2] / it,
    "finished_waiting_lanes_per_iteration": dg[3] / it,
    "done_lanes_per_iteration": dg[4] / it,
    "shading_lanes_per_outer_iteration": dg[6] / max(dg[5], 1),
    "inner_iterations_per_outer": dg[0] / max(dg[5], 1),
}
print(json.dumps(out, indent=1))
