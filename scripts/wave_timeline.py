"""Per-wave timeline of the assist kernel on a config B slab (diagnostic):
when each wave started, when its workgroup's item pool ran dry for it, when it
ended — shows how much of a slab's time is the tail after the pool empties."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402
import rt2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--ns", default="2,4,8")
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
scene = rt2.Scene(sd, 0)
scene.set_variant(92)
n_waves = 256 * 4 * 8
log = torch.zeros((n_waves, 4), dtype=torch.int64, device="cuda")
L = rt2.lib()
L.rt2_scene_set_wave_log.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
for n in [int(x) for x in a.ns.split(",")]:
    sh = rt2.shard(1, 0, n)
    rows = rt2.shard_rows(spec.height, sh)
    acc = torch.zeros((rows, spec.width, 4), device="cuda")
    scene.render(u, 0, spec.frames, sh, acc.data_ptr())  # warm-up
    log.zero_()
    L.rt2_scene_set_wave_log(scene._p, C.c_void_p(log.data_ptr()), n_waves)
    acc.zero_()
    scene.render(u, 0, spec.frames, sh, acc.data_ptr())
    torch.cuda.synchronize()
    L.rt2_scene_set_wave_log(scene._p, None, 0)
    g = log.cpu().numpy().astype(np.float64)
    g = g[g[:, 2] > 0]
    t0 = g[:, 0].min()
    st, dry, end = (g[:, 0] - t0) / 1e5, (g[:, 1] - t0) / 1e5, (g[:, 2] - t0) / 1e5  # ms (10-ns ticks)
    owners = g[:, 3] > 0
    dry_o = dry[owners & (g[:, 1] > 0)]
    q = lambda x: [round(float(np.percentile(x, p)), 2) for p in (0, 10, 50, 90, 99, 100)]
    print(json.dumps({"slab": f"1/{n}", "waves": int(len(g)), "owner_waves": int(owners.sum()),
                      "start_ms_pct": q(st), "owner_pool_dry_ms_pct": q(dry_o) if len(dry_o) else None,
                      "end_ms_pct": q(end), "segments": int(g[:, 3].sum())}), flush=True)
