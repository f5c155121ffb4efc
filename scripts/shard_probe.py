"""Predicts strong-scaling efficiency on one GPU: renders the slab that every
rank r of N would own (rt2_shard {tile_rows, r, N}) and compares the SLOWEST
rank's time with 1/N of the whole image (a job of N ranks ends with its
slowest slab; VERDICT r4: timing rank 0 alone under-reported it).  (The 8-GPU
run itself is the driver's; this shows whether a 1/N slab still fills the
chip.)"""
import argparse
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
ap.add_argument("--traversal", default="brute")
ap.add_argument("--tile-rows", type=int, default=1)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--variants", default="0")
ap.add_argument("--ns", default="1,2,4,8", help="slab counts N to time (1/N of the image each)")
ap.add_argument("--cost-order", type=int, default=-1, help="1/0: most-expensive-first item order on/off")
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
scene = rt2.Scene(sd, 0)
scene.set_traversal(a.traversal)
if a.cost_order >= 0:
    scene.set_cost_order(bool(a.cost_order))


first = {}  # slab image of the first variant, per N: every variant must match it bit for bit


def slab_time_r(sh):
    first_key = (sh.nranks, sh.rank)
    rows = rt2.shard_rows(spec.height, sh)
    acc = torch.zeros((rows, spec.width, 4), device="cuda")
    scene.render(u, 0, spec.frames, sh, acc.data_ptr())
    torch.cuda.synchronize()
    ref = first.setdefault(first_key, acc.clone())
    assert torch.equal(acc, ref), f"slab {sh.rank}/{sh.nranks} differs from the first variant's"
    ts = []
    for _ in range(a.reps):
        acc.zero_()
        torch.cuda.synchronize()
        t = time.perf_counter()
        scene.render(u, 0, spec.frames, sh, acc.data_ptr())
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return min(ts)


for var in [int(v) for v in a.variants.split(",")]:
    scene.set_variant(var)
    per = {}
    for n in [int(x) for x in a.ns.split(",")]:
        per[n] = [slab_time_r(rt2.shard(a.tile_rows, r, n)) for r in range(n)]
        print(json.dumps({"progress": f"variant {var} N={n}", "slab_ms": [round(t * 1e3, 2) for t in per[n]]}),
              file=sys.stderr, flush=True)
    base = max(per[1]) if 1 in per else None
    print(json.dumps({"config": a.config, "traversal": a.traversal, "tile_rows": a.tile_rows, "variant": var, "cost_order": a.cost_order,
                      "name": rt2.lib().rt2_variant_name(var).decode() if var else "auto",
                      "slab_ms_max": {n: round(max(t) * 1e3, 2) for n, t in per.items()},
                      "slab_ms_all": {n: [round(x * 1e3, 2) for x in t] for n, t in per.items()},
                      "predicted_efficiency": {n: round(base / n / max(t), 3) for n, t in per.items()} if base else None}),
          flush=True)
