"""A/B of kernel variants in ONE process, interleaved rounds (cdna guide §5.4 rule 24).
Renders a configuration with each variant, checks every variant's image is
bit-identical to the first variant's, reports median / min ms.  Experiment
variants need the experiment build: make -C raytracing2-fork_amd EXPERIMENTS=1
and RT2_LIB=exp in the environment."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402,F401  (one HIP runtime)
import rt2  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="B")
ap.add_argument("--variants", default="0,67")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--width", type=int, default=0)
ap.add_argument("--height", type=int, default=0)
ap.add_argument("--rays", type=int, default=0)
ap.add_argument("--frames", type=int, default=0)
ap.add_argument("--traversal", default="brute", choices=["brute", "bvh"])
ap.add_argument("--no-split", action="store_true", help="whole-pixel items for F > 1")
ap.add_argument("--cost-order", type=int, default=-1, help="1/0: force most-expensive-first item order on/off")
ap.add_argument("--no-check", default="", help="comma list of variants whose image is not compared (speed-of-light probes)")
ap.add_argument("--dup", default="", help="K,T: the scene's last K triangles repeated T times (every matrix-filter "
                                          "group identical: isolates the record-load cost from the paths)")
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
if a.dup:
    k, t = (int(x) for x in a.dup.split(","))
    tri = sd.triangles()[-k:]
    sd2 = rt2.SceneData()
    for m in sd.materials():
        sd2.add_material(rt2.Material.from_buffer_copy(m.tobytes()))
    sd2.add_triangles(np.concatenate([tri] * t))
    sd = sd2
W, H, R = a.width or spec.width, a.height or spec.height, a.rays or spec.rays
u = rt2.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
scene = rt2.Scene(sd, 0)
scene.set_traversal(a.traversal)
scene.set_frame_split(not a.no_split)
if a.cost_order >= 0:
    scene.set_cost_order(bool(a.cost_order))
F = a.frames or spec.frames
variants = [int(v) for v in a.variants.split(",")]
times = {v: [] for v in variants}
ref = None
sha = {}  # image digest per variant (compare across runs, e.g. with different environments)
import ctypes as C  # noqa: E402
import hashlib  # noqa: E402
diag = {}
for rnd in range(a.rounds):
    for v in variants:
        scene.set_variant(v)
        torch.cuda.synchronize()
        scene.stats(reset=True)
        t = time.perf_counter()
        img = scene.render_host(u, 0, F)
        times[v].append(time.perf_counter() - t)
        scene.stats(reset=True)
        c = (C.c_ulonglong * 32)()
        rt2.lib().rt2_scene_diag_ex(scene._p, c, 32)
        if a.traversal == "bvh":
            diag[v] = dict(segments=c[1], tests_per_segment=c[2] / max(c[1], 1),
                           interior_visits_per_segment=c[3] / max(c[1], 1),
                           refined_visit_frac=c[4] / max(c[3], 1),
                           wave_end_spread_ms=(c[7] - c[6]) * 1e-5 if c[7] > c[6] else None)
        elif c[2]:
            diag[v] = dict(segments=c[1], groups=c[2], groups_with_survivor=c[3], exact_iters=c[4],
                           lane_survivors=c[5], frac_groups_exact=c[3] / c[2], exact_iters_per_group=c[4] / c[2],
                           lane_survivor_rate=c[5] / (c[2] * 64 * 4),
                           wave_end_spread_ms=(c[7] - c[6]) * 1e-5 if c[7] > c[6] else None)
            diag[v]["raw"] = [int(x) for x in c[:16]]
            tt = [c[9], c[10], c[11], c[12]]  # render_mfma diag: shader clocks per phase (advance, sweep, shade, tail)
            if sum(tt):
                diag[v]["clock_share"] = dict(zip(("advance", "sweep", "shade", "tail"),
                                                  [round(x / sum(tt), 4) for x in tt]))
                diag[v]["sweep_clocks_per_group"] = round(c[10] / c[2], 1)
            tf = [c[13], c[14], c[15], c[16], c[17]]  # render_mfma_k5t tile_flow diag: wait, filter, exact, sweep, life
            if tf[4]:
                diag[v]["flow_clock_share"] = dict(
                    wait=round(tf[0] / tf[4], 4), filter=round(tf[1] / tf[4], 4), exact=round(tf[2] / tf[4], 4),
                    sweep=round(tf[3] / tf[4], 4), outside_sweep=round(1 - tf[3] / tf[4], 4))
                diag[v]["filter_clocks_per_group"] = round(tf[1] / c[2], 1)
                diag[v]["flow_clock_share"].update(issue=round(c[18] / tf[4], 4), claimer_wait=round(c[19] / tf[4], 4))
                diag[v]["claims"] = c[20]
                diag[v]["issue_clocks_per_claim"] = round(c[18] / max(c[20], 1), 1)
                diag[v]["claimer_wait_clocks_per_claim"] = round(c[19] / max(c[20], 1), 1)
        if rnd == 0:
            if ref is None:
                ref = img
            if str(v) not in a.no_check.split(","):
                assert np.array_equal(img, ref), f"variant {v} differs"
            sha[v] = hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest()[:16]
st = scene.stats(reset=True)
samples = W * H * R * F
out = {}
for v in variants:
    med = float(np.median(times[v]))
    out[rt2.lib().rt2_variant_name(v).decode()] = dict(variant=v, median_ms=round(med * 1e3, 2),
                                                        min_ms=round(min(times[v]) * 1e3, 2),
                                                        all_ms=[round(t * 1e3, 1) for t in times[v]],
                                                        msamples_s=round(samples / med / 1e6, 2))
print(json.dumps({"config": a.config, "W": W, "H": H, "R": R, "variants": out, "diag": diag, "image_sha256": sha},
                 indent=1))
