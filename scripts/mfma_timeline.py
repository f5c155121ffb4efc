"""Per-wave timeline of the k16 brute-force kernel (diagnostic variants 210 /
222: 3 / 4 waves per SIMD) on config B: the whole image and rank slabs.
Each wave logs start, first lane out of items, end, its segment rounds by kind
(two 32-ray blocks, one, idle under the workgroup's lockstep, cooperative
drain) and its place (XCC, CU, SIMD).  Prints one JSON summary per launch and
saves the raw log (gpurun_out/mfma_timeline_<tag>.npz) for offline analysis."""
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
ap.add_argument("--runs", default="210:1,222:8,210:8", help="variant:N pairs (slab 1/N of the image)")
ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out"))
ap.add_argument("--wg-waves", type=int, default=4, help="waves per workgroup (16 for the resident kernel 287)")
a = ap.parse_args()
sd, spec = rt2.build_config_scene(a.config)
u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
scene = rt2.Scene(sd, 0)
n_log = 16384
log = torch.zeros((n_log, 10), dtype=torch.int64, device="cuda")
L = rt2.lib()
L.rt2_scene_set_wave_log.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32]
os.makedirs(a.out, exist_ok=True)


def pct(x):
    return [round(float(np.percentile(x, q)), 2) for q in (0, 10, 50, 90, 99, 100)] if len(x) else None


for run in a.runs.split(","):
    var, n = (int(v) for v in run.split(":"))
    if not rt2.has_variant(var):
        print(json.dumps({"variant": var, "skipped": "not in this build (RT2_LIB=exp)"}), flush=True)
        continue
    scene.set_variant(var)
    sh = rt2.shard(1, 0, n)
    rows = rt2.shard_rows(spec.height, sh)
    acc = torch.zeros((rows, spec.width, 4), device="cuda")
    scene.render(u, 0, spec.frames, sh, acc.data_ptr())  # warm-up
    log.zero_()
    L.rt2_scene_set_wave_log(scene._p, C.c_void_p(log.data_ptr()), n_log)
    acc.zero_()
    torch.cuda.synchronize()
    scene.render(u, 0, spec.frames, sh, acc.data_ptr())
    torch.cuda.synchronize()
    L.rt2_scene_set_wave_log(scene._p, None, 0)
    g = log.cpu().numpy()
    used = g[:, 2] > 0
    idx = np.flatnonzero(used)
    g = g[used]
    np.savez(os.path.join(a.out, f"mfma_timeline_v{var}_n{n}.npz"), log=g, wave=idx)
    t0 = g[:, 0].min()
    ms = lambda c: (g[:, c] - t0) / 1e5  # 100 MHz s_memrealtime ticks -> ms
    hw = g[:, 7].astype(np.uint64)
    hwid = (hw & 0xFFFFFFFF).astype(np.int64)
    xcc = ((hw >> 32) & 0xF).astype(np.int64)
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    shid = (hwid >> 12) & 1
    se = (hwid >> 13) & 7
    place = ((xcc * 8 + se) * 2 + shid) * 16 + cu
    simd_key = place * 4 + simd
    end = ms(2)
    dry = np.where(g[:, 1] > 0, ms(1), np.nan)
    r2, r1, idle, coop = g[:, 3], g[:, 4], g[:, 5], g[:, 6]
    work = 2 * r2 + r1 + coop  # 32-ray block sweeps (a drain round ~ one block)
    keys, inv = np.unique(simd_key, return_inverse=True)
    simd_work = np.bincount(inv, weights=work)
    simd_end = np.zeros(len(keys))
    np.maximum.at(simd_end, inv, end)
    wg = idx // a.wg_waves
    # per SIMD: how long its last wave ran alone (last end - second-to-last end)
    lone = []
    for k in range(len(keys)):
        e = np.sort(end[inv == k])
        lone.append(e[-1] - e[-2] if len(e) > 1 else 0.0)
    wkeys, winv = np.unique(wg, return_inverse=True)
    wg_end = np.zeros(len(wkeys))
    np.maximum.at(wg_end, winv, end)
    print(json.dumps({
        "variant": var, "name": L.rt2_variant_name(var).decode(), "slab": f"1/{n}", "waves": int(len(g)),
        "simds": int(len(keys)), "cus": int(len(np.unique(place))),
        "launch_ms": round(float(end.max()), 3),
        "start_ms_pct": pct(ms(0)), "first_dry_ms_pct": pct(dry[~np.isnan(dry)]), "end_ms_pct": pct(end),
        "wg_end_ms_pct": pct(wg_end), "simd_end_ms_pct": pct(simd_end),
        "rounds_two_blocks_pct": pct(r2), "rounds_one_block_pct": pct(r1), "rounds_idle_pct": pct(idle),
        "rounds_drain_pct": pct(coop),
        "block_sweeps_total": int(work.sum()), "simd_block_sweeps_pct": pct(simd_work),
        "simd_work_max_over_mean": round(float(simd_work.max() / simd_work.mean()), 4),
        "simd_lone_ms_pct": pct(np.array(lone)),
        "wave_work_pct": pct(work), "wave_work_max_over_mean": round(float(work.max() / work.mean()), 4),
        "clock_ghz_pct": pct((g[:, 9] - g[:, 8]) / np.maximum(g[:, 2] - g[:, 0], 1) / 10.0),
    }), flush=True)
