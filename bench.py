#!/usr/bin/env python3
"""Benchmark of the MI355X render path on BASELINE.json's metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B] [--no-cpu-baseline]

One "step" = one render of the configuration's image (config B: campfire +
Cornell box, 1920x1080, 64 rays/pixel x 1 frame, 8 bounces) —
rt2_render into a device accumulator + the device resolve (+ one RCCL gather of
the framebuffer to rank 0 for N > 1; rows interleaved across ranks, so the
image is fixed as N grows: strong scaling).  Inputs (scene arrays) are
uploaded to HBM before the timed region.  For N > 1 the driver launches one
process per GPU through torch.distributed.run.

Prints ONE JSON line (rank 0):
  value       Msamples/s of the whole job = W*H*R*F*K / max-over-ranks wall time
  roofline    dominant kernel (the render kernel), FP32-VALU-bound: algorithmic
              FLOP = 53 x ray-triangle tests per launch / the
              launch's average HIP-event duration, against 157.3 TFLOP/s; plus
              the north star's HBM-read figure (36 B x tests) against 8 TB/s
  cpu_baseline  the CPU restatement of compute.glsl (oracle/, reference-faithful
              BVH traversal) on the host cores, on a bounded strided pixel sample
              (every k-th pixel in raster order, full spp); the brute-force CPU
              rate is reported beside it
  parity      GPU pixels vs the CPU oracle on those same sampled pixels
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))

METRIC = "Msamples/sec at 1920×1080 Cornell+OBJ; per-pixel RMSE vs CPU ref"
VALU_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (MI355X_MICROARCH.md, chip-level parameters)
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec
FLOP_PER_TEST = 53
FLOP_PER_VISIT = 24        # BVH interior node: 2 boxes x (6 sub + 6 div), compute.glsl:382-408
BYTES_PER_TEST = 36        # a, b, c positions
KERNEL_NAMES = {"brute": "render_smem (rt2_render.hip, variant smem/256/max3f8/coop32/w6)",
                "bvh": "render_bvh3 (rt2_render.hip, variant bvh3/256/t16/w5)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="B")
    ap.add_argument("--tile-rows", type=int, default=1)
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--traversal", default="brute", choices=["brute", "bvh"],
                    help="brute = the north-star kernel (default); bvh = the reference's traversal on the GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-alt", action="store_true", help="skip timing the other traversal beside the headline")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target seconds per CPU baseline mode")
    return ap.parse_args()


def launched_kernel(rt2, scene, traversal):
    """Kernel + variant of the scene's last launch (the auto choice depends on
    the slab size: rank slabs at N > 1 take other variants than the full image)."""
    import ctypes as C
    c = (C.c_ulonglong * 8)()
    lv = C.c_int(-1)
    rt2.lib().rt2_scene_diag(scene._p, c, C.byref(lv))
    name = rt2.lib().rt2_variant_name(lv.value) if lv.value >= 0 else None
    if not name:
        return KERNEL_NAMES[traversal]
    name = name.decode()
    kern = {"smem": "render_smem", "split": "render_split", "tiled": "render_tiled", "resident": "render_resident",
            "bvh3": "render_bvh3", "bvh2": "render_bvh2", "bvh": "render_bvh"}
    for prefix, k in kern.items():
        if name.startswith(prefix):
            return f"{k} (rt2_render.hip, variant {name})"
    return name


def cpu_baseline(sd, spec, u, gpu_image, threads):
    """Times oracle/ (CPU restatement of compute.glsl) on a strided pixel sample
    (every k-th pixel in raster order, full spp) and checks the GPU's pixels
    against it.  Test infrastructure: the oracle is only the checker / baseline
    here, never the measured path."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    tris, mats, nodes = sd.triangles(), sd.materials(), sd.nodes()
    H, W = spec.height, spec.width
    npx_all = H * W
    res = {}
    done = {}
    for mode in ("bvh", "brute"):
        # calibrate on a spread probe, then size the sample to ~cpu_seconds
        nprobe = 4 * threads
        pid = np.linspace(npx_all // 7, npx_all - 1 - npx_all // 7, nprobe).astype(np.int64)
        t0 = time.perf_counter()
        oracle.render_pixels(tris, mats, u, pid % W, pid // W, 0, spec.frames, mode, nodes=nodes, threads=threads)
        dt = max(time.perf_counter() - t0, 1e-3) / nprobe
        n = int(max(threads, min(npx_all, args.cpu_seconds / dt)))
        pid = np.arange(n, dtype=np.int64) * npx_all // n  # n pixels spread evenly in raster order
        xs, ys = pid % W, pid // W
        t0 = time.perf_counter()
        acc, _, segs, tests = oracle.render_pixels(tris, mats, u, xs, ys, 0, spec.frames, mode, nodes=nodes,
                                                   threads=threads)
        dt = time.perf_counter() - t0
        if dt < 0.4 * args.cpu_seconds and n < npx_all:  # the probe over-estimated: resize once
            n = int(min(npx_all, n * args.cpu_seconds / max(dt, 1e-3)))
            pid = np.arange(n, dtype=np.int64) * npx_all // n
            xs, ys = pid % W, pid // W
            t0 = time.perf_counter()
            acc, _, segs, tests = oracle.render_pixels(tris, mats, u, xs, ys, 0, spec.frames, mode, nodes=nodes,
                                                       threads=threads)
            dt = time.perf_counter() - t0
        samples = len(pid) * spec.rays * spec.frames
        res[mode] = dict(value=samples / dt / 1e6, pixels=int(len(pid)), seconds=dt,
                         segments_per_sample=segs / samples, tests_per_segment=tests / max(segs, 1))
        done[mode] = (ys, xs, acc / spec.frames)
    parity = None
    if gpu_image is not None:
        ds = []
        fr = {}
        for mode, (ys, xs, ref) in done.items():
            d = np.abs(gpu_image[ys, xs][..., :3] - ref[..., :3])
            ds.append(d)
            fr[mode] = float((d.max(-1) == 0).mean())
        parity = dict(pixels=int(sum(len(d) for d in ds)), oracle_modes=list(done),
                      exact_pixel_frac_brute=fr["brute"], exact_pixel_frac_bvh=fr["bvh"],
                      rmse=float(np.sqrt(np.concatenate([(d ** 2).ravel() for d in ds]).mean())),
                      max_abs=float(max(d.max() for d in ds)), tolerance_rmse=1e-4)
    return res, parity


def main():
    global args
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist
    import rt2
    from rt2 import dist as rdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # nccl = RCCL over xGMI (one rank per GPU).  RT2_BENCH_BACKEND=gloo is a
        # rehearsal mode for boxes with fewer GPUs than ranks (ranks share
        # devices, collectives staged through host memory); never the measured
        # configuration.
        backend = os.environ.get("RT2_BENCH_BACKEND", "nccl")
        local = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.cuda.current_device()

    sd, spec = rt2.build_config_scene(args.config)
    u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2.Scene(sd, dev)
    scene.set_traversal(args.traversal)
    if args.variant:
        scene.set_variant(args.variant)
    renderer = rdist.DeviceSlabRenderer(scene, u, 0, spec.frames, args.tile_rows, rank, world)

    def step():
        return rdist.render_distributed(renderer, spec.height, spec.width, args.tile_rows, rank, world)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    scene.stats(reset=True)

    stream = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    img = None
    for i in range(args.steps):
        # kernel-only bracket: rt2_render = counter reset + the render kernel, on this stream
        renderer.accum.zero_()
        ev[i][0].record(stream)
        scene.render(u, 0, spec.frames, renderer.sh, renderer.accum.data_ptr(), 0, stream.cuda_stream)
        ev[i][1].record(stream)
        rt2.resolve_rgba32f(renderer.accum.data_ptr(), renderer.rows * spec.width, spec.frames,
                            renderer.image.data_ptr(), stream.cuda_stream)
        img = renderer.image if world == 1 else rdist.gather_image(renderer.image, spec.height, spec.width,
                                                                    args.tile_rows, rank, world)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st = scene.stats(reset=True)
    kernel_name = launched_kernel(rt2, scene, args.traversal)
    t = torch.tensor([elapsed, kern_ms, float(st.tests), float(st.segments), float(st.node_visits)],
                     dtype=torch.float64, device="cuda")
    if world > 1:
        tmax = t.clone()
        dist.all_reduce(tmax[:2], op=dist.ReduceOp.MAX)
        tsum = t.clone()
        dist.all_reduce(tsum[2:], op=dist.ReduceOp.SUM)
        elapsed, kern_ms = float(tmax[0]), float(tmax[1])
        tests, segs, visits = float(tsum[2]), float(tsum[3]), float(tsum[4])
    else:
        tests, segs, visits = float(st.tests), float(st.segments), float(st.node_visits)

    samples_per_step = spec.width * spec.height * spec.rays * spec.frames
    value = samples_per_step * args.steps / elapsed / 1e6
    tests_per_launch = tests / args.steps / world
    visits_per_launch = visits / args.steps / world
    flops = (FLOP_PER_TEST * tests_per_launch + FLOP_PER_VISIT * visits_per_launch) / (kern_ms * 1e-3) / 1e12
    hbm_read = BYTES_PER_TEST * tests_per_launch / (kern_ms * 1e-3) / 1e9

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": f"config {spec.name}: {spec.description}", "width": spec.width,
                   "height": spec.height, "rays_per_pixel": spec.rays, "frames": spec.frames,
                   "max_bounce": spec.bounces, "triangles": sd.num_triangles,
                   "traversal": "brute force" if args.traversal == "brute" else "BVH (compute.glsl:410-460)",
                   "seed": "x + y*W + frame*968824447", "parallelism": f"row-tile x{world}" if world > 1 else "1 GPU",
                   "tile_rows": args.tile_rows},
        "roofline": {"bound": "valu", "achieved": round(flops, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(flops / VALU_PEAK_TFLOPS, 4), "traffic": None,
                     "kernel": kernel_name, "kernel_ms": round(kern_ms, 3),
                     "tests_per_launch": int(tests_per_launch),
                     "node_visits_per_launch": int(visits_per_launch),
                     "flop_model": "53 x ray-triangle tests + 24 x BVH interior visits (2 slab boxes)",
                     "segments_per_sample": round(segs / (samples_per_step * args.steps), 4),
                     "hbm_read_algorithmic": {"achieved": round(hbm_read, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                              "frac": round(hbm_read / HBM_PEAK_GBS, 3),
                                              "note": "36 B x tests; >1 = LDS reuse (effective bandwidth)"}},
        "cpu_baseline": None,
    }
    traffic_file = os.path.join(ROOT, "profiles", f"pmc_config{spec.name}.json")
    if world == 1 and os.path.exists(traffic_file):  # PMC traffic was measured for the 1-GPU launch
        with open(traffic_file) as f:
            out["roofline"]["traffic"] = json.load(f).get("hbm_bytes_per_launch")
        if out["roofline"]["traffic"]:
            # rocprof-measured HBM bandwidth of the launch (PMC bytes / this run's kernel time)
            gbs = out["roofline"]["traffic"] / (kern_ms * 1e-3) / 1e9
            out["roofline"]["hbm_measured"] = {"achieved": round(gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                               "frac": round(gbs / HBM_PEAK_GBS, 4),
                                               "source": f"profiles/pmc_config{spec.name}.json (FETCH_SIZE x2 + "
                                                         f"WRITE_SIZE, MI355X_MICROARCH.md HBM section)"}
    alt = "bvh" if args.traversal == "brute" else "brute"
    # brute force over 100k+ triangles takes minutes per step: not timed beside BVH there
    if world == 1 and not args.no_alt and (alt == "bvh" or sd.num_triangles <= 20000):
        # the other closest-hit algorithm on the same workload, same timing
        # bracket (reported beside the headline, never as `value`)
        img_main = img.clone()
        scene.set_traversal(alt)
        scene.set_variant(0)
        renderer.accum.zero_()
        scene.render(u, 0, spec.frames, renderer.sh, renderer.accum.data_ptr(), 0, stream.cuda_stream)
        torch.cuda.synchronize()
        scene.stats(reset=True)
        ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(args.steps)]
        t1 = time.perf_counter()
        for i in range(args.steps):
            renderer.accum.zero_()
            ev2[i][0].record(stream)
            scene.render(u, 0, spec.frames, renderer.sh, renderer.accum.data_ptr(), 0, stream.cuda_stream)
            ev2[i][1].record(stream)
            rt2.resolve_rgba32f(renderer.accum.data_ptr(), renderer.rows * spec.width, spec.frames,
                                renderer.image.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        el2 = time.perf_counter() - t1
        st2 = scene.stats(reset=True)
        ndiff = int((renderer.image[..., :3] != img_main[..., :3]).any(-1).sum().item())
        d2 = (renderer.image[..., :3] - img_main[..., :3]).double()
        out["alt_traversal"] = {
            "traversal": alt, "value": round(samples_per_step * args.steps / el2 / 1e6, 3),
            "ms_per_step": round(el2 / args.steps * 1e3, 3),
            "kernel": launched_kernel(rt2, scene, alt),
            "kernel_ms": round(float(np.mean([a.elapsed_time(b) for a, b in ev2])), 3),
            "segments_per_sample": round(st2.segments / (samples_per_step * args.steps), 4),
            "tests_per_segment": round(st2.tests / max(st2.segments, 1), 3),
            "node_visits_per_segment": round(st2.node_visits / max(st2.segments, 1), 3),
            "valu_tflops": round((FLOP_PER_TEST * st2.tests + FLOP_PER_VISIT * st2.node_visits) / args.steps
                                 / (float(np.mean([a.elapsed_time(b) for a, b in ev2])) * 1e-3) / 1e12, 3),
            "pixels_differing_from_main": ndiff,
            "rmse_vs_main": float(d2.pow(2).mean().sqrt()),
            "note": "brute force and the reference BVH traversal agree except on exact distance ties"}
        scene.set_traversal(args.traversal)
        scene.set_variant(args.variant)
    if world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        gpu_np = img.cpu().numpy() if img is not None else None
        res, parity = cpu_baseline(sd, spec, u, gpu_np, threads)
        out["cpu_baseline"] = {"value": round(res["bvh"]["value"], 4), "unit": "Msamples/s", "cores": threads,
                               "kind": "port",
                               "sample": f"{res['bvh']['pixels']} of {spec.width * spec.height} pixels, "
                                         f"i = floor(k*{spec.width * spec.height}/{res['bvh']['pixels']}) in raster "
                                         f"order, full spp, reference BVH traversal (compute.glsl:410-460), "
                                         f"{res['bvh']['seconds']:.1f} s",
                               "brute_force": {"value": round(res["brute"]["value"], 4),
                                               "pixels": res["brute"]["pixels"],
                                               "seconds": round(res["brute"]["seconds"], 2)},
                               "gpu_over_cpu_bvh": round(value / res["bvh"]["value"], 1),
                               "gpu_over_cpu_brute": round(value / res["brute"]["value"], 1)}
        out["parity"] = parity
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
