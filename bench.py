#!/usr/bin/env python3
"""Benchmark of the MI355X render path on BASELINE.json's metric.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config B] [--traversal brute|bvh]
                    [--no-cpu-baseline] [--no-alt] [--no-config-c] [--no-config-e] [--no-config-w] [--no-scalar]

--gpus N > 1 without a launcher starts N ranks itself (torch.distributed.run,
one process per GPU, master 127.0.0.1); under a launcher WORLD_SIZE must equal N.

One "step" = one render of the configuration's image (config B: campfire +
Cornell box, 1920x1080, 64 rays/pixel x 1 frame, 8 bounces) —
rt2_render into a device accumulator + the device resolve (+ one RCCL gather of
the framebuffer to rank 0 for N > 1; rows interleaved across ranks, so the
image is fixed as N grows: strong scaling).  Inputs (scene arrays) are
uploaded to HBM before the timed region.  For N > 1 one process per GPU runs
under torch.distributed.run (the driver's launch, or bench.py's own).

Prints ONE JSON line (rank 0):
  value         Msamples/s of the whole job = W*H*R*F*K / max-over-ranks wall time
  roofline      dominant kernel (the render kernel), FP32-VALU-bound: algorithmic
                FLOP = 53 x ray-triangle tests per launch / the
                launch's average HIP-event duration, against 157.3 TFLOP/s; plus
                the north star's HBM-read figure (36 B x tests) against 8 TB/s.
                `traffic` = PMC-measured HBM bytes per launch from
                profiles/pmc_config<X>.json, attached only when that profile was
                taken of the same kernel variant built from the same kernel sources
  cpu_baseline  the CPU restatement of compute.glsl (oracle/, reference-faithful
                BVH traversal) on the host CPUs this job may use (the cgroup CPU
                quota of a GPU box), on a bounded evenly spread pixel sample at
                full spp; the brute-force CPU rate beside it; the host's model,
                core counts and a linear extrapolation to every core of the node
  parity        GPU pixels vs the CPU oracle on those same sampled pixels
  config_C      (1 GPU, config B runs) the north-star target configuration
                (100k triangles, 1920x1080, 256 spp): one brute-force step with
                its own roofline, the BVH kernel, the CPU baseline, parity, and
                whether the >= 10x target is met and by which kernel
  config_E      (1 GPU, config B runs) 1M triangles, mirror box, 16 bounces, 4
                spp: the same legs as config_C
  config_W      (1 GPU, config B runs) config B with the reference's windmill
                model (1,821 triangles = 57 groups: beyond the 38 whose records
                the LDS holds): the same legs
  scalar_valu   (1 GPU) the no-MFMA scalar-path kernel (render_smem) on the
                headline workload with its FP32-VALU roofline and parity
"""
import argparse
import glob
import hashlib
import json
import os
import re
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
BVH_RECORD_BYTES = 64      # BVH: one child-pair record per interior visit (both boxes + entries)
BVH_TRI_BYTES = 48         # BVH: one pre-transformed triangle record per leaf test
L2_PEAK_GBS = 34500.0      # MI355X_MICROARCH.md §L2: ≈34.5 TB/s aggregate
MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense F16/BF16 matrix peak (MI355X_MICROARCH.md; no sparsity)
MAX_CLOCK_GHZ = 2.4        # MI355X_MICROARCH.md chip-level parameters: the clock the dense peaks are quoted at
MFMA_FLOP_PER_PAIR = 320   # render_mfma 16x16x32 form: 5 quantities x 32 k-slots x 2 per (ray, triangle) pair
MFMA_K16_FLOP_PER_PAIR = 256  # the k16 sweep: 8 v_mfma_f32_32x32x16_f16 (32x32x16x2 FLOP each) per 1,024 pairs
MFMA_K5_FLOP_PER_PAIR = 160   # its 5-product form (MfmaSpec::k5): 5 v_mfma_f32_32x32x16_f16 per 1,024 pairs
MFMA_K5_NOTN_FLOP_PER_PAIR = 128  # ... without the -tn term (small scenes): 4 per 1,024 pairs
SCALAR_VARIANT = 136       # render_smem forced (rt2_render.hip): the no-MFMA scalar-path kernel
TARGET_RATIO = 10.0        # north star: >= 10x the CPU reference at config C on 1 GPU
KERNEL_FILES = {"mfmat5": "render_mfma_k5t", "mfmarl2": "render_mfma_k5r", "mfmar": "render_mfma_k5r", "mfma": "render_mfma", "massist": "render_assist", "smem": "render_smem", "split": "render_split", "tiled": "render_tiled", "assist": "render_assist",
                "resident": "render_resident", "bvh4": "render_bvh4", "bvh3": "render_bvh3", "bvh2": "render_bvh2",
                "bvh": "render_bvh"}


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
    ap.add_argument("--no-config-c", action="store_true", help="skip the config C (north-star target) leg")
    ap.add_argument("--no-config-e", action="store_true", help="skip the config E (1M triangles, mirror box) leg")
    ap.add_argument("--no-config-w", action="store_true",
                    help="skip the config W leg (windmill + Cornell box: 57 triangle groups, beyond the 38 the LDS holds)")
    ap.add_argument("--no-scalar", action="store_true",
                    help="skip the scalar-VALU leg (render_smem, the north star's no-MFMA kernel, on the headline workload)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target seconds per CPU baseline mode")
    ap.add_argument("--plumbing", action="store_true",
                    help="launch/collective path only, no GPU (CPU tests of --gpus N): each rank gathers a synthetic "
                         "slab of its image rows and rank 0 checks the assembled image")
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ensure_world(args):
    """`--gpus N` on its own: with no launcher (WORLD_SIZE unset) and N > 1, start
    one fresh process per GPU through torch.distributed.run (master 127.0.0.1)
    and exit with its status — this process has made no GPU call (torch is not
    even imported yet), so nothing is inherited or exec'd from a GPU-initialised
    process.  Under a launcher, WORLD_SIZE must equal --gpus."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks",
                  file=sys.stderr)
            sys.exit(2)
        return
    if args.gpus <= 1:
        return
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def plumbing(args, world, rank):
    """The N-rank launch + gather path without a GPU: rank r's slab holds its own
    image rows (value = row index), gathered to rank 0 and checked there."""
    import torch
    import torch.distributed as dist
    from rt2 import dist as rdist
    H, W = 64, 8
    ids = rdist.slab_row_ids(H, args.tile_rows, rank, world)
    slab = torch.as_tensor(ids, dtype=torch.float32)[:, None, None].expand(len(ids), W, 4).contiguous()
    t0 = time.perf_counter()
    img = rdist.gather_image(slab, H, W, args.tile_rows, rank, world) if world > 1 else slab
    dist.barrier() if world > 1 else None
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    if rank == 0:
        ok = bool((img[:, :, 0] == torch.arange(H, dtype=torch.float32)[:, None]).all())
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Msamples/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "plumbing": True, "gather_ok": ok,
                          "ms_per_step": round(float(el[0]) * 1e3, 3), "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
                          "config": {"workload": "plumbing: row-tile gather of a 64x8 synthetic image",
                                     "parallelism": f"row-tile x{world}" if world > 1 else "1 GPU"}}), flush=True)
    if world > 1:
        dist.destroy_process_group()


# Device sources the brute-force and BVH render kernels are compiled from (one
# translation unit; the launcher policy in rt2_render.hip does not change their
# code).  A PMC profile carries the digest of the sources it was measured on.
KERNEL_SOURCES = ["raytracing2-fork_amd/csrc/device/rt2_math.h", "raytracing2-fork_amd/csrc/device/rt2_sweep.h",
                  "raytracing2-fork_amd/csrc/device/rt2_path.h", "include/rt2_pinned_math.h", "include/rt2.h"]
KERNEL_SOURCES_BY_TRAVERSAL = {"brute": ["raytracing2-fork_amd/csrc/device/rt2_brute.h",  # the brute-force kernels
                                         "raytracing2-fork_amd/csrc/device/rt2_mfma.h",
                                         "raytracing2-fork_amd/csrc/device/rt2_k5_tiles.h",
                                         "raytracing2-fork_amd/csrc/device/rt2_k5_resident.h",
                                         "raytracing2-fork_amd/csrc/device/rt2_assist.h"],
                               "bvh": ["raytracing2-fork_amd/csrc/device/rt2_bvh.h"]}


def _code_only(text):
    """Source text without comments and blank-line differences (a comment edit
    does not change the kernel)."""
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", "", text)
    return "\n".join(line.rstrip() for line in text.splitlines() if line.strip())


def kernel_source_digest(traversal="brute"):
    """sha256 over the code (comments stripped) of one traversal's kernel sources."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES + KERNEL_SOURCES_BY_TRAVERSAL[traversal]:
        h.update(os.path.basename(f).encode())
        with open(os.path.join(ROOT, f), encoding="utf-8") as fh:
            h.update(_code_only(fh.read()).encode())
    return h.hexdigest()


def launched_variant(rt2, scene):
    """Name of the kernel variant of the scene's last launch (the automatic
    choice depends on the slab size: rank slabs at N > 1 take other variants)."""
    import ctypes as C
    c = (C.c_ulonglong * 8)()
    lv = C.c_int(-1)
    rt2.lib().rt2_scene_diag(scene._p, c, C.byref(lv))
    name = rt2.lib().rt2_variant_name(lv.value) if lv.value >= 0 else None
    return name.decode() if name else None


def kernel_label(variant):
    if not variant:
        return None
    for prefix, k in KERNEL_FILES.items():
        if variant.startswith(prefix):
            return f"{k} (rt2_render.hip, variant {variant})"
    return variant


def roofline(tests, visits, kern_ms, segments=0, n_tris=0, variant=None):
    """Roofline of one launch.  Scalar-path / BVH kernels: FP32-VALU bound,
    algorithmic FLOP / kernel time.  The matrix-core kernel (render_mfma): its
    filter products on the MFMA pipe (320 FLOP per ray-triangle pair over the
    16-padded triangle count) against the dense F16 peak, with the
    reference-formulation VALU figure (53 FLOP per test) beside it."""
    flops = (FLOP_PER_TEST * tests + FLOP_PER_VISIT * visits) / (kern_ms * 1e-3) / 1e12
    hbm = BYTES_PER_TEST * tests / (kern_ms * 1e-3) / 1e9
    rf = {"bound": "valu", "achieved": round(flops, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
          "frac": round(flops / VALU_PEAK_TFLOPS, 4), "traffic": None, "kernel_ms": round(kern_ms, 3),
          "tests_per_launch": int(tests), "node_visits_per_launch": int(visits),
          "flop_model": "53 x ray-triangle tests + 24 x BVH interior visits (2 slab boxes)",
          "hbm_read_algorithmic": {"achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(hbm / HBM_PEAK_GBS, 3),
                                   "note": "36 B x tests; >1 = on-chip reuse (effective bandwidth)"}}
    if variant and variant.startswith(("mfma", "massist")) and segments and n_tris:
        kt = re.search(r"/kt\d/", variant) is not None  # the threshold in the K-slots: U, -V, X, Y per block
        k5 = "/k5/" in variant or kt
        k16 = "/k16/" in variant or k5
        group = 32 if k16 else 16
        pairs = segments * (-(-int(n_tris) // group) * group)
        notn = k5 and ("/notn/" in variant or kt)
        fpp = (MFMA_K5_NOTN_FLOP_PER_PAIR if notn else MFMA_K5_FLOP_PER_PAIR if k5 else MFMA_K16_FLOP_PER_PAIR if k16
               else MFMA_FLOP_PER_PAIR)
        mf = fpp * pairs / (kern_ms * 1e-3) / 1e12
        model = ("128 x (ray, triangle) pairs: the threshold in the K-slots, 4 v_mfma_f32_32x32x16_f16 per 32 rays "
                 "x 32 triangles (U, -V, X, Y: one K-half each, the threshold two of its slots), triangles padded to 32"
                 if kt else
                 "128 x (ray, triangle) pairs: the 5-product k16 form without -tn, 4 v_mfma_f32_32x32x16_f16 per "
                 "32 rays x 32 triangles (U, -V, X, Y: one K-half each), triangles padded to 32" if notn else
                 "160 x (ray, triangle) pairs: the 5-product k16 form's 5 v_mfma_f32_32x32x16_f16 per 32 rays x 32 "
                 "triangles (U, -V, X, -tn, Y: one K-half each), triangles padded to 32" if k5 else
                 "256 x (ray, triangle) pairs: the k16 sweep's 8 v_mfma_f32_32x32x16_f16 per 32 rays x 32 "
                 "triangles (U, -V, X: two K-halves each; -tn, Y: one), triangles padded to 32"
                 if k16 else "320 x (ray, triangle) pairs (5 f16x3 products of 32 k-slots per pair, triangles "
                             "padded to 16)")
        rf.update({"bound": "mfma", "achieved": round(mf, 3), "peak": MFMA_F16_PEAK_TFLOPS,
                   "frac": round(mf / MFMA_F16_PEAK_TFLOPS, 4),
                   "pairs_per_s": float(f"{pairs / (kern_ms * 1e-3):.4e}"),
                   "flop_model": model + "; rays = segments (the active lanes) on the matrix cores",
                   "valu_algorithmic": {"achieved": round(flops, 3), "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                                        "frac": round(flops / VALU_PEAK_TFLOPS, 4),
                                        "note": "53 FLOP x tests (the reference formulation) / kernel time: the "
                                                "rate the scalar-path kernels are measured in; the filter runs on "
                                                "the matrix cores, so this is an effective figure"}})
    if visits:
        # the BVH walk is a chain of dependent per-lane gathers: its bound is
        # the cache hierarchy, not the VALU (DESIGN.md §BVH traversal)
        l2 = (BVH_RECORD_BYTES * visits + BVH_TRI_BYTES * tests) / (kern_ms * 1e-3) / 1e9
        rf["l2_read_algorithmic"] = {"achieved": round(l2, 1), "peak": L2_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(l2 / L2_PEAK_GBS, 3),
                                     "note": "64 B per interior visit + 48 B per leaf test, per-lane gathers"}
    return rf


def attach_traffic(rf, config, variant, kern_ms):
    """roofline.traffic from profiles/pmc_config<X>.json — only when that PMC
    profile was taken of this kernel variant built from these kernel sources."""
    path = os.path.join(ROOT, "profiles", f"pmc_config{config}.json")
    if not os.path.exists(path):
        rf["traffic_note"] = f"no PMC profile for config {config}"
        return
    with open(path) as f:
        prof = json.load(f)
    digest = kernel_source_digest("bvh" if config.endswith("_bvh") else "brute")
    if prof.get("kernel_variant") != variant or prof.get("kernel_source_sha256") != digest:
        rf["traffic_note"] = (f"profiles/pmc_config{config}.json was measured on variant "
                              f"{prof.get('kernel_variant')} / sources {str(prof.get('kernel_source_sha256'))[:12]}, "
                              f"not this launch ({variant} / {digest[:12]}): traffic not attached")
        return
    clk = prof.get("clock_ghz")
    if clk and rf.get("bound") == "mfma":
        # the dense peak is quoted at 2.4 GHz; the kernel holds a lower clock
        # under load (DVFS give-back): its own ceiling is peak x clock / 2.4
        pk = rf["peak"] * clk / MAX_CLOCK_GHZ
        rf.update({"clock_ghz": round(clk, 3), "peak_at_clock": round(pk, 1),
                   "frac_at_clock": round(rf["achieved"] / pk, 4),
                   "clock_source": f"profiles/pmc_config{config}.json: GRBM_GUI_ACTIVE / 8 / kernel ns "
                                   "(kernel trace of the same --pmc pass)"})
    b = prof.get("hbm_bytes_per_launch")
    if not b:
        return
    rf["traffic"] = b
    gbs = b / (kern_ms * 1e-3) / 1e9
    rf["hbm_measured"] = {"achieved": round(gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(gbs / HBM_PEAK_GBS, 5),
                          "source": f"profiles/pmc_config{config}.json (FETCH_SIZE x2 + WRITE_SIZE, separate "
                                    f"--pmc passes, MI355X_MICROARCH.md HBM section; kernel sources "
                                    f"{digest[:12]})"}


def progress(msg):
    """One progress line on stderr (the JSON line alone goes to stdout): a
    long run (config D, the C / E legs) shows that it is alive."""
    print(f"bench.py: {msg}", file=sys.stderr, flush=True)


def timed_renders(torch, rt2, scene, u, frames, sh, accum, image, steps, stream):
    """`steps` renders, each bracketed by HIP events on the stream it runs on;
    returns (wall seconds, mean kernel ms, stats)."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    scene.stats(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        accum.zero_()
        ev[i][0].record(stream)
        scene.render(u, 0, frames, sh, accum.data_ptr(), 0, stream.cuda_stream)
        ev[i][1].record(stream)
        rt2.resolve_rgba32f(accum.data_ptr(), accum.shape[0] * accum.shape[1], frames, image.data_ptr(),
                            stream.cuda_stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / steps
    return el, kern_ms, scene.stats(reset=True)


def cpu_baseline(sd, spec, u, gpu_images, threads, seconds):
    """Times oracle/ (CPU restatement of compute.glsl) in both traversals on an
    evenly spread pixel sample (every k-th pixel in raster order, full spp) of
    ~`seconds` each, and checks the GPU images' pixels against it (brute GPU
    image vs brute oracle, BVH vs BVH: bit-exact).  Test infrastructure: the
    oracle is the checker / baseline here, never the measured path."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle
    tris, mats, nodes = sd.triangles(), sd.materials(), sd.nodes()
    H, W = spec.height, spec.width
    npx_all = H * W
    res, done = {}, {}
    for mode in ("bvh", "brute"):
        nprobe = 2 * threads
        pid = np.linspace(npx_all // 7, npx_all - 1 - npx_all // 7, nprobe).astype(np.int64)
        t0 = time.perf_counter()
        oracle.render_pixels(tris, mats, u, pid % W, pid // W, 0, spec.frames, mode, nodes=nodes, threads=threads)
        dt = max(time.perf_counter() - t0, 1e-3) / nprobe
        n = int(max(threads, min(npx_all, seconds / dt)))
        for attempt in range(2):
            pid = np.arange(n, dtype=np.int64) * npx_all // n  # n pixels spread evenly in raster order
            xs, ys = pid % W, pid // W
            t0 = time.perf_counter()
            acc, _, segs, tests = oracle.render_pixels(tris, mats, u, xs, ys, 0, spec.frames, mode, nodes=nodes,
                                                       threads=threads)
            dt = time.perf_counter() - t0
            if attempt == 1 or dt >= 0.4 * seconds or n >= npx_all:
                break
            n = int(min(npx_all, n * seconds / max(dt, 1e-3)))  # the probe over-estimated: resize once
        samples = len(pid) * spec.rays * spec.frames
        res[mode] = dict(value=samples / dt / 1e6, pixels=int(len(pid)), seconds=dt,
                         segments_per_sample=segs / samples, tests_per_segment=tests / max(segs, 1))
        done[mode] = (ys, xs, acc / spec.frames)
    ds, exact = [], {}
    for mode, (ys, xs, ref) in done.items():
        img = gpu_images.get(mode)
        if img is None:
            continue
        d = np.abs(img[ys, xs][..., :3].astype(np.float64) - ref[..., :3])
        ds.append(d)
        exact[mode] = float((d.max(-1) == 0).mean())
    parity = None
    if ds:
        parity = dict(pixels=int(sum(len(d) for d in ds)), pairs="GPU brute vs oracle brute, GPU BVH vs oracle BVH",
                      exact_pixel_frac=exact, rmse=float(np.sqrt(np.concatenate([(d ** 2).ravel() for d in ds]).mean())),
                      max_abs=float(max(d.max() for d in ds)), tolerance_rmse=1e-4)
    return res, parity


def cpu_summary(res, threads, host, sample_desc, gpu_values):
    """cpu_baseline object: the measured rate on the CPUs this job may use, the
    host's core counts, and a linear extrapolation to the whole node."""
    logical, phys = host.get("logical_cpus") or threads, host.get("physical_cores") or threads
    v = res["bvh"]["value"]
    node_hi = v / threads * logical   # every hardware thread at the measured per-thread rate (upper bound)
    node_lo = v / threads * phys      # one thread per physical core (SMT adds nothing)
    out = {"value": round(v, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
           "sample": sample_desc,
           "host": {**host, "threads_used": threads,
                    "note": "threads = the CPUs this job may use: the affinity mask capped by the cgroup CPU quota "
                            "(a GPU box grants a one-GPU job 16 CPUs of its node; more threads would add no CPU "
                            "time and exceed the pool's worker sizing)"},
           "brute_force": {"value": round(res["brute"]["value"], 5), "pixels": res["brute"]["pixels"],
                           "seconds": round(res["brute"]["seconds"], 2)},
           "node_extrapolated": {"value_all_logical_cpus": round(node_hi, 3),
                                 "value_all_physical_cores": round(node_lo, 3),
                                 "note": "linear scaling of the measured per-thread BVH rate to the node's "
                                         f"{logical} hardware threads (upper bound) / {phys} physical cores; "
                                         "an estimate, not a measurement"}}
    for name, g in gpu_values.items():
        out[f"gpu_{name}_over_cpu_bvh"] = round(g / v, 2)
        out[f"gpu_{name}_over_cpu_brute"] = round(g / res["brute"]["value"], 1)
        out[f"gpu_{name}_over_node_extrapolated_bvh"] = round(g / node_hi, 2)
    return out


def config_leg(torch, rt2, stream, threads, host, seconds, do_cpu, name="C"):
    """A second configuration on one GPU, timed beside the headline: config C
    (the north-star target: 100k triangles, 256 spp) or config E (1M
    triangles, mirror box, 16 bounces: the divergence stress).  Brute force (1
    timed step: ~33 s / ~12 s of kernel) with its roofline (PMC traffic from
    profiles/pmc_config<X>.json when it matches), the BVH traversal (3 steps),
    the CPU baseline on the same sample and parity against the oracle."""
    import numpy as np
    sd, spec = rt2.build_config_scene(name)
    u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2.Scene(sd, torch.cuda.current_device())
    sh = rt2.shard()
    accum = torch.zeros((spec.height, spec.width, 4), dtype=torch.float32, device="cuda")
    image = torch.empty_like(accum)
    samples = spec.width * spec.height * spec.rays * spec.frames
    out = {"workload": f"config {name}: {spec.description}", "width": spec.width, "height": spec.height,
           "rays_per_pixel": spec.rays, "frames": spec.frames, "max_bounce": spec.bounces,
           "triangles": sd.num_triangles}
    legs, imgs = {}, {}
    for trav, steps, warm in (("bvh", 3, 1), ("brute", 1 if sd.num_triangles > 20000 else 3, 0 if sd.num_triangles > 20000 else 1)):
        progress(f"config {name}: {trav} ({steps} step(s))")
        scene.set_traversal(trav)
        for _ in range(warm):
            accum.zero_()
            scene.render(u, 0, spec.frames, sh, accum.data_ptr(), 0, stream.cuda_stream)
        el, kern_ms, st = timed_renders(torch, rt2, scene, u, spec.frames, sh, accum, image, steps, stream)
        variant = launched_variant(rt2, scene)
        rf = roofline(st.tests / steps, st.node_visits / steps, kern_ms, st.segments / steps, sd.num_triangles,
                      variant)
        rf["kernel"] = kernel_label(variant)
        attach_traffic(rf, name if trav == "brute" else f"{name}_bvh", variant, kern_ms)
        legs[trav] = {"value": round(samples * steps / el / 1e6, 4), "unit": "Msamples/s", "steps": steps,
                      "ms_per_step": round(el / steps * 1e3, 1), "roofline": rf,
                      "segments_per_sample": round(st.segments / (samples * steps), 4)}
        imgs[trav] = image.cpu().numpy()
    out["brute"], out["bvh"] = legs["brute"], legs["bvh"]
    nd = int((imgs["brute"][..., :3] != imgs["bvh"][..., :3]).any(-1).sum())
    out["pixels_brute_vs_bvh_differing"] = nd
    if do_cpu:
        progress(f"config {name}: CPU baseline and parity sample")
        res, parity = cpu_baseline(sd, spec, u, imgs, threads, seconds)
        desc = (f"{res['bvh']['pixels']} of {spec.width * spec.height} pixels (BVH mode; brute mode "
                f"{res['brute']['pixels']}), evenly spread in raster order, full {spec.rays * spec.frames} spp, "
                f"{res['bvh']['seconds']:.1f} s")
        cb = cpu_summary(res, threads, host, desc, {"brute": legs["brute"]["value"], "bvh": legs["bvh"]["value"]})
        out["cpu_baseline"] = cb
        out["parity"] = parity
        if name != "C":
            return out
        tgt = {"target": f">= {TARGET_RATIO:g}x the CPU reference's Msamples/s at config C on 1 GPU",
               "cpu_reference": f"oracle/ BVH traversal (the reference's algorithm) on {threads} CPUs",
               "brute_ratio": cb["gpu_brute_over_cpu_bvh"], "bvh_ratio": cb["gpu_bvh_over_cpu_bvh"],
               "met_by_brute": cb["gpu_brute_over_cpu_bvh"] >= TARGET_RATIO,
               "met_by_bvh": cb["gpu_bvh_over_cpu_bvh"] >= TARGET_RATIO,
               "bvh_ratio_vs_node_extrapolation": cb["gpu_bvh_over_node_extrapolated_bvh"],
               "met_by_bvh_vs_node_extrapolation": cb["gpu_bvh_over_node_extrapolated_bvh"] >= TARGET_RATIO}
        k = [n for n in ("brute", "bvh") if tgt[f"met_by_{n}"]]
        tgt["statement"] = (f"target met by the {' and '.join(k)} kernel(s)" if k else "target NOT met") + \
            f" against {threads} CPUs; against all {host.get('logical_cpus')} hardware threads of the node " \
            f"(extrapolated) the BVH kernel is {cb['gpu_bvh_over_node_extrapolated_bvh']}x"
        out["north_star_target"] = tgt
    return out


def main():
    args = parse()
    ensure_world(args)  # before any GPU call: may start the N ranks and exit
    import numpy as np
    import torch
    import torch.distributed as dist
    import rt2
    from rt2 import dist as rdist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing:
        if world > 1:
            dist.init_process_group("gloo")
        return plumbing(args, world, rank)
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

    progress(f"config {spec.name}: {args.warmup} warmup step(s)")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    scene.stats(reset=True)
    progress(f"config {spec.name}: {args.steps} timed step(s)")

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
    variant = launched_variant(rt2, scene)
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

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    rf = roofline(tests / args.steps / world, visits / args.steps / world, kern_ms, segs / args.steps / world,
                  sd.num_triangles, variant)
    rf["kernel"] = kernel_label(variant)
    rf["segments_per_sample"] = round(segs / (samples_per_step * args.steps), 4)
    if world == 1:  # PMC traffic was measured for the 1-GPU launch
        attach_traffic(rf, spec.name if args.traversal == "brute" else f"{spec.name}_bvh", variant, kern_ms)
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
        "roofline": rf,
        "cpu_baseline": None,
    }
    gpu_imgs = {args.traversal: img.cpu().numpy() if img is not None else None}
    img_main = img.clone() if img is not None else None  # the headline image (renderer.image is reused below)
    gpu_values = {args.traversal: value}
    alt = "bvh" if args.traversal == "brute" else "brute"
    # brute force over 100k+ triangles takes minutes per step: not timed beside BVH there
    if world == 1 and not args.no_alt and (alt == "bvh" or sd.num_triangles <= 20000):
        # the other closest-hit algorithm on the same workload, same timing
        # bracket (reported beside the headline, never as `value`)
        progress(f"config {spec.name}: the {alt} traversal beside the headline")
        scene.set_traversal(alt)
        scene.set_variant(0)
        renderer.accum.zero_()
        scene.render(u, 0, spec.frames, renderer.sh, renderer.accum.data_ptr(), 0, stream.cuda_stream)
        el2, km2, st2 = timed_renders(torch, rt2, scene, u, spec.frames, renderer.sh, renderer.accum,
                                      renderer.image, args.steps, stream)
        ndiff = int((renderer.image[..., :3] != img_main[..., :3]).any(-1).sum().item())
        d2 = (renderer.image[..., :3] - img_main[..., :3]).double()
        v2 = samples_per_step * args.steps / el2 / 1e6
        gpu_imgs[alt] = renderer.image.cpu().numpy()
        gpu_values[alt] = v2
        out["alt_traversal"] = {
            "traversal": alt, "value": round(v2, 3), "ms_per_step": round(el2 / args.steps * 1e3, 3),
            "kernel": kernel_label(launched_variant(rt2, scene)), "kernel_ms": round(km2, 3),
            "segments_per_sample": round(st2.segments / (samples_per_step * args.steps), 4),
            "tests_per_segment": round(st2.tests / max(st2.segments, 1), 3),
            "node_visits_per_segment": round(st2.node_visits / max(st2.segments, 1), 3),
            "valu_tflops": round((FLOP_PER_TEST * st2.tests + FLOP_PER_VISIT * st2.node_visits) / args.steps
                                 / (km2 * 1e-3) / 1e12, 3),
            "l2_read_algorithmic_gbs": round((BVH_RECORD_BYTES * st2.node_visits + BVH_TRI_BYTES * st2.tests)
                                             / args.steps / (km2 * 1e-3) / 1e9, 1) if st2.node_visits else None,
            "pixels_differing_from_main": ndiff,
            "rmse_vs_main": float(d2.pow(2).mean().sqrt()),
            "note": "brute force and the reference BVH traversal agree except on exact distance ties"}
        scene.set_traversal(args.traversal)
        scene.set_variant(args.variant)
    if world == 1 and args.traversal == "brute" and not args.no_scalar and sd.num_triangles <= 20000:
        # the north star's literal kernel: one work-item per pixel-sample, the
        # reference's 53-FLOP Moller-Trumbore per pair on the FP32 VALU, no
        # MFMA (render_smem forced) — its VALU roofline is the physical one
        # for that kernel; same workload, same bracket, never `value`
        progress(f"config {spec.name}: the scalar-VALU kernel (variant {SCALAR_VARIANT})")
        scene.set_variant(SCALAR_VARIANT)
        renderer.accum.zero_()
        scene.render(u, 0, spec.frames, renderer.sh, renderer.accum.data_ptr(), 0, stream.cuda_stream)
        nsteps = max(1, min(args.steps, 2))
        el3, km3, st3 = timed_renders(torch, rt2, scene, u, spec.frames, renderer.sh, renderer.accum,
                                      renderer.image, nsteps, stream)
        v3 = launched_variant(rt2, scene)
        rf3 = roofline(st3.tests / nsteps, 0, km3, st3.segments / nsteps, sd.num_triangles, v3)
        rf3["kernel"] = kernel_label(v3)
        attach_traffic(rf3, f"{spec.name}_scalar", v3, km3)
        out["scalar_valu"] = {
            "value": round(samples_per_step * nsteps / el3 / 1e6, 3), "unit": "Msamples/s", "steps": nsteps,
            "ms_per_step": round(el3 / nsteps * 1e3, 3), "roofline": rf3,
            "pixels_differing_from_main": int((renderer.image[..., :3] != img_main[..., :3]).any(-1).sum().item()),
            "note": "render_smem (variant 136): scalar-cache triangle records, the exact filtered test on the VALU, "
                    "no MFMA; bit-identical to the headline kernel"}
        scene.set_variant(args.variant)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: the CPU baseline and the parity checker only
    threads, host = oracle.default_threads(), oracle.host_cpu_info()
    if world == 1 and not args.no_cpu_baseline:
        progress(f"config {spec.name}: CPU baseline and parity sample")
        res, parity = cpu_baseline(sd, spec, u, gpu_imgs, threads, args.cpu_seconds)
        desc = (f"{res['bvh']['pixels']} of {spec.width * spec.height} pixels (BVH mode; brute mode "
                f"{res['brute']['pixels']}), i = floor(k*{spec.width * spec.height}/n) in raster order, full spp, "
                f"reference BVH traversal (compute.glsl:410-460), {res['bvh']['seconds']:.1f} s")
        out["cpu_baseline"] = cpu_summary(res, threads, host, desc, gpu_values)
        out["parity"] = parity
    if world == 1 and spec.name == "B" and not (args.no_config_c and args.no_config_e and args.no_config_w):
        scene.close()
        torch.cuda.empty_cache()
        for name, skip in (("C", args.no_config_c), ("E", args.no_config_e), ("W", args.no_config_w)):
            if not skip:
                progress(f"config {name} leg")
                out[f"config_{name}"] = config_leg(torch, rt2, stream, threads, host, args.cpu_seconds,
                                                   not args.no_cpu_baseline, name)
                torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
