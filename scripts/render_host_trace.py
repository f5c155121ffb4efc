"""Repeated rt2_render_host calls for a rocprofv3 HIP API trace: the scene keeps
its render_host buffers, so only the first call may allocate.

  rocprofv3 --hip-trace --stats -d gpurun_out/rh -o run --output-format csv \
      -- python3 scripts/render_host_trace.py
  python3 scripts/render_host_trace.py --summarise gpurun_out/rh   (on the host)
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))


def run(calls: int) -> None:
    import rt2
    sd, spec = rt2.build_config_scene("A")
    u = rt2.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2.Scene(sd, 0)
    for i in range(calls):
        img = scene.render_host(u, 0, 1)
        print(f"call {i}: mean {float(img[..., :3].mean()):.6f}", flush=True)


def summarise(d: str) -> None:
    """Per-call counts of the allocation and synchronisation APIs between
    consecutive rt2_render_host calls (each call ends with one D2H copy)."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Function"] for r in rows]
    # a render_host call = the launches up to and including its D2H copy
    calls, cur = [], []
    for n in names:
        cur.append(n)
        if n in ("hipMemcpy", "hipMemcpyAsync", "hipMemcpyDtoH", "hipMemcpyDtoHAsync", "hipMemcpyWithStream"):
            calls.append(cur)
            cur = []
    watch = ("hipMalloc", "hipFree", "hipDeviceSynchronize", "hipStreamSynchronize", "hipMemcpy", "hipMemcpyAsync",
             "hipMemcpyWithStream", "hipLaunchKernel", "hipExtModuleLaunchKernel", "hipModuleLaunchKernel")
    out = {"trace_dir": d, "api_calls_total": len(names),
           "per_render_host_call": [{w: c.count(w) for w in watch if c.count(w)} for c in calls]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=4)
    ap.add_argument("--summarise", default=None)
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a.calls)
