"""Occupancy API answer and register counts of render-kernel variants."""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import torch  # noqa: E402,F401
import rt2  # noqa: E402

L = rt2.lib()
out = {}
for v in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,67,85,28,53,2").split(",")]:
    a, r, lb = C.c_int(), C.c_int(), C.c_int()
    rc = L.rt2_variant_occupancy(v, C.byref(a), C.byref(r), C.byref(lb))
    out[L.rt2_variant_name(v).decode()] = dict(variant=v, rc=rc, api_blocks_per_cu=a.value, num_regs=r.value,
                                               local_bytes=lb.value)
print(json.dumps(out, indent=1))
