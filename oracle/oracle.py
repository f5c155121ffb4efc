"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/liboracle.so, the CPU
restatement of compute.glsl (rt_oracle.c).  Imported by tests/, by
__graft_entry__.smoke() and by bench.py's cpu_baseline leg; never by the
product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_DUMP = os.path.join(HERE, "_ref", "ref_dump")

_lib = None


def cgroup_cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup v2 CPU controller (cpu.max
    quota / period), or None when unlimited or unavailable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def host_cpu_info() -> dict:
    """The host's CPU as seen from this process: model, logical CPUs, physical
    cores, the affinity mask and the cgroup CPU quota (a GPU box grants a job a
    quota far below its core count)."""
    model, cores_per_socket, sockets = None, None, set()
    try:
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "cpu cores" and cores_per_socket is None:
                cores_per_socket = int(v)
            elif k == "physical id":
                sockets.add(v)
    except OSError:
        pass
    phys = cores_per_socket * max(len(sockets), 1) if cores_per_socket else None
    return {"model": model, "logical_cpus": os.cpu_count(), "physical_cores": phys,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpu_quota": cgroup_cpu_quota()}


def default_threads() -> int:
    """Worker threads for the oracle: every CPU of the affinity mask, capped by
    the cgroup CPU quota (threads beyond the quota add no CPU time)."""
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpu_quota()
    if q:
        n = min(n, max(1, int(q + 0.5)))
    return max(1, n)


def build() -> None:
    subprocess.run(["make", "-C", HERE, "liboracle.so"], check=True, stdout=subprocess.DEVNULL)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.c_void_p
        L.oracle_render.restype = C.c_int
        L.oracle_render.argtypes = [P, C.c_int32, P, C.c_int32, P, C.c_int32, P, C.c_uint32, C.c_uint32, P,
                                    C.c_int32, C.c_int32, C.c_int32, P, P, P, P]
        L.oracle_render_pixels.restype = C.c_int
        L.oracle_render_pixels.argtypes = [P, C.c_int32, P, C.c_int32, P, C.c_int32, P, C.c_uint32, C.c_uint32, P,
                                           C.c_int64, C.c_int32, C.c_int32, P, P, P, P]
        L.oracle_set_textures.restype = C.c_int
        L.oracle_set_textures.argtypes = [P, P, C.c_int32]
        L.oracle_pcg_next.restype = C.c_uint32
        L.oracle_pcg_next.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_float)]
        L.oracle_ray_triangle.restype = C.c_int
        L.oracle_ray_triangle.argtypes = [P, P, P, P]
        L.oracle_sky.restype = None
        L.oracle_sky.argtypes = [P, P]
        L.oracle_tonemap_srgb.restype = C.c_float
        L.oracle_tonemap_srgb.argtypes = [C.c_float]
        L.oracle_pinned.restype = C.c_float
        L.oracle_pinned.argtypes = [C.c_int, C.c_float]
        _lib = L
    return _lib


def render(triangles: np.ndarray, materials: np.ndarray, uniforms, rows, frame_begin: int = 0,
           frame_count: int = 1, mode: str = "brute", nodes: np.ndarray | None = None, threads: int | None = None,
           with_acc8: bool = False):
    """Renders the listed image rows.  Returns (accum[nrows, W, 4] = per-pixel SUM over
    frames, acc8 or None, segments, tests)."""
    tri = np.ascontiguousarray(triangles)
    mat = np.ascontiguousarray(materials)
    assert tri.dtype.itemsize == 80 and mat.dtype.itemsize == 96
    rows = np.ascontiguousarray(rows, dtype=np.int32)
    W = int(uniforms.width)
    acc = np.zeros((len(rows), W, 4), dtype=np.float32)
    acc8 = np.zeros((len(rows), W, 4), dtype=np.uint32) if with_acc8 else None
    segs = C.c_uint64(0)
    tests = C.c_uint64(0)
    nd = None if nodes is None else np.ascontiguousarray(nodes)
    m = {"brute": 0, "bvh": 1}[mode]
    rc = lib().oracle_render(tri.ctypes.data, len(tri), mat.ctypes.data, len(mat),
                             None if nd is None else nd.ctypes.data, 0 if nd is None else len(nd),
                             C.addressof(uniforms), frame_begin, frame_count, rows.ctypes.data, len(rows), m,
                             threads or default_threads(), acc.ctypes.data,
                             None if acc8 is None else acc8.ctypes.data, C.byref(segs), C.byref(tests))
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return acc, acc8, segs.value, tests.value


def render_pixels(triangles: np.ndarray, materials: np.ndarray, uniforms, xs, ys, frame_begin: int = 0,
                  frame_count: int = 1, mode: str = "brute", nodes: np.ndarray | None = None,
                  threads: int | None = None, with_acc8: bool = False):
    """Renders the pixels (xs[i], ys[i]).  Returns (accum[n, 4] = per-pixel SUM over
    frames, acc8 or None, segments, tests)."""
    tri = np.ascontiguousarray(triangles)
    mat = np.ascontiguousarray(materials)
    assert tri.dtype.itemsize == 80 and mat.dtype.itemsize == 96
    px = np.ascontiguousarray(np.stack([np.asarray(xs, np.int32), np.asarray(ys, np.int32)], -1))
    n = len(px)
    acc = np.zeros((n, 4), dtype=np.float32)
    acc8 = np.zeros((n, 4), dtype=np.uint32) if with_acc8 else None
    segs = C.c_uint64(0)
    tests = C.c_uint64(0)
    nd = None if nodes is None else np.ascontiguousarray(nodes)
    m = {"brute": 0, "bvh": 1}[mode]
    rc = lib().oracle_render_pixels(tri.ctypes.data, len(tri), mat.ctypes.data, len(mat),
                                    None if nd is None else nd.ctypes.data, 0 if nd is None else len(nd),
                                    C.addressof(uniforms), frame_begin, frame_count, px.ctypes.data, n, m,
                                    threads or default_threads(), acc.ctypes.data,
                                    None if acc8 is None else acc8.ctypes.data, C.byref(segs), C.byref(tests))
    if rc != 0:
        raise RuntimeError(f"oracle_render_pixels failed: {rc}")
    return acc, acc8, segs.value, tests.value


_tex_keep = None


def set_textures(images) -> None:
    """images: list of uint8 arrays shaped (h, w, channels) in stb layout
    (row 0 first in memory).  Held by the library until the next call."""
    global _tex_keep
    arrs = [np.ascontiguousarray(a, dtype=np.uint8) for a in images]
    whn = np.array([[a.shape[1], a.shape[0], a.shape[2] if a.ndim == 3 else 1] for a in arrs],
                   dtype=np.int32).reshape(-1)
    ptrs = (C.c_void_p * max(len(arrs), 1))(*[a.ctypes.data for a in arrs])
    _tex_keep = (arrs, whn, ptrs)
    rc = lib().oracle_set_textures(whn.ctypes.data if len(arrs) else None, C.addressof(ptrs), len(arrs))
    if rc != 0:
        raise RuntimeError("oracle_set_textures failed")


def pcg_sequence(seed: int, n: int):
    s = C.c_uint32(seed)
    f = C.c_float()
    out = []
    for _ in range(n):
        r = lib().oracle_pcg_next(C.byref(s), C.byref(f))
        out.append((r, f.value))
    return out


def pinned(which: int, x: float) -> float:
    return lib().oracle_pinned(which, x)
