"""Known-answer tests pinning the CPU oracle (oracle/rt_oracle.c) to compute.glsl.

The reference ships no tests or golden renders, so the oracle's
arithmetic is pinned by hand-checkable cases: the PCG hash (compute.glsl:148-154,
integer-exact), Möller–Trumbore decisions (:302-340), tonemap/sRGB (:647-658),
and the pinned transcendentals against the host libm.
"""
import ctypes as C
import math

import numpy as np
import pytest


def pcg_py(state):
    """Pure-Python restatement of random(), compute.glsl:148-154."""
    state = (state * 747796405 + 2891336453) & 0xFFFFFFFF
    r = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & 0xFFFFFFFF
    r = ((r >> 22) ^ r) & 0xFFFFFFFF
    return state, r


def test_pcg_kat(oraclemod):
    # SURVEY.md §8a A10 known answers
    assert [r for r, _ in oraclemod.pcg_sequence(0, 3)] == [129708002, 582399676, 1006035121]
    assert [r for r, _ in oraclemod.pcg_sequence(1, 3)] == [2831084092, 645514520, 2544563910]
    rng = np.random.default_rng(1)
    for seed in rng.integers(0, 2**32, 200, dtype=np.uint64):
        seed = int(seed)
        s = seed
        for r_or, f_or in oraclemod.pcg_sequence(seed, 5):
            s, r = pcg_py(s)
            assert r == r_or
            # result / 4294967295.0 in float: uint -> float (RN), / 2^32
            assert f_or == np.float32(np.float32(r) / np.float32(4294967296.0))


def test_random_can_return_one(oraclemod):
    # float(result) rounds up to 2^32 for result >= 2^32 - 128: random() == 1.0 is reachable
    assert np.float32(np.float32(4294967295) / np.float32(4294967296.0)) == 1.0


def tri(a, b, c):
    t = np.zeros(1, dtype=[("a", "<f4", 4), ("b", "<f4", 4), ("c", "<f4", 4), ("uv", "<f4", 6), ("m", "<i4"),
                           ("p", "<f4")])
    t["a"][0, :3], t["b"][0, :3], t["c"][0, :3] = a, b, c
    return t


def hit(oraclemod, o, d, t):
    o = np.array(o, np.float32)
    d = np.array(d, np.float32)
    dst = C.c_float()
    ok = oraclemod.lib().oracle_ray_triangle(o.ctypes.data, d.ctypes.data, t.ctypes.data, C.byref(dst))
    return bool(ok), dst.value


def test_moller_trumbore_cases(oraclemod):
    # counter-clockwise seen from +z: n = (b-a)x(c-a) = +z; ray going -z hits (det = -d.n > 0)
    t = tri((0, 0, 0), (1, 0, 0), (0, 1, 0))
    ok, dst = hit(oraclemod, (0.25, 0.25, 1), (0, 0, -1), t)
    assert ok and dst == 1.0
    # back face culled (det < 0)
    assert not hit(oraclemod, (0.25, 0.25, -1), (0, 0, 1), t)[0]
    # outside (u < 0, v < 0, 1-u-v < 0)
    assert not hit(oraclemod, (-0.1, 0.25, 1), (0, 0, -1), t)[0]
    assert not hit(oraclemod, (0.25, -0.1, 1), (0, 0, -1), t)[0]
    assert not hit(oraclemod, (0.6, 0.6, 1), (0, 0, -1), t)[0]
    # exactly on an edge / vertex counts (tests are strict < 0)
    assert hit(oraclemod, (0.0, 0.5, 1), (0, 0, -1), t)[0]
    assert hit(oraclemod, (0.0, 0.0, 1), (0, 0, -1), t)[0]
    assert hit(oraclemod, (0.5, 0.5, 1), (0, 0, -1), t)[0]
    # behind the origin / dst <= 1e-6 rejected
    assert not hit(oraclemod, (0.25, 0.25, -1), (0, 0, -1), t)[0]
    assert not hit(oraclemod, (0.25, 0.25, 5e-7), (0, 0, -1), t)[0]
    assert hit(oraclemod, (0.25, 0.25, 2e-6), (0, 0, -1), t)[0]
    # parallel ray: |det| < 1e-10
    assert not hit(oraclemod, (0.25, 0.25, 1), (1, 0, 0), t)[0]
    # degenerate triangle
    assert not hit(oraclemod, (0.25, 0.25, 1), (0, 0, -1), tri((0, 0, 0), (1, 0, 0), (2, 0, 0)))[0]


def test_tonemap_srgb(oraclemod):
    L = oraclemod.lib()
    assert L.oracle_tonemap_srgb(0.0) == 0.0
    for x in (0.01, 0.18, 0.5, 1.0, 4.0):
        a = (x * (2.51 * x + 0.03)) / (x * (2.43 * x + 0.59) + 0.14)
        ref = min(max(a, 0.0), 1.0) ** (1 / 2.2)
        assert abs(L.oracle_tonemap_srgb(x) - ref) < 2e-6
    assert L.oracle_tonemap_srgb(1e6) == 1.0


def ulp_diff(a, b):
    a = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    a = np.where(a < 0, -(a & 0x7FFFFFFF), a)
    b = np.where(b < 0, -(b & 0x7FFFFFFF), b)
    return np.abs(a - b)


@pytest.mark.parametrize("which,fn,lo,hi,tol", [
    (0, math.exp, -87.0, 88.0, 3),
    (1, math.log, 1e-30, 1e30, 3),
    (2, math.acos, -1.0, 1.0, 3),
    (3, math.cos, -3.0, 3.0, 3),
    (4, math.sin, -3.0, 3.0, 3),
])
def test_pinned_math_accuracy(oraclemod, which, fn, lo, hi, tol):
    rng = np.random.default_rng(which)
    if which == 1:
        xs = np.exp(rng.uniform(math.log(lo), math.log(hi), 3000)).astype(np.float32)
    else:
        xs = rng.uniform(lo, hi, 3000).astype(np.float32)
    got = np.array([oraclemod.pinned(which, float(x)) for x in xs], np.float32)
    ref = np.array([fn(float(x)) for x in xs], np.float32)
    err = ulp_diff(got, ref)
    if which in (3, 4):  # near zeros of sin/cos compare absolutely
        small = np.abs(ref) < 1e-3
        assert np.all(np.abs(got[small] - ref[small]) < 1e-7)
        err = err[~small]
    assert err.max() <= tol, (which, err.max())


def test_pinned_pow_srgb(oraclemod):
    xs = np.linspace(0, 1, 2001, dtype=np.float32)
    got = np.array([oraclemod.pinned(5, float(x)) for x in xs], np.float32)
    ref = (xs.astype(np.float64) ** (1.0 / 2.2)).astype(np.float32)
    assert np.max(np.abs(got - ref)) < 1e-6
    assert got[0] == 0.0 and got[-1] == 1.0


def test_sky_reference_values(oraclemod):
    L = oraclemod.lib()
    out = np.zeros(3, np.float32)
    sun = np.array([0.6, 0.3, -0.2], np.float32)
    sun = sun / np.sqrt((sun.astype(np.float64) ** 2).sum())
    d = np.ascontiguousarray(sun, np.float32)
    L.oracle_sky(d.ctypes.data, out.ctypes.data)
    # looking straight at the sun: all four glows ~1 -> base + (15,15,10)*1.43
    assert out[0] > 20 and out[2] > 14
    up = np.array([0, 1, 0], np.float32)
    L.oracle_sky(up.ctypes.data, out.ctypes.data)
    assert np.allclose(out, [0.15, 0.25, 0.65], atol=0.02)
    down = np.array([0, -1, 0], np.float32)
    L.oracle_sky(down.ctypes.data, out.ctypes.data)
    assert np.allclose(out, [0.2, 0.15, 0.1], atol=0.02)
