"""Quick GPU bring-up check: render configs A and B on cuda:0 through the C-ABI
and compare strided rows against the CPU oracle (bit-exact expected)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import rt2  # noqa: E402

x = np.random.default_rng(0).uniform(-20, 20, 4096).astype(np.float32)
dev = rt2.device_selftest(x)
print("selftest div exact:", np.array_equal(dev[:, 0], x / x[(np.arange(4096) * 7 + 3) % 4096]),
      "sqrt exact:", np.array_equal(dev[:, 1], np.sqrt(np.abs(x))))
host = np.array([[oracle.pinned(k, float(v)) for k in range(6)] for v in x[:512]], dtype=np.float32)
print("pinned exp/cos/sin equal:", [np.array_equal(dev[:512, c], host[:, k]) for c, k in ((3, 0), (6, 3), (7, 4))])

for cfg, W, H, R in (("A", 256, 256, 4), ("B", 1920, 1080, 64)):
    sd, spec = rt2.build_config_scene(cfg)
    u = rt2.offline_uniforms(W, H, spec.bounces, R, sd.num_triangles)
    scene = rt2.Scene(sd, 0)
    t = time.time()
    img = scene.render_host(u, 0, 1)
    dt = time.time() - t
    st = scene.stats(reset=True)
    print(f"{cfg}: {W}x{H} R{R} {dt:.3f}s {st.samples / dt / 1e6:.1f} Msamples/s segs/sample {st.segments / st.samples:.3f}")
    t = time.time()
    img = scene.render_host(u, 0, 1)
    dt = time.time() - t
    st = scene.stats(reset=True)
    print(f"{cfg}: 2nd run {dt:.3f}s {st.samples / dt / 1e6:.1f} Msamples/s tests/s {st.tests / dt:.3e}")
    rows = np.arange(0, H, max(1, H // 24))
    acc, _, segs, _ = oracle.render(sd.triangles(), sd.materials(), u, rows, 0, 1, "brute")
    gpu = img[rows]
    diff = np.abs(gpu[..., :3] - acc[..., :3])
    print(f"{cfg}: rows {len(rows)} exact pixels {(diff.max(-1) == 0).mean() * 100:.3f}% maxdiff {diff.max():.3e} "
          f"rmse {np.sqrt((diff ** 2).mean()):.3e}")
