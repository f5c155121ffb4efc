"""Multi-GPU path on one GPU (the 8-GPU run is the driver's).

- Config D (scene B at 3840x2160, 64 rays x 16 frames, 8 bounces — the 8-GPU
  configuration of BASELINE.json): rendered whole, with the per-frame planes
  forced into 4-frame chunks (the chunking path of rt2_render), and as the 8
  row-tile shards the bench uses, each slab rendered on its own; the slabs,
  packed as an RCCL gather leaves them on the root ([rank][max_rows][W]) and
  un-interleaved by rt2_unshard_slabs, must equal the whole image bit for bit;
  2,048 spread pixels at full spp must equal the CPU oracle bit for bit.
- The C-ABI communicator (rt2_comm_*, RCCL): a one-rank communicator's
  rt2_render_host_gather and rt2_gather_slabs reproduce rt2_render_host.
"""
import ctypes as C
import os

import numpy as np
import pytest

from test_gpu_parity import assert_exact

pytestmark = pytest.mark.gpu

N_SHARDS = 8
TILE = 1  # bench.py --tile-rows default


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    torch.cuda.set_device(0)
    return torch


def render_slab(rt2mod, torch, scene, u, frames, sh, rows_alloc=None):
    """Renders a shard into a device accumulator and resolves it on the device;
    returns the resolved slab (rows_alloc rows, zero padded) as a torch tensor."""
    rows = rt2mod.shard_rows(u.height, sh)
    acc = torch.zeros((rows_alloc or rows, u.width, 4), dtype=torch.float32, device="cuda")
    res = torch.zeros_like(acc)
    stream = torch.cuda.current_stream().cuda_stream
    scene.render(u, 0, frames, sh, acc.data_ptr(), 0, stream)
    rt2mod.resolve_rgba32f(acc.data_ptr(), rows * u.width, frames, res.data_ptr(), stream)
    return res


@pytest.fixture(scope="module")
def config_d(rt2mod, config_scene, torch_cuda):
    sd, spec = config_scene("D")
    assert (spec.width, spec.height, spec.rays, spec.frames, spec.bounces) == (3840, 2160, 64, 16, 8)
    u = rt2mod.offline_uniforms(spec.width, spec.height, spec.bounces, spec.rays, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    L = rt2mod.lib()
    L.rt2_scene_set_frame_scratch_cap.argtypes = [C.c_void_p, C.c_ulonglong]
    plane = spec.width * spec.height * 16
    assert L.rt2_scene_set_frame_scratch_cap(scene._p, 4 * plane) == 0  # 4-frame chunks
    whole = render_slab(rt2mod, torch_cuda, scene, u, spec.frames, rt2mod.shard())
    torch_cuda.cuda.synchronize()
    st = scene.stats(reset=True)
    assert st.samples == spec.width * spec.height * spec.rays * spec.frames
    return sd, spec, u, whole


def test_config_D_pixels_match_oracle(rt2mod, oraclemod, config_d):
    """2,048 pixels spread over the 4K image, all 1,024 samples each, bit-exact."""
    sd, spec, u, whole = config_d
    img = whole.cpu().numpy()
    n = 2048
    pid = (np.arange(n, dtype=np.int64) * (spec.width * spec.height)) // n + 977  # off the row starts
    xs, ys = pid % spec.width, pid // spec.width
    acc, _, _, _ = oraclemod.render_pixels(sd.triangles(), sd.materials(), u, xs, ys, 0, spec.frames, "brute")
    assert_exact(img[ys, xs], acc[:, :3] / np.float32(spec.frames), "config D sampled pixels")


def test_config_D_eight_row_tile_shards_assemble(rt2mod, config_d, torch_cuda):
    """The 8 rank slabs (1/8 of the rows each, no frame chunking: 265 MB of
    planes per slab), gathered-layout + rt2_unshard_slabs == the whole image."""
    torch = torch_cuda
    sd, spec, u, whole = config_d
    scene = rt2mod.Scene(sd, 0)
    mr = max(rt2mod.shard_rows(spec.height, rt2mod.shard(TILE, r, N_SHARDS)) for r in range(N_SHARDS))
    gathered = torch.zeros((N_SHARDS, mr, spec.width, 4), dtype=torch.float32, device="cuda")
    for r in range(N_SHARDS):
        sh = rt2mod.shard(TILE, r, N_SHARDS)
        gathered[r] = render_slab(rt2mod, torch, scene, u, spec.frames, sh, rows_alloc=mr)
    image = torch.empty_like(whole)
    rt2mod.unshard_slabs(gathered.data_ptr(), mr, spec.width, spec.height, rt2mod.shard(TILE, 0, N_SHARDS),
                         image.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    diff = (image != whole).any(-1)
    assert not bool(diff.any()), f"{int(diff.sum())} pixels of the assembled shards differ from the whole render"


def test_unshard_uneven_slabs(rt2mod, config_scene, torch_cuda):
    """Ragged layouts: slabs of different heights (50 rows, tiles of 4 over 3
    ranks), padded to max_rows as the gather leaves them."""
    torch = torch_cuda
    sd, spec = config_scene("B")
    W, H, n, tile = 72, 50, 3, 4
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    whole = render_slab(rt2mod, torch, scene, u, 2, rt2mod.shard())
    rows = [rt2mod.shard_rows(H, rt2mod.shard(tile, r, n)) for r in range(n)]
    assert len(set(rows)) > 1
    mr = max(rows)
    gathered = torch.full((n, mr, W, 4), -1.0, dtype=torch.float32, device="cuda")
    for r in range(n):
        gathered[r] = render_slab(rt2mod, torch, scene, u, 2, rt2mod.shard(tile, r, n), rows_alloc=mr)
    image = torch.zeros_like(whole)
    rt2mod.unshard_slabs(gathered.data_ptr(), mr, W, H, rt2mod.shard(tile, 0, n), image.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(image, whole)


def test_comm_one_rank_render_host_gather(rt2mod, config_scene, torch_cuda):
    """rt2_render_host_gather over a one-rank RCCL communicator == rt2_render_host
    (float mean and the 8-bit reference average)."""
    sd, spec = config_scene("B")
    W, H = 96, 54
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 4, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    ref, ref8 = scene.render_host(u, 2, 3, rgb8=True)
    comm = rt2mod.Comm(rt2mod.Comm.unique_id(), 1, 0, 0)
    for tile in (1, 5):
        img, img8 = scene.render_host_gather(u, 2, 3, rt2mod.shard(tile, 0, 1), comm, 0, rgb8=True)
        assert np.array_equal(img, ref) and np.array_equal(img8, ref8)
    comm.check()
    with pytest.raises(rt2mod.RT2Error):  # a shard of another communicator size
        scene.render_host_gather(u, 0, 1, rt2mod.shard(1, 0, 2), comm, 0)
    comm.close()


def test_comm_gather_slabs_one_rank(rt2mod, config_scene, torch_cuda):
    torch = torch_cuda
    sd, spec = config_scene("B")
    W, H = 64, 30
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    slab = render_slab(rt2mod, torch, scene, u, 1, rt2mod.shard())
    image = torch.zeros_like(slab)
    comm = rt2mod.Comm(rt2mod.Comm.unique_id(), 1, 0, 0)
    stream = torch.cuda.current_stream().cuda_stream
    comm.gather_slabs(slab.data_ptr(), W, H, rt2mod.shard(), 0, image.data_ptr(), stream)
    comm.wait(stream)  # rt2_comm_wait: the gather drained under the RT2_COMM_TIMEOUT_S deadline
    comm.check()
    assert torch.equal(image, slab)
    comm.close()


def test_comm_gather_slabs_after_long_render(rt2mod, config_scene, torch_cuda, monkeypatch):
    """INTEGRATION.md's async sequence on ONE stream — rt2_render,
    resolve, rt2_gather_slabs, rt2_comm_wait — with a render many times longer
    than RT2_COMM_TIMEOUT_S.  rt2_comm_wait waits for the rank's own queued
    work (everything before the gather) outside the deadline, then applies the
    deadline to the gather: a healthy job completes, bit-identical."""
    import time
    torch = torch_cuda
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(1920, 1080, spec.bounces, 64, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    ref = scene.render_host(u, 0, 1)
    comm = rt2mod.Comm(rt2mod.Comm.unique_id(), 1, 0, 0)
    stream = torch.cuda.current_stream().cuda_stream
    torch.cuda.synchronize()
    monkeypatch.setenv("RT2_COMM_TIMEOUT_S", "0.02")
    t0 = time.time()
    slab = render_slab(rt2mod, torch, scene, u, 1, rt2mod.shard())  # queued, not waited for
    image = torch.zeros_like(slab)
    comm.gather_slabs(slab.data_ptr(), u.width, u.height, rt2mod.shard(), 0, image.data_ptr(), stream)
    comm.wait(stream)
    assert time.time() - t0 > 3 * 0.02  # the render alone outlasts the deadline several times
    comm.check()
    assert np.array_equal(image.cpu().numpy(), ref)
    comm.close()


@pytest.mark.parametrize("site", ["gather.prepare", "check", "render", "gather.issue", "agree.copy"])
def test_comm_one_rank_injected_faults(rt2mod, config_scene, torch_cuda, site, monkeypatch):
    """The failure sites of rt2_comm_protocol.h under RCCL (RT2_FAULT_AT): the
    call returns < 0 within seconds; after the sites the agreement catches the
    communicator still works, after gather.issue / agree.copy (the rank could
    not take part) it was aborted and refuses further use."""
    import time
    torch = torch_cuda
    sd, spec = config_scene("B")
    W, H = 64, 30
    u = rt2mod.offline_uniforms(W, H, spec.bounces, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    slab = render_slab(rt2mod, torch, scene, u, 1, rt2mod.shard())
    image = torch.zeros_like(slab)
    stream = torch.cuda.current_stream().cuda_stream
    comm = rt2mod.Comm(rt2mod.Comm.unique_id(), 1, 0, 0)
    monkeypatch.setenv("RT2_FAULT_AT", site)
    monkeypatch.setenv("RT2_COMM_TIMEOUT_S", "20")
    t0 = time.time()
    with pytest.raises(rt2mod.RT2Error):
        if site == "gather.prepare":
            comm.gather_slabs(slab.data_ptr(), W, H, rt2mod.shard(), 0, image.data_ptr(), stream)
        else:
            scene.render_host_gather(u, 0, 1, rt2mod.shard(), comm, 0)
    assert time.time() - t0 < 20
    monkeypatch.delenv("RT2_FAULT_AT")
    if site in ("gather.issue", "agree.copy"):
        with pytest.raises(rt2mod.RT2Error):
            comm.check()
    else:
        comm.check()
        img = scene.render_host_gather(u, 0, 1, rt2mod.shard(), comm, 0)
        assert np.array_equal(img, scene.render_host(u, 0, 1))
    comm.close()


def test_comm_render_longer_than_timeout(rt2mod, config_scene, torch_cuda, monkeypatch):
    """the watchdog of rt2_render_host_gather starts after the rank's
    own render (a local render has no peer to wait for), and the render's time
    is slack on the deadlines after it: a healthy render many times longer
    than RT2_COMM_TIMEOUT_S completes, bit-identical to rt2_render_host."""
    import time
    sd, spec = config_scene("B")
    u = rt2mod.offline_uniforms(1920, 1080, spec.bounces, 64, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    ref = scene.render_host(u, 0, 1)
    comm = rt2mod.Comm(rt2mod.Comm.unique_id(), 1, 0, 0)
    monkeypatch.setenv("RT2_COMM_TIMEOUT_S", "0.02")
    t0 = time.time()
    img = scene.render_host_gather(u, 0, 1, rt2mod.shard(), comm, 0)
    assert time.time() - t0 > 3 * 0.02  # the render alone outlasts the deadline several times
    assert np.array_equal(img, ref)
    comm.check()
    comm.close()


def test_torch_nccl_one_rank_gather(rt2mod, config_scene, torch_cuda):
    """bench.py's multi-GPU gather (rt2/dist.py gather_image: dist.gather on the
    nccl backend = RCCL) run for real on a one-rank process group: the gathered
    and un-interleaved image equals the rank's own render bit for bit."""
    import socket

    import torch.distributed as dist
    from rt2 import dist as rdist
    torch = torch_cuda
    sd, spec = config_scene("A")
    W, H = 96, 40
    u = rt2mod.offline_uniforms(W, H, 4, 2, sd.num_triangles)
    scene = rt2mod.Scene(sd, 0)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        renderer = rdist.DeviceSlabRenderer(scene, u, 0, 2, 1, 0, 1)
        slab = renderer().clone()
        img = rdist.gather_image(renderer.image, H, W, 1, 0, 1)
        torch.cuda.synchronize()
        assert torch.equal(img, slab)
        assert np.array_equal(img.cpu().numpy(), scene.render_host(u, 0, 2))
    finally:
        dist.destroy_process_group()


def test_comm_two_ranks(rt2mod, tmp_path):
    """The C-ABI multi-rank paths: two processes, one GPU each, an
    RCCL communicator through rt2_comm_init — rt2_render_host_gather with
    uneven slabs and the 8-bit sums asked for by the root only, rt2_gather_slabs
    of device slabs (both bit-identical to rt2_render_host), and a rank-local
    failure that both ranks report instead of blocking.  Needs two GPUs (the
    driver's 8-GPU node); skipped on a one-GPU box."""
    import subprocess
    import sys
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    worker = os.path.join(os.path.dirname(__file__), "multi_rank_worker.py")
    out, idf = str(tmp_path / "res.json"), str(tmp_path / "comm.id")
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, worker, str(r), "2", idf, out], env=env) for r in range(2)]
    try:
        rcs = [p.wait(timeout=240) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0]
    import json
    res = json.load(open(out))
    assert res == {**res, "render_host_gather": True, "render_host_gather_rgb8": True, "gather_slabs": True,
                   "failure_agreed": True, "fault_gather.prepare@1": True, "fault_render@1": True,
                   "fault_check@0": True, "fault_gather.prepare@0": True, "after_faults": True,
                   "fault_agree.copy@1": True}, res
