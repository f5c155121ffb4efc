"""One rank of tests/test_gpu_multi.py::test_comm_two_ranks (run as a separate
process per GPU): rt2_render_host_gather with uneven slabs and asymmetric
8-bit output pointers, then rt2_gather_slabs, then rank-local failures (a
shard that does not match, and RT2_FAULT_AT injections at every site of
rt2_comm_protocol.h) that every rank must see as an error instead of a hang.  Rank 0 writes its checks
to the JSON file named on the command line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing2-fork_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import rt2  # noqa: E402


def main():
    rank, n, id_file, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
    torch.cuda.set_device(rank)
    if rank == 0:
        uid = rt2.Comm.unique_id()
        with open(id_file + ".tmp", "wb") as f:
            f.write(uid)
        os.replace(id_file + ".tmp", id_file)
    else:
        t0 = time.time()
        while not os.path.exists(id_file):
            if time.time() - t0 > 60:
                raise SystemExit("no communicator id")
            time.sleep(0.05)
        uid = open(id_file, "rb").read()
    comm = rt2.Comm(uid, n, rank, rank)
    sd, spec = rt2.build_config_scene("B")
    W, H, tile = 96, 54, 5  # 54 rows in tiles of 5 over 2 ranks: uneven slabs
    u = rt2.offline_uniforms(W, H, spec.bounces, 4, sd.num_triangles)
    scene = rt2.Scene(sd, rank)
    res = {}
    # the root asks for the 8-bit sums, the other rank does not (round 2 hung here)
    got = scene.render_host_gather(u, 1, 2, rt2.shard(tile, rank, n), comm, 0, rgb8=(rank == 0))
    if rank == 0:
        img, img8 = got
        ref, ref8 = scene.render_host(u, 1, 2, rgb8=True)
        res["render_host_gather"] = bool(np.array_equal(img, ref))
        res["render_host_gather_rgb8"] = bool(np.array_equal(img8, ref8))
    # asynchronous slab gather of a device slab
    sh = rt2.shard(tile, rank, n)
    rows = rt2.shard_rows(H, sh)
    acc = torch.zeros((rows, W, 4), device="cuda")
    slab = torch.empty_like(acc)
    stream = torch.cuda.current_stream().cuda_stream
    scene.render(u, 0, 1, sh, acc.data_ptr(), 0, stream)
    rt2.resolve_rgba32f(acc.data_ptr(), rows * W, 1, slab.data_ptr(), stream)
    image = torch.zeros((H, W, 4), device="cuda") if rank == 0 else None
    comm.gather_slabs(slab.data_ptr(), W, H, sh, 0, image.data_ptr() if rank == 0 else 0, stream)
    comm.wait(stream)  # rt2_comm_wait: the gather drained under the deadline
    comm.check()
    if rank == 0:
        res["gather_slabs"] = bool(np.array_equal(image.cpu().numpy(), scene.render_host(u, 0, 1)))
    # a rank-local failure (rank 1's shard does not match the communicator):
    # every rank returns an error, none blocks in the gather
    bad = rt2.shard(tile, rank, n) if rank == 0 else rt2.shard(tile, 0, n + 1)
    try:
        scene.render_host_gather(u, 0, 1, bad, comm, 0)
        res["failure_agreed"] = False
    except rt2.RT2Error as e:
        res["failure_agreed"] = True
        res["failure_message"] = str(e)
    comm.check()
    # injected failures (RT2_FAULT_AT, include/rt2.h "Failure contract"): a
    # failure the agreement sees makes every rank return < 0 at once
    for site in ("gather.prepare@1", "render@1", "check@0", "gather.prepare@0"):
        os.environ["RT2_FAULT_AT"] = site
        t0 = time.time()
        try:
            if site.startswith("gather."):
                comm.gather_slabs(slab.data_ptr(), W, H, sh, 0, image.data_ptr() if rank == 0 else 0, stream)
            else:
                scene.render_host_gather(u, 0, 1, sh, comm, 0)
            res[f"fault_{site}"] = False
        except rt2.RT2Error:
            res[f"fault_{site}"] = time.time() - t0 < 30
        os.environ.pop("RT2_FAULT_AT")
        comm.check()
    # the communicator still works after them
    got = scene.render_host_gather(u, 0, 1, sh, comm, 0)
    if rank == 0:
        res["after_faults"] = bool(np.array_equal(got, scene.render_host(u, 0, 1)))
    # a rank that cannot take part in the agreement at all: it aborts, and the
    # peers' watchdog aborts theirs at the deadline — every rank returns < 0
    os.environ["RT2_FAULT_AT"] = "agree.copy@1"
    os.environ["RT2_COMM_TIMEOUT_S"] = "10"
    t0 = time.time()
    try:
        scene.render_host_gather(u, 0, 1, sh, comm, 0)
        res["fault_agree.copy@1"] = False
    except rt2.RT2Error:
        res["fault_agree.copy@1"] = time.time() - t0 < 60
    os.environ.pop("RT2_FAULT_AT")
    comm.close()
    if rank == 0:
        with open(out, "w") as f:
            json.dump(res, f)


if __name__ == "__main__":
    main()
