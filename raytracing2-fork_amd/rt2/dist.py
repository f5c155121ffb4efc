"""Multi-GPU render: image-row tiles across ranks + one framebuffer gather.

SURVEY.md §8e: every (pixel, frame) is independent and its seed depends only on
(x, y, frame), so the image shards by rows with no data-path exchange.  Rows are
interleaved in tiles of `tile_rows` (rank r owns tiles t = r, r+N, ...) for load
balance (the cost of an image region depends on what it shows).  Each rank
renders its slab into a device accumulator, resolves it, and the slabs are
gathered to rank 0 with ONE collective (torch.distributed.gather: RCCL's gather
over xGMI when the backend is "nccl"); rank 0 un-interleaves.  The result is
bit-identical to a single-GPU render (same per-pixel arithmetic).

The per-rank slab renderer is injectable so the sharding/gather logic can be
tested on CPU ranks (gloo) with the CPU oracle standing in as the checker's
renderer; the product renderer is `device_slab_renderer` (HIP only).
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np


def slab_row_ids(height: int, tile_rows: int, rank: int, nranks: int) -> np.ndarray:
    """Image rows owned by `rank`, in slab order (== rt2_shard_row)."""
    rows = []
    t = rank
    while t * tile_rows < height:
        rows.extend(range(t * tile_rows, min((t + 1) * tile_rows, height)))
        t += nranks
    return np.array(rows, dtype=np.int32)


def max_slab_rows(height: int, tile_rows: int, nranks: int) -> int:
    return max(len(slab_row_ids(height, tile_rows, r, nranks)) for r in range(nranks))


def assemble(gathered, height: int, width: int, tile_rows: int, nranks: int):
    """Un-interleave gathered slabs [nranks, max_rows, W, C] into the image [H, W, C]."""
    import torch
    out = torch.empty((height, width) + tuple(gathered.shape[3:]), dtype=gathered.dtype, device=gathered.device)
    for r in range(nranks):
        ids = slab_row_ids(height, tile_rows, r, nranks)
        if len(ids):
            out[torch.as_tensor(ids, device=gathered.device, dtype=torch.long)] = gathered[r, :len(ids)]
    return out


def gather_image(slab, height: int, width: int, tile_rows: int, rank: int, nranks: int, group=None, root=0):
    """Gathers every rank's resolved slab to `root` (one RCCL gather); returns the
    full image on root and None elsewhere."""
    import torch
    import torch.distributed as dist
    mr = max_slab_rows(height, tile_rows, nranks)
    dev = slab.device
    if slab.is_cuda and dist.get_backend(group) == "gloo":
        slab = slab.cpu()  # gloo collectives take host tensors
    if slab.shape[0] == mr:
        padded = slab.contiguous()
    else:
        padded = torch.zeros((mr,) + tuple(slab.shape[1:]), dtype=slab.dtype, device=slab.device)
        padded[:slab.shape[0]] = slab
    if rank == root:
        gathered = torch.empty((nranks,) + tuple(padded.shape), dtype=slab.dtype, device=slab.device)
        dist.gather(padded, gather_list=list(gathered.unbind(0)), dst=root, group=group)
        return assemble(gathered, height, width, tile_rows, nranks).to(dev)
    dist.gather(padded, gather_list=None, dst=root, group=group)
    return None


class DeviceSlabRenderer:
    """Renders this rank's slab on its GPU through rt2_render (asynchronous, on torch's current stream)."""

    def __init__(self, scene, uniforms, frame_begin: int, frame_count: int, tile_rows: int, rank: int,
                 nranks: int):
        import torch
        from . import shard, shard_rows
        self.scene, self.u = scene, uniforms
        self.fb, self.fc = frame_begin, frame_count
        self.sh = shard(tile_rows, rank, nranks)
        self.rows = shard_rows(uniforms.height, self.sh)
        dev = torch.device("cuda", torch.cuda.current_device())
        self.accum = torch.zeros((self.rows, uniforms.width, 4), dtype=torch.float32, device=dev)
        self.image = torch.empty_like(self.accum)

    def __call__(self):
        import torch
        from . import resolve_rgba32f
        stream = torch.cuda.current_stream().cuda_stream
        self.accum.zero_()
        self.scene.render(self.u, self.fb, self.fc, self.sh, self.accum.data_ptr(), 0, stream)
        resolve_rgba32f(self.accum.data_ptr(), self.rows * self.u.width, self.fc, self.image.data_ptr(), stream)
        return self.image


def render_distributed(render_slab: Callable[[], "object"], height: int, width: int, tile_rows: int, rank: int,
                       nranks: int, group=None):
    """One distributed frame set: local slab render + one gather."""
    slab = render_slab()
    if nranks == 1:
        return slab
    return gather_image(slab, height, width, tile_rows, rank, nranks, group)
