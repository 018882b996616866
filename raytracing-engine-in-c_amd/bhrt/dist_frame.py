"""Multi-GPU frame assembly: one shard per rank, one gather, one un-permute.

The image is split into cyclic row blocks (block b -> rank b % world; bhrt_rows in
include/bhrt_api.h), so the divergent disk band lands on every GPU. Each rank renders its
rows into ONE contiguous byte buffer holding every SoA field (FrameBuffer), so assembling
the frame is a single collective (torch.distributed.gather: RCCL on GPUs, gloo in the CPU
tests) followed by a device-side permutation back to image order.
"""
import numpy as np
import torch
import torch.distributed as dist

from . import abi

INT_FIELDS = ("result", "steps")


def shard_row_count(H, row_block, shard, world):
    """Rows owned by `shard` (same rule as bhrt_shard_rows)."""
    if world <= 1:
        return H
    n, b = 0, shard
    while b * row_block < H:
        n += min((b + 1) * row_block, H) - b * row_block
        b += world
    return n


def shard_rows_index(H, row_block, shard, world):
    """Image row of each local row of `shard`, in local order."""
    n = shard_row_count(H, row_block, shard, world)
    j = np.arange(n)
    return ((j // row_block) * world + shard) * row_block + j % row_block


class FrameBuffer:
    """All SoA fields of n rays carved from one uint8 tensor (8-byte aligned views)."""

    def __init__(self, n, device, fields=abi.SOA_FIELDS):
        self.n = n
        self.fields = tuple(fields)
        sizes = {f: (4 if f in INT_FIELDS else 8) for f in self.fields}
        self.offsets, o = {}, 0
        for f in sorted(self.fields, key=lambda f: sizes[f]):  # int32 fields first
            if sizes[f] == 8:
                o = (o + 7) // 8 * 8                          # then 8-byte aligned doubles
            self.offsets[f] = (o, o + sizes[f] * n)
            o += sizes[f] * n
        self.nbytes = o
        self.buf = torch.empty(max(o, 8), dtype=torch.uint8, device=device)
        self.views = {f: self.view(self.buf, f) for f in self.fields}

    def view(self, buf, f):
        a, b = self.offsets[f]
        return buf[a:b].view(torch.int32 if f in INT_FIELDS else torch.float64)

    def soa(self):
        from . import lib
        return lib.soa_from_tensors(self.views)


def gather_frame(fb, H, W, row_block, world, rank, gathered=None):
    """Gather every rank's FrameBuffer to rank 0 and return {field: [H, W] tensor} there
    (None on other ranks). All shards must hold the same number of rows (pad H to a
    multiple of world * row_block)."""
    if world == 1:
        return {f: fb.views[f].view(H, W) for f in fb.fields}
    if rank == 0 and gathered is None:
        gathered = [torch.empty_like(fb.buf) for _ in range(world)]
    dist.gather(fb.buf, gathered if rank == 0 else None, dst=0)
    if rank != 0:
        return None
    n_rows = fb.n // W
    img = {}
    for f in fb.fields:
        parts = torch.stack([fb.view(g, f) for g in gathered])  # [world, n_rows*W]
        img[f] = (parts.view(world, n_rows // row_block, row_block, W)
                  .permute(1, 0, 2, 3).reshape(H, W))
    return img
