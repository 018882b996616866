"""Multi-GPU frame assembly: one buffer per rank, one gather per frame, pipelined.

Each rank renders into ONE contiguous byte buffer holding every SoA field (FrameBuffer), so
assembling a frame on rank 0 is a single collective (torch.distributed.gather: RCCL on GPUs,
gloo in the CPU tests). Two ways of splitting the work (FramePipeline.mode):

  * "shards" (strong scaling, one image): cyclic row blocks (block b -> rank b % world;
    bhrt_rows in include/bhrt_api.h), so the divergent disk band lands on every GPU; rank 0
    permutes the gathered shards back to image order on the device.
  * "samples" (weak scaling): every rank traces the whole frame at its own sub-pixel offset
    (sample_offset: rank 0 the pixel centre, rank k the reference's Halton point k), i.e.
    the frame is supersampled across GPUs with the per-GPU work of one frame -- trace_pixel's
    supersampling (raytracer.c:1096-1164) with one sample per GPU. Its exchange is the
    sample average of the colour: ONE reduce (sum) of the three colour planes to rank 0
    (24 B per ray instead of the 96 B of a full gather), which divides by the sample count.
    Every rank's per-ray SoA (hit classes, points, distances) stays resident on its own GPU.

The collective of frame i runs (on the collective's own stream) while frame i+1 renders; a
buffer is reused only after the collective that read it has completed (double buffering).
"""
import numpy as np
import torch
import torch.distributed as dist

from . import abi

INT_FIELDS = ("result", "steps")
RGB_FIELDS = ("rgb_r", "rgb_g", "rgb_b")


def shard_row_count(H, row_block, shard, world):
    """Rows owned by `shard` (same rule as bhrt_shard_rows)."""
    if world <= 1:
        return H
    n, b = 0, shard
    while b * row_block < H:
        n += min((b + 1) * row_block, H) - b * row_block
        b += world
    return n


def padded_shard_rows(H, row_block, world):
    """Rows of every shard's buffer in "shards" mode: the largest shard, in whole blocks, so
    all ranks gather equal-sized buffers. A shard's padding rows map to image rows >= H."""
    if world <= 1:
        return H
    return -(-H // (row_block * world)) * row_block


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


def sample_offset(k):
    """Sub-pixel offset of sample plane k: None (pixel centre) for k = 0, else the Halton
    point of generate_jittered_position's JITTER_HALTON (raytracer.c:900-915)."""
    if k == 0:
        return None
    from . import lib
    return lib.halton(k, 2), lib.halton(k, 3)


class FramePipeline:
    """Double-buffered render -> gather-to-rank-0 -> assemble.

    n = rays per rank buffer: W * H ("samples"), W * padded_shard_rows(...) ("shards", of
    which a rank renders its first W * shard_row_count(...)).
    Per frame: fb = next_buffer(); render into fb; submit(). finish() completes the gathers
    still in flight and returns rank 0's newest assembled frame (None elsewhere):
      shards:  {field: [H, W]}
      samples: world > 1 with rgb rendered: {field: [1, H, W]} of rank 0's own sample plane
               plus "rgb_mean" [3, H, W], the colour averaged over all planes (reduce);
               without rgb: {field: [world, H, W]}, every plane gathered; world 1: the plane.
    """

    def __init__(self, n, device, world, rank, mode, H, W, row_block=8,
                 fields=abi.SOA_FIELDS):
        assert mode in ("shards", "samples")
        self.world, self.rank, self.mode = world, rank, mode
        self.H, self.W, self.row_block = H, W, row_block
        self.bufs = [FrameBuffer(n, device, fields) for _ in range(2)]
        self.reduce = (mode == "samples" and world > 1 and
                       all(c in fields for c in RGB_FIELDS))
        if self.reduce:  # per slot: the colour planes summed over ranks (in place on rank 0)
            self.colour = [torch.empty(3, n, dtype=torch.float64, device=device)
                           for _ in range(2)]
        self.gathered = ([[torch.empty_like(b.buf) for _ in range(world)] for b in self.bufs]
                         if (world > 1 and rank == 0 and not self.reduce) else None)
        self.works = [None, None]
        self.frames = 0
        self.last = None

    def next_buffer(self):
        slot = self.frames % 2
        self._complete(slot)
        return self.bufs[slot]

    def submit(self):
        slot = self.frames % 2
        if self.reduce:
            fb, col = self.bufs[slot], self.colour[slot]
            for i, c in enumerate(RGB_FIELDS):
                col[i].copy_(fb.views[c])
            self.works[slot] = dist.reduce(col, dst=0, op=dist.ReduceOp.SUM, async_op=True)
        elif self.world > 1:
            self.works[slot] = dist.gather(
                self.bufs[slot].buf, self.gathered[slot] if self.rank == 0 else None, dst=0,
                async_op=True)
        else:
            self.works[slot] = True
        self.frames += 1

    def finish(self):
        for k in range(max(self.frames - 2, 0), self.frames):  # oldest first
            self._complete(k % 2)
        return self.last

    def _complete(self, slot):
        w = self.works[slot]
        if w is None:
            return
        if w is not True:
            w.wait()
        self.works[slot] = None
        if self.rank == 0:
            self.last = self._assemble(slot)

    def _assemble(self, slot):
        fb, H, W, world = self.bufs[slot], self.H, self.W, self.world
        parts = self.gathered[slot] if (world > 1 and not self.reduce) else [fb.buf]
        img = {}
        if self.mode == "shards":
            if world == 1:
                return {f: fb.views[f].view(H, W) for f in fb.fields}
            n_rows, B = fb.n // W, self.row_block  # padded_shard_rows
            for f in fb.fields:
                p = torch.stack([fb.view(g, f) for g in parts])  # [world, n_rows*W]
                img[f] = (p.view(world, n_rows // B, B, W).permute(1, 0, 2, 3)
                          .reshape(world * n_rows, W)[:H])
            return img
        if self.reduce:  # rank 0's own plane (sample 0) and the mean colour of all samples
            img = {f: fb.views[f].view(1, H, W) for f in fb.fields}
            img["rgb_mean"] = (self.colour[slot] / world).view(3, H, W)
            return img
        for f in fb.fields:
            img[f] = (fb.views[f].view(1, H, W) if world == 1 else
                      torch.stack([fb.view(g, f) for g in parts]).view(world, H, W))
        if world > 1 and all(c in img for c in RGB_FIELDS):
            img["rgb_mean"] = torch.stack([img[c].mean(dim=0) for c in RGB_FIELDS])
        return img
