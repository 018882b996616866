"""Multi-GPU frame assembly: one shard per rank, ONE gather per frame, pipelined.

A frame is a W x H image split into S cyclic row-block shards (block b -> shard b % S,
bhrt_rows in include/bhrt_api.h), so the divergent regions (the disk band, the image centre
against its edges) land on every shard alike. Rank r renders shard r into ONE contiguous byte
buffer holding every SoA field of its rays (FrameBuffer); the per-ray SoA stays resident on
its GPU. Rank 0 assembles the image -- by default the colour planes, 24 B per ray -- from a
single collective (torch.distributed.gather: RCCL over xGMI on GPUs, gloo in the CPU tests):
the gathered fields are one contiguous byte range of every rank's buffer, so the collective
reads the render target itself, and rank 0 scatters the N shards into their image rows with
one strided copy per field. S may exceed the number of ranks (C5: the 7680x4320 frame is 8
shards of 540 rows; N GPUs render shards 0..N-1 and rank 0 holds those rows of the image).

FramePipeline.mode:
  * "shards" -- the above (bench.py's default; configs.Config.frame gives W, H, S, B).
  * "samples" (opt-in) -- every rank traces the whole W x H frame at its own sub-pixel offset
    (sample_offset: rank 0 the pixel centre, rank k the reference's Halton point k), i.e. the
    frame is supersampled across GPUs with the per-GPU work of one frame: trace_pixel's
    supersampling (raytracer.c:1096-1164) with one sample per GPU. The exchange is the sample
    average of the colour: ONE reduce (sum) of the three colour planes to rank 0, which
    divides by the sample count.

The collective of frame i runs (on the collective's own stream) while frame i+1 renders; a
buffer is reused only after the collective that read it has completed (double buffering).
"""
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist

from . import abi

INT_FIELDS = ("result", "steps")
RGB_FIELDS = ("rgb_r", "rgb_g", "rgb_b")
DISPLAY_FIELD = ("rgba8",)  # the display buffer (4 B per pixel): bench.py's default gather
# per-ray layout of a field in the FrameBuffer: (element dtype, elements per ray)
_LAYOUT = {"result": (torch.int32, 1), "steps": (torch.int32, 1),
           "rgba8": (torch.uint8, 4), "rgba32f": (torch.float32, 4)}


def field_layout(f):
    return _LAYOUT.get(f, (torch.float64, 1))


def field_bytes(f):
    dt, k = field_layout(f)
    return k * torch.empty(0, dtype=dt).element_size()


def shard_row_count(H, row_block, shard, num_shards):
    """Rows owned by `shard` of `num_shards` (same rule as bhrt_shard_rows)."""
    if num_shards <= 1:
        return H
    n, b = 0, shard
    while b * row_block < H:
        n += min((b + 1) * row_block, H) - b * row_block
        b += num_shards
    return n


def padded_shard_rows(H, row_block, num_shards):
    """Rows of every shard's buffer: the largest shard in whole blocks, so all ranks gather
    equal-sized buffers. A shard's padding rows map to image rows >= H."""
    if num_shards <= 1:
        return H
    return -(-H // (row_block * num_shards)) * row_block


def shard_rows_index(H, row_block, shard, num_shards):
    """Image row of each local row of `shard`, in local order."""
    n = shard_row_count(H, row_block, shard, num_shards)
    if num_shards <= 1:
        return np.arange(n)
    j = np.arange(n)
    return ((j // row_block) * num_shards + shard) * row_block + j % row_block


class FrameBuffer:
    """All SoA fields of n rays carved from one uint8 tensor (aligned views): the 4-byte
    fields first (int32 result/steps, the rgba8 display buffer), then the doubles in the order
    given (abi.SOA_FIELDS ends with the colour planes, so they form a contiguous range), then
    the 16-byte rgba32f buffer if requested."""

    def __init__(self, n, device, fields=abi.SOA_FIELDS):
        self.n = n
        self.fields = tuple(fields)
        sizes = {f: field_bytes(f) for f in self.fields}
        self.offsets, o = {}, 0
        for f in sorted(self.fields, key=lambda f: sizes[f]):  # 4-byte fields first (stable)
            if sizes[f] >= 8:
                o = (o + 15) // 16 * 16 if sizes[f] > 8 else (o + 7) // 8 * 8
            self.offsets[f] = (o, o + sizes[f] * n)
            o += sizes[f] * n
        self.nbytes = o
        self.buf = torch.empty(max(o, 8), dtype=torch.uint8, device=device)
        self.views = {f: self.view(self.buf, f) for f in self.fields}

    def view(self, buf, f):
        a, b = self.offsets[f]
        dt, k = field_layout(f)
        v = buf[a:b].view(dt)
        return v.view(-1, k) if k > 1 else v

    def span(self, fields):
        """(first, last) byte of `fields`, which must be one contiguous range of the buffer."""
        rng = sorted(self.offsets[f] for f in fields)
        for (_, b), (a, _) in zip(rng, rng[1:]):
            if a != b:
                raise ValueError(f"fields {fields} are not contiguous in the frame buffer")
        return rng[0][0], rng[-1][1]

    def soa(self):
        """The FrameSoA of this buffer (built once: the pointers never change)."""
        if getattr(self, "_soa", None) is None:
            from . import lib
            self._soa = lib.soa_from_tensors(self.views)
        return self._soa


def sample_offset(k):
    """Sub-pixel offset of sample plane k: None (pixel centre) for k = 0, else the Halton
    point of generate_jittered_position's JITTER_HALTON (raytracer.c:900-915)."""
    if k == 0:
        return None
    from . import lib
    return lib.halton(k, 2), lib.halton(k, 3)


@dataclass
class Assembled:
    """A frame on rank 0.
    image       {field: [H, W]} of the gathered fields. "shards": the image rows of the
                rendered shards 0..N-1 (rows of other shards are 0); "samples": the colour
                averaged over every rank's sample plane.
    local       {field: [rows, W]} rank 0's own per-ray SoA (every field it rendered).
    local_rows  image row of each local row."""
    image: dict
    local: dict
    local_rows: np.ndarray


class FramePipeline:
    """Double-buffered render -> gather-to-rank-0 -> assemble.

    "shards": rank r renders shard first_shard + r of `shards` (default: world) of the W x H
    image into
    next_buffer() (n = W * padded_shard_rows(H, row_block, shards) rays; it fills its first
    W * shard_row_count(...) of them). "samples": every rank renders the whole W x H frame
    (n = W * H) at its own sub-pixel offset.
    `gather`: the fields that travel to rank 0 -- the colour planes by default; they must be
    a contiguous range of the FrameBuffer (the doubles keep `fields` order).
    Per frame: fb = next_buffer(); render into fb; submit(). finish() completes the
    collectives still in flight and returns rank 0's newest Assembled frame (None elsewhere).
    """

    def __init__(self, n, device, world, rank, mode, H, W, row_block=8,
                 fields=abi.SOA_FIELDS, shards=None, gather=RGB_FIELDS, first_shard=0,
                 slots=2, force_collective=False):
        assert mode in ("shards", "samples")
        # the collective runs at world > 1; force_collective runs it at world 1 too (a
        # one-rank process group: the RCCL path exercised on a one-GPU box, tests)
        self.collective = world > 1 or bool(force_collective)
        self.nslots = max(2, int(slots))  # frames in flight: a slot is reused nslots frames later
        self.world, self.rank, self.mode = world, rank, mode
        self.H, self.W, self.row_block = H, W, row_block
        self.shards = (shards or world) if mode == "shards" else 1
        self.first = first_shard  # rank r renders shard first_shard + r
        if mode == "shards" and not 0 <= first_shard <= self.shards - world:
            raise ValueError(f"{world} ranks from shard {first_shard} but {self.shards} shards")
        self.bufs = [FrameBuffer(n, device, fields) for _ in range(self.nslots)]
        fb = self.bufs[0]
        self.gather = tuple(gather) if gather is not None else fb.fields
        self.span = fb.span(self.gather)
        if mode == "samples" and world > 1 and not set(self.gather) <= set(RGB_FIELDS):
            raise ValueError("samples mode reduces the colour planes only")
        self.works = [None] * self.nslots
        # the collective's own GPU time per completed frame (ms), where the process group
        # times its work (RCCL with TORCH_NCCL_ENABLE_TIMING=1: Work._get_duration), filled by
        # collect_timing() once the device has synchronised: wait() only orders the current
        # stream after the collective, and its end event cannot be read before it completes
        self.collective_ms = []
        self.timing_error = None
        self._timed = []
        self.frames = 0
        self.last = None
        self.images = self.gathered = self.colour = None
        self.staged = False
        if mode == "samples":
            if world > 1:  # per slot: the colour planes summed over ranks (in place on rank 0)
                self.colour = [torch.empty(len(self.gather), n, dtype=torch.float64,
                                           device=device) for _ in range(self.nslots)]
            return
        self.direct = not self.collective and self.shards == 1  # the buffer IS the image
        if rank == 0 and not self.direct:
            a, b = self.span
            # one [world, bytes] receive tensor per slot; gather writes rank k's range to row k
            self.gathered = [torch.empty(world, b - a, dtype=torch.uint8, device=device)
                             for _ in range(self.nslots)]
            rows = padded_shard_rows(H, row_block, self.shards) * self.shards
            self.images = [{f: torch.zeros(rows, W, *self._inner(f), dtype=fb.views[f].dtype,
                                        device=device)
                            for f in self.gather} for _ in range(self.nslots)]
        # gloo gathers host tensors only: with device buffers (the one-GPU rehearsal of the
        # N-rank bench, BHRT_BENCH_SHARE_DEVICE) the gathered range travels through host
        # copies; RCCL gathers the device buffers directly
        self.staged = (self.collective and torch.device(device).type != "cpu" and
                       dist.get_backend() == "gloo")
        if self.staged:
            a, b = self.span
            self.host_send = [torch.empty(b - a, dtype=torch.uint8) for _ in range(self.nslots)]
            self.host_recv = ([torch.empty(world, b - a, dtype=torch.uint8)
                               for _ in range(self.nslots)] if rank == 0 else None)

    def next_buffer(self):
        slot = self.frames % self.nslots
        self._complete(slot)
        return self.bufs[slot]

    def submit(self):
        slot = self.frames % self.nslots
        fb = self.bufs[slot]
        a, b = self.span
        if self.mode == "samples":
            if self.world > 1:
                col = self.colour[slot]
                for i, c in enumerate(self.gather):
                    col[i].copy_(fb.views[c])
                self.works[slot] = dist.reduce(col, dst=0, op=dist.ReduceOp.SUM, async_op=True)
            else:
                self.works[slot] = True
        elif self.collective and self.staged:
            self.host_send[slot].copy_(fb.buf[a:b])  # (waits for the render on this stream)
            recv = list(self.host_recv[slot].unbind(0)) if self.rank == 0 else None
            self.works[slot] = dist.gather(self.host_send[slot], recv, dst=0, async_op=True)
        elif self.collective:
            recv = list(self.gathered[slot].unbind(0)) if self.rank == 0 else None
            self.works[slot] = dist.gather(fb.buf[a:b], recv, dst=0, async_op=True)
        else:
            if self.gathered is not None:  # one shard of several: place it in the image
                self.gathered[slot][0].copy_(fb.buf[a:b])
            self.works[slot] = True
        self.frames += 1

    def collect_timing(self):
        """Move the GPU time of every collective completed since the last call into
        collective_ms (call after torch.cuda.synchronize()); unmeasured (gloo, or timing not
        enabled): collective_ms stays as it was and timing_error says why."""
        for w in self._timed:
            try:
                dur = getattr(w, "get_duration", None) or w._get_duration  # (torch 2.10: _get_duration)
                self.collective_ms.append(float(dur()))
            except Exception as e:  # (gloo, or TORCH_NCCL_ENABLE_TIMING unset)
                self.timing_error = repr(e)[:200]
        self._timed.clear()
        return self.collective_ms

    def reset_timing(self):
        self._timed.clear()
        self.collective_ms.clear()
        self.timing_error = None

    def finish(self):
        for k in range(max(self.frames - self.nslots, 0), self.frames):  # oldest first
            self._complete(k % self.nslots)
        return self.last

    def _complete(self, slot):
        w = self.works[slot]
        if w is None:
            return
        if w is not True:
            w.wait()
            self._timed.append(w)
            if self.staged and self.rank == 0:
                self.gathered[slot].copy_(self.host_recv[slot])
        self.works[slot] = None
        if self.rank == 0:
            self.last = self._assemble(slot)

    # Per-frame host work is a handful of tensor ops: every view the assembly needs is built
    # once per slot (a C4 shard of an 8-GPU plan renders in ~0.1 ms, so per-frame Python
    # view-building, ~0.1-0.2 ms, had become the frame rate's bound)
    def _plan(self, slot):
        plans = self.__dict__.setdefault("_plans", {})
        if slot in plans:
            return plans[slot]
        fb, H, W, world = self.bufs[slot], self.H, self.W, self.world
        local, idx = self._local(fb)
        copies, image = [], {}
        if self.mode == "samples":
            if world == 1:
                image = {f: local[f] for f in self.gather}
        elif self.direct:
            image = {f: local[f] for f in self.gather}
        else:
            B, S = self.row_block, self.shards
            nbk = fb.n // W // B                       # blocks per (padded) shard
            src_all = self.gathered[slot]
            a0 = self.span[0]
            for f in self.gather:
                a, b = fb.offsets[f]
                inner = self._inner(f)
                dst = self.images[slot][f]
                raw = src_all[:, a - a0:b - a0]
                if fb.views[f].dtype == torch.uint8 and inner == (4,):
                    # rgba8: one 4-byte word per pixel -- an int32 copy moves 4x fewer
                    # elements than a uint8 one (an 8-shard C4 frame: ~8x faster on rank 0)
                    src = raw.view(torch.int32).view(world, nbk, B, W)
                    d = dst.view(torch.int32).view(nbk, S, B, W)
                else:
                    src = raw.view(fb.views[f].dtype).view(world, nbk, B, W, *inner)
                    d = dst.view(nbk, S, B, W, *inner)
                copies.append((d[:, self.first:self.first + world], src.transpose(0, 1)))
                image[f] = dst[:H]
        plans[slot] = (local, idx, copies, image)
        return plans[slot]

    def _local(self, fb):
        if self.mode == "samples":
            return ({f: fb.views[f].view(self.H, self.W, *self._inner(f)) for f in fb.fields},
                    np.arange(self.H))
        idx = shard_rows_index(self.H, self.row_block, self.first, self.shards)
        rows = fb.n // self.W
        return {f: fb.views[f].view(rows, self.W, *self._inner(f))[:len(idx)]
                for f in fb.fields}, idx

    @staticmethod
    def _inner(f):
        k = field_layout(f)[1]
        return (k,) if k > 1 else ()

    def _assemble(self, slot):
        local, idx, copies, image = self._plan(slot)
        if self.mode == "samples" and self.world > 1:
            image = {f: (self.colour[slot][i] / self.world).view(self.H, self.W)
                     for i, f in enumerate(self.gather)}
        for d, src in copies:
            d.copy_(src)
        return Assembled(image, local, idx)
