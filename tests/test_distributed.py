"""Multi-GPU frame assembly, exercised on CPU with the gloo backend.

bench.py at N > 1 renders one cyclic row-block shard per rank into a packed FrameBuffer,
gathers the buffers to rank 0 with ONE collective and un-permutes them into the image
(bhrt/dist_frame.py). Here each rank renders its shard with the CPU oracle instead of the
GPU (the plumbing under test is identical) and rank 0's assembled frame must equal the
single-process frame bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT
from bhrt import abi, configs
from bhrt.dist_frame import FrameBuffer, gather_frame, shard_row_count, shard_rows_index


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _scene():
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    return c, bh, dk, cfg, configs.camera("B")


def _worker(rank, world, port, W, H, B, out_path):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c, bh, dk, cfg, cam = _scene()
        rows = abi.Rows(B, rank, world)
        n = shard_row_count(H, B, rank, world) * W
        fb = FrameBuffer(n, "cpu")
        part = orc.oracle().render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, rows=rows,
                                         threads=1)
        for f in fb.fields:
            fb.views[f].copy_(torch.from_numpy(part[f]))
        img = gather_frame(fb, H, W, B, world, rank)
        if rank == 0:
            np.savez(out_path, **{f: v.numpy() for f, v in img.items()})
        else:
            assert img is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,B", [(2, 24, 32, 4), (3, 16, 24, 4), (2, 20, 16, 8)])
def test_gloo_gather_reassembles_frame(tmp_path, oracle, world, W, H, B):
    out = str(tmp_path / "frame.npz")
    mp.spawn(_worker, args=(world, _free_port(), W, H, B, out), nprocs=world, join=True)
    c, bh, dk, cfg, cam = _scene()
    want = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    with np.load(out) as got:
        for f in abi.SOA_FIELDS:
            assert np.array_equal(got[f].reshape(-1), want[f], equal_nan=True), f


def test_single_rank_gather_is_identity():
    fb = FrameBuffer(6 * 4, "cpu")
    for f in fb.fields:
        fb.views[f].copy_(torch.arange(24, dtype=fb.views[f].dtype))
    img = gather_frame(fb, 6, 4, 8, 1, 0)
    assert all(img[f].shape == (6, 4) for f in img)
    assert int(img["steps"][5, 3]) == 23


def test_shard_index_matches_library_rule():
    """Python and C (bhrt_shard_rows) agree on which rows a shard owns."""
    from bhrt import lib
    for H in (16, 1080, 2160):
        for world in (1, 2, 4, 8):
            for B in (1, 8):
                rows_all = []
                for s in range(world):
                    n = lib.shard_rows(H, abi.Rows(B, s, world))
                    assert n == shard_row_count(H, B, s, world)
                    rows_all.extend(shard_rows_index(H, B, s, world).tolist())
                assert sorted(rows_all) == list(range(H))


def test_framebuffer_alignment():
    for n in (1, 3, 7, 1000):
        fb = FrameBuffer(n, "cpu")
        for f, (a, b) in fb.offsets.items():
            assert a % (4 if f in ("result", "steps") else 8) == 0
            assert b - a == n * (4 if f in ("result", "steps") else 8)


def _pipeline_worker(rank, world, port, mode, W, H, frames, out_path):
    """bench.py's FramePipeline with oracle-rendered frames: `frames` frames in flight
    through the double-buffered async gathers."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from bhrt.dist_frame import FramePipeline, sample_offset
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c, bh, dk, cfg, cam = _scene()
        B = 4
        if mode == "shards":
            from bhrt.dist_frame import padded_shard_rows
            rows = abi.Rows(B, rank, world)
            n = padded_shard_rows(H, B, world) * W  # renders shard_row_count(...) rows of it
        else:
            rows, n = None, W * H
            off = sample_offset(rank)
            if off is not None:
                cam.use_offset, cam.offset_x, cam.offset_y = 1, off[0], off[1]
        pipe = FramePipeline(n, "cpu", world, rank, mode, H, W, B)
        part = orc.oracle().render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, rows=rows,
                                         threads=1)
        for i in range(frames):
            fb = pipe.next_buffer()
            for f in fb.fields:  # frame i = the rendered frame with steps + i (distinct frames)
                v = torch.from_numpy(part[f])
                fb.views[f][:len(v)].copy_(v + i if f == "steps" else v)
            pipe.submit()
        img = pipe.finish()
        if rank == 0:
            np.savez(out_path, **{f: v.numpy() for f, v in img.items()})
        else:
            assert img is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,frames,H", [(2, "shards", 3, 24), (3, "shards", 4, 24),
                                                 (2, "shards", 2, 20), (3, "shards", 3, 26),
                                                 (2, "samples", 3, 24), (3, "samples", 1, 24),
                                                 (4, "samples", 3, 16)])
def test_pipelined_gather(tmp_path, oracle, world, mode, frames, H):
    W = 16
    out = str(tmp_path / "frame.npz")
    mp.spawn(_pipeline_worker, args=(world, _free_port(), mode, W, H, frames, out),
             nprocs=world, join=True)
    c, bh, dk, cfg, cam = _scene()
    with np.load(out) as got:
        if mode == "shards":
            want = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
            for f in abi.SOA_FIELDS:
                w = want[f] + (frames - 1) if f == "steps" else want[f]
                assert np.array_equal(got[f].reshape(-1), w, equal_nan=True), f
            return
        from bhrt.dist_frame import sample_offset
        planes = []
        for k in range(world):
            cam_k = configs.camera("B")
            off = sample_offset(k)
            if off is not None:
                cam_k.use_offset, cam_k.offset_x, cam_k.offset_y = 1, off[0], off[1]
            planes.append(oracle.render_frame(bh, dk, cfg, cam_k, W, H, c.method, c.flags))
        for f in abi.SOA_FIELDS:  # rank 0 keeps its own plane (sample 0) ...
            w = planes[0][f] + (frames - 1) if f == "steps" else planes[0][f]
            assert got[f].shape[0] == 1
            assert np.array_equal(got[f][0].reshape(-1), w, equal_nan=True), f
        # ... and receives the colour averaged over every rank's plane (one reduce)
        mean = np.stack([np.mean([p[ch] for p in planes], axis=0)
                         for ch in ("rgb_r", "rgb_g", "rgb_b")])
        np.testing.assert_allclose(got["rgb_mean"].reshape(3, -1), mean, rtol=1e-12)
        # the offsets really moved the rays
        assert not np.array_equal(planes[0]["hit_x"], planes[1]["hit_x"], equal_nan=True)
