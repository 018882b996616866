"""Multi-GPU frame assembly, exercised on CPU with the gloo backend.

bench.py at N > 1 renders one cyclic row-block shard per rank into a packed FrameBuffer,
gathers the colour planes (or every field) to rank 0 with ONE collective and scatters them
into the image rows (bhrt/dist_frame.py FramePipeline). Here each rank renders its shard with
the CPU oracle instead of the GPU (the plumbing under test is identical) and rank 0's
assembled frame must equal the single-process frame bit for bit.
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
from bhrt.dist_frame import (DISPLAY_FIELD, FrameBuffer, FramePipeline, RGB_FIELDS,
                             padded_shard_rows, sample_offset, shard_row_count,
                             shard_rows_index)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tiles_worker(rank, world, port, W, H, B, S, gather, frames, cfg_name, max_steps,
                  out_path, slots=2):
    """bench.py's tiles mode: rank r renders shard r of S through FramePipeline, `frames`
    frames in flight through the double-buffered async gathers (frame i = the rendered
    shard with its colour scaled by i + 1, so the frames differ)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = configs.CONFIGS[cfg_name]
        bh, dk, cfg = c.scene()
        if max_steps:
            cfg.max_integration_steps = max_steps
        cam = configs.camera("B")
        rows = abi.Rows(B, rank, S) if S > 1 else None
        n = padded_shard_rows(H, B, S) * W
        fields = abi.SOA_FIELDS + (DISPLAY_FIELD if gather == "rgba8" else ())
        pipe = FramePipeline(n, "cpu", world, rank, "shards", H, W, B, fields, shards=S,
                             gather={"all": None, "image": RGB_FIELDS,
                                     "rgba8": DISPLAY_FIELD}[gather], slots=slots)
        part = orc.oracle().render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, rows=rows,
                                         threads=2)
        for i in range(frames):
            fb = pipe.next_buffer()
            for f in abi.SOA_FIELDS:
                v = torch.from_numpy(part[f])
                fb.views[f][:len(v)].copy_(v * (i + 1) if f in RGB_FIELDS else v)
            if "rgba8" in fields:  # the colour pass's display buffer of frame i
                v = torch.from_numpy(abi.rgba8_from_rgb(*(part[f] * (i + 1)
                                                          for f in RGB_FIELDS)))
                fb.views["rgba8"][:len(v)].copy_(v)
            pipe.submit()
        fr = pipe.finish()
        if rank == 0:
            np.savez(out_path, local_rows=fr.local_rows,
                     **{"img_" + f: v.numpy() for f, v in fr.image.items()},
                     **{"loc_" + f: v.numpy() for f, v in fr.local.items()})
        else:
            assert fr is None
    finally:
        dist.destroy_process_group()


def _run_tiles(tmp_path, world, W, H, B, S, gather, frames=1, cfg_name="C2", max_steps=0,
               slots=2):
    out = str(tmp_path / "frame.npz")
    mp.spawn(_tiles_worker, args=(world, _free_port(), W, H, B, S, gather, frames, cfg_name,
                                  max_steps, out, slots), nprocs=world, join=True)
    with np.load(out) as z:
        return {k: z[k] for k in z.files}


def _c2_frame(oracle, W, H):
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    return oracle.render_frame(bh, dk, cfg, configs.camera("B"), W, H, c.method, c.flags)


@pytest.mark.parametrize("world,W,H,B,gather,frames,slots", [
    (2, 24, 32, 4, "all", 1, 2), (3, 16, 24, 4, "all", 3, 2), (2, 20, 16, 8, "image", 2, 2),
    (3, 16, 26, 4, "image", 4, 2), (2, 16, 20, 8, "all", 3, 2),
    (2, 16, 20, 8, "all", 7, 4), (3, 16, 24, 4, "image", 6, 4)])  # four frames in flight
def test_gloo_tiles_reassemble_frame(tmp_path, oracle, world, W, H, B, gather, frames, slots):
    """Every shard rendered (S = world), padded shards included (H = 26, 20): the image on
    rank 0 is the single-process frame, several frames in flight (two or four buffer slots,
    bench.py --streams auto)."""
    got = _run_tiles(tmp_path, world, W, H, B, world, gather, frames, slots=slots)
    want = _c2_frame(oracle, W, H)
    fields = abi.SOA_FIELDS if gather == "all" else RGB_FIELDS
    assert sorted(k[4:] for k in got if k.startswith("img_")) == sorted(fields)
    for f in fields:
        w = want[f] * frames if f in RGB_FIELDS else want[f]
        assert got["img_" + f].shape == (H, W), f
        assert np.array_equal(got["img_" + f].reshape(-1), w, equal_nan=True), f
    # rank 0 keeps its own shard's every field
    idx = shard_rows_index(H, B, 0, world)
    assert np.array_equal(got["local_rows"], idx)
    assert np.array_equal(got["loc_steps"], want["steps"].reshape(H, W)[idx])


@pytest.mark.parametrize("world,W,H,B,S,frames", [
    (2, 24, 32, 4, 2, 1), (3, 16, 26, 4, 3, 3), (2, 16, 40, 2, 4, 2)])
def test_gloo_rgba8_gather_assembles_display_image(tmp_path, oracle, world, W, H, B, S,
                                                   frames):
    """bench.py's default exchange: ONE gather of the 4-byte rgba8 display buffer (not the
    24-byte f64 colour planes). Rank 0's image is the rendered shards' display pixels, within
    one 8-bit step of the oracle's f64 colour; rows of shards no rank rendered stay 0."""
    got = _run_tiles(tmp_path, world, W, H, B, S, "rgba8", frames)
    assert sorted(k for k in got if k.startswith("img_")) == ["img_rgba8"]
    img = got["img_rgba8"]
    assert img.shape == (H, W, 4) and img.dtype == np.uint8
    want = _c2_frame(oracle, W, H)
    mine = np.concatenate([shard_rows_index(H, B, s, S) for s in range(world)])
    rgb = [want[f].reshape(H, W)[mine] * frames for f in RGB_FIELDS]
    assert np.array_equal(img[mine], abi.rgba8_from_rgb(*rgb))
    for i, v in enumerate(rgb):  # one 8-bit step of the f64 colour (NaN -> 255)
        ref = np.where(np.isnan(v), 255.0, np.minimum(v, 1.0) * 255.0)
        assert np.all(np.abs(img[mine][..., i] - ref) <= 1.0)
    assert not np.delete(img, mine, axis=0).any()
    # rank 0 keeps its own shard's f64 SoA (the per-ray record stays resident per rank)
    idx = shard_rows_index(H, B, 0, S)
    assert np.array_equal(got["loc_steps"], want["steps"].reshape(H, W)[idx])
    # exchange size: 4 B per ray instead of 24
    fb = FrameBuffer(8, "cpu", abi.SOA_FIELDS + DISPLAY_FIELD)
    a, b = fb.span(DISPLAY_FIELD)
    assert b - a == 4 * 8 and fb.span(RGB_FIELDS)[1] - fb.span(RGB_FIELDS)[0] == 24 * 8


def test_gloo_partial_node_frame(tmp_path, oracle):
    """S > world: 2 ranks render shards 0 and 1 of 4; rank 0 holds exactly those image rows."""
    W, H, B, S = 16, 40, 2, 4
    got = _run_tiles(tmp_path, 2, W, H, B, S, "image", 2)
    want = _c2_frame(oracle, W, H)
    mine = np.concatenate([shard_rows_index(H, B, s, S) for s in (0, 1)])
    other = np.setdiff1d(np.arange(H), mine)
    for f in RGB_FIELDS:
        img = got["img_" + f]
        assert np.array_equal(img[mine], 2 * want[f].reshape(H, W)[mine], equal_nan=True), f
        assert not img[other].any(), f


def test_gloo_c5_shards_assemble_8k_layout(tmp_path, oracle):
    """BASELINE C5's node frame: 7680x4320 in 8 shards of 540 rows (cyclic 6-row blocks).
    World 2 renders shards 0 and 1 (2 RKF45 steps per ray keep the CPU render short; the
    layout is what is under test) and rank 0 assembles them into the 7680x4320 image."""
    c = configs.CONFIGS["C5"]
    plan = c.frame(2)
    W, H, S, B = plan.width, plan.height, plan.shards, plan.row_block
    assert (W, H, S, B) == (7680, 4320, 8, 6)
    assert all(shard_row_count(H, B, s, S) == 540 for s in range(S))
    got = _run_tiles(tmp_path, 2, W, H, B, S, "image", 1, "C5", 2)
    bh, dk, cfg = c.scene()
    cfg.max_integration_steps = 2
    rows = np.concatenate([shard_rows_index(H, B, s, S) for s in (0, 1)])
    assert len(rows) == 1080
    for r in rows[::37]:
        want = oracle.render_frame(bh, dk, cfg, configs.camera("B"), W, H, c.method, c.flags,
                                   rows=abi.Rows(1, int(r), H), threads=4)
        for f in RGB_FIELDS:
            assert np.array_equal(got["img_" + f][r], want[f], equal_nan=True), (r, f)
    other = np.setdiff1d(np.arange(H), rows)
    assert not got["img_rgb_r"][other].any()
    assert got["img_rgb_r"][rows].all()  # every pixel of the rendered rows has colour


def _samples_worker(rank, world, port, W, H, frames, out_path):
    """bench.py --weak-mode samples: every rank traces the frame at its own sub-pixel
    offset, one reduce averages the colour on rank 0."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = configs.CONFIGS["C2"]
        bh, dk, cfg = c.scene()
        cam = configs.camera("B")
        off = sample_offset(rank)
        if off is not None:
            cam.use_offset, cam.offset_x, cam.offset_y = 1, off[0], off[1]
        pipe = FramePipeline(W * H, "cpu", world, rank, "samples", H, W)
        part = orc.oracle().render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, threads=1)
        for i in range(frames):
            fb = pipe.next_buffer()
            for f in fb.fields:  # frame i = the rendered frame with steps + i (distinct frames)
                v = torch.from_numpy(part[f])
                fb.views[f].copy_(v + i if f == "steps" else v)
            pipe.submit()
        fr = pipe.finish()
        if rank == 0:
            np.savez(out_path, **{"img_" + f: v.numpy() for f, v in fr.image.items()},
                     **{"loc_" + f: v.numpy() for f, v in fr.local.items()})
        else:
            assert fr is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,frames,H", [(2, 3, 24), (3, 1, 24), (4, 3, 16)])
def test_pipelined_sample_reduce(tmp_path, oracle, world, frames, H):
    W = 16
    out = str(tmp_path / "frame.npz")
    mp.spawn(_samples_worker, args=(world, _free_port(), W, H, frames, out), nprocs=world,
             join=True)
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    planes = []
    for k in range(world):
        cam_k = configs.camera("B")
        off = sample_offset(k)
        if off is not None:
            cam_k.use_offset, cam_k.offset_x, cam_k.offset_y = 1, off[0], off[1]
        planes.append(oracle.render_frame(bh, dk, cfg, cam_k, W, H, c.method, c.flags))
    with np.load(out) as got:
        for f in abi.SOA_FIELDS:  # rank 0 keeps its own plane (sample 0) ...
            w = planes[0][f] + (frames - 1) if f == "steps" else planes[0][f]
            assert np.array_equal(got["loc_" + f].reshape(-1), w, equal_nan=True), f
        # ... and receives the colour averaged over every rank's plane (one reduce)
        for f in RGB_FIELDS:
            mean = np.mean([p[f] for p in planes], axis=0)
            np.testing.assert_allclose(got["img_" + f].reshape(-1), mean, rtol=1e-12)
        # the offsets really moved the rays
        assert not np.array_equal(planes[0]["hit_x"], planes[1]["hit_x"], equal_nan=True)


def test_single_rank_single_shard_is_the_buffer():
    W, H = 4, 6
    pipe = FramePipeline(W * H, "cpu", 1, 0, "shards", H, W, gather=None)
    fb = pipe.next_buffer()
    for f in fb.fields:
        fb.views[f].copy_(torch.arange(24, dtype=fb.views[f].dtype))
    pipe.submit()
    fr = pipe.finish()
    assert all(fr.image[f].shape == (6, 4) for f in fr.image)
    assert int(fr.image["steps"][5, 3]) == 23
    assert fr.image["steps"].data_ptr() == fb.views["steps"].data_ptr()  # no copy


def test_single_rank_one_shard_of_several():
    """N = 1 of a node frame (C5's bench point): shard k's rows land in their image rows."""
    W, H, B, S = 3, 24, 2, 4
    for k in (0, 2):
        n = padded_shard_rows(H, B, S) * W
        pipe = FramePipeline(n, "cpu", 1, 0, "shards", H, W, B, shards=S, first_shard=k)
        fb = pipe.next_buffer()
        for f in RGB_FIELDS:
            fb.views[f].copy_(torch.arange(n, dtype=torch.float64) + 1)
        pipe.submit()
        fr = pipe.finish()
        idx = shard_rows_index(H, B, k, S)
        assert np.array_equal(fr.local_rows, idx)
        img = fr.image["rgb_g"].numpy()
        assert np.array_equal(img[idx], np.arange(1, n + 1).reshape(-1, W)[:len(idx)])
        assert not np.delete(img, idx, axis=0).any()


def test_frame_plans_of_the_configs():
    """C5 = the 7680x4320 frame in 8 equal shards at every N; C1-C3 keep ~one configuration
    frame of rays per GPU at the configuration's aspect; C4 splits its one image."""
    c5 = configs.CONFIGS["C5"]
    for n in (1, 2, 4, 8):
        p = c5.frame(n)
        assert (p.width, p.height, p.shards) == (7680, 4320, 8)
    with pytest.raises(ValueError):
        c5.frame(16)
    for name in ("C1", "C2", "C3"):
        c = configs.CONFIGS[name]
        assert (c.frame(1).width, c.frame(1).height, c.frame(1).shards) == (c.width, c.height, 1)
        for n in (2, 3, 4, 8):
            p = c.frame(n)
            assert p.shards == n and p.height % (p.row_block * n) == 0
            assert abs(p.width * p.height / n / (c.width * c.height) - 1) < 0.02
            assert abs(p.width / p.height - c.width / c.height) < 2e-3
    c2 = configs.CONFIGS["C2"]
    assert (c2.frame(4).width, c2.frame(4).height) == (3840, 2160)
    c4 = configs.CONFIGS["C4"]
    for n in (1, 2, 4, 8):
        assert (c4.frame(n).width, c4.frame(n).height, c4.frame(n).shards) == (3840, 2160, n)


def test_shard_index_matches_library_rule():
    """Python and C (bhrt_shard_rows) agree on which rows a shard owns."""
    from bhrt import lib
    for H in (16, 1080, 2160, 4320):
        for world in (1, 2, 4, 8):
            for B in (1, 6, 8):
                rows_all = []
                for s in range(world):
                    n = lib.shard_rows(H, abi.Rows(B, s, world))
                    assert n == shard_row_count(H, B, s, world)
                    rows_all.extend(shard_rows_index(H, B, s, world).tolist())
                assert sorted(rows_all) == list(range(H))


def test_framebuffer_alignment_and_colour_tail():
    for n in (1, 3, 7, 1000):
        fb = FrameBuffer(n, "cpu")
        for f, (a, b) in fb.offsets.items():
            assert a % (4 if f in ("result", "steps") else 8) == 0
            assert b - a == n * (4 if f in ("result", "steps") else 8)
        a, b = fb.span(RGB_FIELDS)  # the gathered colour planes: one contiguous byte range
        assert b == fb.nbytes and b - a == 24 * n
    with pytest.raises(ValueError):
        FrameBuffer(4, "cpu").span(("result", "rgb_r"))
    fb = FrameBuffer(5, "cpu", abi.SOA_FIELDS + DISPLAY_FIELD)
    assert fb.views["rgba8"].shape == (5, 4) and fb.views["rgba8"].dtype == torch.uint8
    assert fb.offsets["rgba8"][1] <= min(fb.offsets[f][0] for f in RGB_FIELDS)
    assert all(fb.offsets[f][0] % 8 == 0 for f in RGB_FIELDS)
