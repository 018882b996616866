"""The RCCL branch of the N-GPU frame path, run once on one GPU.

bench.py at N > 1 renders shard r on rank r and gathers the rgba8 display range of every rank's
frame buffer to rank 0 with ONE torch.distributed.gather per frame (bhrt/dist_frame.py
FramePipeline.submit), overlapped with the next frames. The driver's 8-GPU run is the first
place that branch would otherwise execute on hardware; here an `nccl` (= RCCL) process group of
world size 1 drives the same code (force_collective) for a shard of C4's 8-GPU plan: the
assembled image rows must equal a one-launch frame's bit for bit, and Work.get_duration()
(TORCH_NCCL_ENABLE_TIMING) must give each gather's GPU time. The reference loop this path
parallelises: raytracer.c:795-804 / blackhole_api.c:236-247.
"""
import socket

import numpy as np
import pytest

from bhrt import abi, configs

pytestmark = pytest.mark.gpu


def test_rccl_gather_of_a_c4_shard_at_world_one(bhrt_lib, monkeypatch):
    import torch
    import torch.distributed as dist
    from bhrt.dist_frame import (DISPLAY_FIELD, FramePipeline, padded_shard_rows,
                                 shard_rows_index)
    monkeypatch.setenv("TORCH_NCCL_ENABLE_TIMING", "1")  # (read when the group is created)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", world_size=1,
                            rank=0, device_id=dev)
    try:
        assert dist.get_backend() == "nccl"
        c = configs.CONFIGS["C4"]
        bh, dk, cfg = c.scene()
        cam = configs.camera("B")
        plan = c.frame(8)
        W, H, S, B = plan.width, plan.height, plan.shards, plan.row_block
        shard = 5
        n = padded_shard_rows(H, B, S) * W
        pipe = FramePipeline(n, dev, 1, 0, "shards", H, W, B, abi.SOA_FIELDS + DISPLAY_FIELD,
                             shards=S, gather=DISPLAY_FIELD, first_shard=shard, slots=2,
                             force_collective=True)
        streams = [torch.cuda.Stream(dev) for _ in range(2)]
        frames = 6  # three per slot: buffers reused behind their gathers
        for k in range(frames):
            s = streams[k % 2]
            with torch.cuda.stream(s):
                fb = pipe.next_buffer()
                bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, plan.rows(shard), c.method,
                                             c.flags, fb.soa(), s.cuda_stream)
                pipe.submit()
        frame = pipe.finish()
        torch.cuda.synchronize()
        pipe.collect_timing()
        assert len(pipe.collective_ms) == frames, pipe.timing_error
        assert all(np.isfinite(v) and v > 0 for v in pipe.collective_ms), pipe.collective_ms
        # the one-launch frame's display buffer (C4 writes rgba8 from the trace kernel)
        full = torch.zeros((W * H, 4), dtype=torch.uint8, device=dev)
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     abi.FrameSoA(rgba8=full.data_ptr()), None)
        want = full.view(H, W, 4).cpu().numpy()
        img = frame.image["rgba8"].cpu().numpy()
        rows = shard_rows_index(H, B, shard, S)
        assert img.shape == (H, W, 4)
        assert np.array_equal(img[rows], want[rows])
        others = np.setdiff1d(np.arange(H), rows)
        assert not img[others].any()  # (rows of shards this one rank did not render)
        bhrt_lib.stats(reset=True)
    finally:
        dist.destroy_process_group()
