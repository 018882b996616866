#!/usr/bin/env python3
"""Does the GPU's recent load set trace_rays_batch's rate? (round 5: the frame time falls under
sustained load and rises after a few ms idle; the batch API is
synchronous, so its chunks see an idle GPU between calls.)

  python tools/batch_idle_probe.py

The C2 camera's 2 M rays through trace_rays_batch (Ray[] in, RayTraceHit[] out), three calls
each: at process start, right after 300 ms of back-to-back device frames, and after 50 ms /
1 s idle. Per call: wall ms and the trace kernels' HIP-event ms (bhrt_get_stats)."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
import torch  # noqa: E402
from bhrt import abi, configs, lib  # noqa: E402

c = configs.CONFIGS["C2"]
bh, dk, cfg = c.scene()
cam = configs.camera("B")
W, H = 1920, 1080
rays = configs.camera_rays(cam, W, H)
hits = np.zeros(W * H, dtype=abi.HIT_DTYPE)
L = lib.load()
args = (rays.ctypes.data, W * H, C.byref(bh), C.byref(dk), C.byref(cfg), hits.ctypes.data, 0)


def calls(what, k=3):
    out = []
    for _ in range(k):
        lib.stats(reset=True)
        t = time.perf_counter()
        assert L.trace_rays_batch(*args) == 0, lib.last_error()
        wall = (time.perf_counter() - t) * 1e3
        st = lib.stats(reset=True)
        out.append(f"{wall:7.2f} ms wall / {st['kernel_ms']:6.2f} ms kernels "
                   f"({W * H / wall / 1e3:6.1f} Mrays/s)")
    print(f"{what:34s} " + " | ".join(out), flush=True)


def sustained(ms, stream=None, count=None):
    n = W * H
    t = {f: torch.empty(n, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                        device="cuda") for f in abi.SOA_FIELDS}
    soa = lib.soa_from_tensors(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    done = 0
    while (time.perf_counter() - t0) * 1e3 < ms and (count is None or done < count):
        for _ in range(4 if count is None else 1):
            lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags, soa, stream)
            done += 1
        torch.cuda.synchronize()
    lib.stats_discard()


def cpu_spin(ms):
    t0 = time.perf_counter()
    x = 0
    while (time.perf_counter() - t0) * 1e3 < ms:
        x += 1


calls("process start")
calls("again")
mode = os.environ.get("PROBE", "frames")
if mode == "spin":  # 300 ms of host busy-spin, no GPU work
    cpu_spin(300)
    calls("after 300 ms host spin")
if mode in ("spin", "torch"):  # torch's HIP context, one tiny op
    torch.zeros(16, device="cuda").add_(1)
    torch.cuda.synchronize()
    calls("after torch's first device op")
if mode == "tiny":  # one 8x8 device frame of the same scene
    tt = {f: torch.empty(64, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                         device="cuda") for f in abi.SOA_FIELDS}
    torch.cuda.synchronize()
    lib.render_frame_device(bh, dk, cfg, cam, 8, 8, None, c.method, c.flags,
                            lib.soa_from_tensors(tt), None)
    torch.cuda.synchronize()
    calls("after one 8x8 device frame")
if mode == "tinyhost":  # one 8x8 host-buffer frame
    arrays, soa8 = abi.alloc_soa(64, abi.SOA_FIELDS)
    assert L.bhrt_render_frame(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), 8, 8,
                               c.method, c.flags, C.byref(soa8)) == 0
    calls("after one 8x8 host frame")
if mode == "tinybatch":  # a 64-ray batch first
    assert L.trace_rays_batch(rays.ctypes.data, 64, C.byref(bh), C.byref(dk), C.byref(cfg),
                              hits.ctypes.data, 0) == 0
    calls("after a 64-ray batch")
if mode == "one":  # a single device frame on libbhrt's stream
    sustained(1e9, count=1)
    calls("after one device frame")
if mode == "torchstream":  # device frames on a torch stream instead of libbhrt's
    s = torch.cuda.Stream()
    sustained(300, stream=s.cuda_stream)
    calls("after 300 ms of frames on a torch stream")
sustained(300)
calls("after 300 ms of device frames")
time.sleep(0.05)
calls("after 50 ms idle")
time.sleep(1.0)
calls("after 1 s idle")
sustained(300)
calls("after 300 ms of device frames")
