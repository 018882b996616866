#!/usr/bin/env python3
"""Why does trace_rays_batch run ~30% slower in a fresh process until one device camera frame
has run (profiles/r05/batch_mode_probe.txt)?

  python tools/batch_fresh_probe.py [mode ...]      (parent: never touches the GPU)

Each mode runs in a fresh child process: trace_rays_batch of the C2 camera's 2 M rays, a few
calls, then the mode's action, then more calls; per call the wall ms. Modes:
  base         calls only
  frame        an 8x8 device camera frame (torch outputs, NULL stream) between the calls
  frame_hits   the same frame writing only result/steps/hit fields (no colour pass)
  rays_dev     64 rays through bhrt_trace_rays_device (NULL stream) instead of a frame
  batch_small  a 64-ray trace_rays_batch instead
  warm1        one drop-in trace_ray BEFORE the first batch call (what the first call's cost is)
  env:K=V,...  base with extra environment (e.g. env:BHRT_STREAM_QUEUE=0)
  MODE@K=V,... a mode with extra environment (e.g. batch_small@BHRT_BATCH_LATE_D2H=0)
"""
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(mode):
    import ctypes as C
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
    import torch
    from bhrt import abi, configs, lib
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 1920, 1080
    rays = configs.camera_rays(cam, W, H)
    hits = np.zeros(W * H, dtype=abi.HIT_DTYPE)
    L = lib.load()
    args = (rays.ctypes.data, W * H, C.byref(bh), C.byref(dk), C.byref(cfg), hits.ctypes.data, 0)

    def calls(what, k):
        out = []
        for _ in range(k):
            t = time.perf_counter()
            assert L.trace_rays_batch(*args) == 0, lib.last_error()
            out.append((time.perf_counter() - t) * 1e3)
        print(f"  {what:28s} " + " ".join(f"{v:6.2f}" for v in out) +
              f"  ms  (last {W * H / out[-1] / 1e3:6.1f} Mrays/s)", flush=True)

    if mode == "warm1":  # one drop-in trace_ray first: context, code object, streams
        t = time.perf_counter()
        hit = abi.RayTraceHit()
        ray = abi.Ray(cam.position, cam.direction)
        L.trace_ray(C.byref(ray), C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(hit))
        print(f"  one trace_ray first: {(time.perf_counter() - t) * 1e3:.2f} ms", flush=True)
    calls("fresh", 4)
    if mode in ("frame", "frame_hits"):
        fields = abi.SOA_FIELDS if mode == "frame" else ("result", "steps", "hit_x", "hit_y",
                                                         "hit_z", "distance")
        tt = {f: torch.empty(64, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                             device="cuda") for f in fields}
        lib.render_frame_device(bh, dk, cfg, cam, 8, 8, None, c.method, c.flags,
                                lib.soa_from_tensors(tt), None)
        torch.cuda.synchronize()
        calls("after an 8x8 device frame", 4)
    elif mode == "rays_dev":
        tt = {f: torch.empty(64, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                             device="cuda") for f in ("result", "steps", "hit_x", "hit_y", "hit_z")}
        d = torch.from_numpy(rays[:64].view(np.uint8)).cuda()
        assert L.bhrt_trace_rays_device(d.data_ptr(), 64, C.byref(bh), C.byref(dk), C.byref(cfg),
                                        c.method, 0, C.byref(lib.soa_from_tensors(tt)), None) == 0
        torch.cuda.synchronize()
        calls("after 64 device rays", 4)
    elif mode == "batch_small":
        assert L.trace_rays_batch(rays.ctypes.data, 64, C.byref(bh), C.byref(dk), C.byref(cfg),
                                  hits.ctypes.data, 0) == 0
        calls("after a 64-ray batch", 4)
    else:
        calls("again", 4)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    modes = sys.argv[1:] or ["base", "frame", "frame_hits", "rays_dev", "batch_small"]
    rc = 0
    for m in modes:
        env = dict(os.environ)
        name = m
        if "@" in m:  # mode@K=V,...: a mode with extra environment
            m, kvs = m.split("@", 1)
            for kv in kvs.split(","):
                k, v = kv.split("=", 1)
                env[k] = v
        elif m.startswith("env:"):
            for kv in m[4:].split(","):
                k, v = kv.split("=", 1)
                env[k] = v
            m = "base"
        print(f"== {name}", flush=True)
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", m], env=env,
                           timeout=300)
        rc = rc or r.returncode
        if r.returncode:
            print(f"   (child exit {r.returncode})", flush=True)
            break
    sys.exit(rc)


if __name__ == "__main__":
    main()
