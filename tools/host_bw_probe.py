"""Where the host-buffer frame time goes (DESIGN.md §4 "Host-buffer frames"): D2H bandwidth
into pinned and pageable memory, host memcpy bandwidth, and bhrt_render_frame per chunk count."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
from bhrt import abi, configs, lib  # noqa: E402

NB = 199065600
dev = torch.empty(NB, dtype=torch.uint8, device="cuda").fill_(1)
pin = torch.empty(NB, dtype=torch.uint8, pin_memory=True)
pag = torch.empty(NB, dtype=torch.uint8)
pag.fill_(0)


def bw(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    return NB / dt / 1e9, dt * 1e3


print("D2H pinned   %.1f GB/s %.2f ms" % bw(lambda: pin.copy_(dev, non_blocking=True)))
print("D2H pageable %.1f GB/s %.2f ms" % bw(lambda: pag.copy_(dev)))
print("H2D pinned   %.1f GB/s %.2f ms" % bw(lambda: dev.copy_(pin, non_blocking=True)))
a = np.ones(NB // 8)
b = np.zeros(NB // 8)
t = time.perf_counter()
for _ in range(3):
    np.copyto(b, a)
dt = (time.perf_counter() - t) / 3
print("host memcpy 1 thread %.1f GB/s %.2f ms" % (NB / dt / 1e9, dt * 1e3))

c = configs.CONFIGS["C2"]
bh, dk, cfg = c.scene()
cam = configs.camera("B")
W, H = 1920, 1080
L = lib.load()
arrays, soa = abi.alloc_soa(W * H)
for x in arrays.values():
    x[...] = 0
for k in (1, 2, 4, 8):
    os.environ["BHRT_HOST_CHUNKS"] = str(k)
    L.bhrt_render_frame(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), W, H, c.method, c.flags, C.byref(soa))
    lib.stats(reset=True)
    t = time.perf_counter()
    for _ in range(3):
        assert L.bhrt_render_frame(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), W, H,
                                   c.method, c.flags, C.byref(soa)) == 0
    dt = (time.perf_counter() - t) / 3
    st = lib.stats(reset=True)
    print(f"render_frame chunks={k}: {dt * 1e3:.2f} ms/frame, {W * H / dt / 1e6:.1f} Mrays/s, "
          f"trace span/launches {st['span_ms'] / max(st['launches'], 1):.3f} ms x {st['launches'] / 3:.0f}")
