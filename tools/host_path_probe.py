"""Host-buffer API timing breakdown for one C2 frame: device-resident kernel time, then
bhrt_render_frame into (a) fresh numpy arrays per frame, (b) the same arrays reused."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
from bhrt import abi, configs, lib  # noqa: E402

c = configs.CONFIGS["C2"]
bh, dk, cfg = c.scene()
cam = configs.camera("B")
W, H = 1920, 1080
L = lib.load()
lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)  # warm-up
lib.stats(reset=True)
t = time.perf_counter()
for _ in range(3):
    lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
fresh = (time.perf_counter() - t) / 3
st = lib.stats(reset=True)
arrays, soa = abi.alloc_soa(W * H)
for a in arrays.values():
    a[...] = 1  # touch every page once, as a render loop's buffers are
t = time.perf_counter()
for _ in range(3):
    assert L.bhrt_render_frame(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), W, H,
                               c.method, c.flags, C.byref(soa)) == 0
reused = (time.perf_counter() - t) / 3
print(f"kernel {st['kernel_ms'] / st['launches']:.2f} ms | host API, fresh arrays "
      f"{fresh * 1e3:.2f} ms | reused arrays {reused * 1e3:.2f} ms")
