"""Shift-argument and lane-occupancy statistics of the trace kernel (diagnostic build).

  make -C raytracing-engine-in-c_amd/csrc stats
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_stats.so python tools/delta_stats.py [--config C2]

For each sincos_shift site (RK stages 2..4 of theta = state[1], then the per-iteration
advances of state[1..3]) prints the fraction of lane evaluations and of wave evaluations whose
|delta| exceeds 0.05 / 0.1 / 0.2 / pi/4, and the mean number of live lanes per wave pass of
the persistent loop. Used to size the shift polynomials.
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

from bhrt import configs, lib  # noqa: E402

SITES = ["stage2 y1", "stage3 y1", "stage4 y1", "advance y1", "advance y2", "advance y3"]
THR = ["0.05", "0.1", "0.2", "pi/4"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--camera", default="B")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    a = ap.parse_args()
    L = lib.load()
    fn = L.bhrt_debug_stats
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * 64)()
    fn(buf, 1)
    c = configs.CONFIGS[a.config]
    bh, dk, cfg = c.scene()
    W = a.width or c.width
    H = a.height or c.height
    lib.render_frame(bh, dk, cfg, configs.camera(a.camera), W, H, c.method, c.flags,
                     fields=("result", "steps"))
    rc = fn(buf, 1)
    assert rc == 0, rc
    v = list(buf)
    print(f"{a.config} {W}x{H}: lane occupancy {v[61] / max(v[60], 1):.2f} of 64 "
          f"over {v[60]} wave passes")
    print(f"{'site':12s} {'lanes':>12s} " + " ".join(f"L>{t:>5s}" for t in THR) + "  " +
          " ".join(f"W>{t:>5s}" for t in THR))
    for s, name in enumerate(SITES):
        b = v[s * 10:(s + 1) * 10]
        lanes, waves = max(b[0], 1), max(b[1], 1)
        print(f"{name:12s} {b[0]:12d} " + " ".join(f"{b[2 + j] / lanes:7.4f}" for j in range(4))
              + "  " + " ".join(f"{b[6 + j] / waves:7.4f}" for j in range(4)))


if __name__ == "__main__":
    main()
