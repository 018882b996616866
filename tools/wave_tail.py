"""Tail of the persistent trace kernel (diagnostic build): per-wave start / queue-exhausted / end
times of one frame's hot k_trace launch.

  make -C raytracing-engine-in-c_amd/csrc stats
  BHRT_LIB=raytracing-engine-in-c_amd/ab/libbhrt_stats.so python tools/wave_tail.py [--config C2]

Prints the launch span, when the ray queue ran dry, how long the waves kept running after that
(percentiles of their exit times) and the fraction of wave-slot time left idle by early exits.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

from bhrt import configs, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--camera", default="B")
    ap.add_argument("--frames", type=int, default=2)
    a = ap.parse_args()
    import torch  # before libbhrt, so both use the one HIP runtime torch loads
    torch.cuda.set_device(0)
    L = lib.load()
    fn = L.bhrt_debug_wave_times
    fn.restype = C.c_int
    fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]
    buf = (C.c_ulonglong * (3 * 16384))()
    ds = L.bhrt_debug_stats
    ds.restype = C.c_int
    ds.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dsb = (C.c_ulonglong * 64)()
    tbf = L.bhrt_debug_time_bins
    tbf.restype = C.c_int
    tbf.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    tbb = (C.c_ulonglong * 256)()
    c = configs.CONFIGS[a.config]
    bh, dk, cfg = c.scene()
    cam = configs.camera(a.camera)
    from bhrt.dist_frame import FrameBuffer
    fb = FrameBuffer(c.width * c.height, torch.device("cuda", 0))
    stream = torch.cuda.current_stream()
    for f in range(a.frames + 1):
        fn(buf, 16384, 1)
        ds(dsb, 1)
        tbf(tbb, 1)
        # the device-resident path: one k_trace launch per frame (the host path chunks it)
        lib.render_frame_device(bh, dk, cfg, cam, c.width, c.height, None, c.method, c.flags,
                                fb.soa(), stream.cuda_stream)
        torch.cuda.synchronize()
        n = fn(buf, 16384, 1)
        ds(dsb, 1)
        v = list(dsb)
        tbf(tbb, 1)
        tb = np.array(list(tbb), dtype=np.float64).reshape(128, 2)
        if f == 0:
            continue  # warm-up
        t = np.frombuffer(buf, dtype=np.uint64, count=3 * n).reshape(n, 3).astype(np.float64)
        t = (t - t[:, 0].min()) / 100.0  # 100 MHz -> microseconds from the first wave start
        start, exh, end = t[:, 0], t[:, 1], t[:, 2]
        span = end.max()
        dry = exh[exh > 0].min() if (exh > 0).any() else float("nan")
        after = end - dry
        busy = (end - start).sum() / (n * span)
        print(f"{a.config} frame {f}: {n} waves, span {span:.0f} us, queue dry at {dry:.0f} us "
              f"({dry / span:.1%}); wave exits after dry: p10 {np.percentile(after, 10):.0f} "
              f"p50 {np.percentile(after, 50):.0f} p90 {np.percentile(after, 90):.0f} "
              f"max {after.max():.0f} us; wave-slot occupancy {busy:.1%}; "
              f"start spread {start.max():.0f} us")
        print(f"   lane occupancy: all passes {v[61] / max(v[60], 1):.2f}/64 over {v[60]}; "
              f"before dry {(v[61] - v[63]) / max(v[60] - v[62], 1):.2f}/64 over {v[60] - v[62]}; "
              f"after dry {v[63] / max(v[62], 1):.2f}/64 over {v[62]} passes "
              f"(lane-iterations after dry: {v[63] / max(v[61], 1):.1%})")
        # throughput per 250 us bin; "ideal" = all lane-iterations at the median full-bin rate
        last = int(np.nonzero(tb[:, 1])[0].max()) + 1
        rate = tb[:last, 0]
        steady = np.median(rate[1:max(2, last - 20)])
        ideal_us = tb[:, 0].sum() / steady * 250.0
        print("   lane-iterations per 250 us bin (x1e6): " +
              " ".join(f"{x / 1e6:.1f}" for x in rate))
        print(f"   steady {steady / 1e6:.2f}e6 per bin -> ideal {ideal_us:.0f} us vs span "
              f"{span:.0f} us: tail loss {1 - ideal_us / span:.1%}; live lanes per pass in the "
              f"last bins: " + " ".join(f"{tb[i, 0] / max(tb[i, 1], 1):.0f}"
                                         for i in range(max(0, last - 16), last)))


if __name__ == "__main__":
    main()
