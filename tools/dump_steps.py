#!/usr/bin/env python3
"""Per-ray step counts of the BASELINE frames, for the wave-scheduler replay (tools/tail_sim.py).

  python tools/dump_steps.py [--configs C2 C4 C5] [--out gpurun_out/steps.npz]

Renders every configuration's whole camera-B image with bhrt_render_frame (the GPU path) and
stores the `steps` and `result` planes (uint16 / uint8, row-major, row 0 = top). C5 is the
7680x4320 node frame (its shards are rows of it). The shard of an N-GPU plan is recovered from
the rows: row r belongs to shard (r // B) % S (configs.Config.frame).
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

from bhrt import configs, lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", nargs="+", default=["C2", "C4", "C5"])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "steps.npz"))
    a = ap.parse_args()
    out = {}
    for name in a.configs:
        c = configs.CONFIGS[name]
        bh, dk, cfg = c.scene()
        cam = configs.camera("B")
        arr = lib.render_frame(bh, dk, cfg, cam, c.width, c.height, c.method, c.flags,
                               fields=("result", "steps"))
        st = arr["steps"].reshape(c.height, c.width)
        out[f"{name}_steps"] = st.astype(np.uint16)
        out[f"{name}_result"] = arr["result"].reshape(c.height, c.width).astype(np.uint8)
        print(name, c.width, "x", c.height, "mean steps", float(st.mean()), "max", int(st.max()),
              flush=True)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    np.savez_compressed(a.out, **out)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
