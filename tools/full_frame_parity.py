#!/usr/bin/env python3
"""Every ray of the BASELINE frames: the HIP path against the oracle, with the knife-edge list.

  python tools/full_frame_parity.py [--configs C1 C2 C3 C4 C5] [--threads 16]
                                    [--out profiles/r03_full_frame_parity.json]

For each configuration the frame BASELINE.json quotes (C1 256x256, C2/C3 1920x1080, C4
3840x2160, C5 the 7680x4320 frame as its 8 shards of 540 rows) is rendered by libbhrt on
cuda:0 (bhrt_render_frame_device, camera B) and by the oracle (oracle.c, OpenMP on --threads
host cores) with each ray's knife-edge margin (the oracle's smallest relative distance from a
threshold of a discontinuous decision). Every ray is compared (conftest.
full_frame_report: class and steps exact, floats within 1e-5 relative, NaN pattern; sky only
for RKF45, where the reference computes it deterministically). A mismatch is "explained" only
if its ray's margin is below 1e-9. Writes one JSON record per configuration / shard.

Test infrastructure: the oracle is the checker here, never the thing measured.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bhrt import abi, configs, lib  # noqa: E402
from conftest import full_frame_report  # noqa: E402
import oracle as orc  # noqa: E402


def gpu_frame(c, bh, dk, cfg, cam, W, H, rows):
    n = W * (H if rows is None else lib.shard_rows(H, rows))
    t = {f: torch.zeros(n, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                        device="cuda") for f in abi.SOA_FIELDS}
    torch.cuda.synchronize()  # (torch fills on its stream, libbhrt renders on its own)
    lib.render_frame_device(bh, dk, cfg, cam, W, H, rows, c.method, c.flags,
                            lib.soa_from_tensors(t), 0)
    torch.cuda.synchronize()
    return {f: v.cpu().numpy() for f, v in t.items()}


def jobs(names):
    for name in names:
        c = configs.CONFIGS[name]
        if name == "C5":  # the node frame's 8 shards (what 8 GPUs render)
            plan = c.frame(8)
            for s in range(plan.shards):
                yield name, c, plan.width, plan.height, plan.rows(s), f"shard {s}/{plan.shards}"
        else:
            yield name, c, c.width, c.height, None, "whole frame"


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--configs", nargs="+", default=["C1", "C2", "C3", "C4", "C5"])
    p.add_argument("--threads", type=int, default=16)
    p.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "full_frame_parity.json"))
    a = p.parse_args()
    torch.cuda.set_device(0)
    lib.load()
    o = orc.oracle()
    cam = configs.camera("B")
    records = []
    for name, c, W, H, rows, what in jobs(a.configs):
        bh, dk, cfg = c.scene()
        t0 = time.perf_counter()
        got = gpu_frame(c, bh, dk, cfg, cam, W, H, rows)
        t1 = time.perf_counter()
        want, margin = o.render_frame_margin(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                             rows=rows, threads=a.threads)
        t2 = time.perf_counter()
        rep = full_frame_report(got, want, margin, c.method == abi.INTEGRATOR_RKF45)
        rep.update(config=name, frame=f"{W}x{H} {what}", camera="B", gpu_s=round(t1 - t0, 3),
                   oracle_s=round(t2 - t1, 1), oracle_threads=a.threads,
                   classes=np.bincount(want["result"], minlength=5).tolist())
        records.append(rep)
        print(json.dumps({k: rep[k] for k in ("config", "frame", "rays", "mismatched_rays",
                                              "knife_edge_rays", "unexplained", "min_margin",
                                              "oracle_s")}), flush=True)
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(records, f, indent=1)
    total = sum(r["rays"] for r in records)
    bad = sum(r["unexplained"] for r in records)
    print(json.dumps({"rays_compared": total, "mismatched": sum(r["mismatched_rays"] for r in records),
                      "knife_edge": sum(r["knife_edge_rays"] for r in records),
                      "unexplained": bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
