#!/usr/bin/env python3
"""Claim-order probe: does a longest-first claim order shorten a frame's drain?

  python tools/order_probe.py [--config C2] [--frames 10]

Renders the configuration's frame (camera B) on cuda:0 through bhrt_render_frame_device, first
in ray id order, then with bhrt_set_claim_order set to the rays sorted by the previous frame's
step count (longest first) and to a two-class order (MAX_STEPS rays first). For each order:
a lone frame (launch + synchronize, ms), frames back to back on one stream and alternating
between two streams (ms per frame), and that every output field is bit-identical to the id
order's. One JSON line per order.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

import torch  # noqa: E402

from bhrt import abi, configs, lib  # noqa: E402
from bhrt.dist_frame import FrameBuffer  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--config", default="C2")
    p.add_argument("--frames", type=int, default=10)
    p.add_argument("--orders", default="id,longest_first,max_steps_first,reverse",
                   help="comma list; also tileWxH (WxH pixel tiles, row-major tiles)")
    a = p.parse_args()
    torch.cuda.set_device(0)
    lib.load()
    c = configs.CONFIGS[a.config]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = c.width, c.height
    rows = None
    n = W * H
    dev = torch.device("cuda", 0)
    fbs = [FrameBuffer(n, dev, abi.SOA_FIELDS), FrameBuffer(n, dev, abi.SOA_FIELDS)]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]

    def render(fb, s):
        with torch.cuda.stream(s):
            lib.render_frame_device(bh, dk, cfg, cam, W, H, rows, c.method, c.flags, fb.soa(),
                                    s.cuda_stream)

    render(fbs[0], streams[0])
    torch.cuda.synchronize()
    ref = {f: t.clone() for f, t in fbs[0].views.items()}
    steps = ref["steps"].to(torch.int64)
    def tiles(tw, th):
        """pixel ids tile by tile (tw x th pixels, tiles row-major, pixels row-major within)"""
        assert W % tw == 0 and H % th == 0, (W, H, tw, th)
        ty, tx, py, px = torch.meshgrid(torch.arange(H // th), torch.arange(W // tw),
                                        torch.arange(th), torch.arange(tw), indexing="ij")
        return ((ty * th + py) * W + tx * tw + px).reshape(-1).to(torch.int32).to(dev)

    orders = {
        "id": None,
        "longest_first": torch.argsort(-steps, stable=True).to(torch.int32),
        "max_steps_first": torch.argsort((ref["result"] != abi.RAY_MAX_STEPS).to(torch.int8),
                                         stable=True).to(torch.int32),
        "reverse": torch.arange(n - 1, -1, -1, device=dev, dtype=torch.int32),
    }
    for name in a.orders.split(","):
        if name.startswith("tile"):
            tw, th = (int(v) for v in name[4:].split("x"))
            order = tiles(tw, th)
        else:
            order = orders[name]
        lib.set_claim_order(order.data_ptr() if order is not None else None,
                            n if order is not None else 0)
        for fb in fbs:
            for t in fb.views.values():
                t.zero_()
        render(fbs[0], streams[0])
        torch.cuda.synchronize()
        same = all(torch.equal(fbs[0].views[f], ref[f]) if not ref[f].is_floating_point() else
                   torch.allclose(fbs[0].views[f], ref[f], rtol=0, atol=0, equal_nan=True)
                   for f in ref)  # (NaN time dilation of rays that end inside rs)
        lone = []
        for _ in range(a.frames):
            t0 = time.perf_counter()
            render(fbs[0], streams[0])
            torch.cuda.synchronize()
            lone.append((time.perf_counter() - t0) * 1e3)
        res = {}
        for ns in (1, 2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(a.frames):
                render(fbs[k % ns], streams[k % ns])
            torch.cuda.synchronize()
            res[f"ms_per_frame_{ns}_streams"] = round((time.perf_counter() - t0) * 1e3 / a.frames, 3)
        lone.sort()
        print(json.dumps({"config": a.config, "order": name, "bit_identical": same,
                          "lone_ms_median": round(lone[len(lone) // 2], 3),
                          "lone_ms_min": round(lone[0], 3), **res,
                          "mrays_s_2_streams": round(n / res["ms_per_frame_2_streams"] / 1e3, 1)}),
              flush=True)
    lib.set_claim_order(None, 0)


if __name__ == "__main__":
    main()
