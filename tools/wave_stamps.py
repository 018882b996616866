#!/usr/bin/env python3
"""Per-wave timeline of the hot trace kernel under bench.py's frame loop (diagnostic build).

  make -C raytracing-engine-in-c_amd/csrc diag     # -> diag/libbhrt_stamps.so
  BHRT_LIB=raytracing-engine-in-c_amd/diag/libbhrt_stamps.so \
      python tools/wave_stamps.py --config C4 --plan-gpus 8 --shard 0 --streams 4 --frames 20 \
      --out gpurun_out/stamps_C4_p8.npz
  python tools/wave_stamps.py --analyse gpurun_out/stamps_C4_p8.npz

The GPU run renders --frames frames the way bench.py does (frames alternate over --streams
streams, every stream warmed first, rank 0's assembly of its shard included) and saves every
wave's record: start and end on the constant 100 MHz clock, CU id, trips of the persistent loop,
refills, lane-iterations, rays -- one row per wave per launch. The analysis prints, for the
timed frames: the window (first wave start to last wave end) per frame, resident waves over
time, how long the chip holds fewer than its full complement of waves, each launch's own
start-to-end, its waves' end-time spread (the tail), and lane utilisation (lane-iterations /
(trips x iterations per trip x 64)).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

SLOTS, WAVES, WORDS = 64, 8192, 8
# bench.py's hardware-queue setting (read when HIP initialises)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 8:
    os.environ["GPU_MAX_HW_QUEUES"] = "8"


def run(a):
    import ctypes as C
    import torch
    from bhrt import abi, configs, lib
    from bhrt.dist_frame import DISPLAY_FIELD, FramePipeline, padded_shard_rows
    L = lib.load()
    L.bhrt_diag_stamps.restype = C.c_long
    L.bhrt_diag_stamps.argtypes = [C.c_void_p, C.c_int]
    c = configs.CONFIGS[a.config]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    plan = c.frame(a.plan_gpus)
    W, H, S, B = plan.width, plan.height, plan.shards, plan.row_block
    rows = plan.rows(a.shard)
    n = padded_shard_rows(H, B, S) * W
    device = torch.device("cuda", 0)
    fields = abi.SOA_FIELDS + DISPLAY_FIELD
    pipe = FramePipeline(n, device, 1, 0, "shards", H, W, B, fields, shards=S,
                         gather=DISPLAY_FIELD, first_shard=a.shard, slots=a.streams)
    streams = [torch.cuda.Stream(device) for _ in range(a.streams)]
    k = [0]

    def step():
        s = streams[k[0] % a.streams]
        k[0] += 1
        with torch.cuda.stream(s):
            fb = pipe.next_buffer()
            lib.render_frame_device(bh, dk, cfg, cam, W, H, rows, c.method, c.flags, fb.soa(),
                                    s.cuda_stream)
            pipe.submit()

    for _ in range(max(a.warmup, a.streams)):
        step()
    pipe.finish()
    torch.cuda.synchronize()
    lib.stats(reset=True)
    if L.bhrt_diag_stamps(None, 1) < 0:
        raise SystemExit("stamp reset failed")
    t0 = time.perf_counter()
    for _ in range(a.frames):
        step()
    pipe.finish()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.frames
    st = lib.stats(reset=True)
    buf = np.zeros(SLOTS * WAVES * WORDS, dtype=np.uint64)
    if L.bhrt_diag_stamps(buf.ctypes.data, 0) < 0:
        raise SystemExit("stamp copy failed")
    buf = buf.reshape(SLOTS, WAVES, WORDS)
    used = [s for s in range(SLOTS) if buf[s, :, 1].any()]
    rec = {f"slot{s}": buf[s][buf[s, :, 1] != 0] for s in used}
    np.savez_compressed(a.out, ms_per_frame=dt * 1e3, frames=a.frames, rays=st["rays"],
                        iterations=st["iterations"], unroll=6 if c.method == abi.INTEGRATOR_RK4
                        else 2, config=a.config, plan=a.plan_gpus, shard=a.shard,
                        streams=a.streams, **rec)
    print(f"{a.config} plan {a.plan_gpus} shard {a.shard}: {dt * 1e3:.4f} ms/frame, "
          f"{len(used)} launches stamped -> {a.out}", flush=True)


def analyse(path):
    z = np.load(path)
    unroll = int(z["unroll"])
    launches = sorted((k for k in z.files if k.startswith("slot")), key=lambda k: int(k[4:]))
    recs = [z[k].astype(np.int64) for k in launches]
    # launch order = order of first wave start
    recs.sort(key=lambda r: r[:, 0].min())
    t_base = min(r[:, 0].min() for r in recs)
    tick_us = 0.01  # 100 MHz
    nfr = len(recs)
    lo = min(r[:, 0].min() for r in recs)
    hi = max(r[:, 1].max() for r in recs)
    print(f"{path}: {z['config']} plan {int(z['plan'])} shard {int(z['shard'])}, "
          f"{int(z['streams'])} streams, host {float(z['ms_per_frame']):.4f} ms/frame, "
          f"{nfr} launches stamped")
    print(f"  window first start..last end {(hi - lo) * tick_us:.1f} us = "
          f"{(hi - lo) * tick_us / nfr:.2f} us per launch")
    # resident waves over time (all launches), 0.5 us bins
    nb = int((hi - lo) // 50) + 1
    occ = np.zeros(nb + 1)
    for r in recs:
        s = (r[:, 0] - lo) / 50.0
        e = (r[:, 1] - lo) / 50.0
        np.add.at(occ, np.floor(s).astype(int), 1)
        np.add.at(occ, np.floor(e).astype(int), -1)
    occ = np.cumsum(occ)[:nb]
    full = np.percentile(occ, 99)
    print(f"  resident waves: max {occ.max():.0f}, p99 {full:.0f}, mean {occ.mean():.0f} "
          f"({occ.mean() / max(full, 1):.3f} of p99)")
    for frac in (0.99, 0.9, 0.75, 0.5):
        print(f"    time with < {frac:.2f} x p99 resident: {(occ < frac * full).mean() * 100:.1f}%")
    tot_li = sum(int(r[:, 4].sum()) for r in recs)
    tot_slots = sum(int((r[:, 3] & 0xffffffff).sum()) for r in recs) * unroll * 64
    print(f"  lane utilisation: lane-iterations / (trips x {unroll} x 64) = "
          f"{tot_li / max(tot_slots, 1):.3f} (upper bound: a trip's later iterations run "
          f"only while some lane goes on)")
    print(f"  refills per wave (mean) {np.mean(np.concatenate([r[:, 3] >> 32 for r in recs])):.2f}, "
          f"trips per wave {np.mean(np.concatenate([r[:, 3] & 0xffffffff for r in recs])):.1f}")
    print("  per launch: start (us from first), duration, wave-start spread (p50/p100), "
          "wave-end spread before last end (p50/p90/p100), waves")
    for i, r in enumerate(recs):
        s0, e1 = r[:, 0].min(), r[:, 1].max()
        ws = (r[:, 0] - s0) * tick_us
        we = (e1 - r[:, 1]) * tick_us
        if i < 6 or i >= nfr - 2:
            print(f"    {i:2d}: {(s0 - t_base) * tick_us:8.1f} {(e1 - s0) * tick_us:7.1f}  "
                  f"start {np.median(ws):6.1f}/{ws.max():6.1f}  end-before-last "
                  f"{np.median(we):6.1f}/{np.percentile(we, 10):6.1f}/{we.max():6.1f}  "
                  f"{len(r)}")
    # the wave with the latest end per launch: how much of it was tail
    durs = np.array([(r[:, 1].max() - r[:, 0].min()) * tick_us for r in recs])
    print(f"  launch duration mean {durs.mean():.1f} us; window / launches "
          f"{(hi - lo) * tick_us / nfr:.1f} us")
    # idle lanes cost: waves alive but whose rays... per-wave duration vs lane-iterations
    dur = np.concatenate([(r[:, 1] - r[:, 0]) for r in recs]) * tick_us
    li = np.concatenate([r[:, 4] for r in recs])
    trips = np.concatenate([r[:, 3] & 0xffffffff for r in recs])
    dur = np.concatenate([(r[:, 1] - r[:, 0]) for r in recs]) * tick_us
    if recs[0].shape[1] >= 8:
        ct = np.concatenate([r[:, 6] & ((1 << 48) - 1) for r in recs]) * tick_us
        cn = np.concatenate([r[:, 6] >> 48 for r in recs])
        first = np.concatenate([r[:, 7] for r in recs]) * tick_us
        print(f"  claims (returning atomics) per wave {cn.mean():.2f}; time in them per wave mean "
              f"{ct.mean():.1f} us ({ct.sum() / max(dur.sum(), 1e-9) * 100:.1f}% of wave time); "
              f"first claim p50 {np.median(first):.2f} / p90 {np.percentile(first, 90):.2f} / max "
              f"{first.max():.2f} us; later claims mean "
              f"{(ct - first).sum() / max((cn - 1).clip(0).sum(), 1):.2f} us")
    print(f"  per wave: duration mean {dur.mean():.1f} us (p10 {np.percentile(dur, 10):.1f}, "
          f"p90 {np.percentile(dur, 90):.1f}), lane-iterations mean {li.mean():.0f}, "
          f"trips mean {trips.mean():.1f}; us per trip {dur.sum() / trips.sum():.3f}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyse", default=None)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--plan-gpus", type=int, default=1)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "stamps.npz"))
    a = ap.parse_args()
    if a.analyse:
        analyse(a.analyse)
    else:
        if a.frames > SLOTS - 8:
            raise SystemExit("at most 56 frames (the control-block ring)")
        run(a)


if __name__ == "__main__":
    main()
