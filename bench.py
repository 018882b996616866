"""Benchmark of the geodesic ray-tracing hot path (BASELINE.json metric) on MI355X.

One "step" = one camera frame of the workload traced by libbhrt.so with every input already
on the device: the frame kernel launch, plus (N > 1) the frame's single RCCL collective and
its assembly on rank 0 (bhrt/dist_frame.py FramePipeline; the collective of frame i overlaps
the rendering of frame i+1, and the timed region ends after the last one). Consecutive frames
alternate between two HIP streams (--streams 2, the default), so the workgroups of frame i+1
take the CUs that frame i's tail -- its last, longest rays draining -- leaves idle
(tools/wave_tail.py: ~9% of a lone C2 launch); --streams 1 runs the frames back to back.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2] [--camera B]

N > 1 is launched by torch.distributed.run, one process per GPU.
  * Weak scaling (C1, C2, C3, C5): every GPU traces the whole configuration frame (1920 x 1080
    for C2) at its own sub-pixel offset -- rank 0 the pixel centres, rank k the reference's
    Halton sample k (trace_pixel's jitter) -- so N GPUs supersample the frame with N samples
    per pixel and every GPU does exactly one frame's work; one RCCL reduce sums the colour
    planes on rank 0, which divides by N (trace_pixel's sample average, raytracer.c:1096-1164).
    (A taller image 1080*N rows high is NOT used: with the fixed vertical FOV its horizontal
    FOV shrinks with N and the per-ray work collapses -- 400 -> 1.6 iterations/ray at N=8.)
  * Strong scaling (C4): one 3840 x 2160 image split into cyclic 8-row blocks (block b ->
    rank b % N), un-permuted on rank 0 after the gather.

The JSON line also carries:
  roofline      FP64 VALU roofline of the trace kernel: algorithmic FLOPs (SURVEY.md 8(a):
                117 per RK4 iteration + 35 per a=0 derivative stage + 4 per far-field stage;
                368 per RKF45 attempt + the same stage costs) / the kernel's GPU time per
                launch: with overlapping frames the HIP-event busy span of the timed launches
                (first start to last end) / launches, else the per-launch HIP-event average.
  cpu_baseline  the compiled reference (oracle/_ref/libref.so, unmodified trace_ray under an
                OpenMP loop) on a row sample of the same frame, rank 0 at N = 1 only; its
                sampled rows double as the parity check "max |dhit|".
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from bhrt import abi, configs, lib  # noqa: E402
from bhrt.dist_frame import FramePipeline, padded_shard_rows, sample_offset  # noqa: E402

FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (and FP64 matrix) peak, AMD spec
METRIC = "Mrays/s (and RK4 steps/s) per GPU + per node; max |Δhit| vs CPU ref"
ROW_BLOCK = 8
FIELDS = abi.SOA_FIELDS


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--config", default="C2")
    p.add_argument("--camera", default="B")
    p.add_argument("--refill", type=int, default=None)
    p.add_argument("--cpu-rows-stride", type=int, default=27,
                   help="CPU baseline samples every k-th image row")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-host-path", action="store_true",
                   help="skip the host-buffer leg (its chunked launches would mix into a "
                        "profiler's per-launch kernel averages)")
    p.add_argument("--streams", type=int, default=2,
                   help="consecutive frames alternate between this many HIP streams, so the "
                        "next frame's rays fill the CUs the tail of the current frame frees")
    p.add_argument("--sample", type=int, default=None,
                   help="weak scaling: trace sample plane K instead of this rank's (to time "
                        "each plane of an N-GPU run on one GPU)")
    return p.parse_args()


def flops(st, method):
    per_iter = 368 if method == abi.INTEGRATOR_RKF45 else 117
    return per_iter * st["iterations"] + 35 * st["stages_full"] + 4 * st["stages_far"]


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.streams not in (1, 2):  # FramePipeline has two buffer slots, one per stream
        raise SystemExit("--streams must be 1 or 2")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    L = lib.load()
    if args.refill:
        L.bhrt_set_refill_threshold(args.refill)

    c = configs.CONFIGS[args.config]
    bh, dk, cfg = c.scene()
    cam = configs.camera(args.camera)
    strong = c.scaling == "strong"
    W, H = c.width, c.bench_height(1)
    if strong:
        rows = abi.Rows(ROW_BLOCK, rank, world) if world > 1 else None
        n = padded_shard_rows(H, ROW_BLOCK, world) * W  # this rank fills its shard_rows
    else:
        rows = None
        n = W * H
        off = sample_offset(rank if args.sample is None else args.sample)
        if off is not None:
            cam.use_offset, cam.offset_x, cam.offset_y = 1, off[0], off[1]
    pipe = FramePipeline(n, device, world, rank, "shards" if strong else "samples", H, W,
                         ROW_BLOCK, FIELDS)
    streams = ([torch.cuda.current_stream()] if args.streams <= 1 else
               [torch.cuda.Stream(device) for _ in range(args.streams)])
    frame_no = [0]

    def step():
        # Frame k renders on streams[k % S]. A persistent k_trace launch ends with a tail in
        # which its last (up to max_steps-iteration) rays drain and CUs fall idle; with S > 1
        # the next frame's workgroups take those CUs (tools/wave_tail.py measures the tail).
        # A frame buffer slot is reused two frames later, on the same stream when S = 2.
        s = streams[frame_no[0] % len(streams)]
        frame_no[0] += 1
        with torch.cuda.stream(s):
            fb = pipe.next_buffer()
            lib.render_frame_device(bh, dk, cfg, cam, W, H, rows, c.method, c.flags, fb.soa(),
                                    s.cuda_stream)
            pipe.submit()

    for _ in range(args.warmup):
        step()
    pipe.finish()
    torch.cuda.synchronize()
    lib.stats(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    frame = pipe.finish()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    st = lib.stats(reset=True)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
        tot = torch.tensor([st["iterations"]], dtype=torch.float64, device=device)
        dist.all_reduce(tot)
        iterations_all = tot.item()
    else:
        iterations_all = st["iterations"]

    if rank != 0:
        dist.destroy_process_group()
        return

    rays_all = float(W * H) * args.steps * (1 if strong else world)
    mrays = rays_all / elapsed / 1e6
    launches = max(st["launches"], 1)
    kern_ms = st["kernel_ms"] / launches
    # GPU time per trace launch: the per-launch HIP-event duration when frames run one after
    # another; with frames alternating between two streams consecutive launches overlap (the
    # next frame fills the CUs the current one's tail frees) and each launch's own start..end
    # interval double-counts the overlap, so the busy span of all timed launches / launches
    span_ms = st["span_ms"] / launches
    dur_ms = span_ms if len(streams) > 1 else kern_ms
    f_launch = flops(st, c.method) / launches
    achieved = f_launch / (dur_ms * 1e-3) / 1e12
    out = {
        "metric": METRIC,
        "value": round(mrays, 3),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": c.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic camera-B frame, no input data)",
        "config": {
            "workload": f"{c.name}: {c.note}",
            "camera": args.camera,
            "sample_plane": None if strong else (rank if args.sample is None else args.sample),
            "width": W,
            "height": H,
            "rays_per_gpu": n,
            "parallelism": ("single GPU" if world == 1 else
                            (f"dp{world}: cyclic {ROW_BLOCK}-row blocks of one image, one RCCL "
                             "gather to rank 0 per frame (overlapped with the next frame)")
                            if strong else
                            (f"dp{world}: one sub-pixel sample plane of the frame per GPU "
                             f"({world} samples/pixel), one RCCL reduce of the colour planes "
                             "to rank 0 per frame (the sample average, overlapped with the "
                             "next frame)")),
        },
        "rk4_steps_per_s": round(iterations_all * (1.0 / elapsed), 1),
        "per_gpu_mrays_s": round(mrays / world, 3),
        "kernel": {
            "name": "k_trace (persistent, wave refill)",
            "avg_ms": round(dur_ms, 4),
            "duration": ("busy span of the timed launches (HIP events, first start to last "
                         "end) / launches: frames alternate between 2 streams and overlap"
                         if len(streams) > 1 else "per-launch HIP-event duration, averaged"),
            "event_avg_ms": round(kern_ms, 4),
            "streams": len(streams),
            "iterations_per_launch": st["iterations"] / max(st["launches"], 1),
            "mean_iterations_per_ray": st["iterations"] / max(st["rays"], 1),
        },
        "roofline": {
            "bound": "valu-fp64",
            "achieved": round(achieved, 4),
            "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": round(achieved / FP64_PEAK_TFLOPS, 5),
            "traffic": traffic_from_profile(args.config),
        },
    }
    if world == 1 and not args.no_host_path:
        out["host_path"] = host_path_rate(c, bh, dk, cfg, cam, W, H)
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], out["max_rel_dhit"], out["class_mismatch"] = cpu_baseline(
            args, c, bh, dk, cfg, cam, frame)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def host_path_rate(c, bh, dk, cfg, cam, W, H, frames=3):
    """bhrt_render_frame into host SoA arrays (allocated and touched once, reused every frame
    as a render loop does): the PCIe-inclusive rate a C caller of the host API sees. Reported
    beside `value`, never as it."""
    import ctypes as C
    arrays, soa = abi.alloc_soa(W * H)
    for a in arrays.values():
        a[...] = 0
    L = lib.load()

    def frame():
        if L.bhrt_render_frame(C.byref(bh), C.byref(dk) if dk else None, C.byref(cfg),
                               C.byref(cam), W, H, c.method, c.flags, C.byref(soa)) != 0:
            raise RuntimeError(lib.last_error())

    frame()
    t0 = time.perf_counter()
    for _ in range(frames):
        frame()
    dt = (time.perf_counter() - t0) / frames
    lib.stats(reset=True)
    return {"mrays_s": round(W * H / dt / 1e6, 3), "ms_per_frame": round(dt * 1e3, 3),
            "bytes_to_host_per_frame": W * H * 96,
            "note": "bhrt_render_frame into reused host arrays; pipelined chunks"}


def traffic_from_profile(config):
    """HBM bytes per trace-kernel launch from the committed rocprofv3 PMC summary (FETCH_SIZE
    x2 per the gfx950 correction + WRITE_SIZE, MI355X_MICROARCH.md 'HBM'), or None."""
    p = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None
    with open(p) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def cpu_baseline(args, c, bh, dk, cfg, cam, frame):
    """The compiled reference (or, if it was not built, the oracle restatement) on every k-th
    row of the same frame; also the parity of those rows against the GPU frame."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    try:
        checker, kind = orc.reference(), "reference"
    except (FileNotFoundError, OSError):
        checker, kind = orc.oracle(), "port"
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    W, H = c.width, c.bench_height(1)
    rows = list(range(0, H, args.cpu_rows_stride))
    got = {f: frame[f].reshape(H, W).cpu().numpy()[rows] for f in FIELDS}
    t0 = time.perf_counter()
    want = []
    for r in rows:
        want.append(checker.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                         rows=abi.Rows(1, r, H), threads=threads))
    dt = time.perf_counter() - t0
    nrays = len(rows) * W
    want = {f: np.stack([w[f] for w in want]) for f in FIELDS}
    mism = int((got["result"] != want["result"]).sum() + (got["steps"] != want["steps"]).sum())
    worst = 0.0
    for f in ("hit_x", "hit_y", "hit_z", "distance", "time_dilation", "rgb_r", "rgb_g", "rgb_b"):
        a, b = got[f], want[f]
        ok = ~(np.isnan(a) | np.isnan(b))
        if ok.any():
            worst = max(worst, float(np.max(np.abs(a[ok] - b[ok]) /
                                            np.maximum(np.abs(b[ok]), 1e-9))))
    base = {"value": round(nrays / dt / 1e6, 5), "unit": "Mrays/s", "cores": threads,
            "kind": kind,
            "sample": f"rows 0,{args.cpu_rows_stride},... of the {W}x{H} frame ({nrays} rays, "
                      f"{dt:.1f} s wall, OpenMP over rays; the reference integrates every ray "
                      f"to its full step budget before the disk scan)"}
    return base, worst, mism


if __name__ == "__main__":
    main()
