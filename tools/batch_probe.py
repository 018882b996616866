"""trace_rays_batch (the reference's batch API: Ray[] in, RayTraceHit[] out) for the C2
camera's 2 M rays: wall time per call with reused arrays, against the trace kernel, for several
chunk counts (BHRT_HOST_CHUNKS; "x" = the default plan) and pack thread counts; BHRT_HOST_TIMING=1 adds libbhrt's
per-call breakdown (staging + issue, waiting for chunks, packing) on stderr."""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
from bhrt import abi, configs, lib  # noqa: E402

c = configs.CONFIGS["C2"]
bh, dk, cfg = c.scene()
cam = configs.camera("B")
W, H = 1920, 1080
rays = configs.camera_rays(cam, W, H)
hits = np.zeros(W * H, dtype=abi.HIT_DTYPE)
L = lib.load()
# PRE_STREAMS=k: k torch streams created and used first (as bench.py's frame streams are), to see
# whether libbhrt's own streams then share hardware queues with busy or idle streams
if int(os.environ.get("PRE_STREAMS", "0")):
    import torch
    ss = [torch.cuda.Stream() for _ in range(int(os.environ["PRE_STREAMS"]))]
    for st in ss:
        with torch.cuda.stream(st):
            torch.zeros(1024, device="cuda").add_(1)
    torch.cuda.synchronize()
# PRE_FRAMES=k: k synchronous host-buffer frames (every field) of the same camera first, as
# bench.py's host-path leg renders before its batch calls
if int(os.environ.get("PRE_FRAMES", "0")):
    arrays, soa = abi.alloc_soa(W * H, abi.SOA_FIELDS)
    for _ in range(int(os.environ["PRE_FRAMES"])):
        assert L.bhrt_render_frame(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), W, H,
                                   c.method, c.flags, C.byref(soa)) == 0
if os.environ.get("WHERE"):  # the CPU (and its NUMA node) this process runs on, per call
    import glob

    def where():
        cpu = int(open("/proc/self/stat").read().rsplit(")", 1)[1].split()[36])
        node = [d.rsplit("node", 1)[1] for d in glob.glob(f"/sys/devices/system/cpu/cpu{cpu}/node*")]
        return f"cpu {cpu} node {','.join(node)}"
    gpus = sorted({open(f).read().strip() for f in glob.glob("/sys/class/drm/renderD*/device/numa_node")})
    print("gpu numa nodes", gpus, "affinity", len(os.sched_getaffinity(0)), "cpus", flush=True)
# PRE_ASYNC=k: k host-buffer frames three in flight (bhrt_render_frame_async, bench.py's async leg)
if int(os.environ.get("PRE_ASYNC", "0")):
    sets = [abi.alloc_soa(W * H, abi.SOA_FIELDS) for _ in range(3)]
    tickets = []
    for i in range(int(os.environ["PRE_ASYNC"])):
        t = C.c_int(0)
        assert L.bhrt_render_frame_async(C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(cam), W,
                                         H, c.method, c.flags, C.byref(sets[i % 3][1]),
                                         C.byref(t)) == 0
        tickets.append(t.value)
        if len(tickets) == 3:
            assert L.bhrt_frame_wait(tickets.pop(0)) == 0
    for t in tickets:
        assert L.bhrt_frame_wait(t) == 0
# PRE_DEVICE=k: k device frames on two torch streams (bench.py's timed frames)
if int(os.environ.get("PRE_DEVICE", "0")):
    import torch
    ss = [torch.cuda.Stream() for _ in range(2)]
    bufs = [{f: torch.zeros(W * H, dtype=torch.int32 if f in ("result", "steps") else
                            torch.float64, device="cuda") for f in abi.SOA_FIELDS} for _ in ss]
    for i in range(int(os.environ["PRE_DEVICE"])):
        st = ss[i % 2]
        lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                lib.soa_from_tensors(bufs[i % 2]), st.cuda_stream)
    torch.cuda.synchronize()
# PRE_PIN=MB: a pinned host buffer of that size allocated (and freed unless PRE_PIN_KEEP=1) first
if int(os.environ.get("PRE_PIN", "0")):
    import torch
    pinned = torch.empty(int(os.environ["PRE_PIN"]) << 20, dtype=torch.uint8, pin_memory=True)
    pinned.fill_(1)
    if os.environ.get("PRE_PIN_KEEP") != "1":
        del pinned
# PRE_PAGEABLE=k: k pageable device-to-host torch copies of a 200 MB tensor first
if int(os.environ.get("PRE_PAGEABLE", "0")):
    import torch
    t = torch.ones(25 << 20, dtype=torch.float64, device="cuda")
    for _ in range(int(os.environ["PRE_PAGEABLE"])):
        t.cpu()
for chunks in os.environ.get("CHUNKS", "4 2 3 6 8").split():
    for threads in (0, 8):
        if chunks == "x":  # the library's default plan
            os.environ.pop("BHRT_HOST_CHUNKS", None)
        else:
            os.environ["BHRT_HOST_CHUNKS"] = chunks
        args = (rays.ctypes.data, W * H, C.byref(bh), C.byref(dk), C.byref(cfg),
                hits.ctypes.data, threads)
        assert L.trace_rays_batch(*args) == 0
        lib.stats(reset=True)
        t = time.perf_counter()
        for _ in range(4):
            assert L.trace_rays_batch(*args) == 0
        dt = (time.perf_counter() - t) / 4
        st = lib.stats(reset=True)
        if os.environ.get("WHERE"):
            print(where(), flush=True)
        print(f"trace_rays_batch 2M rays, {chunks} chunks, num_threads {threads}: "
              f"{dt * 1e3:.2f} ms/call ({W * H / dt / 1e6:.1f} Mrays/s), kernel "
              f"{st['kernel_ms'] / 4:.2f} ms/call over {st['launches'] // 4} launches", flush=True)
