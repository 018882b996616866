"""Does torch's HIP initialisation succeed after libbhrt has driven the device in the same
process? Each case runs in a fresh child process: a libbhrt call sequence, then the first
torch.cuda use. (Diagnosis of a GPU test whose first torch use came after libbhrt's batch
tests and found "No HIP GPUs are available".)"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASE = r'''
import sys, numpy as np
sys.path.insert(0, "{pkg}")
from bhrt import abi, configs, lib
L = lib.load()
print("device_count", L.bhrt_device_count(), flush=True)
c = configs.CONFIGS["C2"]; bh, dk, cfg = c.scene()
rays = configs.camera_rays(configs.camera("B"), 96, 64)
step = "{step}"
if step in ("trace", "batch", "batch_noshared"):
    lib.trace_rays(rays, bh, dk, cfg)
if step in ("batch", "batch_noshared"):
    import os
    if step == "batch_noshared": os.environ["BHRT_SHARED_ORIGIN"] = "0"
    rc, hits = lib.trace_rays_batch(np.resize(rays, 1 << 16), bh, dk, cfg)
    print("batch rc", rc, flush=True)
import torch
print("torch device_count", torch.cuda.device_count(), flush=True)
t = torch.zeros(4, device="cuda")
print("torch ok", t.sum().item(), flush=True)
'''
for step in ("none", "trace", "batch", "batch_noshared"):
    code = CASE.format(pkg=os.path.join(ROOT, "raytracing-engine-in-c_amd"), step=step)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    last = (r.stdout.strip().splitlines() or [""])[-1]
    err = (r.stderr.strip().splitlines() or [""])[-1]
    print(f"{step}: rc {r.returncode}; {last}; {err if r.returncode else ''}", flush=True)
