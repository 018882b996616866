"""Diagnostic: the large-argument ray set of tests/test_gpu_parity.py, traced by the library
named in BHRT_LIB; prints the rays that differ from the oracle."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bhrt import abi, lib
import oracle as orc

rng = np.random.default_rng(7)
n = 256
rays = np.zeros(n, dtype=abi.RAY_DTYPE)
radius = np.concatenate([np.full(64, 25.0), np.full(64, 2.0e6), np.full(64, 2.0**20 - 0.25),
                         2.0 + 10.0 ** rng.uniform(-9.0, -7.0, 64)])
u = rng.normal(size=(n, 3)); u /= np.linalg.norm(u, axis=1)[:, None]
rays["origin"] = u * radius[:, None]
d = rng.normal(size=(n, 3))
rays["direction"] = d / np.linalg.norm(d, axis=1)[:, None]
bh = abi.black_hole(1.0, 0.0)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 120
cfg = abi.sim_config(time_step=0.1, max_dist=1.0e8, max_steps=steps)
got = lib.trace_rays(rays, bh, None, cfg)
want = orc.oracle().trace_rays(rays, bh, None, cfg)
rel = np.abs(got["hit_x"] - want["hit_x"]) / np.maximum(np.abs(want["hit_x"]), 1e-300)
bad = np.nonzero((rel > 1e-9) | (got["result"] != want["result"]) | (got["steps"] != want["steps"]))[0]
print(os.environ.get("BHRT_LIB", "base"), "steps", steps, "bad", bad[:20].tolist())
for i in bad[:6]:
    print(i, rays["origin"][i], rays["direction"][i], "res", got["result"][i], want["result"][i],
          "steps", got["steps"][i], want["steps"][i], "hit", got["hit_x"][i], want["hit_x"][i],
          got["hit_z"][i], want["hit_z"][i], "dist", got["distance"][i], want["distance"][i])
print("max rel hit_x (group1)", float(np.max(rel[:64])))
