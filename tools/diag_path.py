"""Diagnostic: per-iteration path of one ray (GPU integrate_photon_path vs the oracle's)."""
import ctypes as C, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bhrt import abi, lib
import oracle as orc


def run(fn, o4, d3, bh, cfg, maxp):
    path = (abi.Vector3D * maxp)()
    num = C.c_int(0)
    hit = abi.RayTraceHit()
    res = fn(C.byref(abi.Vector4D(*o4)), C.byref(abi.v3(*d3)), C.byref(bh), C.byref(cfg),
             abi.INTEGRATOR_RK4, C.cast(path, C.c_void_p), maxp, C.byref(num), C.byref(hit))
    return res, num.value, np.array([[p.x, p.y, p.z] for p in path[:num.value]])


rng = np.random.default_rng(7)
n = 256
radius = np.concatenate([np.full(64, 25.0), np.full(64, 2.0e6), np.full(64, 2.0**20 - 0.25),
                         2.0 + 10.0 ** rng.uniform(-9.0, -7.0, 64)])
u = rng.normal(size=(n, 3)); u /= np.linalg.norm(u, axis=1)[:, None]
d = rng.normal(size=(n, 3))
d /= np.linalg.norm(d, axis=1)[:, None]
bh = abi.black_hole(1.0, 0.0)
steps = 120
cfg = abi.sim_config(time_step=0.1, max_dist=1.0e8, max_steps=steps)
O = orc.oracle().lib.orc_integrate_photon_path
G = lib.load().integrate_photon_path
for i in [int(a) for a in sys.argv[1:]] or [147]:
    o4 = (0.0, *(u[i] * radius[i]))
    rg = run(G, o4, d[i], bh, cfg, steps + 1)
    ro = run(O, o4, d[i], bh, cfg, steps + 1)
    print("ray", i, "res", rg[:2], ro[:2])
    a, b = rg[2], ro[2]
    m = min(len(a), len(b))
    rel = np.max(np.abs(a[:m] - b[:m]), axis=1) / np.maximum(np.max(np.abs(b[:m]), axis=1), 1e-300)
    first = int(np.argmax(rel > 1e-12)) if (rel > 1e-12).any() else -1
    print(" first step rel>1e-12:", first, "rel there", rel[first] if first >= 0 else 0)
    for k in range(max(first - 2, 0), min(first + 3, m)) if first >= 0 else []:
        print("  ", k, a[k].tolist(), b[k].tolist(), np.linalg.norm(b[k]))
