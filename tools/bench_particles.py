"""update_particles on the GPU: one JSON line.

N disk particles (create_accretion_disk, seeded) plus 1/64 test particles near the hole, so
both the Newtonian and the geodesic update run. Two launch shapes:
  * steps=1 per launch (what bh_update_particles does per frame): HBM-bound, 152 B read +
    152 B written per particle -> roofline against 8 TB/s;
  * steps=S per launch (bhrt_update_particles_steps): particles stay in registers.
Kernel times are HIP events (bhrt_update_particles_steps kernel_ms); the CPU baseline is the
compiled reference's update_particles (or the oracle) on a 20 000-particle sample, 1 core.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from bhrt import abi, lib  # noqa: E402

P = C.POINTER
HBM_PEAK_GBS = 8000.0


def make_system(L, n, seed=5):
    PS = P(abi.ParticleSystem)
    L.particle_system_init.argtypes = [PS, C.c_int]
    L.create_accretion_disk.argtypes = [PS, P(abi.BlackHoleParams), P(abi.AccretionDiskParams),
                                        C.c_int]
    L.add_particle.argtypes = [PS, P(abi.Vector3D), P(abi.Vector3D), C.c_double, C.c_int]
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    dk.thickness_factor = 0.1
    ps = abi.ParticleSystem()
    assert L.particle_system_init(C.byref(ps), n) == 0
    C.CDLL("libc.so.6").srand(seed)
    n_test = n // 64
    assert L.create_accretion_disk(C.byref(ps), C.byref(bh), C.byref(dk), n - n_test) == n - n_test
    rng = np.random.default_rng(seed)
    for _ in range(n_test):
        p = rng.uniform(-30, 30, 3)
        v = rng.normal(scale=0.2, size=3)
        L.add_particle(C.byref(ps), C.byref(abi.v3(*p)), C.byref(abi.v3(*v)), 1.0,
                       abi.PARTICLE_TEST)
    return ps, bh


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 22)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    L = lib.load()
    L.bhrt_update_particles_steps.argtypes = [P(abi.ParticleSystem), P(abi.BlackHoleParams),
                                              P(abi.SimulationConfig), C.c_int, P(C.c_double)]
    ps, bh = make_system(L, args.n)
    cfg = abi.sim_config(0.01, 100.0, 1000, 1e-6)
    ms = C.c_double()

    def run(steps):
        t = []
        for _ in range(args.reps + 1):
            assert L.bhrt_update_particles_steps(C.byref(ps), C.byref(bh), C.byref(cfg), steps,
                                                 C.byref(ms)) == 0, lib.last_error()
            t.append(ms.value)
        return float(np.mean(t[1:]))

    t1 = run(1)
    tS = run(args.steps)
    bytes1 = 2 * 152 * args.n
    out = {
        "workload": f"update_particles, {args.n} particles (1/64 geodesic test particles)",
        "one_step_per_launch": {"kernel_ms": round(t1, 4),
                                "Mparticles_per_s": round(args.n / t1 / 1e3, 1),
                                "roofline": {"bound": "hbm", "achieved": round(bytes1 / t1 / 1e6, 1),
                                             "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                             "frac": round(bytes1 / t1 / 1e6 / HBM_PEAK_GBS, 4)}},
        "steps_per_launch": {"steps": args.steps, "kernel_ms": round(tS, 4),
                             "Gparticle_steps_per_s": round(args.n * args.steps / tS / 1e6, 2)},
    }
    # CPU baseline: the compiled reference (or the oracle) on a sample, one core
    import oracle as orc
    try:
        chk, kind, fn = orc.reference(), "reference", "update_particles"
    except (FileNotFoundError, OSError):
        chk, kind, fn = orc.oracle(), "port", None
    m = 20000
    sample = np.ctypeslib.as_array(ps.particles, shape=(args.n,)).view(np.uint8)
    arr = (abi.Particle * m)()
    C.memmove(arr, ps.particles, m * 152)
    t0 = time.perf_counter()
    reps = 20
    if fn:
        sub = abi.ParticleSystem(C.cast(arr, P(abi.Particle)), m, m, m + 1, None)
        f = getattr(chk.lib, fn)
        f.argtypes = [P(abi.ParticleSystem), P(abi.BlackHoleParams), P(abi.SimulationConfig)]
        for _ in range(reps):
            f(C.byref(sub), C.byref(bh), C.byref(cfg))
    else:
        f = chk.lib.orc_update_particles
        f.argtypes = [C.c_void_p, C.c_int, P(abi.BlackHoleParams), P(abi.SimulationConfig), C.c_int]
        f(C.addressof(arr), m, C.byref(bh), C.byref(cfg), reps)
    dt = time.perf_counter() - t0
    del sample
    out["cpu_baseline"] = {"value": round(m * reps / dt / 1e6, 3), "unit": "Mparticle-steps/s",
                           "cores": 1, "kind": kind,
                           "sample": f"{m} particles x {reps} steps ({dt:.2f} s)"}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
