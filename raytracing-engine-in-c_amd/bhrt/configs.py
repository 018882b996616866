"""The five BASELINE.json configurations and the three cameras.

C1..C5 follow BASELINE.json "configs" in order. Camera B ("inclined 80 deg") is the primary
camera of every benchmark; A is the README camera, V the visualizer default.
"""
from dataclasses import dataclass

from . import abi

CAMERAS = {
    # README.md:78-79
    "A": dict(position=(0.0, 0.0, 30.0), direction=(0.0, 0.0, -1.0), up=(0.0, 1.0, 0.0), fov=60.0),
    # pos (0, -29.544, 5.209), looking at the origin, up +z
    "B": dict(position=(0.0, -29.544, 5.209), direction=(0.0, 29.544, -5.209), up=(0.0, 0.0, 1.0),
              fov=60.0),
    # src/visualization/renderer.h:393-398
    "V": dict(position=(0.0, 0.0, 75.0), direction=(0.0, 0.0, -75.0), up=(0.0, 1.0, 0.0), fov=40.0),
}


def camera(name="B"):
    c = CAMERAS[name]
    return abi.Camera(abi.v3(*c["position"]), abi.v3(*c["direction"]), abi.v3(*c["up"]), c["fov"])


@dataclass(frozen=True)
class Config:
    name: str
    width: int
    height: int
    spin: float
    disk: bool
    method: int
    tol: float
    max_steps: int
    flags: int
    gpus: int          # GPUs the configuration is quoted on
    note: str
    scaling: str = "weak"  # bench.py at N GPUs: "weak" = N x gpu_rows rows, "strong" = height
    gpu_rows: int = 0      # rows per GPU under weak scaling (0: height)

    def bench_height(self, n_gpus):
        """Image rows bench.py renders on n_gpus GPUs."""
        if self.scaling == "strong":
            return self.height
        return (self.gpu_rows or self.height) * n_gpus

    def scene(self):
        bh = abi.black_hole(1.0, self.spin)
        dk = abi.disk(bh.isco_radius, 20.0, 1.0, 1.0) if self.disk else None
        cfg = abi.sim_config(0.1, 100.0, self.max_steps, self.tol)
        return bh, dk, cfg


CONFIGS = {
    "C1": Config("C1", 256, 256, 0.0, False, abi.INTEGRATOR_RK4, 1e-6, 1000, 0, 0,
                 "256x256 Schwarzschild, RK4 dt=0.1, no disk (CPU plumbing case)"),
    "C2": Config("C2", 1920, 1080, 0.0, True, abi.INTEGRATOR_RK4, 1e-6, 1000, 0, 1,
                 "1920x1080 Schwarzschild + disk (ISCO-20M), RK4, 1 GPU"),
    "C3": Config("C3", 1920, 1080, 0.0, True, abi.INTEGRATOR_RKF45, 1e-6, 1000, 0, 1,
                 "1920x1080 Schwarzschild + disk, RKF45 tol 1e-6, 1 GPU"),
    "C4": Config("C4", 3840, 2160, 0.9, True, abi.INTEGRATOR_RK4, 1e-6, 1000,
                 abi.BHRT_FLAG_DOPPLER, 8,
                 "3840x2160 Kerr a=0.9 + disk + Doppler/beaming, RK4, 8 GPUs", "strong"),
    "C5": Config("C5", 7680, 4320, 0.99, False, abi.INTEGRATOR_RKF45, 1e-8, 2000, 0, 8,
                 "7680x4320 Kerr a=0.99, RKF45 tol 1e-8, 2000 steps, 8 GPUs weak scaling: one "
                 "7680x540 slab per GPU", "weak", 540),
}
