"""The five BASELINE.json configurations and the three cameras.

C1..C5 follow BASELINE.json "configs" in order. Camera B ("inclined 80 deg") is the primary
camera of every benchmark; A is the README camera, V the visualizer default.
"""
import math
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


def camera_rays(cam, width, height):
    """Pixel-centre rays of a camera frame as a Ray array (abi.RAY_DTYPE), row 0 = top: the
    camera basis and pixel mapping of calculate_ray_direction (raytracer.c:999-1039), in numpy
    -- synthetic input for the ray-array APIs (bench.py's trace_rays_batch leg)."""
    import numpy as np

    def norm(v):
        n = np.sqrt((v[..., 0] * v[..., 0] + v[..., 1] * v[..., 1]) + v[..., 2] * v[..., 2])
        return v * (1.0 / n)[..., None]

    d = np.array([cam.direction.x, cam.direction.y, cam.direction.z])
    up0 = np.array([cam.up.x, cam.up.y, cam.up.z])
    fwd = norm(d)
    right = norm(np.cross(fwd, up0))
    up = np.cross(right, fwd)
    plane_h = 2.0 * math.tan(cam.fov_deg * math.pi / 180.0 / 2.0)
    plane_w = plane_h * (width / height)
    px = (2.0 * ((np.arange(width) + 0.5) / width) - 1.0) * plane_w
    py = (1.0 - 2.0 * ((np.arange(height) + 0.5) / height)) * plane_h
    v = (fwd[None, None, :] + right[None, None, :] * px[None, :, None]) + \
        up[None, None, :] * py[:, None, None]
    rays = np.zeros(width * height, dtype=abi.RAY_DTYPE)
    rays["origin"] = (cam.position.x, cam.position.y, cam.position.z)
    rays["direction"] = norm(v).reshape(-1, 3)
    return rays


def row_block_for(height, shards):
    """Rows per cyclic block: the largest B <= 8 that splits `height` into `shards` equal
    shards of whole blocks (C5: 4320 rows / 8 shards -> B = 6, 540 rows each), else 8 (the
    shards are then padded to whole blocks, dist_frame.padded_shard_rows)."""
    if shards <= 1:
        return 8
    for b in range(8, 0, -1):
        if height % (b * shards) == 0:
            return b
    return 8


@dataclass(frozen=True)
class FramePlan:
    """What bench.py renders at N GPUs: a width x height image split into
    `shards` cyclic row-block shards (block b -> shard b % shards, bhrt_rows); rank r renders
    shard r and rank 0 assembles the image rows of shards 0..N-1 from ONE gather."""
    width: int
    height: int
    shards: int
    row_block: int
    note: str

    def rows(self, shard):
        """bhrt_rows of `shard` (None: the whole image is one shard)."""
        return abi.Rows(self.row_block, shard, self.shards) if self.shards > 1 else None


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
    # bench.py at N GPUs (frame()):
    #   "strong"       the width x height image split into N shards (C4);
    #   "weak-tiles"   an image with N times the pixels of width x height at the same aspect
    #                  and field of view, split into N shards: N = 1 is the configuration
    #                  frame itself and every GPU keeps one frame's worth of rays (C1-C3);
    #   "weak-shards"  the width x height image is the node frame of `node_shards` GPUs; N
    #                  GPUs render N of its `node_shards` shards (C5: 7680x4320 in 8 shards of
    #                  540 rows; N = 1 is shard 0, N = 8 the whole image)
    scaling: str = "weak-tiles"
    node_shards: int = 0

    def frame(self, n_gpus):
        """The FramePlan of n_gpus GPUs."""
        n = max(1, int(n_gpus))
        if self.scaling == "weak-shards":
            if n > self.node_shards:
                raise ValueError(f"{self.name}: at most {self.node_shards} GPUs render the "
                                 f"{self.width}x{self.height} frame's {self.node_shards} shards")
            S = self.node_shards
            return FramePlan(self.width, self.height, S, row_block_for(self.height, S),
                             f"{self.width}x{self.height} frame, shards 0..{n - 1} of {S}")
        if self.scaling == "strong" or n == 1:
            return FramePlan(self.width, self.height, n, row_block_for(self.height, n),
                             f"{self.width}x{self.height} frame in {n} shards")
        # n x the pixels at the same aspect: height = height * sqrt(n) rounded to a multiple
        # of n (equal shards; row_block_for picks the block), width from the aspect
        # (calculate_ray_direction takes aspect = W / H, raytracer.c:1013). n = 4 is exactly
        # 2x each side (C2: 3840x2160).
        H = max(n, int(round(self.height * math.sqrt(n) / n)) * n)
        W = int(round(self.width * H / self.height))
        return FramePlan(W, H, n, row_block_for(H, n),
                         f"{W}x{H} frame ({n} x the {self.width}x{self.height} rays at its "
                         f"aspect and field of view) in {n} shards")

    def display_fields(self):
        """The device fields of the visualizer's display call: rgba8 alone where the trace
        kernel writes the colour at each ray's exit (bhrt_kernel.h BHRT_COLOUR_IN_TRACE: a disk
        scene traced with RKF45, or with RK4 at a != 0: C3, C4), else also result and the hit
        point that the separate colour pass reads (bhrt_api.c colour_args_bad)."""
        fused = self.disk and (self.method == abi.INTEGRATOR_RKF45 or self.spin != 0.0)
        return ("rgba8",) if fused else ("result", "hit_x", "hit_y", "rgba8")

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
                 "7680x4320 Kerr a=0.99, RKF45 tol 1e-8, 2000 steps, 8 GPUs weak scaling: "
                 "shard k/8 (540 rows in cyclic 6-row blocks) per GPU", "weak-shards", 8),
}
