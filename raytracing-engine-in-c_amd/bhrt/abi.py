"""ctypes mirror of include/bhrt_types.h and the bhrt_* extension structs of include/bhrt_api.h.

Pure data definitions: usable against libbhrt.so (the product), the oracle
(oracle/liboracle.so) and the compiled reference driver (oracle/_ref/libref.so), which all
share the reference's ABI (blackhole_types.h:15-115, raytracer.h:16-106).
"""
import ctypes as C

import numpy as np

RAY_HORIZON, RAY_DISK, RAY_BACKGROUND, RAY_MAX_DISTANCE, RAY_MAX_STEPS, RAY_ERROR = range(6)
INTEGRATOR_RK4, INTEGRATOR_RKF45, INTEGRATOR_LEAPFROG, INTEGRATOR_YOSHIDA = range(4)
JITTER_NONE, JITTER_REGULAR_GRID, JITTER_RANDOM, JITTER_HALTON, JITTER_BLUE_NOISE = range(5)
BHRT_FLAG_DOPPLER = 1


class Vector3D(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class Vector4D(C.Structure):
    _fields_ = [("t", C.c_double), ("x", C.c_double), ("y", C.c_double), ("z", C.c_double)]


class Ray(C.Structure):
    _fields_ = [("origin", Vector3D), ("direction", Vector3D)]


class SchwarzschildMetric(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("g_tt", "g_rr", "g_thth", "g_phph")]


class BlackHoleParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "mass", "schwarzschild_radius", "spin", "charge", "r_plus", "r_minus",
        "isco_radius", "ergosphere_radius")]


class AccretionDiskParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "inner_radius", "outer_radius", "temperature_scale", "density_scale",
        "thickness_factor", "alpha_viscosity")]


class SimulationConfig(C.Structure):
    _fields_ = [("time_step", C.c_double), ("max_ray_distance", C.c_double),
                ("max_integration_steps", C.c_int), ("tolerance", C.c_double),
                ("use_adaptive_step", C.c_int), ("use_gpu_raytracing", C.c_int),
                ("doppler_factor", C.c_double), ("hawking_temp_factor", C.c_double),
                ("enable_doppler", C.c_int), ("enable_gravitational_redshift", C.c_int),
                ("show_accretion_disk", C.c_int)]


class SupersamplingParams(C.Structure):
    _fields_ = [("samples_per_pixel", C.c_int), ("jitter_method", C.c_int),
                ("jitter_strength", C.c_double)]


class AdaptiveSamplingParams(C.Structure):
    _fields_ = [("enable_adaptive", C.c_int), ("min_samples", C.c_int),
                ("max_samples", C.c_int), ("convergence_threshold", C.c_double),
                ("edge_threshold", C.c_double)]


class RayTraceHit(C.Structure):
    _fields_ = [("result", C.c_int), ("hit_position", Vector3D), ("hit_normal", Vector3D),
                ("distance", C.c_double), ("steps", C.c_int), ("time_dilation", C.c_double),
                ("sky_direction", Vector3D), ("doppler_factor", C.c_double),
                ("temperature", C.c_double), ("color", C.c_double * 3),
                ("redshift", C.c_double), ("optical_depth", C.c_double)]


class GPUShaderParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "mass", "spin", "schwarzschild_radius", "disk_inner_radius", "disk_outer_radius",
        "disk_temp_scale", "observer_distance", "fov")]


class Camera(C.Structure):
    _fields_ = [("position", Vector3D), ("direction", Vector3D), ("up", Vector3D),
                ("fov_deg", C.c_double), ("use_offset", C.c_int), ("offset_x", C.c_double),
                ("offset_y", C.c_double)]


class Rows(C.Structure):
    _fields_ = [("row_block", C.c_int), ("shard", C.c_int), ("num_shards", C.c_int)]


SOA_FIELDS = ("result", "steps", "hit_x", "hit_y", "hit_z", "distance", "time_dilation",
              "sky_x", "sky_y", "sky_z", "rgb_r", "rgb_g", "rgb_b")
SOA_DTYPES = {f: (np.int32 if f in ("result", "steps") else np.float64) for f in SOA_FIELDS}
# display path: 4 values per pixel (bhrt_frame_soa.rgba32f / rgba8)
DISPLAY_FIELDS = ("rgba32f", "rgba8")
SOA_DTYPES.update(rgba32f=np.float32, rgba8=np.uint8)


def rgba8_from_rgb(r, g, b):
    """The display conversion of bhrt_frame_soa.rgba8 in numpy (renderer.cpp:2090-2125):
    (unsigned char)(std::min(1.0f, (float)v) * 255.0f) per channel (NaN -> 255, truncation),
    alpha 255. Returns uint8 [n, 4]."""
    out = np.empty(np.shape(r) + (4,), dtype=np.uint8)
    for i, v in enumerate((r, g, b)):
        f = np.asarray(v).astype(np.float32)
        with np.errstate(invalid="ignore"):
            m = np.where(f < np.float32(1.0), f, np.float32(1.0))
        out[..., i] = (m * np.float32(255.0)).astype(np.uint8)
    out[..., 3] = 255
    return out


class FrameSoA(C.Structure):
    _fields_ = [(f, C.c_void_p) for f in SOA_FIELDS + DISPLAY_FIELDS]


class Stats(C.Structure):
    _fields_ = [("rays", C.c_uint64), ("iterations", C.c_uint64), ("stages_full", C.c_uint64),
                ("stages_far", C.c_uint64), ("stages_kerr", C.c_uint64),
                ("launches", C.c_uint64), ("kernel_ms", C.c_double),
                ("rays_redone", C.c_uint64), ("span_ms", C.c_double),
                ("redo_launches", C.c_uint64), ("frame_ms", C.c_double),
                ("frame_ms_max", C.c_double), ("frames_timed", C.c_uint64),
                ("attempts_untested", C.c_uint64)]


# numpy view of RayTraceHit (160 B, offsets pinned in include/bhrt_types.h)
HIT_DTYPE = np.dtype({
    "names": ["result", "hit_position", "hit_normal", "distance", "steps", "time_dilation",
              "sky_direction", "doppler_factor", "temperature", "color", "redshift",
              "optical_depth"],
    "formats": [np.int32, (np.float64, 3), (np.float64, 3), np.float64, np.int32, np.float64,
                (np.float64, 3), np.float64, np.float64, (np.float64, 3), np.float64, np.float64],
    "offsets": [0, 8, 32, 56, 64, 72, 80, 104, 112, 120, 144, 152],
    "itemsize": 160})
RAY_DTYPE = np.dtype([("origin", np.float64, 3), ("direction", np.float64, 3)])

# particle_sim.h:15-75 (Particle 152 B, ParticleSystem 32 B; pinned in bhrt_types.h)
PARTICLE_TEST, PARTICLE_DISK, PARTICLE_HAWKING, PARTICLE_JET = 0, 1, 2, 3


class Particle(C.Structure):
    _fields_ = [("position", Vector3D), ("velocity", Vector3D), ("acceleration", Vector3D),
                ("mass", C.c_double), ("energy", C.c_double), ("angular_momentum", C.c_double),
                ("proper_time", C.c_double), ("coordinate_time", C.c_double),
                ("type", C.c_int), ("active", C.c_int), ("id", C.c_int), ("age", C.c_double),
                ("temperature", C.c_double), ("time_dilation", C.c_double)]


class ParticleSystem(C.Structure):
    _fields_ = [("particles", C.POINTER(Particle)), ("capacity", C.c_int), ("count", C.c_int),
                ("next_id", C.c_int), ("blackhole", C.c_void_p)]


PARTICLE_DTYPE = np.dtype({
    "names": ["position", "velocity", "acceleration", "mass", "energy", "angular_momentum",
              "proper_time", "coordinate_time", "type", "active", "id", "age", "temperature",
              "time_dilation"],
    "formats": [(np.float64, 3), (np.float64, 3), (np.float64, 3)] + [np.float64] * 5 +
               [np.int32] * 3 + [np.float64] * 3,
    "offsets": [0, 24, 48, 72, 80, 88, 96, 104, 112, 116, 120, 128, 136, 144],
    "itemsize": 152})


def particles_view(ps):
    """numpy view (no copy) of ps.particles[0:count]."""
    if ps.count <= 0:
        return np.zeros(0, dtype=PARTICLE_DTYPE)
    buf = (C.c_char * (ps.count * 152)).from_address(C.addressof(ps.particles.contents))
    return np.frombuffer(buf, dtype=PARTICLE_DTYPE)


assert C.sizeof(Particle) == 152 and C.sizeof(ParticleSystem) == 32
assert C.sizeof(RayTraceHit) == 160 and C.sizeof(SimulationConfig) == 72
assert C.sizeof(BlackHoleParams) == 64 and C.sizeof(AccretionDiskParams) == 48


def v3(x, y, z):
    return Vector3D(float(x), float(y), float(z))


def alloc_soa(n, fields=SOA_FIELDS):
    """Host SoA arrays (numpy) + the FrameSoA struct pointing at them."""
    arrays = {f: np.zeros((n, 4) if f in DISPLAY_FIELDS else n, dtype=SOA_DTYPES[f])
              for f in fields}
    soa = FrameSoA(**{f: a.ctypes.data for f, a in arrays.items()})
    return arrays, soa


def _isco(mass, spin):
    """get_isco_radius (spacetime.c:285-308), used only to build configs."""
    import math
    M, a = mass, spin * mass
    if spin == 0.0:
        return 6.0 * M
    z1 = 1.0 + pow(1.0 - a * a / (M * M), 1.0 / 3.0) * (
        pow(1.0 + a / M, 1.0 / 3.0) + pow(1.0 - a / M, 1.0 / 3.0))
    z2 = math.sqrt(3.0 * a * a / (M * M) + z1 * z1)
    return M * (3.0 + z2 - math.sqrt((3.0 - z1) * (3.0 + z1 + 2.0 * z2)))


def black_hole(mass=1.0, spin=0.0, charge=0.0):
    """initialize_black_hole_params (spacetime.c:331-366), for spin >= 0, charge == 0."""
    import math
    bh = BlackHoleParams()
    bh.mass, bh.spin, bh.charge = mass, spin, charge
    bh.schwarzschild_radius = 2.0 * mass
    if spin == 0.0 and charge == 0.0:
        bh.r_plus, bh.r_minus, bh.ergosphere_radius = 2.0 * mass, 0.0, 2.0 * mass
    else:
        a = spin * mass
        s = math.sqrt(mass * mass - a * a - charge * charge)
        bh.r_plus, bh.r_minus, bh.ergosphere_radius = mass + s, mass - s, 2.0 * mass
    bh.isco_radius = _isco(mass, spin)
    return bh


def disk(inner, outer=20.0, tscale=1.0, density=1.0):
    d = AccretionDiskParams()
    d.inner_radius, d.outer_radius, d.temperature_scale, d.density_scale = inner, outer, tscale, density
    return d


def sim_config(time_step=0.1, max_dist=100.0, max_steps=1000, tol=1e-6):
    c = SimulationConfig()
    c.time_step, c.max_ray_distance, c.max_integration_steps, c.tolerance = (
        time_step, max_dist, max_steps, tol)
    return c
