"""ctypes binding of libbhrt.so (the product: HIP kernels behind the C ABI of include/bhrt_api.h).

There is no CPU path here or in the library: if libbhrt.so is missing, or HIP is unusable,
calls raise BhrtError. Tests and the bench call the library through this module.
"""
import ctypes as C
import os

import numpy as np

from . import abi

_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_DEFAULT_PATH = os.path.join(_PKG_DIR, "libbhrt.so")
LIB_PATH = os.environ.get("BHRT_LIB", _DEFAULT_PATH)


class BhrtError(RuntimeError):
    pass


_lib = None

# exported symbols and their prototypes (restype, argtypes)
_P = C.POINTER
_PROTOS = {
    "trace_ray": (C.c_int, [_P(abi.Ray), _P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                            _P(abi.SimulationConfig), _P(abi.RayTraceHit)]),
    "trace_rays_batch": (C.c_int, [C.c_void_p, C.c_int, _P(abi.BlackHoleParams),
                                   _P(abi.AccretionDiskParams), _P(abi.SimulationConfig),
                                   C.c_void_p, C.c_int]),
    "integrate_photon_path": (C.c_int, [_P(abi.Vector4D), _P(abi.Vector3D),
                                        _P(abi.BlackHoleParams), _P(abi.SimulationConfig), C.c_int,
                                        C.c_void_p, C.c_int, _P(C.c_int), _P(abi.RayTraceHit)]),
    "trace_pixel": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _P(abi.Vector3D),
                              _P(abi.Vector3D), _P(abi.Vector3D), C.c_double,
                              _P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                              _P(abi.SimulationConfig), _P(abi.SupersamplingParams),
                              _P(abi.AdaptiveSamplingParams), _P(C.c_double * 3)]),
    "bhrt_render_frame": (C.c_int, [_P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                                    _P(abi.SimulationConfig), _P(abi.Camera), C.c_int, C.c_int,
                                    C.c_int, C.c_int, _P(abi.FrameSoA)]),
    "bhrt_render_frame_async": (C.c_int, [_P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                                          _P(abi.SimulationConfig), _P(abi.Camera), C.c_int,
                                          C.c_int, C.c_int, C.c_int, _P(abi.FrameSoA),
                                          _P(C.c_int)]),
    "bhrt_frame_wait": (C.c_int, [C.c_int]),
    "bhrt_render_frame_device": (C.c_int, [_P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                                           _P(abi.SimulationConfig), _P(abi.Camera), C.c_int,
                                           C.c_int, _P(abi.Rows), C.c_int, C.c_int,
                                           _P(abi.FrameSoA), C.c_void_p]),
    "bhrt_render_frame_gather": (C.c_int, [_P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
                                           _P(abi.SimulationConfig), _P(abi.Camera), C.c_int,
                                           C.c_int, C.c_int, C.c_int, _P(abi.FrameSoA), C.c_int,
                                           C.c_int, C.c_void_p]),
    "bhrt_trace_rays": (C.c_int, [C.c_void_p, C.c_int, _P(abi.BlackHoleParams),
                                  _P(abi.AccretionDiskParams), _P(abi.SimulationConfig), C.c_int,
                                  C.c_int, _P(abi.FrameSoA)]),
    "bhrt_trace_rays_device": (C.c_int, [C.c_void_p, C.c_int, _P(abi.BlackHoleParams),
                                         _P(abi.AccretionDiskParams), _P(abi.SimulationConfig),
                                         C.c_int, C.c_int, _P(abi.FrameSoA), C.c_void_p]),
    "bhrt_shard_rows": (C.c_int, [C.c_int, _P(abi.Rows)]),
    "bhrt_get_stats": (C.c_int, [_P(abi.Stats), C.c_int]),
    "bhrt_device_count": (C.c_int, []),
    "bhrt_set_refill_threshold": (None, [C.c_int]),
    "bhrt_set_claim_order": (C.c_int, [C.c_void_p, C.c_int]),
    "bhrt_last_error": (C.c_char_p, []),
    "bh_initialize": (C.c_void_p, []),
    "bh_shutdown": (None, [C.c_void_p]),
    "bh_configure_black_hole": (C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_double]),
    "bh_configure_accretion_disk": (C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_double,
                                              C.c_double]),
    "bh_configure_simulation": (C.c_int, [C.c_void_p, C.c_double, C.c_double, C.c_int,
                                          C.c_double]),
    "bh_trace_ray": (C.c_int, [C.c_void_p, _P(C.c_double * 3), _P(C.c_double * 3),
                               _P(abi.RayTraceHit)]),
    "bh_trace_rays_batch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]),
    "bh_get_version": (None, [_P(C.c_int), _P(C.c_int), _P(C.c_int)]),
    "bh_calculate_time_dilation": (C.c_int, [C.c_void_p, _P(C.c_double * 3),
                                             _P(C.c_double * 3), _P(C.c_double)]),
    "calculate_disk_temperature": (None, [_P(abi.Vector3D), _P(abi.BlackHoleParams),
                                          _P(abi.AccretionDiskParams), _P(C.c_double),
                                          _P(C.c_double * 3)]),
    "apply_relativistic_effects": (None, [_P(abi.Vector3D), _P(abi.Vector3D),
                                          _P(abi.BlackHoleParams), _P(C.c_double * 3),
                                          _P(C.c_double)]),
    "temperature_to_rgb": (None, [C.c_double, _P(C.c_double * 3)]),
    "halton_sequence": (C.c_double, [C.c_int, C.c_int]),
    "get_isco_radius": (C.c_double, [_P(abi.BlackHoleParams)]),
    "initialize_black_hole_params": (None, [_P(abi.BlackHoleParams), C.c_double, C.c_double,
                                            C.c_double]),
    "check_disk_intersection": (C.c_int, [_P(abi.Vector3D), _P(abi.Vector3D), _P(abi.Vector3D),
                                          _P(abi.AccretionDiskParams), _P(abi.Vector3D)]),
}


def _one_hip_runtime():
    """Import torch (if installed) before libbhrt is mapped. The torch wheel carries its own HIP
    runtime, torch/lib/libamdhip64.so, whose SONAME is libamdhip64.so.7 -- the name libbhrt.so
    needs. Loaded first, it is the process's one runtime and libbhrt binds to it (torch's device
    buffers and streams are then libbhrt's too). Loaded after libbhrt, torch -- which needs the
    library by its file name -- maps a second runtime next to /opt/rocm's, and its device
    initialisation fails ("No HIP GPUs are available", tools/torch_after_lib.py).
    BHRT_PY_NO_TORCH=1 skips it (a torch-free process then runs /opt/rocm's runtime)."""
    if os.environ.get("BHRT_PY_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    except Exception as e:  # a broken torch (its bundled HIP runtime failed to load): go on
        import warnings     # with /opt/rocm's runtime, which libbhrt finds by its SONAME
        warnings.warn(f"torch failed to import ({e!r}); libbhrt binds /opt/rocm's HIP runtime")


def load(path=None):
    """Load libbhrt.so once; raise BhrtError (never fall back) if it is not there."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise BhrtError(f"libbhrt.so not built at {p} (run __graft_entry__.build())")
    _one_hip_runtime()
    lib = C.CDLL(p)
    older = p != _DEFAULT_PATH  # an A/B build of an earlier revision may lack newer entry points
    for name, (res, args) in _PROTOS.items():
        if older and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _ptr(x):
    return C.byref(x) if x is not None else None


def last_error():
    return (load().bhrt_last_error() or b"").decode()


def _check(rc, what):
    if rc != 0:
        raise BhrtError(f"{what} failed: {last_error()}")


def render_frame(bh, dk, cfg, cam, width, height, method=abi.INTEGRATOR_RK4, flags=0,
                 fields=abi.SOA_FIELDS):
    """bhrt_render_frame into host numpy arrays (all visible GPUs)."""
    arrays, soa = abi.alloc_soa(width * height, fields)
    _check(load().bhrt_render_frame(_ptr(bh), _ptr(dk), _ptr(cfg), _ptr(cam), width, height,
                                    method, flags, C.byref(soa)), "bhrt_render_frame")
    return arrays


def trace_rays(rays, bh, dk, cfg, method=abi.INTEGRATOR_RK4, flags=0, fields=abi.SOA_FIELDS):
    """bhrt_trace_rays: rays is a numpy array of abi.RAY_DTYPE."""
    rays = np.ascontiguousarray(rays, dtype=abi.RAY_DTYPE)
    arrays, soa = abi.alloc_soa(len(rays), fields)
    _check(load().bhrt_trace_rays(rays.ctypes.data, len(rays), _ptr(bh), _ptr(dk), _ptr(cfg),
                                  method, flags, C.byref(soa)), "bhrt_trace_rays")
    return arrays


def trace_rays_batch(rays, bh, dk, cfg):
    """The drop-in trace_rays_batch; returns (rc, hits as abi.HIT_DTYPE array)."""
    rays = np.ascontiguousarray(rays, dtype=abi.RAY_DTYPE)
    hits = np.zeros(len(rays), dtype=abi.HIT_DTYPE)
    rc = load().trace_rays_batch(rays.ctypes.data, len(rays), _ptr(bh), _ptr(dk), _ptr(cfg),
                                 hits.ctypes.data, 0)
    return rc, hits


def soa_from_tensors(tensors):
    """FrameSoA pointing at device tensors (torch), keyed by abi.SOA_FIELDS names."""
    return abi.FrameSoA(**{f: t.data_ptr() for f, t in tensors.items()})


def render_frame_device(bh, dk, cfg, cam, width, height, rows, method, flags, soa, stream):
    """Asynchronous launch into device SoA buffers on a hipStream_t (int handle or None)."""
    _check(load().bhrt_render_frame_device(_ptr(bh), _ptr(dk), _ptr(cfg), _ptr(cam), width,
                                           height, _ptr(rows), method, flags, C.byref(soa),
                                           C.c_void_p(stream) if stream else None),
           "bhrt_render_frame_device")


def render_frame_gather(bh, dk, cfg, cam, width, height, method, flags, soa, ndev=0, shards=0,
                        stream=None):
    """bhrt_render_frame_gather: the frame rendered by ndev devices in `shards` cyclic shards and
    gathered into root-device SoA buffers (the current device) on a hipStream_t."""
    _check(load().bhrt_render_frame_gather(_ptr(bh), _ptr(dk), _ptr(cfg), _ptr(cam), width,
                                           height, method, flags, C.byref(soa), int(ndev),
                                           int(shards),
                                           C.c_void_p(stream) if stream else None),
           "bhrt_render_frame_gather")


def set_claim_order(d_order_ptr, n):
    """bhrt_set_claim_order: the claim order (device int32 permutation of [0, n)) of this
    thread's next device camera frames of n rays; None / 0 = the default order. Raises if the
    array is not a permutation of [0, n)."""
    _check(load().bhrt_set_claim_order(d_order_ptr, int(n)), "bhrt_set_claim_order")


def shard_rows(height, rows):
    return load().bhrt_shard_rows(height, C.byref(rows))


def stats(reset=False):
    s = abi.Stats()
    _check(load().bhrt_get_stats(C.byref(s), 1 if reset else 0), "bhrt_get_stats")
    return {f: getattr(s, f) for f, _ in abi.Stats._fields_}


def stats_discard():
    """bhrt_get_stats(NULL, 1): wait for this thread's launches and drop their counters unread
    (no event timing: the cheap reset before a timed region)."""
    _check(load().bhrt_get_stats(None, 1), "bhrt_get_stats")


def halton(index, base):
    """halton_sequence (raytracer.c:852-863), libbhrt's host export."""
    L = load()
    L.halton_sequence.restype = C.c_double
    L.halton_sequence.argtypes = [C.c_int, C.c_int]
    return L.halton_sequence(index, base)
