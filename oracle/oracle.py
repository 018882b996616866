"""TEST INFRASTRUCTURE ONLY: Python loaders for the CPU checkers.

  liboracle.so       the C restatement of the reference (oracle.c), "port" baseline
  _ref/libref.so     the compiled reference + driver (ref_driver.c), "reference" baseline

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "raytracing-engine-in-c_amd"))
from bhrt import abi  # noqa: E402

ORACLE_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libref.so")

_P = C.POINTER
_FRAME_ARGS = [_P(abi.BlackHoleParams), _P(abi.AccretionDiskParams), _P(abi.SimulationConfig),
               _P(abi.Camera), C.c_int, C.c_int, _P(abi.Rows), C.c_int, C.c_int,
               _P(abi.FrameSoA), C.c_int]
_RAYS_ARGS = [C.c_void_p, C.c_int, _P(abi.BlackHoleParams), _P(abi.AccretionDiskParams),
              _P(abi.SimulationConfig), C.c_int, C.c_int, _P(abi.FrameSoA), C.c_int]


class Checker:
    """Common frame/batch interface over the oracle or the compiled reference."""

    def __init__(self, path, prefix):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = C.CDLL(path)
        self.path = path
        self._frame = getattr(self.lib, prefix + "render_frame")
        self._frame.argtypes = _FRAME_ARGS
        self._frame.restype = C.c_int
        self._rays = getattr(self.lib, prefix + "trace_rays")
        self._rays.argtypes = _RAYS_ARGS
        self._rays.restype = C.c_int
        self.quiet = getattr(self.lib, "refdrv_quiet", None)

    def render_frame(self, bh, dk, cfg, cam, width, height, method=abi.INTEGRATOR_RK4, flags=0,
                     rows=None, threads=0, fields=abi.SOA_FIELDS):
        n = width * (height if rows is None else _shard_rows(height, rows))
        arrays, soa = abi.alloc_soa(n, fields)
        if self.quiet:
            self.quiet(1)
        try:
            rc = self._frame(C.byref(bh), C.byref(dk) if dk else None, C.byref(cfg), C.byref(cam),
                             width, height, C.byref(rows) if rows else None, method, flags,
                             C.byref(soa), threads)
        finally:
            if self.quiet:
                self.quiet(0)
        assert rc == 0
        return arrays

    def render_frame_margin(self, bh, dk, cfg, cam, width, height, method=abi.INTEGRATOR_RK4,
                            flags=0, rows=None, threads=0, fields=abi.SOA_FIELDS):
        """render_frame plus every ray's knife-edge margin (oracle only; oracle.c "knife-edge
        margins"): returns (arrays, margin)."""
        fn = self.lib.orc_render_frame_margin
        fn.argtypes = _FRAME_ARGS[:-1] + [C.c_void_p, C.c_int]
        fn.restype = C.c_int
        n = width * (height if rows is None else _shard_rows(height, rows))
        arrays, soa = abi.alloc_soa(n, fields)
        margin = np.empty(n, dtype=np.float64)
        rc = fn(C.byref(bh), C.byref(dk) if dk else None, C.byref(cfg), C.byref(cam), width,
                height, C.byref(rows) if rows else None, method, flags, C.byref(soa),
                margin.ctypes.data, threads)
        assert rc == 0
        return arrays, margin

    def trace_rays(self, rays, bh, dk, cfg, method=abi.INTEGRATOR_RK4, flags=0, threads=0,
                   fields=abi.SOA_FIELDS):
        rays = np.ascontiguousarray(rays, dtype=abi.RAY_DTYPE)
        arrays, soa = abi.alloc_soa(len(rays), fields)
        if self.quiet:
            self.quiet(1)
        try:
            rc = self._rays(rays.ctypes.data, len(rays), C.byref(bh), C.byref(dk) if dk else None,
                            C.byref(cfg), method, flags, C.byref(soa), threads)
        finally:
            if self.quiet:
                self.quiet(0)
        assert rc == 0
        return arrays


def _shard_rows(H, rows):
    if rows is None or rows.num_shards <= 1:
        return H
    n, b = 0, rows.shard
    while b * rows.row_block < H:
        n += min((b + 1) * rows.row_block, H) - b * rows.row_block
        b += rows.num_shards
    return n


def oracle():
    return Checker(ORACLE_PATH, "orc_")


def reference():
    return Checker(REF_PATH, "refdrv_")
