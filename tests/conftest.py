"""Shared test plumbing.

Markers: `gpu` = needs a real MI355X (run with -m gpu). Everything else runs on CPU.

Comparison policy:
  * oracle vs golden (compiled reference): integers exact, floats rtol 1e-12;
  * libbhrt (GPU) vs golden / oracle: integers exact, floats rtol 1e-5 (north_star);
  * NaN == NaN; RayTraceHit.sky_direction is compared only where the reference computes it
    deterministically (RKF45 / no-op integrators): for RK4 it integrates uninitialised heap
    memory in the reference.
"""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, os.path.join(ROOT, "raytracing-engine-in-c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from bhrt import abi  # noqa: E402

INT_FIELDS = ("result", "steps")
FLOAT_FIELDS = ("hit_x", "hit_y", "hit_z", "distance", "time_dilation", "rgb_r", "rgb_g", "rgb_b")
SKY_FIELDS = ("sky_x", "sky_y", "sky_z")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def golden(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_names(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def scene_from(g):
    """(bh, disk or None, cfg) from a fixture's scene arrays."""
    bh = abi.BlackHoleParams(*[float(x) for x in g["bh"]])
    dk = abi.AccretionDiskParams(*[float(x) for x in g["disk"]]) if bool(g["has_disk"]) else None
    cfg = abi.SimulationConfig()
    cfg.time_step, cfg.max_ray_distance, cfg.tolerance = [float(x) for x in g["cfg_f"]]
    cfg.max_integration_steps = int(g["cfg_steps"])
    return bh, dk, cfg


def camera_from(g):
    c = [float(x) for x in g["cam"]]
    return abi.Camera(abi.v3(*c[0:3]), abi.v3(*c[3:6]), abi.v3(*c[6:9]), c[9])


def rays_from(g):
    r = np.zeros(len(g["rays"]), dtype=abi.RAY_DTYPE)
    r["origin"] = g["rays"][:, 0:3]
    r["direction"] = g["rays"][:, 3:6]
    return r


def compare(got, want, rtol, check_sky, what="", fields=None):
    """Assert SoA equality under the policy above; returns max relative float error."""
    fields = fields or (INT_FIELDS + FLOAT_FIELDS + (SKY_FIELDS if check_sky else ()))
    worst = 0.0
    for f in fields:
        a, b = np.asarray(got[f]), np.asarray(want[f])
        assert a.shape == b.shape, (what, f, a.shape, b.shape)
        if f in INT_FIELDS:
            bad = np.nonzero(a != b)[0]
            assert bad.size == 0, f"{what}: {f} differs at {bad[:10]}: got {a[bad[:10]]} want {b[bad[:10]]}"
            continue
        nan_a, nan_b = np.isnan(a), np.isnan(b)
        assert (nan_a == nan_b).all(), f"{what}: {f} NaN pattern differs at {np.nonzero(nan_a != nan_b)[0][:10]}"
        ok = ~nan_a
        diff = np.abs(a[ok] - b[ok])
        scale = np.maximum(np.abs(a[ok]), np.abs(b[ok]))
        tol = rtol * scale + (1e-300 if rtol < 1e-9 else 1e-9)
        bad = np.nonzero(diff > tol)[0]
        assert bad.size == 0, (f"{what}: {f} rel err {np.max(diff[bad] / np.maximum(scale[bad], 1e-300)):.3e} "
                               f"at {np.nonzero(ok)[0][bad[:5]]}")
        if diff.size:
            worst = max(worst, float(np.max(diff / np.maximum(scale, 1e-300))))
    return worst


KNIFE_EDGE = 1e-9  # rays whose reference margin to a threshold is below this


def full_frame_report(got, want, margin, check_sky, rtol=1e-5):
    """Every-ray comparison of a GPU frame with the oracle's (integers exact, floats within
    rtol, NaN pattern identical), with the oracle's knife-edge margin of each ray: a mismatch
    on a ray whose margin is below KNIFE_EDGE is a listed knife-edge ray, any other is a
    parity failure. Returns a JSON-able dict; report["unexplained"] must be 0."""
    n = len(want["result"])
    bad = np.zeros(n, dtype=bool)
    rep = {"rays": int(n)}
    for f in INT_FIELDS:
        d = np.asarray(got[f]) != np.asarray(want[f])
        rep[f + "_mismatch"] = int(d.sum())
        bad |= d
    worst = {}
    for f in FLOAT_FIELDS + (SKY_FIELDS if check_sky else ()):
        a, b = np.asarray(got[f]), np.asarray(want[f])
        na, nb = np.isnan(a), np.isnan(b)
        d = na != nb
        ok = ~(na | nb)
        rel = np.zeros(n)
        rel[ok] = np.abs(a[ok] - b[ok]) / np.maximum(np.maximum(np.abs(a[ok]), np.abs(b[ok])),
                                                     1e-300)
        small = ok & (np.abs(a - b) <= 1e-9)  # (values at ~0: absolute floor, as in compare)
        d |= (rel > rtol) & ~small
        rep[f + "_violations"] = int(d.sum())
        worst[f] = float(rel[ok & ~bad].max()) if (ok & ~bad).any() else 0.0
        bad |= d
    knife = margin < KNIFE_EDGE
    rep["max_rel_err_on_matching_rays"] = worst
    rep["mismatched_rays"] = int(bad.sum())
    rep["knife_edge_rays"] = int(knife.sum())
    rep["mismatches_on_knife_edge"] = int((bad & knife).sum())
    rep["unexplained"] = int((bad & ~knife).sum())
    rep["unexplained_ids"] = np.nonzero(bad & ~knife)[0][:20].tolist()
    rep["knife_edge_ids"] = np.nonzero(knife)[0][:200].tolist()
    rep["min_margin"] = float(np.nanmin(margin)) if n else None
    edges = [0, 1e-12, 1e-9, 1e-6, 1e-3, np.inf]
    rep["margin_histogram"] = {f"[{lo:g},{hi:g})": int(((margin >= lo) & (margin < hi)).sum())
                               for lo, hi in zip(edges, edges[1:])}
    return rep


def fixture_outputs(g):
    return {k[4:]: v for k, v in g.items() if k.startswith("out_")}


def sky_pinned(method):
    return int(method) != abi.INTEGRATOR_RK4


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc
    return orc.oracle()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def bhrt_lib():
    """libbhrt.so on a GPU box; a GPU test that gets here without HIP must fail, not skip."""
    from bhrt import lib
    lib.load()
    assert lib.load().bhrt_device_count() > 0, "gpu test without a HIP device: " + lib.last_error()
    return lib
