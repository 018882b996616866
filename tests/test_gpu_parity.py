"""Parity of the HIP path (libbhrt.so on an MI355X) with the reference.

  * against the golden fixtures made by the compiled reference (small frames of every
    BASELINE config, edge rays, main.c's KAT, recorded paths, trace_pixel);
  * against the oracle on larger frames of every config;
  * at BASELINE's full size (1920x1080, C2) through size-independent properties: sampled
    rows equal the oracle's, determinism, shard reassembly, counter identities.

Tolerance: integers (class, steps) bit-exact; floats 1e-5 relative (BASELINE north_star).
"""
import ctypes as C
import os

import numpy as np
import pytest

from conftest import (ROOT, camera_from, compare, fixture_outputs, full_frame_report, golden,
                      golden_names, rays_from, scene_from, sky_pinned)
from bhrt import abi, configs

pytestmark = pytest.mark.gpu
RTOL = 1e-5


@pytest.mark.parametrize("name", golden_names("frame_"))
def test_frames_vs_reference(bhrt_lib, name):
    g = golden(name)
    bh, dk, cfg = scene_from(g)
    got = bhrt_lib.render_frame(bh, dk, cfg, camera_from(g), int(g["W"]), int(g["H"]),
                                int(g["method"]), int(g["flags"]))
    compare(got, fixture_outputs(g), RTOL, sky_pinned(g["method"]), name)


@pytest.mark.parametrize("name", golden_names("rays_"))
def test_rays_vs_reference(bhrt_lib, name):
    g = golden(name)
    bh, dk, cfg = scene_from(g)
    got = bhrt_lib.trace_rays(rays_from(g), bh, dk, cfg, int(g["method"]), int(g["flags"]))
    compare(got, fixture_outputs(g), RTOL, sky_pinned(g["method"]), name)


def test_main_kat_through_context_api(bhrt_lib):
    """main.c's five rays through bh_* exactly as main.c drives them."""
    L = bhrt_lib.load()
    g = golden("kat_main5")
    ctx = L.bh_initialize()
    assert L.bh_configure_black_hole(ctx, 1.0, 0.0, 0.0) == 0
    assert L.bh_configure_accretion_disk(ctx, 6.0, 20.0, 1.0, 1.0) == 0
    assert L.bh_configure_simulation(ctx, 0.1, 100.0, 1000, 1.0e-6) == 0
    rays = rays_from(g)
    hits = np.zeros(5, dtype=abi.HIT_DTYPE)
    hits["color"] = 7.0  # fields the reference never writes must stay untouched
    assert L.bh_trace_rays_batch(ctx, rays.ctypes.data, hits.ctypes.data, 5) == 0
    L.bh_shutdown(ctx)
    np.testing.assert_array_equal(hits["result"], g["result"])
    np.testing.assert_array_equal(hits["steps"], g["steps"])
    np.testing.assert_allclose(hits["hit_position"], g["hit_position"], rtol=RTOL, atol=1e-9)
    np.testing.assert_allclose(hits["distance"], g["distance"], rtol=RTOL)
    np.testing.assert_allclose(hits["time_dilation"], g["time_dilation"], rtol=RTOL)
    assert (hits["color"] == 7.0).all()


def test_trace_ray_and_bh_trace_ray(bhrt_lib):
    """Single-ray entry points: trace_ray (raw direction) and bh_trace_ray (normalises)."""
    L = bhrt_lib.load()
    g = golden("kat_main5")
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    cfg = abi.sim_config(0.1, 100.0, 1000, 1e-6)
    for i, row in enumerate(g["rays"]):
        ray = abi.Ray(abi.v3(*row[0:3]), abi.v3(*row[3:6]))
        hit = abi.RayTraceHit()
        res = L.trace_ray(C.byref(ray), C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(hit))
        assert res == g["result"][i] == hit.result and hit.steps == g["steps"][i]
        np.testing.assert_allclose([hit.hit_position.x, hit.hit_position.y, hit.hit_position.z],
                                   g["hit_position"][i], rtol=RTOL, atol=1e-9)
    assert L.trace_ray(C.byref(abi.Ray(abi.v3(0, 0, 30), abi.v3(0, 0, -1))), C.byref(bh), None,
                       C.byref(cfg), None) == abi.RAY_MAX_STEPS


def test_paths_vs_reference(bhrt_lib):
    L = bhrt_lib.load()
    g = golden("paths")
    for i in range(int(g["ncases"])):
        inp = g[f"case{i}_in"]
        o4, d3, spin, method, steps, maxp = inp[0:4], inp[4:7], inp[7], int(inp[8]), int(inp[9]), int(inp[10])
        bh = abi.black_hole(1.0, float(spin))
        cfg = abi.sim_config(0.1, 100.0, steps, 1e-6 if spin == 0 else 1e-8)
        path = (abi.Vector3D * max(maxp, 1))()
        num = C.c_int(0)
        hit = abi.RayTraceHit()
        res = L.integrate_photon_path(C.byref(abi.Vector4D(*o4)), C.byref(abi.v3(*d3)),
                                      C.byref(bh), C.byref(cfg), method, C.cast(path, C.c_void_p),
                                      maxp, C.byref(num), C.byref(hit))
        assert [res, num.value, hit.result, hit.steps] == list(g[f"case{i}_res"]), i
        h = g[f"case{i}_hit"]
        np.testing.assert_allclose([hit.hit_position.x, hit.hit_position.y, hit.hit_position.z,
                                    hit.distance, hit.time_dilation], h[:5], rtol=RTOL, atol=1e-9)
        if method != abi.INTEGRATOR_RK4:
            np.testing.assert_allclose([hit.sky_direction.x, hit.sky_direction.y,
                                        hit.sky_direction.z], h[5:8], rtol=RTOL, atol=1e-9)
        stored = g[f"case{i}_path"]
        got = np.array([[p.x, p.y, p.z] for p in path[:len(stored)]]).reshape(-1, 3)
        np.testing.assert_allclose(got, stored, rtol=RTOL, atol=1e-9)


def test_trace_pixel_vs_reference(bhrt_lib):
    L = bhrt_lib.load()
    g = golden("trace_pixel")
    W, H = int(g["W"]), int(g["H"])
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    cfg = abi.sim_config(0.1, 100.0, 1000, 1e-6)
    for cam, px, py, res, r, gg, b in g["rows"]:
        c = configs.camera(chr(int(cam)))
        col = (C.c_double * 3)()
        got = L.trace_pixel(int(px), int(py), W, H, C.byref(c.position), C.byref(c.direction),
                            C.byref(c.up), c.fov_deg, C.byref(bh), C.byref(dk), C.byref(cfg),
                            None, None, C.byref(col))
        assert got == int(res)
        if got != abi.RAY_DISK:
            np.testing.assert_allclose(list(col), [r, gg, b], rtol=RTOL)


def test_trace_pixel_supersampling(bhrt_lib, oracle):
    """Regular-grid and Halton supersampling average the per-sample colours."""
    L = bhrt_lib.load()
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    cfg = abi.sim_config(0.1, 100.0, 1000, 1e-6)
    c = configs.camera("B")
    lib_o = oracle.lib
    lib_o.orc_jittered_offset.argtypes = [C.c_int, C.c_int, C.c_int, C.c_double, C.c_void_p, C.c_void_p]
    lib_o.orc_camera_ray_direction.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                               C.c_int, C.c_void_p, C.c_void_p]
    for jm, spp, strength in ((abi.JITTER_REGULAR_GRID, 4, 1.0), (abi.JITTER_HALTON, 5, 0.5)):
        ss = abi.SupersamplingParams(spp, jm, strength)
        for px, py in ((3, 5), (12, 8)):
            col = (C.c_double * 3)()
            L.trace_pixel(px, py, 24, 16, C.byref(c.position), C.byref(c.direction), C.byref(c.up),
                          c.fov_deg, C.byref(bh), C.byref(dk), C.byref(cfg), C.byref(ss), None,
                          C.byref(col))
            rays = np.zeros(spp, dtype=abi.RAY_DTYPE)
            for s in range(spp):
                ox, oy = C.c_double(), C.c_double()
                lib_o.orc_jittered_offset(s, spp, jm, strength, C.byref(ox), C.byref(oy))
                d = abi.Vector3D()
                lib_o.orc_camera_ray_direction(px, py, ox.value, oy.value, 24, 16, C.byref(c), C.byref(d))
                rays[s]["origin"] = (c.position.x, c.position.y, c.position.z)
                rays[s]["direction"] = (d.x, d.y, d.z)
            want = oracle.trace_rays(rays, bh, dk, cfg)
            np.testing.assert_allclose(list(col), [want["rgb_r"].mean(), want["rgb_g"].mean(),
                                                   want["rgb_b"].mean()], rtol=RTOL)


LARGER = [("C1", "B", 96, 96), ("C2", "B", 320, 180), ("C2", "A", 160, 90), ("C3", "B", 96, 54),
          ("C4", "B", 384, 216), ("C5", "B", 192, 108), ("C2", "V", 160, 90)]


@pytest.mark.parametrize("cname,camname,W,H", LARGER)
def test_larger_frames_vs_oracle(bhrt_lib, oracle, cname, camname, W, H):
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera(camname)
    got = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    want = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    compare(got, want, RTOL, c.method != abi.INTEGRATOR_RK4, f"{cname}/{camname} {W}x{H}")


def test_full_size_c2_properties(bhrt_lib, oracle):
    """C2 at BASELINE size (1920x1080): sampled rows equal the oracle's; two renders are
    bit-identical; a 3-way cyclic shard render reassembles to the same frame; the kernel's
    work counters satisfy the per-ray identities."""
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = c.width, c.height
    bhrt_lib.stats(reset=True)
    a = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    st = bhrt_lib.stats(reset=True)
    b = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    for f in abi.SOA_FIELDS:
        assert np.array_equal(a[f], b[f], equal_nan=True), f
    # counters: every ray once; executed iterations = steps (+1 for HORIZON/MAX_DISTANCE)
    assert st["rays"] == W * H
    extra = np.isin(a["result"], (abi.RAY_HORIZON, abi.RAY_MAX_DISTANCE)).sum()
    assert st["iterations"] == int(a["steps"].astype(np.int64).sum() + extra)
    # (the per-branch stage split is checked against counted stages in
    # test_stage_counts_are_counted; no ray of a camera frame needs the redo pass)
    assert st["redo_launches"] == 0 and st["rays_redone"] == 0, st
    # rows 0, 53, 106, ... against the oracle (same pixels, same camera)
    rows = list(range(0, H, 53))
    samp = {f: a[f].reshape(H, W)[rows].ravel() for f in abi.SOA_FIELDS}
    want = {f: [] for f in abi.SOA_FIELDS}
    for r in rows:
        o = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                rows=abi.Rows(1, r, H))
        for f in abi.SOA_FIELDS:
            want[f].append(o[f])
    compare(samp, {f: np.concatenate(v) for f, v in want.items()}, RTOL, False, "C2 full rows")
    # shard reassembly through the device API
    import torch
    frame = {f: np.empty(W * H, dtype=abi.SOA_DTYPES[f]) for f in abi.SOA_FIELDS}
    for s in range(3):
        rows_s = abi.Rows(8, s, 3)
        n = bhrt_lib.shard_rows(H, rows_s) * W
        t = {f: torch.empty(n, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                            device="cuda") for f in abi.SOA_FIELDS}
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, rows_s, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), None)
        torch.cuda.synchronize()
        bhrt_lib.stats()
        local = {f: t[f].cpu().numpy().reshape(-1, W) for f in t}
        for j in range(n // W):
            g = ((j // 8) * 3 + s) * 8 + j % 8
            for f in abi.SOA_FIELDS:
                frame[f][g * W:(g + 1) * W] = local[f][j]
    for f in abi.SOA_FIELDS:
        assert np.array_equal(frame[f], a[f], equal_nan=True), f


def _render_shard(bhrt_lib, c, plan, shard):
    """bench.py's per-rank render: shard `shard` of the plan's frame through the device API;
    returns {field: [rows, W] numpy} and the image row of each local row."""
    import torch
    from bhrt.dist_frame import shard_rows_index
    W, H = plan.width, plan.height
    bh, dk, cfg = c.scene()
    rows = plan.rows(shard)
    n = (bhrt_lib.shard_rows(H, rows) if rows else H) * W
    t = {f: torch.empty(n, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                        device="cuda") for f in abi.SOA_FIELDS}
    bhrt_lib.stats(reset=True)
    bhrt_lib.render_frame_device(bh, dk, cfg, configs.camera("B"), W, H, rows, c.method,
                                 c.flags, bhrt_lib.soa_from_tensors(t), None)
    torch.cuda.synchronize()
    st = bhrt_lib.stats(reset=True)
    return ({f: v.cpu().numpy().reshape(-1, W) for f, v in t.items()}, st,
            shard_rows_index(H, plan.row_block, shard, plan.shards))


# BASELINE sizes of the other configs: sampled rows of what bench.py renders at N = 1 (C5:
# shard 0 of the 7680x4320 frame; C4's whole 3840x2160 image; C3's 1920x1080 frame) and of
# one more shard of an N-GPU plan, against the oracle rendering the same image rows.
@pytest.mark.parametrize("cname,n_gpus,shard,stride", [
    ("C3", 1, 0, 54), ("C4", 1, 0, 135), ("C4", 8, 5, 17), ("C5", 1, 0, 45), ("C5", 8, 7, 45),
    ("C2", 8, 3, 96)])
def test_full_size_shard_rows_vs_oracle(bhrt_lib, oracle, cname, n_gpus, shard, stride):
    c = configs.CONFIGS[cname]
    plan = c.frame(n_gpus)
    W, H = plan.width, plan.height
    got, st, idx = _render_shard(bhrt_lib, c, plan, shard)
    assert st["rays"] == got["result"].size == len(idx) * W
    if c.method == abi.INTEGRATOR_RK4:  # executed iterations = steps (+1 HORIZON/MAX_DISTANCE)
        extra = np.isin(got["result"], (abi.RAY_HORIZON, abi.RAY_MAX_DISTANCE)).sum()
        assert st["iterations"] == int(got["steps"].astype(np.int64).sum() + extra)
    assert st["redo_launches"] == 0 and st["rays_redone"] == 0, st
    if cname == "C5":  # the 16:9 frame's work per ray (golden frame_C5_B: ~50 attempts)
        assert 30 < st["iterations"] / st["rays"] < 70, st["iterations"] / st["rays"]
    local = list(range(0, len(idx), stride))
    bh, dk, cfg = c.scene()
    want = {f: [] for f in abi.SOA_FIELDS}
    for j in local:
        o = oracle.render_frame(bh, dk, cfg, configs.camera("B"), W, H, c.method, c.flags,
                                rows=abi.Rows(1, int(idx[j]), H))
        for f in abi.SOA_FIELDS:
            want[f].append(o[f])
    compare({f: got[f][local].ravel() for f in abi.SOA_FIELDS},
            {f: np.concatenate(v) for f, v in want.items()}, RTOL,
            c.method != abi.INTEGRATOR_RK4, f"{cname} {W}x{H} shard {shard}/{plan.shards}")


def test_device_api_on_torch_stream(bhrt_lib):
    """bhrt_render_frame_device on a torch stream: asynchronous, ordered with torch work."""
    import torch
    c = configs.CONFIGS["C4"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 256, 144
    s = torch.cuda.Stream()
    t = {f: torch.full((W * H,), -1, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                       device="cuda") for f in abi.SOA_FIELDS}
    s.wait_stream(torch.cuda.current_stream())  # (the fills ran on torch's current stream)
    with torch.cuda.stream(s):
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), s.cuda_stream)
        counts = torch.bincount(t["result"].long(), minlength=5)
    s.synchronize()
    host = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    for f in abi.SOA_FIELDS:
        assert np.array_equal(t[f].cpu().numpy(), host[f], equal_nan=True), f
    assert counts.sum().item() == W * H


@pytest.mark.parametrize("cname", ["C1", "C4"])
def test_overlapping_frames_on_two_streams(bhrt_lib, cname):
    """bench.py's pipelined mode: consecutive frames on alternating streams, in flight together
    (launch scratch is per stream), each equal to a lone render; span_ms covers the launches."""
    import torch
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = (c.width, c.height) if cname == "C1" else (640, 360)
    ref = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = [{f: torch.full((W * H,), -1, dtype=torch.int32 if f in ("result", "steps")
                           else torch.float64, device="cuda") for f in abi.SOA_FIELDS}
            for _ in range(4)]
    torch.cuda.synchronize()
    bhrt_lib.stats(reset=True)
    for k, t in enumerate(bufs):
        s = streams[k % 2]
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), s.cuda_stream)
    torch.cuda.synchronize()
    st = bhrt_lib.stats(reset=True)
    assert st["launches"] == 4 and st["rays"] == 4 * W * H
    assert st["span_ms"] > 0.0
    for t in bufs:
        for f in abi.SOA_FIELDS:
            assert np.array_equal(t[f].cpu().numpy(), ref[f], equal_nan=True), f


@pytest.mark.parametrize("cname", ["C2", "C4", "C5"])
def test_refill_threshold_does_not_change_results(bhrt_lib, cname):
    """The wave refill policy (0 = the per-scene default) is a speed knob only."""
    L = bhrt_lib.load()
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    outs = []
    for thr in (0, 1, 8, 64):
        L.bhrt_set_refill_threshold(thr)
        outs.append(bhrt_lib.render_frame(bh, dk, cfg, cam, 200, 120, c.method, c.flags))
    L.bhrt_set_refill_threshold(0)
    for o in outs[1:]:
        for f in abi.SOA_FIELDS:
            assert np.array_equal(o[f], outs[0][f], equal_nan=True), f


@pytest.mark.parametrize("cname", ["C1", "C2", "C3", "C4", "C5"])
def test_claim_order_does_not_change_results(bhrt_lib, monkeypatch, cname):
    """bhrt_set_claim_order (the queue position -> ray id permutation of device camera frames)
    is a speed knob only: the default tiled order (64-pixel tiles, geodesic.hip claim_ray), ray
    id order (BHRT_TILES=0), scattered tiles (BHRT_TILE_SCATTER=1), a random permutation and
    the reversed order give the same frame
    bit for bit, on the in-kernel set-up paths (C2-C5) and the k_init table path (C1); a
    permutation of another length is ignored."""
    import torch
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 200, 120
    n = W * H
    g = torch.Generator().manual_seed(7)
    orders = [None, torch.randperm(n, generator=g).to(torch.int32).cuda(),
              torch.arange(n - 1, -1, -1, dtype=torch.int32, device="cuda"),
              torch.arange(n + 64, dtype=torch.int32, device="cuda")]  # wrong length: ignored
    orders.insert(1, "ids")
    orders.insert(2, "scatter")
    outs = []
    try:
        for order in orders:
            monkeypatch.delenv("BHRT_TILES", raising=False)
            monkeypatch.delenv("BHRT_TILE_SCATTER", raising=False)
            if isinstance(order, str) and order == "ids":  # ray id order, not the default tiles
                monkeypatch.setenv("BHRT_TILES", "0")
                order = None
            elif isinstance(order, str):  # "scatter": the tiles visited with a coprime stride
                monkeypatch.setenv("BHRT_TILE_SCATTER", "1")
                order = None
            bhrt_lib.set_claim_order(order.data_ptr() if order is not None else None,
                                     order.numel() if order is not None else 0)
            t = {f: torch.full((n,), -1, dtype=torch.int32 if f in ("result", "steps")
                               else torch.float64, device="cuda") for f in abi.SOA_FIELDS}
            torch.cuda.synchronize()  # (torch fills on its stream, libbhrt renders on its own)
            bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                         bhrt_lib.soa_from_tensors(t), 0)
            torch.cuda.synchronize()
            outs.append({f: v.cpu().numpy() for f, v in t.items()})
        # an array that is not a permutation is rejected (claim_ray would index the outputs
        # with it) and the default order stays
        bad = torch.zeros(n, dtype=torch.int32, device="cuda")
        with pytest.raises(bhrt_lib.BhrtError):
            bhrt_lib.set_claim_order(bad.data_ptr(), n)
        # a set order applies to device-API frames only: the chunks of a host-buffer frame of
        # the same ray count never take it
        perm = next(o for o in orders if torch.is_tensor(o))  # the random permutation
        bhrt_lib.set_claim_order(perm.data_ptr(), n)
        host = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
        outs.append(host)
    finally:
        bhrt_lib.set_claim_order(None, 0)
    for o in outs[1:]:
        for f in abi.SOA_FIELDS:
            assert np.array_equal(o[f], outs[0][f], equal_nan=True), f


@pytest.mark.parametrize("cname", ["C2", "C4"])
def test_gather_frame_equals_device_frame(bhrt_lib, cname):
    """bhrt_render_frame_gather: the frame in 1, 2, 3 and 5 cyclic shards,
    each rendered into its device's shard buffer and copied straight into its image rows on the
    root (one 2-D copy per field and shard, plus the partial last block: 412 rows = 51.5
    blocks), equals the one-launch device frame bit for bit, every field and the display
    buffers. On a one-GPU box every shard is the root's (same-device copies); the peer path
    (xGMI copies, cross-device ordering) runs on the simulated devices of
    tests/test_multidevice_host.py."""
    import torch
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    fields = abi.SOA_FIELDS + abi.DISPLAY_FIELDS
    ndev = bhrt_lib.load().bhrt_device_count()  # every device (the peer path with >= 2)

    def new(W, H):
        t = {}
        for f in fields:
            dt = {"result": torch.int32, "steps": torch.int32, "rgba32f": torch.float32,
                  "rgba8": torch.uint8}.get(f, torch.float64)
            shape = (W * H, 4) if f in abi.DISPLAY_FIELDS else (W * H,)
            t[f] = torch.full(shape, 7, dtype=dt, device="cuda")
        return t

    def same(t, ref, what):
        for f in fields:
            assert torch.equal(t[f], ref[f]) or (
                t[f].is_floating_point() and
                bool(((t[f] == ref[f]) | (t[f].isnan() & ref[f].isnan())).all())), (what, f)

    sizes = ((320, 412), (480, 600))
    refs = []
    for W, H in sizes:
        refs.append(new(W, H))
        # (torch filled the buffers on its stream; libbhrt renders on its own, non-blocking one)
        torch.cuda.synchronize()
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(refs[-1]), 0)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    (W, H), ref = sizes[0], refs[0]
    for shards in sorted({1, 2, 3, 5, 2 * ndev}):
        t = new(W, H)
        torch.cuda.synchronize()
        bhrt_lib.render_frame_gather(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), ndev, shards, s.cuda_stream)
        s.synchronize()
        same(t, ref, shards)
    # back to back with no wait: the larger frame grows every device's shard buffers while the
    # smaller one's copies may still be queued (freed only after those copies ran)
    outs = [new(W, H) for W, H in sizes]
    torch.cuda.synchronize()
    for (W, H), t in zip(sizes, outs):
        bhrt_lib.render_frame_gather(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), ndev, 2 * ndev + 1,
                                     s.cuda_stream)
    s.synchronize()
    for t, ref, wh in zip(outs, refs, sizes):
        same(t, ref, wh)


def test_empty_and_degenerate_inputs(bhrt_lib):
    bh, cfg = abi.black_hole(), abi.sim_config()
    r = bhrt_lib.trace_rays(np.zeros(0, dtype=abi.RAY_DTYPE), bh, None, cfg)
    assert all(len(v) == 0 for v in r.values())
    rc, hits = bhrt_lib.trace_rays_batch(np.zeros(0, dtype=abi.RAY_DTYPE), bh, None, cfg)
    assert rc == -1
    one = bhrt_lib.render_frame(bh, None, cfg, configs.camera("A"), 1, 1)
    assert one["result"][0] == abi.RAY_MAX_STEPS


def test_c_caller_drop_in(bhrt_lib, tmp_path):
    """A plain C program using the reference API (bh_* + trace batch) gets main.c's known
    answers from libbhrt.so."""
    import subprocess
    from test_abi import build_c_demo
    out = subprocess.run([build_c_demo(tmp_path)], check=True, capture_output=True, text=True).stdout
    g = golden("kat_main5")
    lines = [l.split() for l in out.strip().splitlines()]
    for i in range(5):
        _, res, steps, x, y, z, dist, td = lines[i]
        assert int(res) == g["result"][i] and int(steps) == g["steps"][i]
        np.testing.assert_allclose([float(x), float(y), float(z)], g["hit_position"][i], rtol=RTOL, atol=1e-9)
        np.testing.assert_allclose([float(dist), float(td)], [g["distance"][i], g["time_dilation"][i]], rtol=RTOL)
    assert lines[5][0] == "frame" and sum(int(v) for v in lines[5][1:]) == 64 * 36


def _ulp_stable(oracle, rays, bh, disk, cfg):
    """Rays whose oracle result (class, steps, hit to 1e-9) is unchanged when the origin
    moves by one ulp either way: the inputs the reference itself treats as well-conditioned."""
    base = oracle.trace_rays(rays, bh, disk, cfg)
    keep = np.ones(len(rays), dtype=bool)
    for direction in (np.inf, -np.inf):
        moved = rays.copy()
        moved["origin"] = np.nextafter(rays["origin"], direction)
        o = oracle.trace_rays(moved, bh, disk, cfg)
        keep &= (o["result"] == base["result"]) & (o["steps"] == base["steps"])
        for f in ("hit_x", "hit_y", "hit_z", "distance"):
            keep &= np.abs(o[f] - base[f]) <= 1e-7 * np.maximum(np.abs(base[f]), 1.0)
    return keep


def test_large_argument_rays_take_the_redo_path(bhrt_lib, oracle):
    """Rays whose sincos arguments reach |x| >= 2^20 are evicted from the hot trace kernel,
    which has no large-argument reduction, and re-traced by its HUGE instantiation
    (geodesic.hip k_trace). Results must equal the oracle's for every ray, whichever kernel
    finished it.

    Groups of 64: (1) |origin| 25; (2) |origin| 2e6; (3) 0.25 below 2^20, where state[1]
    (read as theta by ray_derivatives) rises through 2^20 in the first steps (checked with
    an instrumented oracle) -- with the carried trig (BHRT_TRIG_CHAIN) such rays are
    reached by exact shifts and need no large-argument evaluation; (4) 1e-8..1e-7 outside
    the horizon, where dt/dlambda is huge and single RK stages jump state[1] past 2^20, so
    the shift does not apply and the ray is evicted. No group sits at |origin| = 15 rs (the
    far-field threshold) and no direction is exactly radial (v_phi would be a cancellation
    residual that FMA contraction decides, switching the far-field branch through
    impact_parameter > 0); group (4) keeps only the rays whose oracle result survives a
    one-ulp move of the origin (_ulp_stable); so does every other group."""
    rng = np.random.default_rng(7)
    n = 320
    rays = np.zeros(n, dtype=abi.RAY_DTYPE)
    radius = np.concatenate([np.full(64, 25.0), np.full(64, 2.0e6), np.full(64, 2.0**20 - 0.25),
                             2.0 + 10.0 ** rng.uniform(-8.0, -7.0, 128)])
    u = rng.normal(size=(n, 3))
    u /= np.linalg.norm(u, axis=1)[:, None]
    rays["origin"] = u * radius[:, None]
    d = rng.normal(size=(n, 3))
    rays["direction"] = d / np.linalg.norm(d, axis=1)[:, None]
    bh = abi.black_hole(1.0, 0.0)
    cfg = abi.sim_config(time_step=0.1, max_dist=1.0e8, max_steps=120)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    for disk in (None, dk):
        keep = _ulp_stable(oracle, rays, bh, disk, cfg)
        sel = rays[keep]
        assert all(keep[a:b].sum() >= 16 for a, b in ((0, 64), (64, 128), (128, 192), (192, n)))
        bhrt_lib.stats(reset=True)
        got = bhrt_lib.trace_rays(sel, bh, disk, cfg)
        st = bhrt_lib.stats(reset=True)
        want = oracle.trace_rays(sel, bh, disk, cfg)
        compare(got, want, RTOL, False, "large-argument rays")
        assert st["rays"] == len(sel)
        assert st["rays_redone"] > 0, st


@pytest.mark.parametrize("method", [abi.INTEGRATOR_RK4, abi.INTEGRATOR_RKF45])
def test_unbounded_far_field_launch_takes_the_redo_path(bhrt_lib, oracle, method):
    """geodesic.hip repair_at_refill: the far-field instantiations drop the per-iteration state
    recovery (and RKF45's literal accept quotient) only where bhrt_api.c far_bounded proves that
    no state can overflow. A tiny black hole (M = 1e-3: the far-field factor 2M / (15 rs)^2 is
    2.2, so h S C > 1/2) is not provable: every ray is handed to the HUGE redo pass, whose
    literal per-iteration checks must give the oracle's frame (camera B origin beyond 15 rs,
    so the frame runs the FAR instantiations). A normal scene hands over none."""
    cam = configs.camera("B")
    dk = abi.disk(0.006, 0.04, 1.0, 1.0)
    W, H = 40, 24
    for mass, expect_all in ((1.0e-3, True), (1.0, False)):
        bh = abi.black_hole(mass, 0.0)
        cfg = abi.sim_config(0.1, 100.0, 300, 1e-6)
        bhrt_lib.stats(reset=True)
        got = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, method, 0)
        st = bhrt_lib.stats(reset=True)
        want = oracle.render_frame(bh, dk, cfg, cam, W, H, method, 0)
        compare(got, want, RTOL, method != abi.INTEGRATOR_RK4, f"far-field M={mass}")
        assert st["rays"] == W * H, st
        assert st["rays_redone"] == (W * H if expect_all else 0), st


def _display_u8(v):
    """(unsigned char)(std::min(1.0f, v) * 255.0f), renderer.cpp:2113-2116, on x86."""
    v = v.astype(np.float32)
    m = np.where(v < np.float32(1.0), v, np.float32(1.0)).astype(np.float32)
    with np.errstate(invalid="ignore"):
        return (np.trunc(m * np.float32(255.0)).astype(np.int64) & 0xFF).astype(np.uint8)


@pytest.mark.parametrize("cname,fuse", [("C2", "1"), ("C4", "1"), ("C4", "0"), ("C3", "1"),
                                        ("C3", "0")])
def test_display_path_rgba(bhrt_lib, oracle, monkeypatch, cname, fuse):
    """the visualizer's texture buffer (float RGBA with alpha 1, then
    RGBA8 by its own conversion) produced by the colour pass, row 0 = top. C3 (RKF45 with a
    disk) and C4 (RK4 Kerr with a disk) write the colour in the trace kernel
    (BHRT_FUSE_COLOUR, default on): both forms are run, and must give the same
    buffers bit for bit (colour_of is compiled without FP contraction in both)."""
    monkeypatch.setenv("BHRT_FUSE_COLOUR", fuse)
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 96, 54
    fields = abi.SOA_FIELDS + abi.DISPLAY_FIELDS
    got = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, fields=fields)
    if cname in ("C3", "C4"):  # the other colour form gives every output bit for bit
        monkeypatch.setenv("BHRT_FUSE_COLOUR", "0" if fuse == "1" else "1")
        other = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags, fields=fields)
        other_only = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                           fields=abi.DISPLAY_FIELDS)
        monkeypatch.setenv("BHRT_FUSE_COLOUR", fuse)
        for f in fields:
            assert np.array_equal(other[f], got[f], equal_nan=True), f
        assert np.array_equal(other_only["rgba8"], got["rgba8"])
    rgb = np.stack([got["rgb_r"], got["rgb_g"], got["rgb_b"]], axis=1)
    f32 = got["rgba32f"]
    assert np.array_equal(f32[:, :3], rgb.astype(np.float32), equal_nan=True)
    assert (f32[:, 3] == 1.0).all()
    assert np.array_equal(got["rgba8"], _display_u8(f32))
    # the display fields alone (no per-ray outputs requested) give the same image
    only = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                 fields=abi.DISPLAY_FIELDS)
    assert np.array_equal(only["rgba8"], got["rgba8"])
    assert np.array_equal(only["rgba32f"], f32, equal_nan=True)
    # and the colours are the oracle's (frame colour contract) to the float32 rounding
    want = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    w32 = np.stack([want["rgb_r"], want["rgb_g"], want["rgb_b"]], axis=1).astype(np.float32)
    ok = ~np.isnan(w32)
    assert np.array_equal(np.isnan(f32[:, :3]), ~ok)
    np.testing.assert_allclose(f32[:, :3][ok], w32[ok], rtol=1e-5, atol=1e-6)
    assert np.abs(got["rgba8"][:, :3].astype(int) - _display_u8(w32).astype(int)).max() <= 1


@pytest.mark.parametrize("cname", ["C1", "C2", "C3", "C4", "C5"])
def test_display_fields_device_frame(bhrt_lib, cname):
    """bench.py's display_resident leg (and --fields display): a device frame that asks only
    for Config.display_fields() -- rgba8 alone where the colour is written in the trace
    kernel -- is accepted and gives the rgba8 of the every-field frame bit for bit."""
    import torch
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 96, 54
    n = W * H

    def frame(fields):
        t = {f: torch.full((n, 4) if f == "rgba8" else (n,), 7,
                           dtype={"rgba8": torch.uint8, "result": torch.int32,
                                  "steps": torch.int32}.get(f, torch.float64), device="cuda")
             for f in fields}
        torch.cuda.synchronize()
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), None)
        torch.cuda.synchronize()
        return {f: v.cpu().numpy() for f, v in t.items()}

    fused = c.display_fields() == ("rgba8",)
    assert fused == (cname in ("C3", "C4"))
    only = frame(c.display_fields())
    full = frame(abi.SOA_FIELDS + ("rgba8",))
    for f in c.display_fields():
        assert np.array_equal(only[f], full[f], equal_nan=True), f


def test_sub_pixel_offset_frames(bhrt_lib, oracle):
    """bhrt_camera.use_offset: frames at trace_pixel's jitter offsets (the weak-scaling sample
    planes of bench.py) against the oracle."""
    from bhrt.dist_frame import sample_offset
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    for k in (1, 2, 5):
        cam = configs.camera("B")
        cam.use_offset, (cam.offset_x, cam.offset_y) = 1, sample_offset(k)
        got = bhrt_lib.render_frame(bh, dk, cfg, cam, 64, 36, c.method, c.flags)
        want = oracle.render_frame(bh, dk, cfg, cam, 64, 36, c.method, c.flags)
        compare(got, want, RTOL, False, f"sample {k}")


def test_host_frame_chunks_equal_device_frame(bhrt_lib, monkeypatch):
    """bhrt_render_frame traces a host-buffer frame in pipelined chunks (cyclic row-block
    shards, copies overlapped with tracing, staged and un-permuted on the host); any chunk
    count gives the device frame (416 rows = 52 row blocks: uneven shards, partial last
    blocks)."""
    import torch
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H = 640, 416
    t = {f: torch.zeros(W * H, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                        device="cuda") for f in abi.SOA_FIELDS}
    torch.cuda.synchronize()  # (torch fills on its stream, libbhrt renders on its own)
    bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                 bhrt_lib.soa_from_tensors(t), 0)
    torch.cuda.synchronize()
    ref = {f: v.cpu().numpy() for f, v in t.items()}
    for chunks in ("1", "3", "4", "8"):
        monkeypatch.setenv("BHRT_HOST_CHUNKS", chunks)
        got = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
        for f in abi.SOA_FIELDS:
            assert np.array_equal(got[f], ref[f], equal_nan=True), (chunks, f)


def _frame_soa_in_one_buffer(n, fields, offset=0):
    """Caller arrays carved back to back out of ONE host allocation (fields share pages, and
    the first starts `offset` bytes into a page)."""
    sizes = [n * (16 if f == "rgba32f" else 4 if f in ("result", "steps", "rgba8") else 8)
             for f in fields]
    buf = np.zeros(sum(sizes) + offset + 64, dtype=np.uint8)
    arrays, p = {}, offset
    for f, sz in zip(fields, sizes):
        dt = abi.SOA_DTYPES[f]
        shape = (n, 4) if f in abi.DISPLAY_FIELDS else (n,)
        arrays[f] = buf[p:p + sz].view(dt).reshape(shape)
        p += sz
    soa = abi.FrameSoA(**{f: a.ctypes.data for f, a in arrays.items()})
    return buf, arrays, soa


def test_async_frames_in_flight_equal_sync_frames(bhrt_lib):
    """bhrt_render_frame_async: four frames of different scenes queued back to back (three in
    flight, the fourth waits for the oldest slot), into separate host arrays -- one set
    carved out of a single allocation at an odd page offset -- each equals the synchronous
    frame; waiting twice, or for a ticket never issued, is an error."""
    L = bhrt_lib.load()
    W, H = 1024, 576  # 590 k rays, 56 MB of fields, 2 chunks
    jobs = [("C2", "B"), ("C4", "B"), ("C3", "A"), ("C2", "V")]
    outs, keep = [], []
    for i, (cname, camname) in enumerate(jobs):
        fields = abi.SOA_FIELDS + (abi.DISPLAY_FIELDS if i == 1 else ())
        if i == 2:
            buf, arrays, soa = _frame_soa_in_one_buffer(W * H, fields, offset=1000)
            keep.append(buf)
        else:
            arrays, soa = abi.alloc_soa(W * H, fields)
        outs.append((arrays, soa))
    tickets = []
    for (cname, camname), (arrays, soa) in zip(jobs, outs):
        c = configs.CONFIGS[cname]
        bh, dk, cfg = c.scene()
        t = C.c_int(0)
        assert L.bhrt_render_frame_async(C.byref(bh), C.byref(dk) if dk else None,
                                         C.byref(cfg), C.byref(configs.camera(camname)), W,
                                         H, c.method, c.flags, C.byref(soa),
                                         C.byref(t)) == 0, bhrt_lib.last_error()
        tickets.append(t.value)
    assert len(set(tickets)) == 4 and min(tickets) > 0
    # the fourth issue took the oldest frame's slot and completed frame 1 first; frame
    # 1's own wait still returns its result, once
    for t in tickets:
        assert L.bhrt_frame_wait(t) == 0, bhrt_lib.last_error()
    assert L.bhrt_frame_wait(tickets[0]) == -1  # already waited for
    assert L.bhrt_frame_wait(tickets[-1]) == -1
    assert L.bhrt_frame_wait(max(tickets) + 100) == -1
    for (cname, camname), (arrays, _) in zip(jobs, outs):
        c = configs.CONFIGS[cname]
        bh, dk, cfg = c.scene()
        want = bhrt_lib.render_frame(bh, dk, cfg, configs.camera(camname), W, H, c.method,
                                     c.flags, fields=tuple(arrays))
        for f in arrays:
            assert np.array_equal(arrays[f], want[f], equal_nan=True), (cname, camname, f)


def _default_stream_filled_outputs(torch, n):
    """SoA output tensors of n rays whose fills are still queued on torch's default stream
    (the legacy null stream) when this returns: a busy kernel first, then a poison fill of
    every field (ints -7 / floats 1e300 through fill_, the hit point through zero_, a memset),
    so a render that is not ordered after the default stream finds its outputs overwritten.
    The caller must not synchronise before rendering."""
    assert torch.cuda.current_stream().cuda_stream == 0  # (torch's default = the null stream)
    t = {f: torch.empty(n, dtype=torch.int32 if f in ("result", "steps") else torch.float64,
                        device="cuda") for f in abi.SOA_FIELDS}
    torch.cuda.synchronize()  # (allocation done; everything below stays queued)
    sleep = getattr(torch.cuda, "_sleep", None)
    if sleep is not None:
        sleep(20_000_000)
    else:  # a few ms of GPU work on the default stream instead
        a = torch.ones(2048, 2048, device="cuda")
        for _ in range(8):
            a = a @ a * 1e-3
    for f, v in t.items():
        if f in ("hit_x", "hit_y", "hit_z"):
            v.zero_()
        else:
            v.fill_(-7 if f in ("result", "steps") else 1e300)
    return t


def test_null_stream_trace_rays_device_orders_after_default_stream(bhrt_lib, oracle):
    """bhrt_trace_rays_device(..., NULL): the rays are uploaded and the outputs poison-filled
    on the default stream, the launch takes hip_stream NULL, the results are read back on the
    default stream -- no host sync in between. Every ray against the oracle (C5's Kerr a = 0.99
    RKF45 scene, a 160x90 camera's rays)."""
    import torch
    c = configs.CONFIGS["C5"]
    bh, dk, cfg = c.scene()
    rays = configs.camera_rays(configs.camera("B"), 160, 90)
    n = len(rays)
    want = oracle.trace_rays(rays, bh, dk, cfg, c.method, c.flags)
    L = bhrt_lib.load()
    t = _default_stream_filled_outputs(torch, n)
    d_rays = torch.from_numpy(rays.view(np.uint8)).to("cuda", non_blocking=True)
    assert L.bhrt_trace_rays_device(d_rays.data_ptr(), n, C.byref(bh), C.byref(dk) if dk else None,
                                    C.byref(cfg), c.method, c.flags,
                                    C.byref(bhrt_lib.soa_from_tensors(t)), None) == 0
    got = {f: v.cpu().numpy() for f, v in t.items()}
    compare(got, want, RTOL, sky_pinned(c.method), "C5 rays, NULL stream")


@pytest.mark.parametrize("tol", [1e-8, 2.0**-30, 1e-12])
def test_accept_all_attempts_equal_the_tested_ones(bhrt_lib, oracle, monkeypatch, tol):
    """rkf45_attempt ACC (geodesic.hip): on the zero-acceleration RKF45 paths an attempt's error
    is rounding alone, so for tol >= 2^-30 the host lets every attempt through without the
    accept test. The frame must be bit-identical to the one that runs the test
    (BHRT_ACCEPT_ALL=0) and equal the oracle; below 2^-30 (1e-12) the test runs either way.
    C5's scene (Kerr a = 0.99, RKF45, no disk) on a 192x108 camera-B frame."""
    c = configs.CONFIGS["C5"]
    bh, dk, cfg = c.scene()
    cfg.tolerance = tol
    cam = configs.camera("B")
    W, H = 192, 108
    bhrt_lib.stats(reset=True)
    got = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    st = bhrt_lib.stats(reset=True)  # (bench.py credits untested attempts 27 ops, not 54)
    assert st["iterations"] > 0
    assert st["attempts_untested"] == (st["iterations"] if tol >= 2.0**-30 else 0), st
    monkeypatch.setenv("BHRT_ACCEPT_ALL", "0")
    tested = bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    st = bhrt_lib.stats(reset=True)
    assert st["iterations"] > 0 and st["attempts_untested"] == 0, st
    for f in abi.SOA_FIELDS:
        assert np.array_equal(got[f], tested[f], equal_nan=True), f
    want = oracle.render_frame(bh, dk, cfg, cam, W, H, c.method, c.flags)
    compare(got, want, RTOL, True, f"C5 tol={tol}")


def test_wrong_no_evict_proof_is_reported(bhrt_lib, monkeypatch):
    """the redo launch is left out where the host proves that no ray can be evicted
    (origin_no_evict). If that proof were wrong for a scene, the evicted rays must not keep
    stale outputs silently: k_trace marks them RAY_ERROR and the next harvest (bhrt_get_stats)
    fails with the count. Forced here with the test knob BHRT_ASSUME_NO_EVICT on a scene that
    hands every ray over (M = 1e-3: the far-field bound is unprovable,
    test_unbounded_far_field_launch_takes_the_redo_path)."""
    cam = configs.camera("B")
    dk = abi.disk(0.006, 0.04, 1.0, 1.0)
    bh = abi.black_hole(1.0e-3, 0.0)
    cfg = abi.sim_config(0.1, 100.0, 300, 1e-6)
    bhrt_lib.stats(reset=True)
    monkeypatch.setenv("BHRT_ASSUME_NO_EVICT", "1")
    got = bhrt_lib.render_frame(bh, dk, cfg, cam, 40, 24, abi.INTEGRATOR_RK4, 0)
    assert (got["result"] == abi.RAY_ERROR).all(), np.unique(got["result"])
    with pytest.raises(bhrt_lib.BhrtError, match="redo pass"):
        bhrt_lib.stats(reset=True)
    monkeypatch.delenv("BHRT_ASSUME_NO_EVICT")
    assert bhrt_lib.stats(reset=True)["launches"] == 0  # (the error is reported once)
    got = bhrt_lib.render_frame(bh, dk, cfg, cam, 40, 24, abi.INTEGRATOR_RK4, 0)
    assert not (got["result"] == abi.RAY_ERROR).any()
    assert bhrt_lib.stats(reset=True)["rays_redone"] == 40 * 24


@pytest.mark.parametrize("cname", ["C1", "C2", "C3", "C4", "C5"])
def test_full_frame_every_ray_vs_oracle(bhrt_lib, oracle, cname):
    """Every ray of the frame bench.py renders at N = 1 (camera B) against the oracle: C1
    256x256, C2 and C3 1920x1080, C4 3840x2160 (8.3 M rays), C5 shard 0 of the 7680x4320
    frame (540 rows, 4.1 M rays). Classes and steps exact, floats within 1e-5, NaN pattern; a
    mismatch is allowed only on a listed knife-edge ray (oracle margin to a threshold < 1e-9,
    SURVEY.md 7(f)). tools/full_frame_parity.py also runs the other seven C5 shards."""
    import torch
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    plan = c.frame(1) if cname != "C5" else c.frame(8)
    W, H = plan.width, plan.height
    rows = plan.rows(0)
    n = W * (H if rows is None else bhrt_lib.shard_rows(H, rows))
    # The outputs are filled on torch's default stream (the legacy null stream) behind a busy
    # kernel, rendered with hip_stream NULL and read back on the default stream, with no host
    # sync anywhere: NULL orders the frame after the fills and before the reads (null_fence,
    # bhrt_api.c). Round 5 needed a torch.cuda.synchronize() on each side (a fill still queued
    # behind the trace kernel overwrote 3.37 M rays of C5's frame).
    t = _default_stream_filled_outputs(torch, n)
    bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, rows, c.method, c.flags,
                                 bhrt_lib.soa_from_tensors(t), None)
    got = {f: v.cpu().numpy() for f, v in t.items()}
    del t
    want, margin = oracle.render_frame_margin(bh, dk, cfg, cam, W, H, c.method, c.flags,
                                              rows=rows, threads=16)
    rep = full_frame_report(got, want, margin, sky_pinned(c.method))
    print(cname, {k: rep[k] for k in ("rays", "mismatched_rays", "knife_edge_rays",
                                      "min_margin", "max_rel_err_on_matching_rays")})
    assert rep["unexplained"] == 0, rep
    assert rep["rays"] == n


def test_frames_with_freed_arrays_and_pageable_copies(bhrt_lib, monkeypatch):
    """A render loop that reallocates: every frame's caller arrays are freed right after the
    frame (some carved out of one allocation at odd offsets, some small enough to come from
    the heap next to other allocations), two frames in flight, and after every frame pageable
    torch D2H copies and heap allocations that re-use the freed memory. libbhrt never
    page-locks caller memory (the registered path and its faults were
    removed in round 3); every frame must equal the device frame and every pageable copy its
    source."""
    import torch
    L = bhrt_lib.load()
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    cams = [configs.camera("B"), configs.camera("A")]
    W, H = 768, 432  # 332 k rays, 32 MB of fields, 2 chunks
    refs = []
    for cam in cams:
        t = {f: torch.zeros(W * H, dtype=torch.int32 if f in ("result", "steps") else
                            torch.float64, device="cuda") for f in abi.SOA_FIELDS}
        torch.cuda.synchronize()  # (torch fills on its stream, libbhrt renders on its own)
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     bhrt_lib.soa_from_tensors(t), 0)
        torch.cuda.synchronize()
        refs.append({f: v.cpu().numpy() for f, v in t.items()})
    src = torch.arange(1 << 20, dtype=torch.float64, device="cuda")
    for it in range(6):
        junk = [np.full(777 + 13 * k, k, dtype=np.uint8) for k in range(64)]  # heap neighbours
        sets = []
        for j in range(2):
            if (it + j) % 2:
                buf, arrays, soa = _frame_soa_in_one_buffer(W * H, abi.SOA_FIELDS,
                                                            offset=(1000 * it + 24 * j) % 4096)
            else:
                buf = None
                arrays, soa = abi.alloc_soa(W * H)
            sets.append((buf, arrays, soa))
        tickets = []
        for j, (_, _, soa) in enumerate(sets):
            t = C.c_int(0)
            cam = cams[j]
            assert L.bhrt_render_frame_async(C.byref(bh), C.byref(dk), C.byref(cfg),
                                             C.byref(cam), W, H, c.method, c.flags,
                                             C.byref(soa), C.byref(t)) == 0, bhrt_lib.last_error()
            tickets.append(t.value)
        for t in tickets:
            assert L.bhrt_frame_wait(t) == 0, bhrt_lib.last_error()
        for j, (_, arrays, _) in enumerate(sets):
            for f in abi.SOA_FIELDS:
                assert np.array_equal(arrays[f], refs[j][f], equal_nan=True), (it, j, f)
        del sets, arrays, soa, buf
        for k in range(8):  # pageable copies into freshly allocated (recycled) host memory
            n = (1 << 12) << k
            host = src[:n].cpu()
            assert host[-1].item() == n - 1 and bool((host[:7] == src[:7].cpu()).all())
        del junk


def test_small_claimed_launches(bhrt_lib, oracle):
    """Launches of a few workgroups on the block-claim paths (Kerr / RKF45 scenes: claim_div
    1): the claim-size shift is computed for grids smaller than the queue count too."""
    g = golden("rays_rkf45_kerr")
    bh, dk, cfg = scene_from(g)
    rays = rays_from(g)
    for n in (1, 3, 64, 65, 700):
        sub = np.resize(rays, n)
        got = bhrt_lib.trace_rays(sub, bh, dk, cfg, int(g["method"]), int(g["flags"]))
        want = oracle.trace_rays(sub, bh, dk, cfg, int(g["method"]), int(g["flags"]))
        compare(got, want, RTOL, sky_pinned(g["method"]), f"n={n}")
    c = configs.CONFIGS["C4"]
    bh, dk, cfg = c.scene()
    for W, H in ((4, 3), (40, 17)):
        got = bhrt_lib.render_frame(bh, dk, cfg, configs.camera("B"), W, H, c.method, c.flags)
        want = oracle.render_frame(bh, dk, cfg, configs.camera("B"), W, H, c.method, c.flags)
        compare(got, want, RTOL, False, f"C4 {W}x{H}")


@pytest.mark.parametrize("n,weights", [
    (65536, None), (300_001, None), ((1 << 20) + 7, None),
    (2_073_600, None),  # the default weighted plan (>= 1 M rays per device)
    (300_001, "1,1,1,1"), (300_001, "2,5,5,3,1"), (1 << 17, "1,2,3,4,5,6,7,8")])
def test_large_batch_pipelined_equals_soa_trace(bhrt_lib, monkeypatch, n, weights):
    """trace_rays_batch at n >= 65536 takes the chunked path (rays staged through pinned
    memory, chunks on two trace streams, results packed into RayTraceHit[] by OpenMP
    threads): every hit must equal the one-shot SoA trace of the same rays, and sky_direction
    must stay untouched for rays that did not escape (raytracer.c:299-333). Chunk plans
    (BHRT_BATCH_WEIGHTS) change how rays are dealt over chunks, never the results."""
    if weights:
        monkeypatch.setenv("BHRT_BATCH_WEIGHTS", weights)
    rng = np.random.default_rng(n)
    bh, dk, cfg = configs.CONFIGS["C2"].scene()
    rays = np.zeros(n, dtype=abi.RAY_DTYPE)
    rays["origin"] = (0.0, 2.0, -30.0)
    d = rng.normal(size=(n, 3)) * (0.25, 0.25, 1.0) + (0.0, 0.0, 1.0)
    rays["direction"] = d / np.linalg.norm(d, axis=1, keepdims=True)
    ref = bhrt_lib.trace_rays(rays, bh, dk, cfg)
    rc, hits = bhrt_lib.trace_rays_batch(rays, bh, dk, cfg)
    assert rc == 0
    assert np.array_equal(hits["result"], ref["result"])
    assert np.array_equal(hits["steps"], ref["steps"])
    for i, ax in enumerate("xyz"):
        assert np.array_equal(hits["hit_position"][:, i], ref["hit_" + ax], equal_nan=True)
    assert np.array_equal(hits["distance"], ref["distance"], equal_nan=True)
    assert np.array_equal(hits["time_dilation"], ref["time_dilation"], equal_nan=True)
    esc = hits["result"] == abi.RAY_MAX_DISTANCE
    assert esc.any() and (~esc).any()
    for i, ax in enumerate("xyz"):
        assert np.array_equal(hits["sky_direction"][esc, i], ref["sky_" + ax][esc])
    assert not hits["sky_direction"][~esc].any()


@pytest.mark.parametrize("cname", ["C1", "C2", "C3", "C4", "C5"])
def test_shared_origin_ray_arrays_vs_oracle(bhrt_lib, oracle, monkeypatch, cname):
    """Ray arrays whose rays all start at one point (a camera's rays passed as Ray[]: the
    visualizer's trace_rays_batch) are set up inside the trace kernel from the host's origin
    block, as camera frames are (kparams.rays_shared; C1 keeps the set-up pass, with the
    far-field decision from the host): every ray against the oracle, through the one-launch
    path and the pipelined trace_rays_batch, which must agree bit for bit; with
    BHRT_SHARED_ORIGIN=0 (the per-ray k_init table) the same rays agree with the oracle too."""
    c = configs.CONFIGS[cname]
    bh, dk, cfg = c.scene()
    W, H = 96, 64
    rays = configs.camera_rays(configs.camera("B"), W, H)
    want = oracle.trace_rays(rays, bh, dk, cfg, c.method, c.flags)
    got = bhrt_lib.trace_rays(rays, bh, dk, cfg, c.method, c.flags)
    compare(got, want, RTOL, sky_pinned(c.method), f"{cname} shared origin")
    if c.method == abi.INTEGRATOR_RK4:  # trace_rays_batch is RK4 (trace_ray's integrator)
        big = np.resize(rays, 1 << 16)  # >= 65536 rays: the pipelined chunks
        ref = bhrt_lib.trace_rays(big, bh, dk, cfg)
        rc, hits = bhrt_lib.trace_rays_batch(big, bh, dk, cfg)
        assert rc == 0
        assert np.array_equal(hits["result"], ref["result"])
        assert np.array_equal(hits["steps"], ref["steps"])
        for i, ax in enumerate("xyz"):
            assert np.array_equal(hits["hit_position"][:, i], ref["hit_" + ax], equal_nan=True)
        assert np.array_equal(hits["distance"], ref["distance"], equal_nan=True)
    monkeypatch.setenv("BHRT_SHARED_ORIGIN", "0")
    gen = bhrt_lib.trace_rays(rays, bh, dk, cfg, c.method, c.flags)
    compare(gen, want, RTOL, sky_pinned(c.method), f"{cname} per-ray set-up")
    # The two set-ups of the same ray: the shared one takes the origin's angles and
    # their sin/cos from the host's glibc (the reference's own values), the per-ray one from the
    # device's libm, so a ray's low-order bits can depend on whether every ray of its chunk
    # shares its origin. Bound that: classes and steps equal, floats within 1e-9 relative
    # (observed: a few ulp).
    for f in ("result", "steps"):
        assert np.array_equal(got[f], gen[f]), f
    for f in ("hit_x", "hit_y", "hit_z", "distance", "time_dilation"):
        a, b = got[f], gen[f]
        ok = ~(np.isnan(a) | np.isnan(b))
        assert np.array_equal(np.isnan(a), np.isnan(b)), f
        rel = np.abs(a[ok] - b[ok]) / np.maximum(np.abs(b[ok]), 1e-300)
        assert rel.size == 0 or float(rel.max()) <= 1e-9, (f, float(rel.max()))


def test_torch_after_libbhrt_in_a_fresh_process():
    """A process that loads libbhrt before it first uses torch on the GPU still has ONE HIP
    runtime (bhrt.lib imports torch before mapping libbhrt: torch's bundled libamdhip64 then
    serves both), so torch's device initialisation works and its buffers go to libbhrt."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from bhrt import lib\n"
            "assert lib.load().bhrt_device_count() > 0\n"
            "import torch\n"
            "t = torch.zeros(8, device='cuda'); torch.cuda.synchronize(); print('ok', t.sum().item())\n"
            % str(os.path.join(ROOT, "raytracing-engine-in-c_amd")))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "ok 0.0" in r.stdout, r.stderr[-2000:]


def test_rkf45_accept_band(bhrt_lib):
    """The trace kernel's RKF45 accept test (geodesic.hip rkf45_accept): the
    division-free fast form -- q = err * rcp(scale) decides outside a +-2^-40 band around
    tol, the IEEE quotient inside it -- must make the reference's decision
    RN(max_i RN(err_i / scale_i) / tol) <= 1 (math_util.c:376-405) exactly, including
    quotients landing ON tol, one ulp either side, on and around the band's edges, several
    components in the band at once, and the literal path's tolerances (0, subnormal, Inf,
    NaN, negative). Operands are run through the kernel's own device code
    (bhrt_check_rkf45_accept) and checked against numpy's IEEE division."""
    import torch
    L = bhrt_lib.load()
    L.bhrt_check_rkf45_accept.restype = C.c_int
    L.bhrt_check_rkf45_accept.argtypes = [C.c_void_p] * 3 + [C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(45)
    errs, scales, tols = [], [], []
    rel = [0.0, 2.0 ** -40, -2.0 ** -40, 2.0 ** -41, -2.0 ** -41, 2.0 ** -39, -2.0 ** -39,
           2.0 ** -52, -2.0 ** -52, 1e-9, -1e-9]
    for _ in range(4000):
        tol = 10.0 ** rng.uniform(-12, -3)
        if rng.random() < 0.2:
            tol = rng.choice([1e-6, 1e-8])
        scale = np.full(6, 10.0 ** rng.uniform(-10, 3))
        scale[rng.random(6) < 0.2] = 1e-10  # BH_EPSILON floor
        scale *= rng.uniform(1, 2, 6)
        err = tol * scale * 10.0 ** rng.uniform(-6, -1, 6)  # clearly accepted components
        for c in rng.choice(6, size=rng.integers(1, 4), replace=False):
            q = tol * (1.0 + rng.choice(rel))
            e = q * scale[c]
            for _ in range(int(rng.integers(-3, 4))):  # nudge a few ulps either way
                e = np.nextafter(e, np.inf if rng.random() < 0.5 else 0.0)
            err[c] = e
        errs.append(err)
        scales.append(scale)
        tols.append(tol)
    for t in (0.0, 5e-324, np.inf, np.nan, -1e-6, 2.2250738585072014e-308):  # literal path
        for big in (0.0, np.inf):
            err = np.full(6, 1e-20)
            err[0] = big
            errs.append(err)
            scales.append(np.ones(6))
            tols.append(t)
    E, S, T = np.array(errs), np.array(scales), np.array(tols)
    n = len(T)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (E.ravel(), S.ravel(), T)]
    out = torch.zeros(2 * n, dtype=torch.int32, device="cuda")
    assert L.bhrt_check_rkf45_accept(*(d.data_ptr() for d in dev), n, out.data_ptr(),
                                     C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().reshape(n, 2)
    with np.errstate(invalid="ignore", divide="ignore"):
        max_err = np.max(E / S, axis=1)
        want = (max_err / T) <= 1.0
    assert np.array_equal(got[:, 1], want.astype(np.int32)), "literal form vs numpy"
    assert np.array_equal(got[:, 0], want.astype(np.int32)), np.nonzero(got[:, 0] != want)[0][:10]
    near = np.abs(max_err / T - 1.0) <= 2.0 ** -39
    assert near.sum() > 1000 and want[near].any() and (~want[near]).any()  # the band was hit


# Small frames of every config, and cameras A / V; "FAR" is C2's scene at M = 0.5 (15 rs = 15,
# so camera B's origin lies beyond it: the far-field instantiations, and long rays whose
# state[0] -- read as r by ray_derivatives -- passes 15 rs, so stages take either branch)
STAGE_CASES = [("C1", "B", 64, 48), ("C2", "B", 96, 54), ("C2", "V", 96, 54), ("C2", "A", 64, 36),
               ("C3", "B", 96, 54), ("C3", "V", 64, 36), ("C4", "B", 128, 72), ("C4", "V", 96, 54),
               ("C5", "B", 128, 72), ("FAR", "B", 64, 36)]


def _stage_scene(cname):
    """(bh, disk, cfg, method, flags) of a STAGE_CASES entry"""
    if cname == "FAR":
        return (abi.black_hole(0.5, 0.0), abi.disk(3.0, 20.0, 1.0, 1.0),
                abi.sim_config(0.1, 100.0, 1000, 1e-6), abi.INTEGRATOR_RK4, 0)
    c = configs.CONFIGS[cname]
    return (*c.scene(), c.method, c.flags)


_COUNT_CHILD = r"""
import json, sys
sys.path.insert(0, sys.argv[1])
sys.path.insert(0, sys.argv[2])
from bhrt import configs, lib
from test_gpu_parity import _stage_scene
out = []
for cname, camname, W, H in json.loads(sys.argv[3]):
    bh, dk, cfg, method, flags = _stage_scene(cname)
    lib.stats(reset=True)
    f = lib.render_frame(bh, dk, cfg, configs.camera(camname), W, H, method, flags)
    st = lib.stats(reset=True)
    out.append({"stats": {k: st[k] for k in ("rays", "iterations", "stages_full", "stages_far",
                                             "stages_kerr")},
                "frame": {k: v.tobytes().hex() for k, v in f.items()}})
print(json.dumps(out))
"""


def test_stage_counts_are_counted(bhrt_lib):
    """bench.py's FLOP credit (roofline.flops_per_launch) is computed from the kernel's stage
    counters, and the hot instantiations DERIVE the per-branch split from the iterations
    (iterations x 4 or 6, minus the far-field stages, which are counted). The stage-counting
    build (diag/libbhrt_count.so, BHRT_COUNT_STAGES: every stage's branch counted one by one, as
    the redo pass does) must give the same rays, iterations and a=0 / far-field / Kerr stage
    counts on every config -- and the same frame bit for bit (counting changes no arithmetic)."""
    import json
    import subprocess
    import sys
    lib_count = os.path.join(ROOT, "raytracing-engine-in-c_amd", "diag", "libbhrt_count.so")
    assert os.path.exists(lib_count), "diag/libbhrt_count.so not built (__graft_entry__.build())"
    env = dict(os.environ, BHRT_LIB=lib_count)
    r = subprocess.run([sys.executable, "-c", _COUNT_CHILD,
                        os.path.join(ROOT, "raytracing-engine-in-c_amd"),
                        os.path.join(ROOT, "tests"), json.dumps(STAGE_CASES)],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    counted = json.loads(r.stdout.strip().splitlines()[-1])
    for (cname, camname, W, H), cnt in zip(STAGE_CASES, counted):
        bh, dk, cfg, method, flags = _stage_scene(cname)
        bhrt_lib.stats(reset=True)
        f = bhrt_lib.render_frame(bh, dk, cfg, configs.camera(camname), W, H, method, flags)
        st = bhrt_lib.stats(reset=True)
        what = f"{cname}/{camname} {W}x{H}"
        derived = {k: st[k] for k in cnt["stats"]}
        assert derived == cnt["stats"], (what, derived, cnt["stats"])
        per_stage = 4 if method == abi.INTEGRATOR_RK4 else 6
        assert sum(st[k] for k in ("stages_full", "stages_far", "stages_kerr")) == \
            per_stage * st["iterations"], what
        for k, v in f.items():
            assert v.tobytes().hex() == cnt["frame"][k], (what, k)
    # the far-field scene takes both branches (a real split, not one branch for all)
    far = counted[STAGE_CASES.index(("FAR", "B", 64, 36))]["stats"]
    assert far["stages_far"] > 0 and far["stages_full"] > 0, far


@pytest.mark.parametrize("cname,camname,W,H", STAGE_CASES)
def test_redo_pass_left_out_where_no_ray_can_need_it(bhrt_lib, monkeypatch, cname, camname, W,
                                                     H):
    """bhrt_api.c origin_no_evict proves from the scene and the shared origin that no ray of a
    camera frame can be handed to the redo pass, and the launcher then leaves that launch out
     -- on every BASELINE frame (camera B); the bound is conservative, so a
    scene it cannot prove (RKF45 from camera V's far origin) keeps the launch. With the launch
    forced back (BHRT_SKIP_REDO=0) it must find nothing to re-trace, and the frame must be the
    same bit for bit; a ray array with one shared origin is proved the same way, an array of
    distinct origins is not."""
    bh, dk, cfg, method, flags = _stage_scene(cname)
    cam = configs.camera(camname)
    frames = []
    skipped = None
    for skip in ("1", "0"):
        monkeypatch.setenv("BHRT_SKIP_REDO", skip)
        bhrt_lib.stats(reset=True)
        frames.append(bhrt_lib.render_frame(bh, dk, cfg, cam, W, H, method, flags))
        st = bhrt_lib.stats(reset=True)
        assert st["rays_redone"] == 0, (skip, st)
        if skip == "1":
            skipped = st["redo_launches"] == 0
            assert skipped or st["redo_launches"] == st["launches"], st
        else:
            assert st["redo_launches"] == st["launches"], st
    if camname == "B":
        assert skipped, f"{cname}: the BASELINE frame should be proved eviction-free"
    for k in frames[0]:
        assert np.array_equal(frames[0][k], frames[1][k], equal_nan=True), k
    monkeypatch.setenv("BHRT_SKIP_REDO", "1")
    rays = configs.camera_rays(cam, W, H)
    bhrt_lib.stats(reset=True)
    bhrt_lib.trace_rays(rays, bh, dk, cfg, method, flags)
    st = bhrt_lib.stats(reset=True)
    assert st["redo_launches"] == (0 if skipped else st["launches"]), st
    rays["origin"][1::2, 0] += 1e-3  # two origins: per-ray set-up, not provable here
    bhrt_lib.stats(reset=True)
    bhrt_lib.trace_rays(rays, bh, dk, cfg, method, flags)
    st = bhrt_lib.stats(reset=True)
    assert st["redo_launches"] == st["launches"] > 0, st


def test_control_ring_wraps(bhrt_lib):
    """600 device frames back to back on one stream, no sync between them: the launch that
    finds the thread's control ring full (256 slots, bhrt_api.c BHRT_RING) harvests it and
    zeroes it, twice here. Every frame must be the first one bit for bit (a slot reused
    without its queue heads zeroed would skip rays) and the statistics must count every launch
    once; a discarding reset (bhrt_get_stats(NULL, 1)) drops pending launches unread."""
    import torch
    c = configs.CONFIGS["C2"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H, frames = 16, 16, 600
    n = W * H

    def bufs():
        return {f: torch.full((n,), 7, dtype=torch.int32 if f in ("result", "steps") else
                              torch.float64, device="cuda") for f in abi.SOA_FIELDS}

    first = bufs()
    torch.cuda.synchronize()
    bhrt_lib.stats(reset=True)
    bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                 bhrt_lib.soa_from_tensors(first), None)
    torch.cuda.synchronize()
    one = bhrt_lib.stats(reset=True)
    assert one["launches"] == 1 and one["rays"] == n, one
    ring = [bufs() for _ in range(3)]
    torch.cuda.synchronize()
    soas = [bhrt_lib.soa_from_tensors(b) for b in ring]
    for k in range(frames):
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     soas[k % 3], None)
    torch.cuda.synchronize()
    st = bhrt_lib.stats(reset=True)
    assert st["launches"] == frames and st["rays"] == frames * n, st
    assert st["iterations"] == frames * one["iterations"], (st, one)
    for b in ring:
        for f in abi.SOA_FIELDS:
            assert torch.equal(b[f], first[f]) or (
                b[f].dtype == torch.float64 and
                torch.equal(torch.isnan(b[f]), torch.isnan(first[f])) and
                torch.equal(b[f].nan_to_num(0.0), first[f].nan_to_num(0.0))), f
    for k in range(5):
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     soas[k % 3], None)
    bhrt_lib.stats_discard()
    st = bhrt_lib.stats(reset=True)
    assert st["launches"] == 0 and st["rays"] == 0, st


@pytest.mark.gpu
def test_control_ring_wraps_across_streams(bhrt_lib):
    """The ring-full launch harvests the older half of the control ring only and reuses it
    (bhrt_api.c harvest): 700 frames rotating over three caller streams, no sync between them,
    so the refilled half is zeroed on one stream while the newer half's frames still run on the
    others, and every stream's first launch after the fill waits for it. Every frame must equal
    the first bit for bit and the statistics must count every launch once."""
    import torch
    c = configs.CONFIGS["C4"]
    bh, dk, cfg = c.scene()
    cam = configs.camera("B")
    W, H, frames = 16, 16, 700
    n = W * H

    def bufs():
        return {f: torch.full((n,), 7, dtype=torch.int32 if f in ("result", "steps") else
                              torch.float64, device="cuda") for f in abi.SOA_FIELDS}

    first = bufs()
    torch.cuda.synchronize()
    bhrt_lib.stats(reset=True)
    bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                 bhrt_lib.soa_from_tensors(first), None)
    torch.cuda.synchronize()
    one = bhrt_lib.stats(reset=True)
    assert one["launches"] == 1 and one["rays"] == n, one
    streams = [torch.cuda.Stream() for _ in range(3)]
    ring = [bufs() for _ in range(3)]
    torch.cuda.synchronize()
    soas = [bhrt_lib.soa_from_tensors(b) for b in ring]
    for k in range(frames):
        s = streams[k % 3]
        bhrt_lib.render_frame_device(bh, dk, cfg, cam, W, H, None, c.method, c.flags,
                                     soas[k % 3], s.cuda_stream)
    torch.cuda.synchronize()
    st = bhrt_lib.stats(reset=True)
    assert st["launches"] == frames and st["rays"] == frames * n, st
    assert st["iterations"] == frames * one["iterations"], (st, one)
    for b in ring:
        for f in abi.SOA_FIELDS:
            assert torch.equal(b[f], first[f]) or (
                b[f].dtype == torch.float64 and
                torch.equal(torch.isnan(b[f]), torch.isnan(first[f])) and
                torch.equal(b[f].nan_to_num(0.0), first[f].nan_to_num(0.0))), f
