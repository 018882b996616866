"""The C ABI of libbhrt.so, checked without a GPU: it loads, exports every symbol declared
in include/*.h, keeps the reference's struct layouts and argument checks, its host-side
scalar helpers agree bit-for-bit with the reference, and the GPU entry points fail loudly
(no CPU fallback) when there is no HIP device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden, gpu_available
from bhrt import abi, lib

HEADERS = [os.path.join(ROOT, "include", h) for h in ("bhrt_api.h",)]


def declared_functions():
    names = []
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        src = re.sub(r"typedef[^;]*;", "", src)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(([^;{]*)\)\s*;", src):
            name = m.group(1)
            if name not in ("if", "sizeof", "BHRT_STATIC_ASSERT"):
                names.append(name)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    L = lib.load()
    names = declared_functions()
    assert len(names) >= 45, names
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_reference_entry_points_are_declared():
    """The drop-in set: the reference's WASM export list (Makefile:47, ray part) plus the
    ray tracer API of raytracer.h."""
    names = set(declared_functions())
    for n in ("bh_initialize", "bh_shutdown", "bh_configure_black_hole",
              "bh_configure_accretion_disk", "bh_configure_simulation", "bh_trace_ray",
              "bh_trace_rays_batch", "bh_calculate_time_dilation", "bh_get_version",
              "trace_ray", "trace_rays_batch", "integrate_photon_path", "trace_pixel",
              "check_disk_intersection", "calculate_disk_temperature",
              "apply_relativistic_effects", "halton_sequence", "generate_gpu_shader_params"):
        assert n in names, n


def test_struct_layouts():
    assert C.sizeof(abi.FrameSoA) == 15 * 8  # 13 per-ray fields + 2 display fields
    assert abi.FrameSoA.rgba8.offset == 14 * 8
    assert C.sizeof(abi.RayTraceHit) == 160 == abi.HIT_DTYPE.itemsize
    assert C.sizeof(abi.Ray) == 48 == abi.RAY_DTYPE.itemsize
    assert C.sizeof(abi.SimulationConfig) == 72
    assert abi.SimulationConfig.tolerance.offset == 24
    assert abi.RayTraceHit.sky_direction.offset == 80
    assert abi.RayTraceHit.color.offset == 120


def test_host_helpers_match_reference():
    """Scalar helpers of the ray path exported by libbhrt (host C) vs the reference."""
    L = lib.load()
    g = golden("shading")
    for t, want in zip(g["t2rgb_in"], g["t2rgb_out"]):
        o = (C.c_double * 3)()
        L.temperature_to_rgb(float(t), C.byref(o))
        np.testing.assert_array_equal(list(o), want)
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    for p, v, w_t, w_rel in zip(g["disk_pos"], g["disk_vel"], g["disk_temp_out"],
                                g["relativistic_out"]):
        T = C.c_double()
        col = (C.c_double * 3)()
        L.calculate_disk_temperature(C.byref(abi.v3(*p)), C.byref(bh), C.byref(dk), C.byref(T),
                                     C.byref(col))
        np.testing.assert_array_equal([T.value] + list(col), w_t)
        dop = C.c_double()
        L.apply_relativistic_effects(C.byref(abi.v3(*p)), C.byref(abi.v3(*v)), C.byref(bh),
                                     C.byref(col), C.byref(dop))
        np.testing.assert_array_equal(list(col) + [dop.value], w_rel)
    for i, b, want in g["halton"]:
        assert L.halton_sequence(int(i), int(b)) == want
    for s, want in zip(g["bh_spins"], g["bh_params"]):
        bhp = abi.BlackHoleParams()
        L.initialize_black_hole_params(C.byref(bhp), 1.0, float(s), 0.0)
        np.testing.assert_array_equal([getattr(bhp, f) for f, _ in bhp._fields_], want)
    for row, want in zip(g["cdi_in"], g["cdi_out"]):
        q = abi.Vector3D()
        h = L.check_disk_intersection(C.byref(abi.v3(*row[0:3])), C.byref(abi.v3(*row[3:6])),
                                      C.byref(abi.v3(*row[6:9])), C.byref(dk), C.byref(q))
        np.testing.assert_array_equal([h, q.x, q.y, q.z] if h else [0, 0, 0, 0], want)
    L2 = C.CDLL(lib.LIB_PATH)
    L2.cartesian_to_spherical.argtypes = [C.c_void_p, C.c_void_p]
    L2.spherical_to_cartesian.argtypes = [C.c_void_p, C.c_void_p]
    for p, w1, w2 in zip(g["cs_in"], g["c2s_out"], g["s2c_out"]):
        o, o2 = abi.Vector3D(), abi.Vector3D()
        L2.cartesian_to_spherical(C.byref(abi.v3(*p)), C.byref(o))
        L2.spherical_to_cartesian(C.byref(o), C.byref(o2))
        np.testing.assert_array_equal([o.x, o.y, o.z], w1)
        np.testing.assert_array_equal([o2.x, o2.y, o2.z], w2)


def test_context_api_validation():
    """bh_* return codes (blackhole_api.c:100-176, 188-190, 231-233, 464-476)."""
    L = lib.load()
    ctx = L.bh_initialize()
    assert ctx
    try:
        assert L.bh_configure_black_hole(ctx, 0.0, 0.0, 0.0) == -1
        assert L.bh_configure_black_hole(ctx, 1.0, -0.1, 0.0) == -1
        assert L.bh_configure_black_hole(ctx, 1.0, 1.1, 0.0) == -1
        assert L.bh_configure_black_hole(ctx, 1.0, 0.5, 0.0) == 0
        assert L.bh_configure_accretion_disk(ctx, 6.0, 6.0, 1.0, 1.0) == -1
        assert L.bh_configure_accretion_disk(ctx, -1.0, 20.0, 1.0, 1.0) == -1
        assert L.bh_configure_accretion_disk(ctx, 6.0, 20.0, 0.0, 1.0) == -1
        assert L.bh_configure_accretion_disk(ctx, 6.0, 20.0, 1.0, 1.0) == 0
        assert L.bh_configure_simulation(ctx, 0.0, 100.0, 1000, 1e-6) == -1
        assert L.bh_configure_simulation(ctx, 0.1, 100.0, 0, 1e-6) == -1
        assert L.bh_configure_simulation(ctx, 0.1, 100.0, 1000, 0.0) == -1
        assert L.bh_configure_simulation(ctx, 0.1, 100.0, 1000, 1e-6) == 0
        assert L.bh_trace_rays_batch(ctx, None, None, 5) == -1
        assert L.bh_trace_ray(None, None, None, None) == -1
        r = C.c_double()
        p1, p2 = (C.c_double * 3)(10, 0, 0), (C.c_double * 3)(0, 20, 0)
        assert L.bh_calculate_time_dilation(ctx, C.byref(p1), C.byref(p2), C.byref(r)) == 0
        want = (1.0 / np.sqrt(1.0 - 2.0 / 10.0)) / (1.0 / np.sqrt(1.0 - 2.0 / 20.0))
        assert r.value == want
    finally:
        L.bh_shutdown(ctx)
    a, b, c = C.c_int(), C.c_int(), C.c_int()
    L.bh_get_version(C.byref(a), C.byref(b), C.byref(c))
    assert (a.value, b.value, c.value) == (0, 1, 0)


def test_batch_argument_checks():
    """trace_rays_batch returns -1 for NULL rays/blackhole/hits or num_rays <= 0
    (raytracer.c:791-793), before touching any device."""
    L = lib.load()
    bh, cfg = abi.black_hole(), abi.sim_config()
    rays = np.zeros(4, dtype=abi.RAY_DTYPE)
    hits = np.zeros(4, dtype=abi.HIT_DTYPE)
    assert L.trace_rays_batch(None, 4, C.byref(bh), None, C.byref(cfg), hits.ctypes.data, 0) == -1
    assert L.trace_rays_batch(rays.ctypes.data, 0, C.byref(bh), None, C.byref(cfg), hits.ctypes.data, 0) == -1
    assert L.trace_rays_batch(rays.ctypes.data, -3, C.byref(bh), None, C.byref(cfg), hits.ctypes.data, 0) == -1
    assert L.trace_rays_batch(rays.ctypes.data, 4, None, None, C.byref(cfg), hits.ctypes.data, 0) == -1
    assert L.trace_rays_batch(rays.ctypes.data, 4, C.byref(bh), None, C.byref(cfg), None, 0) == -1


def test_shard_rows_partition():
    """Cyclic row blocks: every image row belongs to exactly one shard."""
    for H in (1, 7, 64, 1080, 2160, 4320):
        for N in (1, 2, 3, 4, 8):
            for B in (1, 8, 16):
                seen = []
                for s in range(N):
                    rows = abi.Rows(B, s, N)
                    n = lib.shard_rows(H, rows)
                    for j in range(n):
                        seen.append(((j // B) * N + s) * B + j % B)
                assert sorted(seen) == list(range(H)), (H, N, B)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback_without_gpu():
    """On a machine without a HIP device the tracer must fail loudly, not compute on the CPU."""
    L = lib.load()
    bh, cfg = abi.black_hole(), abi.sim_config()
    rays = np.zeros(2, dtype=abi.RAY_DTYPE)
    rays["origin"] = (0, 0, 30)
    rays["direction"] = (0, 0, -1)
    hits = np.zeros(2, dtype=abi.HIT_DTYPE)
    assert L.trace_rays_batch(rays.ctypes.data, 2, C.byref(bh), None, C.byref(cfg),
                              hits.ctypes.data, 0) == -1
    assert (hits["result"] == abi.RAY_ERROR).all()
    assert lib.last_error()
    with pytest.raises(lib.BhrtError):
        lib.render_frame(bh, None, cfg, abi.Camera(abi.v3(0, 0, 30), abi.v3(0, 0, -1),
                                                   abi.v3(0, 1, 0), 60.0), 4, 4)


def build_c_demo(tmp_path):
    """Compile examples/trace_demo.c, a C caller written against the reference's header
    names (include/blackhole_api.h etc. forward to bhrt_api.h), and link it to libbhrt.so."""
    import subprocess
    exe = str(tmp_path / "trace_demo")
    path = os.path.abspath(lib.LIB_PATH)  # BHRT_LIB may name an A/B build (ab/libbhrt_*.so)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "trace_demo.c"), path,
                    f"-Wl,-rpath,{os.path.dirname(path)}", "-lm", "-o", exe], check=True)
    return exe


def test_c_demo_links_against_drop_in_headers(tmp_path):
    assert os.path.exists(build_c_demo(tmp_path))


def test_shader_data_matches_reference():
    """bh_generate_shader_data (blackhole_api.c:495-608) writes the reference's 124-byte
    parameter block bit for bit (tests/golden/shader_data.npz, from the compiled reference)
    over 120 context / argument combinations, leaves the 32nd word alone, and rejects NULL
    arguments with the reference's code."""
    L = lib.load()
    V, I, D, F = C.c_void_p, C.c_int, C.c_double, C.c_float
    L.bh_generate_shader_data.argtypes = [V, V, V, V, I, I, F, I, I, I, V]
    L.bh_generate_shader_data.restype = I
    g = golden("shader_data")
    for ctx_in, call, vec, want, rc in zip(g["ctx"], g["call"], g["vecs"], g["out"], g["rc"]):
        ctx = L.bh_initialize()
        assert L.bh_configure_black_hole(ctx, ctx_in[0], ctx_in[1], 0.0) == 0
        if ctx_in[10]:
            assert L.bh_configure_accretion_disk(ctx, *[float(x) for x in ctx_in[2:6]]) == 0
        if ctx_in[11]:
            assert L.bh_configure_simulation(ctx, float(ctx_in[6]), float(ctx_in[7]),
                                             int(ctx_in[8]), float(ctx_in[9])) == 0
        v = np.ascontiguousarray(vec[:9].reshape(3, 3), dtype=np.float32)
        buf = np.full(32, 0x7fbadbad, dtype=np.uint32)
        got_rc = L.bh_generate_shader_data(ctx, v[0].ctypes.data, v[1].ctypes.data,
                                           v[2].ctypes.data, int(call[0]), int(call[1]),
                                           F(float(vec[9])), int(call[2]), int(call[3]),
                                           int(call[4]), buf.ctypes.data)
        L.bh_shutdown(ctx)
        assert got_rc == rc
        bad = np.nonzero(buf != want)[0]
        assert bad.size == 0, (ctx_in, call, bad, buf[bad], want[bad])
    z = np.zeros(3, dtype=np.float32)
    out = np.zeros(32, dtype=np.float32)
    ctx = L.bh_initialize()
    got = [L.bh_generate_shader_data(None, z.ctypes.data, z.ctypes.data, z.ctypes.data, 8, 8,
                                     F(60.0), 0, 0, 0, out.ctypes.data),
           L.bh_generate_shader_data(ctx, None, z.ctypes.data, z.ctypes.data, 8, 8, F(60.0), 0,
                                     0, 0, out.ctypes.data),
           L.bh_generate_shader_data(ctx, z.ctypes.data, z.ctypes.data, z.ctypes.data, 8, 8,
                                     F(60.0), 0, 0, 0, None)]
    L.bh_shutdown(ctx)
    assert got == list(g["null_rc"])
