"""The oracle (oracle/oracle.c, CPU restatement) against the compiled reference's outputs.

This pins the checker before it is trusted: every golden fixture was produced by the
reference's own code (tests/golden/gen_golden.py). Integers must match exactly and floats to
1e-12 relative; in practice the restatement is bit-identical.
"""
import ctypes as C

import numpy as np
import pytest

from conftest import (camera_from, compare, fixture_outputs, golden, golden_names, rays_from,
                      scene_from, sky_pinned)
from bhrt import abi

RTOL = 1e-12


@pytest.mark.parametrize("name", golden_names("frame_"))
def test_oracle_frames(oracle, name):
    g = golden(name)
    bh, dk, cfg = scene_from(g)
    got = oracle.render_frame(bh, dk, cfg, camera_from(g), int(g["W"]), int(g["H"]),
                              int(g["method"]), int(g["flags"]))
    compare(got, fixture_outputs(g), RTOL, sky_pinned(g["method"]), name)


@pytest.mark.parametrize("name", golden_names("rays_"))
def test_oracle_rays(oracle, name):
    g = golden(name)
    bh, dk, cfg = scene_from(g)
    got = oracle.trace_rays(rays_from(g), bh, dk, cfg, int(g["method"]), int(g["flags"]))
    compare(got, fixture_outputs(g), RTOL, sky_pinned(g["method"]), name)


def test_survey_known_answers(oracle):
    """main.c's five rays, values measured on the compiled reference."""
    g = golden("kat_main5")
    want = [
        (1, 2, (-2.2992673403577877, -5.6736347755292318, -0.52476540250735937), 37.705004165768464, 1.2176178453429627),
        (1, 2, (3.5472538113851115, -5.5170749989085612, -0.022351897354905503), 37.633357669793476, 1.1994516658756558),
        (1, 1, (12.674041311671116, -1.4391340336998424, 0.0), 35.326380926108079, 1.0890140546042),
        (1, 1, (6.5668414588749302, -1.6289075348719388, 0.0), 33.672673854178058, 1.1914915803661377),
        (1, 1, (0.0, 17.265660841181191, 5.4789059106332427), 53.424265571100214, 1.0602427684073148),
    ]
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    cfg = abi.sim_config(0.1, 100.0, 1000, 1e-6)
    got = oracle.trace_rays(rays_from(g), bh, dk, cfg)
    for i, (res, steps, hp, dist, td) in enumerate(want):
        assert g["result"][i] == res and g["steps"][i] == steps
        assert tuple(g["hit_position"][i]) == hp
        assert g["distance"][i] == dist and g["time_dilation"][i] == td
        assert got["result"][i] == res and got["steps"][i] == steps
        assert (got["hit_x"][i], got["hit_y"][i], got["hit_z"][i]) == hp
        assert got["distance"][i] == dist and got["time_dilation"][i] == td


def test_survey_shading_known_answers(oracle):
    """SURVEY.md section 4 shading KATs, on the oracle's colour functions."""
    lib = oracle.lib
    lib.orc_calculate_disk_temperature.argtypes = [C.c_void_p] * 5
    lib.orc_apply_relativistic_effects.argtypes = [C.c_void_p] * 5
    lib.orc_temperature_to_rgb.argtypes = [C.c_double, C.c_void_p]
    lib.orc_halton_sequence.restype = C.c_double
    lib.orc_halton_sequence.argtypes = [C.c_int, C.c_int]
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    T = C.c_double()
    rgb = (C.c_double * 3)()
    lib.orc_calculate_disk_temperature(C.byref(abi.v3(10, 0, 0)), C.byref(bh), C.byref(dk),
                                       C.byref(T), rgb)
    assert T.value == 15985.451076336421
    assert tuple(rgb) == (0.24446553098811544, 0.085408662096262036, 0.0)
    base = tuple(rgb)
    dop = C.c_double()
    lib.orc_apply_relativistic_effects(C.byref(abi.v3(10, 0, 0)), C.byref(abi.v3(0, 1, 0)),
                                       C.byref(bh), rgb, C.byref(dop))
    assert tuple(rgb) == (0.81478980696545855, 0.43238135186232657, 0.0) and dop.value == 1.5
    rgb2 = (C.c_double * 3)(*base)
    lib.orc_apply_relativistic_effects(C.byref(abi.v3(10, 0, 0)), C.byref(abi.v3(0, 0, -1)),
                                       C.byref(bh), rgb2, C.byref(dop))
    assert tuple(rgb2) == (0.2702744437982279, 0.085408662096262036, 0.0) and dop.value == 1.0
    lib.orc_temperature_to_rgb(5000.0, rgb)
    assert tuple(rgb) == (0.04275190074006642, 0.0, 0.0)
    assert lib.orc_halton_sequence(5, 2) == 0.625
    assert lib.orc_halton_sequence(7, 3) == 0.55555555555555558


def test_oracle_shading_fixture(oracle):
    """Oracle colour/geometry helpers vs the reference's, on the fixture's sweeps."""
    g = golden("shading")
    lib = oracle.lib
    lib.orc_temperature_to_rgb.argtypes = [C.c_double, C.c_void_p]
    for t, want in zip(g["t2rgb_in"], g["t2rgb_out"]):
        o = (C.c_double * 3)()
        lib.orc_temperature_to_rgb(float(t), o)
        np.testing.assert_array_equal(np.array(list(o)), want)
    lib.orc_calculate_disk_temperature.argtypes = [C.c_void_p] * 5
    lib.orc_apply_relativistic_effects.argtypes = [C.c_void_p] * 5
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    for p, v, w_t, w_rel in zip(g["disk_pos"], g["disk_vel"], g["disk_temp_out"],
                                g["relativistic_out"]):
        T = C.c_double()
        col = (C.c_double * 3)()
        lib.orc_calculate_disk_temperature(C.byref(abi.v3(*p)), C.byref(bh), C.byref(dk),
                                           C.byref(T), col)
        np.testing.assert_array_equal(np.array([T.value] + list(col)), w_t)
        dop = C.c_double()
        lib.orc_apply_relativistic_effects(C.byref(abi.v3(*p)), C.byref(abi.v3(*v)),
                                           C.byref(bh), col, C.byref(dop))
        np.testing.assert_array_equal(np.array(list(col) + [dop.value]), w_rel)
    lib.orc_halton_sequence.restype = C.c_double
    lib.orc_halton_sequence.argtypes = [C.c_int, C.c_int]
    for i, b, want in g["halton"]:
        assert lib.orc_halton_sequence(int(i), int(b)) == want
    lib.orc_initialize_black_hole_params.argtypes = [C.c_void_p, C.c_double, C.c_double,
                                                     C.c_double]
    for s, want in zip(g["bh_spins"], g["bh_params"]):
        bhp = abi.BlackHoleParams()
        lib.orc_initialize_black_hole_params(C.byref(bhp), 1.0, float(s), 0.0)
        np.testing.assert_array_equal([getattr(bhp, f) for f, _ in bhp._fields_], want)
        # the Python config builder agrees with the reference too
        py = abi.black_hole(1.0, float(s))
        np.testing.assert_array_equal([getattr(py, f) for f, _ in py._fields_], want)
    lib.orc_check_disk_intersection.argtypes = [C.c_void_p] * 5
    for row, want in zip(g["cdi_in"], g["cdi_out"]):
        q = abi.Vector3D()
        h = lib.orc_check_disk_intersection(C.byref(abi.v3(*row[0:3])), C.byref(abi.v3(*row[3:6])),
                                            C.byref(abi.v3(*row[6:9])), C.byref(dk), C.byref(q))
        np.testing.assert_array_equal([h, q.x, q.y, q.z] if h else [0, 0, 0, 0], want)


def test_oracle_paths(oracle):
    """integrate_photon_path with recorded paths, incl. no-op integrators and max_positions 0."""
    g = golden("paths")
    lib = oracle.lib
    lib.orc_integrate_photon_path.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                              C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.orc_integrate_photon_path.restype = C.c_int
    for i in range(int(g["ncases"])):
        inp = g[f"case{i}_in"]
        o4, d3, spin, method, steps, maxp = inp[0:4], inp[4:7], inp[7], int(inp[8]), int(inp[9]), int(inp[10])
        bh = abi.black_hole(1.0, float(spin))
        cfg = abi.sim_config(0.1, 100.0, steps, 1e-6 if spin == 0 else 1e-8)
        path = (abi.Vector3D * max(maxp, 1))()
        num = C.c_int(0)
        hit = abi.RayTraceHit()
        res = lib.orc_integrate_photon_path(C.byref(abi.Vector4D(*o4)), C.byref(abi.v3(*d3)),
                                            C.byref(bh), C.byref(cfg), method, path, maxp,
                                            C.byref(num), C.byref(hit))
        want_res = g[f"case{i}_res"]
        assert [res, num.value, hit.result, hit.steps] == list(want_res), i
        h = g[f"case{i}_hit"]
        got_h = [hit.hit_position.x, hit.hit_position.y, hit.hit_position.z, hit.distance,
                 hit.time_dilation]
        np.testing.assert_allclose(got_h, h[:5], rtol=RTOL)
        if method != abi.INTEGRATOR_RK4:
            np.testing.assert_allclose([hit.sky_direction.x, hit.sky_direction.y,
                                        hit.sky_direction.z], h[5:8], rtol=RTOL)
        stored = g[f"case{i}_path"]
        np.testing.assert_allclose(np.array([[p.x, p.y, p.z] for p in path[:len(stored)]]).reshape(-1, 3),
                                   stored, rtol=RTOL)


def test_camera_restatement_pinned_by_trace_pixel(oracle):
    """The pixel->direction restatement (raytracer.c:999-1039) is static in the reference; it is
    pinned through the reference's own trace_pixel: same class for every sampled pixel and, for
    non-disk pixels, the same sky-gradient colour (a function of the direction's y)."""
    g = golden("trace_pixel")
    from bhrt import configs
    W, H = int(g["W"]), int(g["H"])
    bh = abi.black_hole(1.0, 0.0)
    dk = abi.disk(6.0, 20.0, 1.0, 1.0)
    cfg = abi.sim_config(0.1, 100.0, 1000, 1e-6)
    frames = {c: oracle.render_frame(bh, dk, cfg, configs.camera(c), W, H) for c in "ABV"}
    for cam, px, py, res, r, gg, b in g["rows"]:
        f = frames[chr(int(cam))]
        i = int(py) * W + int(px)
        assert f["result"][i] == int(res)
        if int(res) != abi.RAY_DISK:
            np.testing.assert_array_equal([f["rgb_r"][i], f["rgb_g"][i], f["rgb_b"][i]], [r, gg, b])


def test_numpy_camera_rays_match_the_oracle(oracle):
    """configs.camera_rays (bench.py's synthetic Ray[] input) follows calculate_ray_direction:
    checked against the oracle's restatement on a pixel sample of every camera."""
    import ctypes as C
    from bhrt import abi, configs
    O = oracle.lib
    O.orc_camera_ray_direction.argtypes = [C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                           C.c_int, C.POINTER(abi.Camera), C.POINTER(abi.Vector3D)]
    W, H = 320, 180
    for name in ("A", "B", "V"):
        cam = configs.camera(name)
        rays = configs.camera_rays(cam, W, H)
        d = abi.Vector3D()
        for y in range(0, H, 17):
            for x in range(0, W, 23):
                O.orc_camera_ray_direction(x, y, 0.5, 0.5, W, H, C.byref(cam), C.byref(d))
                got = rays["direction"][y * W + x]
                assert np.allclose(got, (d.x, d.y, d.z), rtol=0, atol=1e-15), (name, x, y)


def test_knife_edge_margins(oracle):
    """orc_render_frame_margin (the knife-edge list of tools/full_frame_parity.py and the
    full-frame GPU tests): outputs identical to orc_render_frame for every config, margins
    positive, and a ray put exactly on a threshold gets margin 0 -- here max_ray_distance set
    to the distance a MAX_DISTANCE ray reaches at its exit iteration."""
    from bhrt import abi, configs
    cam = configs.camera("B")
    for name in ("C1", "C2", "C3", "C4", "C5"):
        c = configs.CONFIGS[name]
        bh, dk, cfg = c.scene()
        a = oracle.render_frame(bh, dk, cfg, cam, 40, 24, c.method, c.flags, threads=4)
        b, m = oracle.render_frame_margin(bh, dk, cfg, cam, 40, 24, c.method, c.flags,
                                          threads=4)
        for f in a:
            assert np.array_equal(a[f], b[f], equal_nan=True), (name, f)
        assert np.all(m > 0) and np.all(np.isfinite(m)), name
    c = configs.CONFIGS["C4"]
    bh, dk, cfg = c.scene()
    f, m = oracle.render_frame_margin(bh, None, cfg, cam, 40, 24, c.method, 0, threads=4)
    i = int(np.nonzero(f["result"] == abi.RAY_MAX_DISTANCE)[0][0])
    assert m[i] > 1e-9
    # a distance threshold exactly at the (k-1)-th partial sum is hit by rounding only: put
    # it at the distance this ray reports and the exit decision is taken at margin 0
    cfg.max_ray_distance = float(f["distance"][i])
    f2, m2 = oracle.render_frame_margin(bh, None, cfg, cam, 40, 24, c.method, 0, threads=4)
    assert f2["result"][i] == abi.RAY_MAX_DISTANCE and m2[i] == 0.0
