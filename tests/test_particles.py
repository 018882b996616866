"""The particle system (src/particle_sim.c, the particle half of src/blackhole_api.c) and the
scalar spacetime helpers (src/spacetime.c), SURVEY.md 8(f) ranks 2 and 4.

  * CPU: the oracle's update_particles equals the compiled reference bit for bit; libbhrt's
    host creation (seeded rand() stream), bookkeeping, argument checks and spacetime helpers
    equal the reference bit for bit; update_particles fails loudly without a GPU.
  * GPU: update_particles (HIP kernel, one lane per particle) against the reference's
    snapshots after 1, 10 and 60 steps, and the visualizer's bh_* sequence.

Fixtures: tests/golden/particles.npz and spacetime_helpers.npz (gen_golden.py).
"""
import ctypes as C

import numpy as np
import pytest

from conftest import golden, gpu_available
from bhrt import abi, lib

P = C.POINTER
LIBC = C.CDLL("libc.so.6")
FIELDS = (("pos", "position"), ("vel", "velocity"), ("type", "type"), ("active", "active"),
          ("id", "id"), ("age", "age"), ("temp", "temperature"), ("mass", "mass"),
          ("tdil", "time_dilation"))
STEP_FIELDS = (("pos", "position"), ("vel", "velocity"), ("active", "active"), ("age", "age"),
               ("tdil", "time_dilation"))


def _bind(L):
    PS = P(abi.ParticleSystem)
    L.particle_system_init.argtypes = [PS, C.c_int]
    L.particle_system_cleanup.argtypes = [PS]
    L.create_accretion_disk.argtypes = [PS, P(abi.BlackHoleParams), P(abi.AccretionDiskParams),
                                        C.c_int]
    L.generate_hawking_radiation.argtypes = [PS, P(abi.BlackHoleParams), C.c_int,
                                             P(abi.SimulationConfig)]
    L.add_particle.argtypes = [PS, P(abi.Vector3D), P(abi.Vector3D), C.c_double, C.c_int]
    L.update_particles.argtypes = [PS, P(abi.BlackHoleParams), P(abi.SimulationConfig)]
    L.bhrt_update_particles_steps.argtypes = [PS, P(abi.BlackHoleParams),
                                              P(abi.SimulationConfig), C.c_int, P(C.c_double)]
    L.bh_initialize.restype = C.c_void_p
    L.bh_shutdown.argtypes = [C.c_void_p]
    L.bh_configure_black_hole.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_double]
    L.bh_configure_accretion_disk.argtypes = [C.c_void_p] + [C.c_double] * 4
    L.bh_configure_simulation.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_int,
                                          C.c_double]
    L.bh_create_particle_system.restype = C.c_void_p
    L.bh_create_particle_system.argtypes = [C.c_void_p, C.c_int]
    L.bh_destroy_particle_system.argtypes = [C.c_void_p, C.c_void_p]
    L.bh_add_test_particle.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_double]
    L.bh_create_accretion_disk_particles.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.bh_generate_hawking_radiation.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.bh_update_particles.argtypes = [C.c_void_p, C.c_void_p]
    L.bh_get_particle_data.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_void_p, P(C.c_int)]
    return L


def _case(g, c):
    pre = f"case{c}_"
    bh = abi.BlackHoleParams(*g[pre + "bh"])
    dk = abi.AccretionDiskParams(*g[pre + "disk"])
    cfg = abi.sim_config(float(g[pre + "in"][4]), 100.0, 1000, 1e-6)
    cfg.hawking_temp_factor = 1.0
    return pre, bh, dk, cfg


def _system_from_fixture(L, g, pre):
    """A libbhrt ParticleSystem holding the fixture's initial particles."""
    n = int(g[pre + "in"][5])
    ps = abi.ParticleSystem()
    assert L.particle_system_init(C.byref(ps), n) == 0
    ps.count = n
    a = abi.particles_view(ps)
    a[:] = np.zeros(n, dtype=abi.PARTICLE_DTYPE)
    for k, f in FIELDS:
        a[f] = g[pre + "init_" + k]
    return ps, a


def _check_steps(a, g, pre, s, exact):
    for k, f in STEP_FIELDS:
        got, want = a[f], g[pre + f"s{s}_" + k]
        if exact or k == "active":
            assert np.array_equal(got, want, equal_nan=True), (pre, s, k)
            continue
        bad_nan = np.isnan(got) != np.isnan(want)
        assert not bad_nan.any(), (pre, s, k, np.nonzero(bad_nan)[0][:5])
        ok = ~np.isnan(want)
        scale = np.maximum(np.abs(want[ok]), 1e-300)
        rel = np.abs(got[ok] - want[ok]) / scale
        tol = 1e-5 + 1e-9 / scale
        assert (rel <= tol).all(), (pre, s, k, float(rel.max()))


# ------------------------------------------------------------------ CPU: oracle and host

def test_oracle_update_particles_matches_reference(oracle):
    g = golden("particles")
    O = oracle.lib
    O.orc_update_particles.argtypes = [C.c_void_p, C.c_int, P(abi.BlackHoleParams),
                                       P(abi.SimulationConfig), C.c_int]
    for c in range(int(g["ncases"])):
        pre, bh, dk, cfg = _case(g, c)
        n = int(g[pre + "in"][5])
        a = np.zeros(n, dtype=abi.PARTICLE_DTYPE)
        for k, f in FIELDS:
            a[f] = g[pre + "init_" + k]
        done = 0
        for s in g["steps"]:
            O.orc_update_particles(a.ctypes.data, n, C.byref(bh), C.byref(cfg), int(s) - done)
            done = int(s)
            _check_steps(a, g, pre, int(s), exact=True)


def test_host_particle_creation_matches_reference():
    """Seeded creation draws the reference's rand() sequence: disk and Hawking particles,
    then test particles, bit for bit (host C, particle_sim.c:108-133, 339-503)."""
    L = _bind(lib.load())
    g = golden("particles")
    for c in range(int(g["ncases"])):
        pre, bh, dk, cfg = _case(g, c)
        spin, seed, n_disk, n_hawk = g[pre + "in"][:4]
        ps = abi.ParticleSystem()
        assert L.particle_system_init(C.byref(ps), 400) == 0
        LIBC.srand(int(seed))
        made = [L.create_accretion_disk(C.byref(ps), C.byref(bh), C.byref(dk), int(n_disk)),
                L.generate_hawking_radiation(C.byref(ps), C.byref(bh), int(n_hawk), C.byref(cfg))]
        for t in g["tests"]:
            made.append(L.add_particle(C.byref(ps), C.byref(abi.v3(*t[0:3])),
                                       C.byref(abi.v3(*t[3:6])), float(t[6]), abi.PARTICLE_TEST))
        assert made == list(g[pre + "made"])
        a = abi.particles_view(ps)
        for k, f in FIELDS:
            if k == "tdil":
                continue  # set by the fixture script, not by creation
            assert np.array_equal(a[f], g[pre + "init_" + k], equal_nan=True), (pre, k)
        L.particle_system_cleanup(C.byref(ps))


def test_particle_api_argument_checks():
    """blackhole_api.c:256-429 return codes; capacity limits of particle_sim.c."""
    L = _bind(lib.load())
    ctx = L.bh_initialize()
    try:
        assert L.bh_create_particle_system(ctx, 0) is None
        assert L.bh_create_particle_system(None, 10) is None
        sysp = L.bh_create_particle_system(ctx, 3)
        assert sysp
        pos, vel = (C.c_double * 3)(1, 2, 3), (C.c_double * 3)(0, 0.1, 0)
        assert L.bh_add_test_particle(ctx, sysp, pos, vel, -1.0) == -1
        assert L.bh_add_test_particle(ctx, None, pos, vel, 1.0) == -1
        assert [L.bh_add_test_particle(ctx, sysp, pos, vel, 1.0) for _ in range(4)] == [1, 2, 3, -1]
        assert L.bh_create_accretion_disk_particles(ctx, sysp, 0) == -1
        assert L.bh_generate_hawking_radiation(ctx, sysp, -1) == -1
        assert L.bh_generate_hawking_radiation(ctx, sysp, 5) == -1  # over capacity
        assert L.bh_update_particles(None, sysp) == -1
        buf = np.zeros(9)
        typ = np.zeros(3, dtype=np.int32)
        cnt = C.c_int(0)
        assert L.bh_get_particle_data(ctx, sysp, buf.ctypes.data, buf.ctypes.data,
                                      typ.ctypes.data, C.byref(cnt)) == -1
        cnt = C.c_int(2)
        assert L.bh_get_particle_data(ctx, sysp, buf.ctypes.data, buf[3:].ctypes.data,
                                      typ.ctypes.data, C.byref(cnt)) == 0
        assert cnt.value == 2 and list(buf[:3]) == [1, 2, 3]
        L.bh_destroy_particle_system(ctx, sysp)
        # disk particles need a configured disk (blackhole_api.c:327-329)
        sysp = L.bh_create_particle_system(ctx, 10)
        assert L.bh_create_accretion_disk_particles(ctx, sysp, 5) == 0
        L.bh_destroy_particle_system(ctx, sysp)
    finally:
        L.bh_shutdown(ctx)


def test_spacetime_helpers_match_reference():
    """spacetime.h scalar helpers (host C restatements) bit for bit on a grid of inputs."""
    L = lib.load()
    D, V = C.c_double, C.c_void_p
    for f, a, r in (("calculate_effective_potential", [D, D, V], D),
                    ("calculate_ergosphere_radius", [D, V], D),
                    ("calculate_kerr_metric_bl", [V, D, D, V], C.c_int),
                    ("calculate_inverse_kerr_metric", [V, D, D, V], C.c_int),
                    ("calculate_kerr_christoffel", [V, D, D, V], C.c_int),
                    ("calculate_kerr_isco", [D, D, C.c_bool], D),
                    ("calculate_kerr_event_horizon", [D, D], D),
                    ("calculate_kerr_ergosphere", [D, D, D], D),
                    ("calculate_frame_dragging", [V, D, D, V], C.c_int),
                    ("calculate_kerr_geodesic", [V, V, D, D, V], C.c_int),
                    ("calculate_christoffel_symbols", [D, D, V, V], None),
                    ("geodesic_equation", [V, V, V, V], None)):
        getattr(L, f).argtypes, getattr(L, f).restype = a, r
    g = golden("spacetime_helpers")
    r, th, l, vel = g["r"], g["th"], g["l"], g["vel"]
    for si, spin in enumerate(g["spins"]):
        bh = abi.black_hole(1.0, float(spin))
        a = float(spin)
        for i in range(len(r)):
            w = {k: g[f"s{si}_{k}"][i] for k in ("veff", "ergo", "bl", "inv", "kchr", "isco",
                                                   "hor", "kergo", "drag", "kgeo", "chr", "geo",
                                                   "rc")}
            pos = np.array([0.0, r[i], th[i], 0.3])
            v = np.ascontiguousarray(vel[i])
            km = (D * 7)()
            got = {"veff": L.calculate_effective_potential(r[i], l[i], C.byref(bh)),
                   "ergo": L.calculate_ergosphere_radius(th[i], C.byref(bh))}
            rc = [L.calculate_kerr_metric_bl(pos.ctypes.data, a, 1.0, km)]
            got["bl"] = [km[0], km[1], km[2], km[4], km[5]]
            rc.append(L.calculate_inverse_kerr_metric(pos.ctypes.data, a, 1.0, km))
            got["inv"] = [km[0], km[1], km[2], km[4], km[5]]
            G = np.zeros(64)
            rc.append(L.calculate_kerr_christoffel(pos.ctypes.data, a, 1.0, G.ctypes.data))
            got["kchr"] = G
            got["isco"] = [L.calculate_kerr_isco(a, 1.0, True), L.calculate_kerr_isco(a, 1.0, False)]
            got["hor"] = L.calculate_kerr_event_horizon(a, 1.0)
            got["kergo"] = L.calculate_kerr_ergosphere(a, 1.0, th[i])
            v3 = np.zeros(3)
            rc.append(L.calculate_frame_dragging(pos.ctypes.data, a, 1.0, v3.ctypes.data))
            got["drag"] = v3
            acc = np.zeros(4)
            rc.append(L.calculate_kerr_geodesic(pos.ctypes.data, v.ctypes.data, a, 1.0,
                                                acc.ctypes.data))
            got["kgeo"] = acc
            G2 = np.zeros(64)
            L.calculate_christoffel_symbols(r[i], th[i], C.byref(bh), G2.ctypes.data)
            got["chr"] = G2
            acc2 = np.zeros(4)
            L.geodesic_equation(pos.ctypes.data, v.ctypes.data, C.byref(bh), acc2.ctypes.data)
            got["geo"] = acc2
            got["rc"] = rc
            for k in w:
                assert np.array_equal(np.asarray(got[k], dtype=np.float64),
                                      np.asarray(w[k], dtype=np.float64), equal_nan=True), (spin, i, k)


@pytest.mark.skipif(gpu_available(), reason="checks the no-GPU behaviour")
def test_update_particles_needs_a_gpu():
    L = _bind(lib.load())
    g = golden("particles")
    pre, bh, dk, cfg = _case(g, 0)
    ps, a = _system_from_fixture(L, g, pre)
    before = a.copy()
    assert L.update_particles(C.byref(ps), C.byref(bh), C.byref(cfg)) == -1
    assert lib.last_error()
    assert np.array_equal(abi.particles_view(ps), before)
    L.particle_system_cleanup(C.byref(ps))


# ------------------------------------------------------------------ GPU

@pytest.mark.gpu
def test_update_particles_gpu_vs_reference(bhrt_lib):
    L = _bind(bhrt_lib.load())
    g = golden("particles")
    for c in range(int(g["ncases"])):
        pre, bh, dk, cfg = _case(g, c)
        ps, a = _system_from_fixture(L, g, pre)
        done = 0
        for s in g["steps"]:
            while done < int(s):
                assert L.update_particles(C.byref(ps), C.byref(bh), C.byref(cfg)) == 0
                done += 1
            # the reference's test-particle update diverges exponentially (positions ~1e40
            # after 10 steps); one-ulp trig differences are compared after 1 step only
            geo = (a["type"] == abi.PARTICLE_TEST)
            if int(s) == 1:
                _check_steps(a, g, pre, 1, exact=False)
            else:
                sub = {k: a[f][~geo] for k, f in STEP_FIELDS}
                for k, f in STEP_FIELDS:
                    want = g[pre + f"s{s}_" + k][~geo]
                    if k == "active":
                        assert np.array_equal(sub[k], want)
                    else:
                        np.testing.assert_allclose(sub[k], want, rtol=1e-5, atol=1e-9)
                assert np.array_equal(a["active"], g[pre + f"s{s}_active"])
        L.particle_system_cleanup(C.byref(ps))


@pytest.mark.gpu
def test_update_particles_steps_equals_single_steps(bhrt_lib):
    """bhrt_update_particles_steps(k) is k update_particles calls in one device round trip."""
    L = _bind(bhrt_lib.load())
    g = golden("particles")
    pre, bh, dk, cfg = _case(g, 0)
    ps1, a1 = _system_from_fixture(L, g, pre)
    ps2, a2 = _system_from_fixture(L, g, pre)
    for _ in range(10):
        assert L.update_particles(C.byref(ps1), C.byref(bh), C.byref(cfg)) == 0
    ms = C.c_double(-1.0)
    assert L.bhrt_update_particles_steps(C.byref(ps2), C.byref(bh), C.byref(cfg), 10,
                                         C.byref(ms)) == 0
    assert ms.value >= 0.0
    for f in abi.PARTICLE_DTYPE.names:  # bitwise, field by field (the struct has padding)
        b1 = np.ascontiguousarray(a1[f]).view(np.uint8)
        b2 = np.ascontiguousarray(a2[f]).view(np.uint8)
        assert np.array_equal(b1, b2), f


@pytest.mark.gpu
def test_visualizer_particle_sequence(bhrt_lib):
    """renderer.cpp:879-1005: create 5000-capacity system, 3000 disk particles, update per
    frame, read back for rendering -- against the reference's run with the same seed."""
    L = _bind(bhrt_lib.load())
    g = golden("particles")
    ctx = L.bh_initialize()
    assert L.bh_configure_black_hole(ctx, 1.0, 0.0, 0.0) == 0
    assert L.bh_configure_accretion_disk(ctx, 6.0, 20.0, 1.0, 1.0) == 0
    assert L.bh_configure_simulation(ctx, 0.05, 100.0, 1000, 1e-6) == 0
    sysp = L.bh_create_particle_system(ctx, 5000)
    LIBC.srand(777)
    made = L.bh_create_accretion_disk_particles(ctx, sysp, 3000)
    for _ in range(5):
        assert L.bh_update_particles(ctx, sysp) == 0
    pos, vel = np.zeros(5000 * 3), np.zeros(5000 * 3)
    typ = np.zeros(5000, dtype=np.int32)
    cnt = C.c_int(5000)
    rc = L.bh_get_particle_data(ctx, sysp, pos.ctypes.data, vel.ctypes.data, typ.ctypes.data,
                                C.byref(cnt))
    L.bh_destroy_particle_system(ctx, sysp)
    L.bh_shutdown(ctx)
    n = cnt.value
    assert [made, rc, n] == list(g["viz_made"])
    np.testing.assert_allclose(pos[:3 * n].reshape(n, 3), g["viz_pos"], rtol=1e-5, atol=1e-9)
    np.testing.assert_allclose(vel[:3 * n].reshape(n, 3), g["viz_vel"], rtol=1e-5, atol=1e-9)
    assert np.array_equal(typ[:n], g["viz_type"])
