/* asan_driver.c -- host code under AddressSanitizer + UBSan.
 *
 * Built by tests/test_sanitizers.py with -fsanitize=address,undefined from: the oracle
 * (oracle/oracle.c), libbhrt's host C (bhrt_api.c, particles.c, kerr_helpers.c) and the
 * stubs below for the three device launchers (geodesic.hip / particles.hip are device code,
 * not instrumented; without a GPU every device entry point must fail cleanly anyway). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bhrt_api.h"
#include "bhrt_kernel.h"
#include "oracle.h"

int bhrt_trace_untested(const bhrt_kparams* kp) { (void)kp; return 0; }
int bhrt_launch_trace(const bhrt_kparams* kp, void* stream, void* ev0, void* ev1) {
    (void)kp; (void)stream; (void)ev0; (void)ev1;
    return 100; /* hipErrorNoDevice */
}
int bhrt_launch_path(const bhrt_kparams* kp, const double* o, const double* d, Vector3D* p,
                     int m, int* n, int nin, void* st) {
    (void)kp; (void)o; (void)d; (void)p; (void)m; (void)n; (void)nin; (void)st;
    return 100;
}
int bhrt_launch_particles(Particle* d, int count, const bhrt_particle_k* k, int steps,
                          void* stream, void* ev0, void* ev1) {
    (void)d; (void)count; (void)k; (void)steps; (void)stream; (void)ev0; (void)ev1;
    return 100;
}

static void soa_alloc(bhrt_frame_soa* s, int n) {
    memset(s, 0, sizeof *s);
    s->result = calloc(n, 4); s->steps = calloc(n, 4);
    double** f[] = {&s->hit_x, &s->hit_y, &s->hit_z, &s->distance, &s->time_dilation,
                    &s->sky_x, &s->sky_y, &s->sky_z, &s->rgb_r, &s->rgb_g, &s->rgb_b};
    for (unsigned i = 0; i < sizeof f / sizeof *f; i++) *f[i] = calloc(n, 8);
}
static void soa_free(bhrt_frame_soa* s) {
    void* p[] = {s->result, s->steps, s->hit_x, s->hit_y, s->hit_z, s->distance,
                 s->time_dilation, s->sky_x, s->sky_y, s->sky_z, s->rgb_r, s->rgb_g, s->rgb_b};
    for (unsigned i = 0; i < sizeof p / sizeof *p; i++) free(p[i]);
}

static int checks, total;
#define CHECK(x) (total++, checks += !!(x))

int main(void) {
    /* oracle frames: the five configurations' scenes, whole and sharded */
    const double spins[] = {0.0, 0.0, 0.0, 0.9, 0.99};
    const int methods[] = {INTEGRATOR_RK4, INTEGRATOR_RK4, INTEGRATOR_RKF45, INTEGRATOR_RK4,
                           INTEGRATOR_RKF45};
    for (int c = 0; c < 5; c++) {
        BlackHoleParams bh;
        orc_initialize_black_hole_params(&bh, 1.0, spins[c], 0.0);
        AccretionDiskParams dk = {bh.isco_radius, 20.0, 1.0, 1.0, 0.0, 0.0};
        SimulationConfig cfg = {0};
        cfg.time_step = 0.1; cfg.max_ray_distance = 100.0;
        cfg.max_integration_steps = c == 4 ? 200 : 120; cfg.tolerance = c == 4 ? 1e-8 : 1e-6;
        bhrt_camera cam = {{0, -29.544, 5.209}, {0, 29.544, -5.209}, {0, 0, 1}, 60.0, c & 1,
                           0.25, 0.75};
        bhrt_frame_soa s;
        soa_alloc(&s, 24 * 16);
        CHECK(orc_render_frame(&bh, c == 0 ? NULL : &dk, &cfg, &cam, 24, 16, NULL,
                               (IntegrationMethod)methods[c], c == 3, &s, 1) == 0);
        bhrt_rows rows = {4, 1, 3};
        CHECK(orc_render_frame(&bh, &dk, &cfg, &cam, 24, 16, &rows,
                               (IntegrationMethod)methods[c], 0, &s, 1) == 0);
        soa_free(&s);
    }
    /* edge rays through the oracle */
    BlackHoleParams bh;
    orc_initialize_black_hole_params(&bh, 1.0, 0.0, 0.0);
    AccretionDiskParams dk = {6.0, 20.0, 1.0, 1.0, 0.1, 0.0};
    SimulationConfig cfg = {0};
    cfg.time_step = 0.1; cfg.max_ray_distance = 100.0; cfg.max_integration_steps = 150;
    cfg.tolerance = 1e-6; cfg.hawking_temp_factor = 1.0;
    Ray rays[6] = {{{0, 0, 2.05}, {0, 0, 1}}, {{0.3, 0.2, 0.4}, {1, 0, 0}},
                   {{0, 0, 30}, {0, 0, -1}}, {{0, 0, 30}, {NAN, 0, -1}},
                   {{0, 0, 30}, {0, 0, 0}}, {{1e7, 0, 0}, {-1, 0.1, 0}}};
    bhrt_frame_soa s;
    soa_alloc(&s, 6);
    CHECK(orc_trace_rays(rays, 6, &bh, &dk, &cfg, INTEGRATOR_RK4, 0, &s, 1) == 0);
    CHECK(orc_trace_rays(rays, 6, &bh, &dk, &cfg, INTEGRATOR_RKF45, 0, &s, 1) == 0);
    soa_free(&s);
    Vector3D path[64];
    int num = 0;
    RayTraceHit hit;
    Vector4D o4 = {0, 0, 0, 30};
    Vector3D d3 = {0.3, 0, -1};
    orc_integrate_photon_path(&o4, &d3, &bh, &cfg, INTEGRATOR_RK4, path, 64, &num, &hit);
    CHECK(num > 0);

    /* libbhrt host code: particles (creation, bookkeeping, the no-GPU update) */
    ParticleSystem ps;
    CHECK(particle_system_init(&ps, 300) == 0);
    srand(7);
    CHECK(create_accretion_disk(&ps, &bh, &dk, 200) == 200);
    CHECK(generate_hawking_radiation(&ps, &bh, 50, &cfg) == 50);
    Vector3D p = {10, 0, 0}, v = {0, 0.3, 0.05};
    CHECK(add_particle(&ps, &p, &v, 1.0, PARTICLE_TEST) > 0);
    CHECK(update_particles(&ps, &bh, &cfg) == -1); /* no device */
    orc_update_particles(ps.particles, ps.count, &bh, &cfg, 20);
    OrbitalParams op;
    CHECK(calculate_particle_orbit(&ps, ps.count, &bh, &op) == 0);
    CHECK(remove_particle(&ps, 3) == 0 && find_particle(&ps, 3) == NULL);
    particle_system_cleanup(&ps);
    BHContextHandle ctx = bh_initialize();
    CHECK(bh_configure_black_hole(ctx, 1.0, 0.5, 0.0) == BH_SUCCESS);
    CHECK(bh_configure_accretion_disk(ctx, 6.0, 20.0, 1.0, 1.0) == BH_SUCCESS);
    void* sys = bh_create_particle_system(ctx, 64);
    CHECK(bh_create_accretion_disk_particles(ctx, sys, 40) == 40);
    double pos[3 * 64], vel[3 * 64];
    int types[64], cnt = 64;
    CHECK(bh_get_particle_data(ctx, sys, pos, vel, types, &cnt) == BH_SUCCESS && cnt == 40);
    CHECK(bh_update_particles(ctx, sys) == BH_ERROR_SIMULATION);
    bh_destroy_particle_system(ctx, sys);

    /* libbhrt host code: ray API without a device, scalar helpers, shader data */
    RayTraceHit hits[6];
    CHECK(trace_rays_batch(rays, 6, &bh, &dk, &cfg, hits, 0) == -1);
    CHECK(bh_trace_rays_batch(ctx, rays, hits, 6) != BH_SUCCESS);
    double rgb[3], T, dop;
    Vector3D q, pt = {10, 0, 0}, vt = {0, 1, 0}, nn = {10, 0.1, 0.2};
    calculate_disk_temperature(&pt, &bh, &dk, &T, rgb);
    apply_relativistic_effects(&pt, &vt, &bh, rgb, &dop);
    CHECK(check_disk_intersection(&pt, &vt, &nn, &dk, &q) >= 0);
    float out[64 * 36 * 4];
    float obs[3] = {0, 0, 30}, dir[3] = {0, 0, -1}, up[3] = {0, 1, 0};
    CHECK(bh_generate_shader_data(ctx, obs, dir, up, 64, 36, 60.0f, 1, 1, 1, out) >= -4);
    bh_shutdown(ctx);

    /* spacetime.h helpers */
    double G[4][4][4], pos4[4] = {0, 5.0, 1.0, 0.3}, v4[4] = {1, 0.1, 0.01, 0.02}, acc[4];
    KerrMetric km;
    CHECK(calculate_kerr_metric_bl(pos4, 0.9, 1.0, &km) == 0);
    CHECK(calculate_inverse_kerr_metric(pos4, 0.9, 1.0, &km) == 0);
    CHECK(calculate_kerr_geodesic(pos4, v4, 0.9, 1.0, acc) == 0);
    geodesic_equation(pos4, v4, &bh, acc);
    calculate_christoffel_symbols(5.0, 0.0, &bh, G); /* pole: cot(0) */
    BlackHoleMetric bm = calculate_metric(5.0, 1.0, &bh);
    CHECK(bm.is_kerr == 0);
    printf("asan driver: %d of %d checks passed\n", checks, total);
    return checks == total ? 0 : 1;
}
