/*
 * trace_demo.c -- a C caller of libbhrt.so written against the reference's API, the way
 * the reference's own smoke test drives it (src/main.c: bh_initialize, configure the black
 * hole / disk / simulation, bh_trace_rays_batch over five rays), plus one camera frame
 * through the bhrt_render_frame extension.
 *
 *   gcc -std=c99 -Iinclude examples/trace_demo.c -Lraytracing-engine-in-c_amd -lbhrt \
 *       -Wl,-rpath,$PWD/raytracing-engine-in-c_amd -lm -o trace_demo && ./trace_demo
 *
 * Output: one line per ray "i result steps x y z distance time_dilation" (%.17g), then
 * the frame's class histogram.
 */
#include <stdio.h>
#include <stdlib.h>

#include "blackhole_api.h"

int main(void) {
    BHContextHandle ctx = bh_initialize();
    if (!ctx) return 1;
    if (bh_configure_black_hole(ctx, 1.0, 0.0, 0.0) != BH_SUCCESS ||
        bh_configure_accretion_disk(ctx, 6.0, 20.0, 1.0, 1.0) != BH_SUCCESS ||
        bh_configure_simulation(ctx, 0.1, 100.0, 1000, 1.0e-6) != BH_SUCCESS)
        return 2;

    const double o[5][3] = {{0, 0, 30}, {0, 0, 30}, {0, 0, 30}, {0, 0, 30}, {30, 0, 0}};
    const double d[5][3] = {{0, 0, -1}, {0.2, 0, -1}, {0.5, 0, -1}, {0.3, 0, -1}, {-1, 0, 0.1}};
    Ray rays[5];
    RayTraceHit hits[5];
    for (int i = 0; i < 5; i++) {
        rays[i].origin.x = o[i][0]; rays[i].origin.y = o[i][1]; rays[i].origin.z = o[i][2];
        rays[i].direction.x = d[i][0]; rays[i].direction.y = d[i][1]; rays[i].direction.z = d[i][2];
    }
    BHErrorCode rc = bh_trace_rays_batch(ctx, rays, hits, 5);
    if (rc != BH_SUCCESS) {
        fprintf(stderr, "bh_trace_rays_batch: %d (%s)\n", rc, bhrt_last_error());
        return 3;
    }
    for (int i = 0; i < 5; i++)
        printf("%d %d %d %.17g %.17g %.17g %.17g %.17g\n", i, hits[i].result, hits[i].steps,
               hits[i].hit_position.x, hits[i].hit_position.y, hits[i].hit_position.z,
               hits[i].distance, hits[i].time_dilation);

    /* one 64x36 camera-B frame through the extension API (host SoA, every visible GPU) */
    enum { W = 64, H = 36 };
    static int32_t result[W * H];
    bhrt_frame_soa soa = {0};
    soa.result = result;
    BlackHoleParams bh;
    initialize_black_hole_params(&bh, 1.0, 0.0, 0.0);
    AccretionDiskParams disk = {bh.isco_radius, 20.0, 1.0, 1.0, 0.0, 0.0};
    SimulationConfig cfg = {0};
    cfg.time_step = 0.1;
    cfg.max_ray_distance = 100.0;
    cfg.max_integration_steps = 1000;
    cfg.tolerance = 1e-6;
    bhrt_camera cam = {{0, -29.544, 5.209}, {0, 29.544, -5.209}, {0, 0, 1}, 60.0};
    if (bhrt_render_frame(&bh, &disk, &cfg, &cam, W, H, INTEGRATOR_RK4, 0, &soa) != 0) {
        fprintf(stderr, "bhrt_render_frame: %s\n", bhrt_last_error());
        return 4;
    }
    int hist[6] = {0};
    for (int i = 0; i < W * H; i++) hist[result[i]]++;
    printf("frame %d %d %d %d %d\n", hist[0], hist[1], hist[2], hist[3], hist[4]);
    bh_shutdown(ctx);
    return 0;
}
