/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Frame/batch driver around the COMPILED REFERENCE (oracle/_ref/libref.so is built from the
 * unmodified sources under /root/reference/src by oracle/Makefile; no reference source is
 * copied into this repository). It calls the reference's own trace_ray,
 * integrate_photon_path, check_disk_intersection, calculate_disk_temperature and
 * apply_relativistic_effects; only the static calculate_ray_direction
 * (raytracer.c:999-1039) is taken from the oracle restatement, and it is pinned separately
 * against the reference's trace_pixel (tests/test_oracle_golden.py).
 *
 * Used to generate tests/golden/ and as the "reference" CPU baseline of bench.py
 * (OpenMP parallel-for over rays; the reference itself is single-threaded).
 * The reference prints debug lines per ray / per RKF45 attempt; refdrv_quiet(1) sends
 * fd 1 to /dev/null around the traced region.
 */
#include "oracle.h"

#include <fcntl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* reference symbols (same prototypes as include/bhrt_api.h declares) */
RayTraceResult trace_ray(const Ray*, const BlackHoleParams*, const AccretionDiskParams*,
                         const SimulationConfig*, RayTraceHit*);
RayTraceResult integrate_photon_path(const Vector4D*, const Vector3D*, const BlackHoleParams*,
                                     const SimulationConfig*, IntegrationMethod, Vector3D*, int,
                                     int*, RayTraceHit*);
int check_disk_intersection(const Vector3D*, const Vector3D*, const Vector3D*,
                            const AccretionDiskParams*, Vector3D*);
void calculate_disk_temperature(const Vector3D*, const BlackHoleParams*,
                                const AccretionDiskParams*, double*, double[3]);
void apply_relativistic_effects(const Vector3D*, const Vector3D*, const BlackHoleParams*,
                                double[3], double*);
double vector3D_length(const Vector3D v);
Vector3D vector3D_sub(const Vector3D a, const Vector3D b);
double calculate_time_dilation(double r, const BlackHoleParams* blackhole);

static int saved_fd = -1;
void refdrv_quiet(int on) {
    fflush(stdout);
    if (on && saved_fd < 0) {
        int devnull = open("/dev/null", O_WRONLY);
        if (devnull < 0) return;
        saved_fd = dup(1);
        dup2(devnull, 1);
        close(devnull);
    } else if (!on && saved_fd >= 0) {
        dup2(saved_fd, 1);
        close(saved_fd);
        saved_fd = -1;
    }
}

/* trace_ray, or (method != RK4) integrate_photon_path + trace_ray's disk scan
 * (raytracer.c:698-759): the C3 composition of SURVEY.md 8(d). */
static RayTraceResult ref_trace(const Ray* ray, const BlackHoleParams* bh,
                                const AccretionDiskParams* disk, const SimulationConfig* cfg,
                                IntegrationMethod method, RayTraceHit* hit) {
    if (method == INTEGRATOR_RK4) return trace_ray(ray, bh, disk, cfg, hit);
    Vector4D pos = {0.0, ray->origin.x, ray->origin.y, ray->origin.z};
    int maxp = 0, np = 0;
    Vector3D* path = NULL;
    if (disk) {
        maxp = cfg->max_integration_steps;
        path = (Vector3D*)malloc((size_t)(maxp > 0 ? maxp : 1) * sizeof(Vector3D));
    }
    RayTraceResult res = integrate_photon_path(&pos, &ray->direction, bh, cfg, method, path, maxp,
                                               &np, hit);
    if (disk && path && np > 1) {
        for (int i = 1; i < np; i++) {
            Vector3D q;
            if (check_disk_intersection(&path[i], &ray->direction, &path[i - 1], disk, &q)) {
                hit->result = RAY_DISK;
                hit->hit_position = q;
                double d = 0.0;
                for (int j = 1; j <= i; j++) d += vector3D_length(vector3D_sub(path[j], path[j - 1]));
                d += vector3D_length(vector3D_sub(q, path[i - 1]));
                hit->distance = d;
                hit->steps = i;
                hit->time_dilation = calculate_time_dilation(vector3D_length(q), bh);
                res = RAY_DISK;
                break;
            }
        }
    }
    free(path);
    return res;
}

static void colour(int res, const Vector3D* q, const Vector3D* dir, const BlackHoleParams* bh,
                   const AccretionDiskParams* disk, int flags, double rgb[3]) {
    if (res == RAY_DISK) {
        double T;
        calculate_disk_temperature(q, bh, disk, &T, rgb);
        if (flags & BHRT_FLAG_DOPPLER) apply_relativistic_effects(q, dir, bh, rgb, NULL);
    } else if (res == RAY_HORIZON) {
        rgb[0] = rgb[1] = rgb[2] = 0.0;
    } else { /* raytracer.c:1150-1157 */
        double t = 0.5 * (dir->y + 1.0);
        rgb[0] = (1.0 - t) * 1.0 + t * 0.5;
        rgb[1] = (1.0 - t) * 1.0 + t * 0.7;
        rgb[2] = (1.0 - t) * 1.0 + t * 1.0;
    }
}

static void put(const bhrt_frame_soa* o, long i, const RayTraceHit* h, const double rgb[3]) {
    if (o->result) o->result[i] = h->result;
    if (o->steps) o->steps[i] = h->steps;
    if (o->hit_x) o->hit_x[i] = h->hit_position.x;
    if (o->hit_y) o->hit_y[i] = h->hit_position.y;
    if (o->hit_z) o->hit_z[i] = h->hit_position.z;
    if (o->distance) o->distance[i] = h->distance;
    if (o->time_dilation) o->time_dilation[i] = h->time_dilation;
    int sky = h->result == RAY_MAX_DISTANCE;
    if (o->sky_x) o->sky_x[i] = sky ? h->sky_direction.x : 0.0;
    if (o->sky_y) o->sky_y[i] = sky ? h->sky_direction.y : 0.0;
    if (o->sky_z) o->sky_z[i] = sky ? h->sky_direction.z : 0.0;
    if (o->rgb_r) o->rgb_r[i] = rgb[0];
    if (o->rgb_g) o->rgb_g[i] = rgb[1];
    if (o->rgb_b) o->rgb_b[i] = rgb[2];
}

int refdrv_render_frame(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                        const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                        const bhrt_rows* rows, IntegrationMethod method, int flags,
                        const bhrt_frame_soa* out, int nthreads) {
    if (!bh || !cfg || !cam || !out || W <= 0 || H <= 0) return -1;
    long n = (long)orc_shard_rows(H, rows) * W;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (long i = 0; i < n; i++) {
        int x = (int)(i % W), y = orc_shard_row((int)(i / W), rows);
        Vector3D dir;
        orc_camera_ray_direction(x, y, cam->use_offset ? cam->offset_x : 0.5,
                                 cam->use_offset ? cam->offset_y : 0.5, W, H, cam, &dir);
        Ray ray = {cam->position, dir};
        RayTraceHit h;
        memset(&h, 0, sizeof h);
        ref_trace(&ray, bh, disk, cfg, method, &h);
        double rgb[3];
        colour(h.result, &h.hit_position, &dir, bh, disk, flags, rgb);
        put(out, i, &h, rgb);
    }
    return 0;
}

int refdrv_trace_rays(const Ray* rays, int n, const BlackHoleParams* bh,
                      const AccretionDiskParams* disk, const SimulationConfig* cfg,
                      IntegrationMethod method, int flags, const bhrt_frame_soa* out,
                      int nthreads) {
    if (!rays || !bh || !cfg || !out || n <= 0) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        RayTraceHit h;
        memset(&h, 0, sizeof h);
        ref_trace(&rays[i], bh, disk, cfg, method, &h);
        double rgb[3];
        colour(h.result, &h.hit_position, &rays[i].direction, bh, disk, flags, rgb);
        put(out, i, &h, rgb);
    }
    return 0;
}
