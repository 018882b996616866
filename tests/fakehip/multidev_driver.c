/* multidev_driver.c -- libbhrt's host layer (bhrt_api.c) on SIMULATED devices (fake_hip.c):
 * frames split over two devices and several chunks, DMA'd or staged into caller arrays,
 * frames in flight (bhrt_render_frame_async), ray batches split over the devices and the
 * pipelined trace_rays_batch, all from two host threads at once. Built by
 * tests/test_multidevice_host.py under ASan+UBSan and under TSan.
 *
 * The trace launcher is a stub that checks the launch against the simulated device that is
 * current (every buffer of the launch must be that device's memory) and writes an encoding
 * of the ray's IMAGE pixel index (camera frames: the kernel's cyclic row-block map) or of
 * its input ray (ray arrays) into every output field, so the test sees exactly where every
 * value landed. Test infrastructure only. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "bhrt_api.h"
#include "bhrt_kernel.h"

int fakehip_kind_of(const void* p, size_t n);
int fakehip_current_device(void);
void fakehip_declare_host(const void* p, size_t n);
void fakehip_forget_host(const void* p);

static int g_fail;
#define CHECK(x, ...)                                                        \
    do {                                                                     \
        if (!(x)) {                                                          \
            fprintf(stderr, "CHECK failed %s:%d: %s: ", __FILE__, __LINE__, #x); \
            fprintf(stderr, __VA_ARGS__);                                    \
            fputc('\n', stderr);                                             \
            __atomic_add_fetch(&g_fail, 1, __ATOMIC_RELAXED);                \
        }                                                                    \
    } while (0)

static const size_t fsize[15] = {4, 4, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 16, 4};

static void on_device(const void* p, size_t n, const char* what) {
    if (!p) return;
    const int k = fakehip_kind_of(p, n);
    if (k != fakehip_current_device()) {
        fprintf(stderr, "launch buffer %s (%zu B) is memory kind %d, launching on device %d\n",
                what, n, k, fakehip_current_device());
        abort();
    }
}

/* the value every field gets for image pixel / input ray v */
static double enc(int f, long v) { return (double)v * 4.0 + f + 0.25; }

static long g_shared_launches; /* ray launches that took the shared-origin set-up */
int bhrt_trace_untested(const bhrt_kparams* kp) { (void)kp; return 0; }
int bhrt_launch_trace(const bhrt_kparams* kp, void* stream, void* ev0, void* ev1) {
    (void)stream; (void)ev0; (void)ev1;
    const long n = kp->n;
    void* const* out = (void* const*)&kp->out;
    for (int f = 0; f < 15; f++) on_device(out[f], fsize[f] * n, "output field");
    on_device(kp->ctl, 8 * 8, "control block");
    on_device(kp->qhead, 8, "queue heads");
    on_device(kp->init, (size_t)(BHRT_INIT_FIELDS + 1) * 8 * n, "init table");
    if (kp->src == BHRT_SRC_RAYS && !kp->rays_shared) on_device(kp->rays, sizeof(Ray) * n, "rays");
    if (kp->src == BHRT_SRC_RAYS && kp->rays_shared) {
        on_device(kp->dirs, 8 * ((size_t)kp->dir_stride * (n - 1) + 3), "directions");
        if (kp->rays) on_device(kp->rays, sizeof(Ray) * n, "rays");
    }
    for (long i = 0; i < n; i++) {
        long v;
        if (kp->src == BHRT_SRC_CAMERA) {
            const long W = kp->cam.width, j = i / W, px = i % W;
            long py = j;
            if (kp->cam.rows.num_shards > 1) {
                const long B = kp->cam.rows.row_block;
                py = ((j / B) * kp->cam.rows.num_shards + kp->cam.rows.shard) * B + j % B;
            }
            v = py * W + px;
        } else if (kp->rays_shared) { /* one origin (the host said so): the id rides in dx */
            if (kp->rays && (memcmp(&kp->rays[i].origin.x, &kp->cam.pos[0], 8) ||
                             memcmp(&kp->rays[i].origin.y, &kp->cam.pos[1], 8) ||
                             memcmp(&kp->rays[i].origin.z, &kp->cam.pos[2], 8))) {
                fprintf(stderr, "rays_shared launch with a ray off the shared origin\n");
                abort();
            }
            v = (long)kp->dirs[(size_t)i * kp->dir_stride];
        } else {
            v = (long)kp->rays[i].origin.x;
        }
        if (kp->out.result) kp->out.result[i] = (int)(v % 5);
        if (kp->out.steps) kp->out.steps[i] = (int)v;
        double* d[11] = {kp->out.hit_x, kp->out.hit_y, kp->out.hit_z, kp->out.distance,
                         kp->out.time_dilation, kp->out.sky_x, kp->out.sky_y, kp->out.sky_z,
                         kp->out.rgb_r, kp->out.rgb_g, kp->out.rgb_b};
        for (int f = 0; f < 11; f++)
            if (d[f]) d[f][i] = enc(f + 2, v);
        if (kp->out.rgba32f)
            for (int c = 0; c < 4; c++) kp->out.rgba32f[4 * i + c] = (float)(v + c);
        if (kp->out.rgba8)
            for (int c = 0; c < 4; c++) kp->out.rgba8[4 * i + c] = (uint8_t)(v + c);
    }
    kp->ctl[1] += (unsigned long long)n; /* rays */
    if (kp->src == BHRT_SRC_RAYS && kp->rays_shared)
        __atomic_fetch_add(&g_shared_launches, 1, __ATOMIC_RELAXED);
    return 0;
}
int bhrt_launch_path(const bhrt_kparams* kp, const double* o, const double* d, Vector3D* p,
                     int m, int* nn, int nin, void* st) {
    (void)kp; (void)o; (void)d; (void)p; (void)m; (void)nn; (void)nin; (void)st;
    return 100;
}
int bhrt_launch_particles(Particle* d, int count, const bhrt_particle_k* k, int steps,
                          void* stream, void* ev0, void* ev1) {
    (void)d; (void)count; (void)k; (void)steps; (void)stream; (void)ev0; (void)ev1;
    return 100;
}

typedef struct {
    void* base;
    bhrt_frame_soa soa;
} host_soa;

/* caller arrays for n pixels: the fields in `mask` (bit f = field f of bhrt_frame_soa), either
 * separate allocations or carved back to back out of one allocation at an odd offset */
static host_soa soa_new(long n, unsigned mask, int one_buffer) {
    host_soa h;
    memset(&h, 0, sizeof h);
    size_t total = 0;
    for (int f = 0; f < 15; f++)
        if (mask >> f & 1) total += fsize[f] * n;
    char* p = NULL;
    if (one_buffer) {
        h.base = malloc(total + 4096 + 1000);
        memset(h.base, 0x5A, total + 4096 + 1000);
        p = (char*)h.base + 1000;
    }
    void** slot = (void**)&h.soa;
    for (int f = 0; f < 15; f++) {
        if (!(mask >> f & 1)) continue;
        if (one_buffer) {
            slot[f] = p;
            p += fsize[f] * n;
        } else {
            slot[f] = malloc(fsize[f] * n);
            memset(slot[f], 0x5A, fsize[f] * n);
        }
        fakehip_declare_host(slot[f], fsize[f] * n);
    }
    return h;
}
static void soa_free(host_soa* h) {
    void** slot = (void**)&h->soa;
    for (int f = 0; f < 15; f++)
        if (slot[f]) fakehip_forget_host(slot[f]);
    if (h->base) {
        free(h->base);
        return;
    }
    for (int f = 0; f < 15; f++) free(slot[f]);
}

static void check_frame(const host_soa* h, long n, const char* what) {
    const bhrt_frame_soa* s = &h->soa;
    long bad = 0;
    for (long p = 0; p < n && bad < 3; p++) {
        if (s->result && s->result[p] != (int)(p % 5)) bad++;
        if (s->steps && s->steps[p] != (int)p) bad++;
        double* d[11] = {s->hit_x, s->hit_y, s->hit_z, s->distance, s->time_dilation, s->sky_x,
                         s->sky_y, s->sky_z, s->rgb_r, s->rgb_g, s->rgb_b};
        for (int f = 0; f < 11; f++)
            if (d[f] && d[f][p] != enc(f + 2, p)) bad++;
        if (s->rgba32f && s->rgba32f[4 * p + 3] != (float)(p + 3)) bad++;
        if (s->rgba8 && s->rgba8[4 * p + 1] != (uint8_t)(p + 1)) bad++;
        if (bad) fprintf(stderr, "%s: pixel %ld wrong\n", what, p);
    }
    CHECK(bad == 0, "%s", what);
}

static void run(BlackHoleParams* bh, SimulationConfig* cfg, AccretionDiskParams* dk, int tid) {
    const bhrt_camera cam = {{0, -29.544, 5.209}, {0, 29.544, -5.209}, {0, 0, 1}, 60.0, 0, 0.5, 0.5};
    const unsigned ALL = (1u << 13) - 1, RGB_DISPLAY = (1u << 0) | (1u << 2) | (1u << 3) |
                                                        (7u << 10) | (3u << 13);
    /* synchronous frames: sizes below and above the DMA threshold, uneven shard heights */
    const int sizes[][2] = {{64, 40}, {333, 77}, {1024, 523}, {1920, 1080}};
    for (int i = 0; i < 4; i++) {
        const int W = sizes[i][0], H = sizes[i][1];
        const long n = (long)W * H;
        for (int v = 0; v < 3; v++) {
            host_soa h = soa_new(n, v == 1 ? RGB_DISPLAY : ALL, v == 2);
            char what[96];
            snprintf(what, sizeof what, "thread %d frame %dx%d variant %d", tid, W, H, v);
            CHECK(bhrt_render_frame(bh, dk, cfg, &cam, W, H, INTEGRATOR_RK4, 0, &h.soa) == 0,
                  "%s: %s", what, bhrt_last_error());
            check_frame(&h, n, what);
            soa_free(&h);
        }
    }
    /* a discarding reset (bench.py's, before its timed frames) drops this thread's pending
     * launches unread; the frames below are counted afresh */
    {
        bhrt_stats z;
        CHECK(bhrt_get_stats(NULL, 1) == 0, "discarding stats reset: %s", bhrt_last_error());
        CHECK(bhrt_get_stats(&z, 0) == 0 && z.launches == 0 && z.rays == 0 && z.kernel_ms == 0.0,
              "stats after a discarding reset: %llu launches", (unsigned long long)z.launches);
    }
    /* frames in flight: 5 queued (the 4th and 5th wait for the oldest slots) */
    {
        const int W = 1500, H = 900;
        const long n = (long)W * H;
        host_soa h[5];
        int t[5];
        for (int k = 0; k < 5; k++) {
            h[k] = soa_new(n, k & 1 ? RGB_DISPLAY : ALL, k == 2);
            CHECK(bhrt_render_frame_async(bh, dk, cfg, &cam, W, H, INTEGRATOR_RK4, 0, &h[k].soa,
                                          &t[k]) == 0 && t[k] > 0,
                  "async issue %d: %s", k, bhrt_last_error());
        }
        /* three slots: the 4th and 5th issues completed the 1st and 2nd frames, whose own
         * waits still return their result (0) once */
        for (int k = 0; k < 5; k++) CHECK(bhrt_frame_wait(t[k]) == 0, "wait %d: %s", k, bhrt_last_error());
        CHECK(bhrt_frame_wait(t[0]) == -1, "second wait of an implicitly completed ticket");
        CHECK(bhrt_frame_wait(t[4]) == -1, "second wait of a ticket");
        for (int k = 0; k < 5; k++) {
            check_frame(&h[k], n, "async frame");
            soa_free(&h[k]);
        }
    }
    /* device frames gathered on a root device (bhrt_render_frame_gather): every root, one
     * shard per device and more shards than devices, uneven heights (a partial last block) */
    {
        const int gsz[][2] = {{64, 40}, {333, 77}, {200, 123}};
        const int gshards[] = {0, 3, 5};
        for (int root = 0; root < 2; root++)
            for (int i = 0; i < 3; i++)
                for (int j = 0; j < 3; j++) {
                    const int W = gsz[i][0], H = gsz[i][1];
                    const long n = (long)W * H;
                    const unsigned mask = j == 1 ? RGB_DISPLAY : ALL;
                    CHECK(hipSetDevice(root) == hipSuccess, "set root");
                    bhrt_frame_soa dev;
                    memset(&dev, 0, sizeof dev);
                    void** slot = (void**)&dev;
                    for (int f = 0; f < 15; f++)
                        if (mask >> f & 1) CHECK(hipMalloc(&slot[f], fsize[f] * n) == hipSuccess, "malloc");
                    char what[96];
                    snprintf(what, sizeof what, "thread %d gather root %d %dx%d shards %d", tid, root,
                             W, H, gshards[j]);
                    CHECK(bhrt_render_frame_gather(bh, dk, cfg, &cam, W, H, INTEGRATOR_RK4, 0, &dev,
                                                   0, gshards[j], NULL) == 0,
                          "%s: %s", what, bhrt_last_error());
                    int cur = -1;
                    CHECK(hipGetDevice(&cur) == hipSuccess && cur == root, "%s: root stays current", what);
                    host_soa h = soa_new(n, mask, 0);
                    void** hs = (void**)&h.soa;
                    for (int f = 0; f < 15; f++)
                        if (slot[f]) {
                            CHECK(hipMemcpy(hs[f], slot[f], fsize[f] * n, hipMemcpyDeviceToHost) ==
                                      hipSuccess, "readback");
                            hipFree(slot[f]);
                        }
                    check_frame(&h, n, what);
                    soa_free(&h);
                }
        CHECK(hipSetDevice(0) == hipSuccess, "reset device");
    }
    /* ray batches: SoA split over the devices, and the pipelined RayTraceHit path */
    /* pass 2: every ray at one origin (its id in direction.x): the shared-origin set-up */
    for (int pass = 0; pass < 3; pass++) {
        const long n = pass ? 300001 : 100003;
        Ray* rays = (Ray*)calloc(n, sizeof(Ray));
        for (long i = 0; i < n; i++) {
            if (pass == 2) {
                rays[i].origin.x = 1.0;
                rays[i].origin.y = -2.0;
                rays[i].origin.z = 30.0;
                rays[i].direction.x = (double)i;
            } else {
                rays[i].origin.x = (double)i;
            }
            rays[i].direction.z = 1.0;
        }
        const long shared0 = __atomic_load_n(&g_shared_launches, __ATOMIC_RELAXED);
        if (!pass) {
            host_soa h = soa_new(n, ALL, 0);
            CHECK(bhrt_trace_rays(rays, (int)n, bh, dk, cfg, INTEGRATOR_RK4, 0, &h.soa) == 0,
                  "bhrt_trace_rays: %s", bhrt_last_error());
            check_frame(&h, n, "bhrt_trace_rays");
            soa_free(&h);
        } else {
            RayTraceHit* hits = (RayTraceHit*)malloc(n * sizeof(RayTraceHit));
            for (long i = 0; i < n; i++) {
                memset(&hits[i], 0, sizeof hits[i]);
                hits[i].hit_normal.x = -7.0; /* never written by trace_ray */
            }
            CHECK(trace_rays_batch(rays, (int)n, bh, dk, cfg, hits, 4) == 0, "trace_rays_batch: %s",
                  bhrt_last_error());
            long bad = 0;
            for (long i = 0; i < n; i++) {
                const int sky = (int)(i % 5) == RAY_MAX_DISTANCE;
                if (hits[i].steps != (int)i || (int)hits[i].result != (int)(i % 5) ||
                    hits[i].hit_position.y != enc(3, i) || hits[i].distance != enc(5, i) ||
                    hits[i].hit_normal.x != -7.0 ||
                    hits[i].sky_direction.x != (sky ? enc(7, i) : 0.0))
                    bad++;
            }
            CHECK(bad == 0, "trace_rays_batch: %ld hits wrong", bad);
            /* (the other thread's launches count too: only "at least one" is per-thread) */
            if (pass == 2)
                CHECK(__atomic_load_n(&g_shared_launches, __ATOMIC_RELAXED) > shared0,
                      "shared-origin batch took the per-ray set-up");
            free(hits);
        }
        free(rays);
    }
    bhrt_stats st;
    CHECK(bhrt_get_stats(&st, 1) == 0 && st.launches > 0 && st.rays > 0, "stats");
    /* the control ring: 700 device frames over three streams with no wait between them. The
     * launch that finds the ring full harvests its older half and reuses those slots (bhrt_api.c
     * harvest); the launcher above adds each launch's rays to its slot's counter, so a slot
     * reused without being zeroed, or a launch counted twice or never, shows in the total. */
    {
        const int W = 16, H = 8, frames = 700;
        const long n = (long)W * H;
        CHECK(hipSetDevice(0) == hipSuccess, "ring: device");
        bhrt_frame_soa dev;
        memset(&dev, 0, sizeof dev);
        void** slot = (void**)&dev;
        for (int f = 0; f < 15; f++)
            if (ALL >> f & 1) CHECK(hipMalloc(&slot[f], fsize[f] * n) == hipSuccess, "ring: malloc");
        hipStream_t s3[3];
        for (int k = 0; k < 3; k++)
            CHECK(hipStreamCreateWithFlags(&s3[k], 0) == hipSuccess, "ring: stream");
        for (int k = 0; k < frames; k++)
            CHECK(bhrt_render_frame_device(bh, dk, cfg, &cam, W, H, NULL, INTEGRATOR_RK4, 0, &dev,
                                           s3[k % 3]) == 0,
                  "ring: frame %d: %s", k, bhrt_last_error());
        CHECK(bhrt_get_stats(&st, 1) == 0 && st.launches == (uint64_t)frames &&
                  st.rays == (uint64_t)(frames * n),
              "ring: %llu launches, %llu rays (want %d, %ld)", (unsigned long long)st.launches,
              (unsigned long long)st.rays, frames, frames * n);
        for (int f = 0; f < 15; f++)
            if (slot[f]) hipFree(slot[f]);
    }
}

static BlackHoleParams g_bh;
static SimulationConfig g_cfg;
static AccretionDiskParams g_dk;

static void* thread_main(void* arg) {
    run(&g_bh, &g_cfg, &g_dk, (int)(long)arg);
    return NULL;
}

int main(void) {
    CHECK(bhrt_device_count() == 2, "two simulated devices, got %d", bhrt_device_count());
    initialize_black_hole_params(&g_bh, 1.0, 0.0, 0.0);
    g_dk.inner_radius = 6.0;
    g_dk.outer_radius = 20.0;
    g_dk.temperature_scale = 1.0;
    g_cfg.time_step = 0.1;
    g_cfg.max_ray_distance = 100.0;
    g_cfg.max_integration_steps = 1000;
    g_cfg.tolerance = 1e-6;
    const char* nt = getenv("DRIVER_THREADS");
    const int threads = nt ? atoi(nt) : 2;
    pthread_t th[8];
    for (int i = 0; i < threads; i++) pthread_create(&th[i], NULL, thread_main, (void*)(long)i);
    for (int i = 0; i < threads; i++) pthread_join(th[i], NULL);
    if (g_fail) {
        fprintf(stderr, "%d checks failed\n", g_fail);
        return 1;
    }
    printf("multidev driver: all checks passed (%d threads)\n", threads);
    return 0;
}
