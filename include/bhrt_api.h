/*
 * bhrt_api.h -- C ABI of libbhrt.so, the MI355X geodesic ray tracer.
 *
 * Two groups of entry points:
 *
 *  1. Drop-in: the reference engine's own symbols, same names, arguments, return codes and
 *     struct layouts (bhrt_types.h). Each declaration names the reference interface it
 *     replaces. The ray-tracing ones (trace_ray, trace_rays_batch, integrate_photon_path,
 *     trace_pixel, bh_trace_ray, bh_trace_rays_batch) run on the GPU; there is no CPU
 *     fallback: if HIP is unavailable they return the reference's error value and
 *     bhrt_last_error() says why.
 *
 *  2. Extension (bhrt_*): whole-frame rendering with device-resident SoA outputs, row
 *     sharding for multi-GPU, and launch statistics. This is what bench.py drives.
 *
 * Host buffers are always caller-owned; nothing is retained across calls.
 */
#ifndef BHRT_API_H
#define BHRT_API_H

#include "bhrt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define BLACKHOLE_API_VERSION_MAJOR 0
#define BLACKHOLE_API_VERSION_MINOR 1
#define BLACKHOLE_API_VERSION_PATCH 0

#define BH_PI 3.14159265358979323846
#define BH_EPSILON 1.0e-10
#define BH_TWO_PI 6.28318530717958647692

typedef enum {
    BH_SUCCESS = 0,
    BH_ERROR_INVALID_PARAMETER = -1,
    BH_ERROR_MEMORY_ALLOCATION = -2,
    BH_ERROR_INITIALIZATION = -3,
    BH_ERROR_SIMULATION = -4
} BHErrorCode; /* include/blackhole_api.h:30-36 */

typedef struct BHContext_t* BHContextHandle; /* include/blackhole_api.h:40 */

/* ================================ 1. drop-in symbols ==================================== */

/* --- ray tracing (GPU) --- */

/* replaces raytracer.h:129-133 / src/raytracer.c:684-767 */
RayTraceResult trace_ray(const Ray* ray, const BlackHoleParams* blackhole,
                         const AccretionDiskParams* disk, const SimulationConfig* config,
                         RayTraceHit* hit);

/* replaces raytracer.h:205-212 / src/raytracer.c:782-807. Returns -1 if rays, blackhole or
 * hits is NULL or num_rays <= 0, else 0. num_threads is ignored (the GPU decides). */
int trace_rays_batch(const Ray* rays, int num_rays, const BlackHoleParams* blackhole,
                     const AccretionDiskParams* disk, const SimulationConfig* config,
                     RayTraceHit* hits, int num_threads);

/* replaces raytracer.h:181-190 / src/raytracer.c:338-679 */
RayTraceResult integrate_photon_path(const Vector4D* position, const Vector3D* direction,
                                     const BlackHoleParams* blackhole,
                                     const SimulationConfig* config, IntegrationMethod method,
                                     Vector3D* path_positions, int max_positions,
                                     int* num_positions, RayTraceHit* hit);

/* replaces raytracer.h:151-165 / src/raytracer.c:1044-1167 (see DESIGN.md for the colour
 * of disk samples, which the reference reads from an uninitialised field) */
RayTraceResult trace_pixel(int pixel_x, int pixel_y, int width, int height,
                           const Vector3D* camera_position, const Vector3D* camera_direction,
                           const Vector3D* camera_up, double fov,
                           const BlackHoleParams* blackhole, const AccretionDiskParams* disk,
                           const SimulationConfig* config, const SupersamplingParams* ss_params,
                           const AdaptiveSamplingParams* as_params, double color_out[3]);

/* --- ray-path helpers (host scalar code, same arithmetic as the device) --- */
int check_disk_intersection(const Vector3D* position, const Vector3D* velocity,
                            const Vector3D* prev_position, const AccretionDiskParams* disk,
                            Vector3D* hit_position);                     /* raytracer.c:159 */
void calculate_disk_temperature(const Vector3D* position, const BlackHoleParams* blackhole,
                                const AccretionDiskParams* disk, double* temperature,
                                double color[3]);                        /* raytracer.c:201 */
void apply_relativistic_effects(const Vector3D* position, const Vector3D* velocity,
                                const BlackHoleParams* blackhole, double color[3],
                                double* doppler_factor);                 /* raytracer.c:233 */
void generate_gpu_shader_params(const BlackHoleParams* blackhole,
                                const AccretionDiskParams* disk, double observer_distance,
                                double fov, GPUShaderParams* params);     /* raytracer.c:818 */
double halton_sequence(int index, int base);                             /* raytracer.c:852 */

/* spacetime.h */
void initialize_black_hole_params(BlackHoleParams* blackhole, double mass, double spin,
                                  double charge);                        /* spacetime.c:331 */
double get_isco_radius(const BlackHoleParams* blackhole);                /* spacetime.c:285 */
SchwarzschildMetric calculate_schwarzschild_metric(double r, const BlackHoleParams* bh);
                                                                         /* spacetime.c:15 */
double calculate_time_dilation(double r, const BlackHoleParams* blackhole);/* spacetime.c:192 */
void cartesian_to_spherical(const Vector3D* cartesian, Vector3D* spherical);/* spacetime.c:201 */
void spherical_to_cartesian(const Vector3D* spherical, Vector3D* cartesian);/* spacetime.c:229 */
KerrMetric calculate_kerr_metric(double r, double theta, const BlackHoleParams* blackhole);
                                                                         /* spacetime.c:38 */
BlackHoleMetric calculate_metric(double r, double theta, const BlackHoleParams* blackhole);
                                                                         /* spacetime.c:74 */
double calculate_effective_potential(double r, double l, const BlackHoleParams* blackhole);
                                                                         /* spacetime.c:242 */
double calculate_ergosphere_radius(double theta, const BlackHoleParams* blackhole);
                                                                         /* spacetime.c:314 */
int calculate_kerr_metric_bl(const double position[4], double a, double M, KerrMetric* metric);
                                                                         /* spacetime.c:377 */
int calculate_inverse_kerr_metric(const double position[4], double a, double M,
                                  KerrMetric* inv_metric);               /* spacetime.c:429 */
int calculate_kerr_christoffel(const double position[4], double a, double M,
                               double christoffel[4][4][4]);             /* spacetime.c:483 */
double calculate_kerr_isco(double a, double M, bool prograde);           /* spacetime.c:548 */
double calculate_kerr_event_horizon(double a, double M);                 /* spacetime.c:565 */
double calculate_kerr_ergosphere(double a, double M, double theta);      /* spacetime.c:577 */
int calculate_frame_dragging(const double position[4], double a, double M, double velocity[3]);
                                                                         /* spacetime.c:590 */
int calculate_kerr_geodesic(const double position[4], const double velocity[4], double a,
                            double M, double acceleration[4]);           /* spacetime.c:624 */
void calculate_christoffel_symbols(double r, double theta, const BlackHoleParams* blackhole,
                                   double christoffel[4][4][4]);         /* spacetime.c:93 */
void geodesic_equation(const double position[4], const double velocity[4],
                       const BlackHoleParams* blackhole, double acceleration[4]);
                                                                         /* spacetime.c:166 */

/* math_util.h */
Vector3D vector3D_add(const Vector3D a, const Vector3D b);               /* math_util.c:31 */
Vector3D vector3D_sub(const Vector3D a, const Vector3D b);               /* math_util.c:49 */
Vector3D vector3D_scale(const Vector3D v, double scale);                 /* math_util.c:67 */
double   vector3D_dot(const Vector3D a, const Vector3D b);               /* math_util.c:85 */
Vector3D vector3D_cross(const Vector3D a, const Vector3D b);             /* math_util.c:100 */
double   vector3D_length(const Vector3D v);                              /* math_util.c:111 */
Vector3D vector3D_normalize(const Vector3D v);                           /* math_util.c:115 */
void rk4_integrate(ODEFunction f, double* y, int n, double t, double h, void* params);
                                                                         /* math_util.c:162 */
int rkf45_integrate(ODEFunction f, double y[], int n, double* t, double h_try, double* h_next,
                    double eps_rel, void* params);                       /* math_util.c:212 */
void temperature_to_rgb(double temperature, double rgb[3]);              /* math_util.c:463 */
double clamp(double value, double min, double max);                      /* math_util.c:505 */
void leapfrog_integrate(ODEFunctionSecondOrder f, double* x, double* v, int n, double t,
                        double dt, void* params);                        /* math_util.c:125 */

/* particle_sim.h -- host bookkeeping; update_particles runs on the GPU (one lane per
 * particle). */
int particle_system_init(ParticleSystem* system, int initial_capacity);   /* particle_sim.c:73 */
void particle_system_cleanup(ParticleSystem* system);                    /* particle_sim.c:96 */
int add_particle(ParticleSystem* system, const Vector3D* position, const Vector3D* velocity,
                 double mass, ParticleType type);                        /* particle_sim.c:108 */
int update_particles(ParticleSystem* system, const BlackHoleParams* blackhole,
                     const SimulationConfig* config);                    /* particle_sim.c:505 */
/* defined (non-static) by the reference but not declared in its headers */
Particle* find_particle(ParticleSystem* system, int particle_id);        /* particle_sim.c:138 */
int remove_particle(ParticleSystem* system, int particle_id);            /* particle_sim.c:155 */
int calculate_particle_orbit(const ParticleSystem* system, int particle_id,
                             const BlackHoleParams* blackhole, OrbitalParams* params);
                                                                         /* particle_sim.c:571 */
int calculate_circular_orbit(double r, const BlackHoleParams* blackhole, Vector3D* velocity);
                                                                         /* particle_sim.c:604 */
int create_accretion_disk(ParticleSystem* system, const BlackHoleParams* blackhole,
                          const AccretionDiskParams* disk, int num_particles);
                                                                         /* particle_sim.c:339 */
int generate_hawking_radiation(ParticleSystem* system, const BlackHoleParams* blackhole,
                               int num_particles, const SimulationConfig* config);
                                                                         /* particle_sim.c:427 */

/* --- context API (include/blackhole_api.h:47-255, src/blackhole_api.c) --- */
BHContextHandle bh_initialize(void);                                     /* blackhole_api.c:52 */
void bh_shutdown(BHContextHandle context);                               /* blackhole_api.c:85 */
double blackhole_get_mass(BHContextHandle context);                      /* blackhole_api.c:33 */
void bh_calculate_orbital_velocity(BHContextHandle context, double r, double* v_phi);
                                                                         /* blackhole_api.c:42 */
BHErrorCode bh_configure_black_hole(BHContextHandle context, double mass, double spin,
                                    double charge);                      /* blackhole_api.c:94 */
BHErrorCode bh_configure_accretion_disk(BHContextHandle context, double inner_radius,
                                        double outer_radius, double temperature_scale,
                                        double density_scale);           /* blackhole_api.c:123 */
BHErrorCode bh_configure_simulation(BHContextHandle context, double time_step,
                                    double max_ray_distance, int max_integration_steps,
                                    double tolerance);                   /* blackhole_api.c:153 */
BHErrorCode bh_trace_ray(BHContextHandle context, const double origin[3],
                         const double direction[3], RayTraceHit* hit);   /* blackhole_api.c:182 */
BHErrorCode bh_trace_rays_batch(BHContextHandle context, const Ray* rays, RayTraceHit* hits,
                                int count);                              /* blackhole_api.c:225 */
void* bh_create_particle_system(BHContextHandle context, int capacity); /* blackhole_api.c:256 */
void bh_destroy_particle_system(BHContextHandle context, void* system);  /* blackhole_api.c:280 */
int bh_add_test_particle(BHContextHandle context, void* system, const double position[3],
                         const double velocity[3], double mass);         /* blackhole_api.c:296 */
int bh_create_accretion_disk_particles(BHContextHandle context, void* system,
                                       int num_particles);               /* blackhole_api.c:318 */
int bh_generate_hawking_radiation(BHContextHandle context, void* system, int num_particles);
                                                                         /* blackhole_api.c:343 */
BHErrorCode bh_update_particles(BHContextHandle context, void* system);  /* blackhole_api.c:364 */
BHErrorCode bh_get_particle_data(BHContextHandle context, void* system, double* positions,
                                 double* velocities, int* types, int* count);
                                                                         /* blackhole_api.c:384 */
BHErrorCode bh_calculate_time_dilation(BHContextHandle context, const double position1[3],
                                       const double position2[3], double* time_ratio);
                                                                         /* blackhole_api.c:432 */
void bh_get_version(int* major, int* minor, int* patch);                 /* blackhole_api.c:464 */
BHErrorCode bh_generate_shader_data(void* context, const float observer_pos[3],
                                    const float observer_dir[3], const float up_vector[3],
                                    int width, int height, float fov, int enable_doppler,
                                    int enable_redshift, int show_disk, float* output_buffer);
                                                                         /* blackhole_api.c:495 */

/* ================================ 2. bhrt extension ===================================== */

/* Pinhole camera of trace_pixel/calculate_ray_direction (raytracer.c:999-1039); fov in
 * degrees. Rays go through the pixel centres (offset 0.5, 0.5) unless use_offset is set:
 * then every pixel uses (offset_x, offset_y), e.g. one sample of trace_pixel's jitter
 * (generate_jittered_position, raytracer.c:868-932). A zero-initialised tail means centres. */
typedef struct {
    Vector3D position;
    Vector3D direction;
    Vector3D up;
    double   fov_deg;
    int      use_offset;
    double   offset_x, offset_y;
} bhrt_camera;

/* Frame flags */
#define BHRT_FLAG_DOPPLER 1 /* disk colour through apply_relativistic_effects (config C4) */

/* Structure-of-arrays frame. Element i is the i-th ray of the launch (for a camera frame:
 * the i-th pixel of the shard, row-major over the shard's rows). Any pointer may be NULL,
 * in which case that field is not produced. Pointers are device pointers for the *_device
 * calls and host pointers otherwise. */
typedef struct {
    int32_t* result;        /* RayTraceResult                                            */
    int32_t* steps;         /* RayTraceHit.steps                                         */
    double*  hit_x;         /* RayTraceHit.hit_position                                  */
    double*  hit_y;
    double*  hit_z;
    double*  distance;
    double*  time_dilation;
    double*  sky_x;         /* RayTraceHit.sky_direction, written for MAX_DISTANCE only  */
    double*  sky_y;
    double*  sky_z;
    double*  rgb_r;         /* frame colour contract, DESIGN.md section 3                */
    double*  rgb_g;
    double*  rgb_b;
    /* display path (renderer.cpp:2090-2125, the visualizer's texture buffer): 4 values per
     * pixel, row 0 = top image row */
    float*   rgba32f;       /* (float)rgb and alpha 1.0f: the compute shader's RayOutput   */
    uint8_t* rgba8;         /* (unsigned char)(std::min(1.0f, v) * 255.0f) of rgba32f      */
} bhrt_frame_soa;

/* Cyclic row-block sharding of an image across num_shards GPUs: block b (rows
 * [b*row_block, (b+1)*row_block)) belongs to shard b % num_shards. {0,0,1} = whole image. */
typedef struct {
    int row_block;
    int shard;
    int num_shards;
} bhrt_rows;

/* Launch statistics accumulated on the calling thread since the last reset. */
typedef struct {
    uint64_t rays;          /* rays traced                                               */
    uint64_t iterations;    /* executed RK4 iterations / RKF45 attempts                  */
    uint64_t stages_full;   /* ray_derivatives evaluations, a=0 strong-field branch      */
    uint64_t stages_far;    /* ... far-field branch                                      */
    uint64_t stages_kerr;   /* ... spin != 0 branch                                      */
    uint64_t launches;      /* trace-kernel launches timed                               */
    double   kernel_ms;     /* sum of HIP-event durations of those launches              */
    uint64_t rays_redone;   /* rays re-traced on the large-argument sincos path          */
    double   span_ms;       /* per GPU: first trace-kernel start to last trace-kernel end
                               since the reset (summed over GPUs); launches overlapping on
                               several streams make this, not kernel_ms, the GPU time     */
    uint64_t redo_launches; /* of those launches, how many were followed by the redo pass
                               (left out where no ray can need it)   */
    /* per launch, the frame's execution window on the GPU's constant-rate wall clock: its
     * first trace wave's start to its last store (the trace kernel's last wave, or the separate
     * colour pass's last workgroup) -- the frame's completion latency once it runs */
    double   frame_ms;      /* sum over the timed launches                               */
    double   frame_ms_max;  /* the longest                                               */
    uint64_t frames_timed;  /* launches with a window (0 where the clock rate is unknown) */
    uint64_t attempts_untested; /* of `iterations`, the RKF45 attempts run without the error
                               estimate and accept test: launches where the host proved every
                               attempt passes (zero-acceleration paths)     */
} bhrt_stats;

/* Number of rows of an image of `height` rows owned by shard rows->shard. */
int bhrt_shard_rows(int height, const bhrt_rows* rows);

/* Render (a shard of) a camera frame into DEVICE SoA buffers on `hip_stream` (a
 * hipStream_t). Asynchronous: returns after the launch. hip_stream NULL behaves like a launch
 * on the legacy default stream: the frame is ordered after all work the caller queued there
 * (e.g. a hipMemset or a torch fill of the output arrays) and before all work queued there
 * afterwards (e.g. a hipMemcpy of the results); the kernels run on the library's per-thread
 * stream, linked to the default stream by two event waits. BHRT_NULL_STREAM=unordered drops
 * that ordering (the library's stream alone). Returns 0, or -1 on invalid arguments / HIP
 * failure (see bhrt_last_error). */
int bhrt_render_frame_device(const BlackHoleParams* blackhole, const AccretionDiskParams* disk,
                             const SimulationConfig* config, const bhrt_camera* camera,
                             int width, int height, const bhrt_rows* rows,
                             IntegrationMethod method, int flags,
                             const bhrt_frame_soa* device_out, void* hip_stream);

/* One camera frame rendered by several GPUs and gathered on the calling thread's CURRENT device
 * (the root) -- the north star's "image tiled across the GPUs, one gather at frame end", from C:
 * the image is split into `shards` cyclic row-block shards of 8 rows (<= 0: one per device),
 * shard s rendered by device (root + s) mod ndev into that device's own buffers (ndev <= 0:
 * every visible device), and the root copies every shard straight into its image rows of
 * device_out -- device-to-device over xGMI for the peers (peer access enabled on first use),
 * one strided 2-D copy per field and shard. device_out: root-device buffers of width * height
 * elements per field (NULL fields are not produced). Asynchronous on hip_stream (a root-device
 * hipStream_t): the frame is complete when that stream's work is; NULL = ordered like the
 * root's legacy default stream, as for bhrt_render_frame_device. A
 * one-shard frame is bhrt_render_frame_device on the root. Replaces the reference's serial
 * per-pixel loop (raytracer.c:795-804 / blackhole_api.c:225-250) on a multi-GPU node. */
int bhrt_render_frame_gather(const BlackHoleParams* blackhole, const AccretionDiskParams* disk,
                             const SimulationConfig* config, const bhrt_camera* camera,
                             int width, int height, IntegrationMethod method, int flags,
                             const bhrt_frame_soa* device_out, int ndev, int shards,
                             void* hip_stream);

/* Same, into HOST buffers; splits the image over every visible GPU (cyclic row blocks)
 * and returns when the frame is complete. */
int bhrt_render_frame(const BlackHoleParams* blackhole, const AccretionDiskParams* disk,
                      const SimulationConfig* config, const bhrt_camera* camera, int width,
                      int height, IntegrationMethod method, int flags,
                      const bhrt_frame_soa* host_out);

/* Asynchronous form of bhrt_render_frame: queues the frame and returns a ticket (> 0) in
 * *ticket; the host arrays receive the frame through libbhrt's pinned staging (caller memory
 * is never page-locked) and must not be read or freed before bhrt_frame_wait(ticket) returns. Three
 * frames may be in flight per host thread; a fourth issue first completes the oldest frame,
 * whose own bhrt_frame_wait then returns its result (once). Each frame needs its own arrays. */
int bhrt_render_frame_async(const BlackHoleParams* blackhole, const AccretionDiskParams* disk,
                            const SimulationConfig* config, const bhrt_camera* camera, int width,
                            int height, IntegrationMethod method, int flags,
                            const bhrt_frame_soa* host_out, int* ticket);

/* Wait for a frame queued by bhrt_render_frame_async; 0 when its host arrays are complete. */
int bhrt_frame_wait(int ticket);

/* Trace n rays already resident on the device (AoS Ray[n]) into DEVICE SoA buffers.
 * method RK4 with disk != NULL is trace_ray; RKF45 with a disk is integrate_photon_path
 * plus trace_ray's disk scan (config C3). hip_stream as for bhrt_render_frame_device (NULL:
 * ordered like the legacy default stream). */
int bhrt_trace_rays_device(const Ray* device_rays, int n, const BlackHoleParams* blackhole,
                           const AccretionDiskParams* disk, const SimulationConfig* config,
                           IntegrationMethod method, int flags,
                           const bhrt_frame_soa* device_out, void* hip_stream);

/* Host-buffer variant of the above (host Ray[n] in, host SoA out), multi-GPU split. */
int bhrt_trace_rays(const Ray* rays, int n, const BlackHoleParams* blackhole,
                    const AccretionDiskParams* disk, const SimulationConfig* config,
                    IntegrationMethod method, int flags, const bhrt_frame_soa* host_out);

/* Diagnostic: both forms of the trace kernel's RKF45 accept test (the division-free fast
 * form and the reference's literal quotient, geodesic.hip rkf45_accept) on n cases of DEVICE
 * arrays err[6n], scale[6n], tol[n]; d_out[2i] / d_out[2i+1] = the two decisions. Returns 0
 * or a hipError_t value; asynchronous on hip_stream. */
int bhrt_check_rkf45_accept(const double* err, const double* scale, const double* tol, int n,
                            int* out, void* hip_stream);

/* Copy and optionally reset this thread's statistics (waits for the timed launches, then reads
 * their counters with a synchronous copy on the legacy default stream, i.e. also after the
 * caller's default-stream work). out == NULL with reset != 0 drops the pending launches'
 * counters unread (no per-launch event timing): the cheap reset before a timed region. Returns
 * -1 if a launch whose redo pass was proved unnecessary handed a ray to it (bhrt_last_error). */
int bhrt_get_stats(bhrt_stats* out, int reset);

/* Number of GPUs libbhrt will use (HIP_VISIBLE_DEVICES / BHRT_MAX_DEVICES respected). */
int bhrt_device_count(void);

/* Tuning knob: refill a wavefront's finished lanes once at least this many are idle
 * (1..64; 0 = per scene: 8 for RK4 at spin 0, else 64). Affects speed only. */
void bhrt_set_refill_threshold(int lanes);

/* Tuning knob: the order in which this thread's next bhrt_render_frame_device calls of n rays
 * claim their rays -- d_order, an int array on the CURRENT device holding a permutation of
 * [0, n) (NULL or n = 0: the default order). Results are the same in any order; only the
 * schedule changes. The array is checked to be a permutation here (one D2H copy): returns 0,
 * or -1 (and the default order) if it is not. It applies only to device-API frames of exactly
 * n rays on the device that was current here, never to the chunks of bhrt_render_frame[_async]
 * host frames. libbhrt keeps the pointer: it must stay valid until the order is cleared
 * (bhrt_set_claim_order(NULL, 0)) or replaced. The check is a blocking copy on the legacy null
 * stream, which is NOT ordered after work on non-blocking streams (torch's, libbhrt's own):
 * synchronise the stream that wrote d_order before this call. The check costs a D2H copy, a
 * host sync and an O(n) scan per call; BHRT_TRUST_CLAIM_ORDER=1 skips it (the caller then
 * guarantees a permutation). Returns int since round 4 (void before). */
int bhrt_set_claim_order(const int* d_order, int n);

/* update_particles (particle_sim.c:505-566) applied `steps` times in one device round trip:
 * the particle array is copied to the GPU once, stepped `steps` times by the HIP kernel and
 * copied back (steps == 1 is exactly update_particles). Returns 0, or -1 on invalid
 * arguments / HIP failure. If kernel_ms is not NULL it receives the kernels' HIP-event time. */
int bhrt_update_particles_steps(ParticleSystem* system, const BlackHoleParams* blackhole,
                                const SimulationConfig* config, int steps, double* kernel_ms);

/* Last error message of the calling thread ("" if none). */
const char* bhrt_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* BHRT_API_H */
