/*
 * bhrt_types.h -- value types of the geodesic ray-tracing ABI.
 *
 * These are the structs and enums that cross the C boundary of the reference engine
 * (Klaudiusz321/raytracing-engine-in-c). Names, member order and therefore the x86-64 SysV
 * layout are the reference's, so a caller compiled against the reference headers can link
 * against libbhrt.so unchanged:
 *
 *   Vector3D / Vector4D / Ray / SchwarzschildMetric    include/blackhole_types.h:15-47
 *   BlackHoleParams / AccretionDiskParams              include/blackhole_types.h:77-98
 *   SimulationConfig                                   include/blackhole_types.h:103-115
 *   RayTraceResult / IntegrationMethod / JitterMethod  include/raytracer.h:16-44
 *   SupersamplingParams / AdaptiveSamplingParams       include/raytracer.h:49-64
 *   RayTraceHit                                        include/raytracer.h:79-92
 *   GPUShaderParams                                    include/raytracer.h:97-106
 *
 * The layout is pinned by the static asserts at the bottom (offsets measured on the compiled
 * reference).
 */
#ifndef BHRT_TYPES_H
#define BHRT_TYPES_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- geometry ---------------------------------------------------------------------------- */
typedef struct { double x, y, z; } Vector3D;
typedef struct { double t, x, y, z; } Vector4D;

/* origin + direction; trace_ray does not require a unit direction (it normalises a copy) */
typedef struct { Vector3D origin; Vector3D direction; } Ray;

typedef struct { double g_tt, g_rr, g_thth, g_phph; } SchwarzschildMetric;

/* include/blackhole_types.h:53-72 (Kerr helpers of spacetime.c) */
typedef struct {
    double g_tt, g_tphi, g_rr, g_thth;
    double g_thetatheta;         /* set by calculate_kerr_metric_bl only                    */
    double g_phiphi, g_phit;
} KerrMetric;

typedef struct {
    int is_kerr;
    union {
        SchwarzschildMetric schwarzschild;
        KerrMetric kerr;
    } metric;
} BlackHoleMetric;

/* ---- physical scene ---------------------------------------------------------------------- */
typedef struct {
    double mass;                 /* M, geometric units                                   */
    double schwarzschild_radius; /* rs = 2M for every spin (spacetime.c:338,348,358)      */
    double spin;                 /* a/M; the ray path only asks "== 0 ?"                   */
    double charge;
    double r_plus;
    double r_minus;
    double isco_radius;
    double ergosphere_radius;
} BlackHoleParams;

typedef struct {
    double inner_radius;
    double outer_radius;
    double temperature_scale;
    double density_scale;
    double thickness_factor;
    double alpha_viscosity;
} AccretionDiskParams;

typedef struct {
    double time_step;            /* "dt" of the radius step schedule                       */
    double max_ray_distance;     /* path-length budget                                     */
    int    max_integration_steps;/* iteration budget                                       */
    double tolerance;            /* RKF45 eps_rel                                          */
    int    use_adaptive_step;    /* never read on the ray path                             */
    int    use_gpu_raytracing;   /* never read on the ray path                             */
    double doppler_factor;       /* never read on the ray path                             */
    double hawking_temp_factor;
    int    enable_doppler;
    int    enable_gravitational_redshift;
    int    show_accretion_disk;
} SimulationConfig;

/* ---- ray tracing results ----------------------------------------------------------------- */
typedef enum {
    RAY_HORIZON,
    RAY_DISK,
    RAY_BACKGROUND,
    RAY_MAX_DISTANCE,
    RAY_MAX_STEPS,
    RAY_ERROR
} RayTraceResult;

typedef enum {
    INTEGRATOR_RK4,
    INTEGRATOR_RKF45,
    INTEGRATOR_LEAPFROG,
    INTEGRATOR_YOSHIDA
} IntegrationMethod;

typedef enum {
    JITTER_NONE,
    JITTER_REGULAR_GRID,
    JITTER_RANDOM,
    JITTER_HALTON,
    JITTER_BLUE_NOISE
} JitterMethod;

typedef struct {
    int          samples_per_pixel;
    JitterMethod jitter_method;
    double       jitter_strength;
} SupersamplingParams;

typedef struct {
    int    enable_adaptive;
    int    min_samples;
    int    max_samples;
    double convergence_threshold;
    double edge_threshold;
} AdaptiveSamplingParams;

typedef struct {
    RayTraceResult result;
    Vector3D hit_position;
    Vector3D hit_normal;         /* never written by trace_ray                              */
    double   distance;
    int      steps;
    double   time_dilation;
    Vector3D sky_direction;      /* MAX_DISTANCE only; see DESIGN.md "unpinned fields"      */
    double   doppler_factor;     /* never written by trace_ray                              */
    double   temperature;        /* never written by trace_ray                              */
    double   color[3];           /* never written by trace_ray                              */
    double   redshift;           /* never written by trace_ray                              */
    double   optical_depth;      /* never written by trace_ray                              */
} RayTraceHit;

typedef struct {
    double mass, spin, schwarzschild_radius;
    double disk_inner_radius, disk_outer_radius, disk_temp_scale;
    double observer_distance, fov;
} GPUShaderParams;

/* ODE right-hand sides used by the generic host integrators (math_util.h:163, 173) */
typedef void (*ODEFunction)(double t, const double y[], double dydt[], void* params);
typedef void (*ODEFunctionSecondOrder)(double t, const double x[], const double v[], double a[],
                                       void* params);

/* ---- particle simulation (include/particle_sim.h:15-75) ---------------------------------- */
typedef enum {
    PARTICLE_TEST,
    PARTICLE_DISK,
    PARTICLE_HAWKING,
    PARTICLE_JET
} ParticleType;

typedef struct {
    Vector3D position;
    Vector3D velocity;
    Vector3D acceleration;       /* never written by the reference                          */
    double mass;
    double energy;               /* never written by the reference                          */
    double angular_momentum;     /* never written by the reference                          */
    double proper_time;          /* never written by the reference                          */
    double coordinate_time;      /* never written by the reference                          */
    ParticleType type;
    int active;
    int id;
    double age;
    double temperature;
    double time_dilation;        /* written by the geodesic update only                     */
} Particle;

typedef struct {
    double semi_major_axis;
    double eccentricity;
    double inclination;
    double longitude_of_ascending_node;
    double argument_of_periapsis;
    double mean_anomaly;
    double specific_angular_momentum;
    double specific_energy;
} OrbitalParams;

typedef struct {
    Particle* particles;
    int capacity;
    int count;
    int next_id;
    BlackHoleParams* blackhole;  /* never set by the reference                               */
} ParticleSystem;

/* ---- layout pins (x86-64 SysV) --------------------------------------------- */
#if defined(__cplusplus)
#define BHRT_STATIC_ASSERT(c, m) static_assert(c, m)
#else
#define BHRT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#endif
BHRT_STATIC_ASSERT(sizeof(Vector3D) == 24, "Vector3D");
BHRT_STATIC_ASSERT(sizeof(Ray) == 48, "Ray");
BHRT_STATIC_ASSERT(sizeof(BlackHoleParams) == 64, "BlackHoleParams");
BHRT_STATIC_ASSERT(sizeof(AccretionDiskParams) == 48, "AccretionDiskParams");
BHRT_STATIC_ASSERT(sizeof(SimulationConfig) == 72, "SimulationConfig");
BHRT_STATIC_ASSERT(offsetof(SimulationConfig, tolerance) == 24, "SimulationConfig.tolerance");
BHRT_STATIC_ASSERT(offsetof(SimulationConfig, show_accretion_disk) == 64, "SimulationConfig.show");
BHRT_STATIC_ASSERT(sizeof(RayTraceHit) == 160, "RayTraceHit");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, hit_position) == 8, "RayTraceHit.hit_position");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, distance) == 56, "RayTraceHit.distance");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, steps) == 64, "RayTraceHit.steps");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, time_dilation) == 72, "RayTraceHit.time_dilation");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, sky_direction) == 80, "RayTraceHit.sky_direction");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, color) == 120, "RayTraceHit.color");
BHRT_STATIC_ASSERT(offsetof(RayTraceHit, optical_depth) == 152, "RayTraceHit.optical_depth");
BHRT_STATIC_ASSERT(sizeof(RayTraceResult) == 4, "enum size");
BHRT_STATIC_ASSERT(sizeof(KerrMetric) == 56, "KerrMetric");
BHRT_STATIC_ASSERT(sizeof(BlackHoleMetric) == 64, "BlackHoleMetric");
BHRT_STATIC_ASSERT(sizeof(Particle) == 152, "Particle");
BHRT_STATIC_ASSERT(offsetof(Particle, type) == 112, "Particle.type");
BHRT_STATIC_ASSERT(offsetof(Particle, age) == 128, "Particle.age");
BHRT_STATIC_ASSERT(offsetof(Particle, time_dilation) == 144, "Particle.time_dilation");
BHRT_STATIC_ASSERT(sizeof(ParticleSystem) == 32, "ParticleSystem");
BHRT_STATIC_ASSERT(sizeof(OrbitalParams) == 64, "OrbitalParams");

#ifdef __cplusplus
}
#endif
#endif /* BHRT_TYPES_H */
