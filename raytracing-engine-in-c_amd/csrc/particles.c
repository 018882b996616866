/*
 * particles.c -- the reference's particle system (src/particle_sim.c, the particle half of
 * src/blackhole_api.c) for the visualizer's per-frame calls (renderer.cpp:879-1005).
 *
 * Bookkeeping and creation stay on the host, in the reference's arithmetic: creation draws
 * from the C library's rand() stream in the reference's order (particle_sim.c:339-503), so a
 * caller that seeds srand() gets the reference's particles. update_particles runs on the GPU
 * (particles.hip): the particle array goes to the device, is stepped and comes back. There is
 * no CPU fallback; without a HIP device update_particles returns -1 (bh_update_particles
 * BH_ERROR_SIMULATION) and bhrt_last_error() says why.
 */
#define _GNU_SOURCE
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#pragma GCC visibility push(default)
#include "../../include/bhrt_api.h"
#pragma GCC visibility pop
#include "bhrt_host.h"
#include "bhrt_kernel.h"

#define PS_PI 3.14159265358979323846 /* particle_sim.c:15 */

/* ======================================================================================= */
/* geodesic_equation on the host (spacetime.c:95-187), for drop-in callers                  */
/* ======================================================================================= */
void calculate_christoffel_symbols(double r, double theta, const BlackHoleParams* bh,
                                   double G[4][4][4]) {
    memset(G, 0, 4 * 4 * 4 * sizeof(double));
    if (bh->spin == 0.0) {
        const double rs = bh->schwarzschild_radius;
        if (r <= rs + BH_EPSILON) r = rs + BH_EPSILON;
        const double st = sin(theta), ct = cos(theta);
        G[0][0][1] = G[0][1][0] = rs / (2.0 * r * (r - rs));
        G[1][0][0] = rs * (r - rs) / (2.0 * r * r * r);
        G[1][1][1] = -rs / (2.0 * r * (r - rs));
        G[1][2][2] = -(r - rs);
        G[1][3][3] = -(r - rs) * st * st;
        G[2][1][2] = G[2][2][1] = 1.0 / r;
        G[2][3][3] = -st * ct;
        G[3][1][3] = G[3][3][1] = 1.0 / r;
        G[3][2][3] = G[3][3][2] = ct / st;
    } else {
        const double M = bh->mass, a = bh->spin * M;
        if (r <= bh->r_plus + BH_EPSILON) r = bh->r_plus + BH_EPSILON;
        const double st = sin(theta), ct = cos(theta);
        const double st2 = st * st, ct2 = ct * ct;
        const double Sigma = r * r + a * a * ct2;
        const double Sigma_sq = Sigma * Sigma;
        G[0][0][1] = M * (r * r - a * a * ct2) / Sigma_sq;
        G[0][1][0] = G[0][0][1];
        G[0][1][3] = -a * M * st2 * (r * r - a * a * ct2) / Sigma_sq;
        G[0][3][1] = G[0][1][3];
    }
}

void geodesic_equation(const double position[4], const double velocity[4],
                       const BlackHoleParams* bh, double acceleration[4]) {
    double G[4][4][4];
    memset(acceleration, 0, 4 * sizeof(double));
    calculate_christoffel_symbols(position[1], position[2], bh, G);
    for (int mu = 0; mu < 4; mu++)
        for (int al = 0; al < 4; al++)
            for (int be = 0; be < 4; be++)
                acceleration[mu] -= G[mu][al][be] * velocity[al] * velocity[be];
}

/* math_util.c:125-157 */
void leapfrog_integrate(ODEFunctionSecondOrder f, double* x, double* v, int n, double t,
                        double dt, void* params) {
    double* a = (double*)malloc((size_t)(n > 0 ? n : 1) * sizeof(double));
    if (!a) return;
    f(t, x, v, a, params);
    for (int i = 0; i < n; i++) v[i] += 0.5 * dt * a[i];
    for (int i = 0; i < n; i++) x[i] += dt * v[i];
    f(t + dt, x, v, a, params);
    for (int i = 0; i < n; i++) v[i] += 0.5 * dt * a[i];
    free(a);
}

/* ======================================================================================= */
/* particle_sim.h                                                                           */
/* ======================================================================================= */
int particle_system_init(ParticleSystem* system, int capacity) { /* particle_sim.c:73-94 */
    if (system == NULL || capacity <= 0) return -1;
    system->particles = (Particle*)malloc((size_t)capacity * sizeof(Particle));
    if (system->particles == NULL) return -1;
    system->capacity = capacity;
    system->count = 0;
    system->next_id = 1;
    srand((unsigned int)time(NULL));
    return 0;
}

void particle_system_cleanup(ParticleSystem* system) { /* particle_sim.c:96-103 */
    if (system != NULL && system->particles != NULL) {
        free(system->particles);
        system->particles = NULL;
        system->capacity = 0;
        system->count = 0;
    }
}

int add_particle(ParticleSystem* system, const Vector3D* position, const Vector3D* velocity,
                 double mass, ParticleType type) { /* particle_sim.c:108-133 */
    if (system->count >= system->capacity) return -1;
    Particle* p = &system->particles[system->count++];
    p->id = system->next_id++;
    p->position = *position;
    p->velocity = *velocity;
    p->mass = mass;
    p->type = type;
    p->active = 1;
    p->age = 0.0;
    p->temperature = 0.0;
    return p->id;
}

Particle* find_particle(ParticleSystem* system, int particle_id) { /* particle_sim.c:138-150 */
    if (system == NULL || particle_id <= 0) return NULL;
    for (int i = 0; i < system->count; i++)
        if (system->particles[i].id == particle_id && system->particles[i].active)
            return &system->particles[i];
    return NULL;
}

int remove_particle(ParticleSystem* system, int particle_id) { /* particle_sim.c:155-168 */
    if (system == NULL || particle_id <= 0) return -1;
    for (int i = 0; i < system->count; i++)
        if (system->particles[i].id == particle_id) {
            system->particles[i].active = 0;
            return 0;
        }
    return -1;
}

/* Keplerian elements of a test particle (particle_sim.c:173-227, calculate_orbit_parameters) */
static void orbit_parameters(const Vector3D* position, const Vector3D* velocity,
                             const BlackHoleParams* bh, OrbitalParams* params) {
    const double r = vector3D_length(*position);
    const double v = vector3D_length(*velocity);
    const Vector3D l_vec = vector3D_cross(*position, *velocity);
    const double L = vector3D_length(l_vec);
    const double E = 0.5 * v * v - bh->mass / r;
    const Vector3D r_hat = vector3D_normalize(*position);
    const Vector3D term1 = vector3D_scale(r_hat, v * v - bh->mass / r);
    const double r_dot_v = vector3D_dot(*position, *velocity);
    const Vector3D term2 = vector3D_scale(*velocity, r_dot_v);
    const Vector3D e_vec = vector3D_scale(vector3D_sub(term1, term2), 1.0 / bh->mass);
    const double e = vector3D_length(e_vec);
    double a;
    if (E < 0)
        a = -bh->mass / (2.0 * E);
    else if (E > 0)
        a = bh->mass / (2.0 * E);
    else
        a = INFINITY;
    params->semi_major_axis = a;
    params->eccentricity = e;
    params->inclination = acos(l_vec.z / L);
    params->specific_angular_momentum = L;
    params->specific_energy = E;
}

int calculate_particle_orbit(const ParticleSystem* system, int particle_id,
                             const BlackHoleParams* bh, OrbitalParams* params) {
    /* particle_sim.c:571-599 */
    if (system == NULL || bh == NULL || params == NULL) return -1;
    for (int i = 0; i < system->count; i++) {
        const Particle* p = &system->particles[i];
        if (p->id == particle_id && p->active) {
            orbit_parameters(&p->position, &p->velocity, bh, params);
            return 0;
        }
    }
    return -1;
}

/* find_particle(system, id) for the id add_particle just returned: ids are unique and the
 * new particle is the last one, so this is the reference's lookup without its O(count) scan
 * (which makes creating N particles O(N^2) there). */
static Particle* just_added(ParticleSystem* system, int id) {
    Particle* p = &system->particles[system->count - 1];
    return (p->id == id && p->active) ? p : NULL;
}

static double urand(void) { return (double)rand() / RAND_MAX; }

int create_accretion_disk(ParticleSystem* system, const BlackHoleParams* bh,
                          const AccretionDiskParams* disk, int num_particles) {
    /* particle_sim.c:339-422 */
    if (system == NULL || bh == NULL || disk == NULL || num_particles <= 0) return -1;
    if (system->count + num_particles > system->capacity) return -1;
    double inner = disk->inner_radius, outer = disk->outer_radius;
    if (inner < bh->isco_radius) inner = bh->isco_radius;
    if (inner < bh->schwarzschild_radius) inner = bh->schwarzschild_radius * 1.1;
    int created = 0;
    for (int i = 0; i < num_particles; i++) {
        const double t = (double)i / (num_particles - 1);
        const double r = inner + (outer - inner) * sqrt(t);
        const double phi = urand() * 2.0 * PS_PI;
        Vector3D pos;
        pos.x = r * cos(phi);
        pos.y = r * sin(phi);
        pos.z = (urand() - 0.5) * disk->thickness_factor * r;
        const double v_orbit = sqrt(bh->mass / r);
        Vector3D vel = {-pos.y * v_orbit / r, pos.x * v_orbit / r, 0.0};
        const double v_random = v_orbit * 0.05;
        vel.x += (urand() - 0.5) * v_random;
        vel.y += (urand() - 0.5) * v_random;
        vel.z += (urand() - 0.5) * v_random;
        const double temperature = disk->temperature_scale * 10000.0 * pow(inner / r, 0.75);
        const int id = add_particle(system, &pos, &vel, 0.0, PARTICLE_DISK);
        if (id < 0) break;
        Particle* p = just_added(system, id);
        if (p != NULL) p->temperature = temperature;
        created++;
    }
    return created;
}

int generate_hawking_radiation(ParticleSystem* system, const BlackHoleParams* bh,
                               int num_particles, const SimulationConfig* config) {
    /* particle_sim.c:427-500 */
    if (system == NULL || bh == NULL || num_particles <= 0) return -1;
    if (system->count + num_particles > system->capacity) return -1;
    double hawking_temp = 1.0 / (8.0 * PS_PI * bh->mass);
    hawking_temp *= config->hawking_temp_factor;
    int created = 0;
    for (int i = 0; i < num_particles; i++) {
        const double theta = urand() * PS_PI;
        const double phi = urand() * 2.0 * PS_PI;
        const double r = bh->schwarzschild_radius * 1.01;
        const double st = sin(theta), ct = cos(theta), sp = sin(phi), cp = cos(phi);
        const Vector3D pos = {r * st * cp, r * st * sp, r * ct};
        Vector3D vel = vector3D_scale(vector3D_normalize(pos), 1.0 * 0.9);
        vel.x += (urand() - 0.5) * 0.2;
        vel.y += (urand() - 0.5) * 0.2;
        vel.z += (urand() - 0.5) * 0.2;
        vel = vector3D_scale(vector3D_normalize(vel), 1.0 * 0.9);
        const int id = add_particle(system, &pos, &vel, 0.0, PARTICLE_HAWKING);
        if (id < 0) break;
        Particle* p = just_added(system, id);
        if (p != NULL) p->temperature = hawking_temp;
        created++;
    }
    return created;
}

int calculate_circular_orbit(double r, const BlackHoleParams* bh, Vector3D* velocity) {
    /* particle_sim.c:604-624 */
    if (r <= get_isco_radius(bh)) return -1;
    const double v = sqrt(bh->mass / r);
    velocity->x = -v * sin(0.0);
    velocity->y = v * cos(0.0);
    velocity->z = 0.0;
    return 0;
}

/* ---- the GPU update ---- */
typedef struct {
    int device;
    hipStream_t stream;
    hipEvent_t ev0, ev1;
    Particle* d_buf;
    size_t cap;
} pctx_t;

#define PCTX_MAX_DEV 16
static _Thread_local pctx_t* g_pctx[PCTX_MAX_DEV];

/* the calling thread's stream, events and device buffer on the current device */
static pctx_t* pctx_get(void) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= PCTX_MAX_DEV) {
        bhrt_set_err("no HIP device for update_particles");
        return NULL;
    }
    if (g_pctx[dev]) return g_pctx[dev];
    pctx_t* c = (pctx_t*)calloc(1, sizeof *c);
    if (!c) return NULL;
    c->device = dev;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        bhrt_set_err("cannot create the particle stream on device %d", dev);
        free(c);
        return NULL;
    }
    g_pctx[dev] = c;
    return c;
}

#define PHIP(call)                                                                            \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess) {                                                               \
            bhrt_set_err("%s failed: %s", #call, hipGetErrorString(e_));                      \
            return -1;                                                                        \
        }                                                                                     \
    } while (0)

int bhrt_update_particles_steps(ParticleSystem* system, const BlackHoleParams* bh,
                                const SimulationConfig* config, int steps, double* kernel_ms) {
    if (system == NULL || bh == NULL || config == NULL || steps < 0) {
        bhrt_set_err("invalid argument");
        return -1;
    }
    if (kernel_ms) *kernel_ms = 0.0;
    const int n = system->count;
    if (n <= 0 || steps == 0) return 0;
    pctx_t* c = pctx_get();
    if (!c) return -1;
    const size_t bytes = (size_t)n * sizeof(Particle);
    if (c->cap < bytes) {
        if (c->d_buf) (void)hipFree(c->d_buf);
        c->d_buf = NULL;
        c->cap = 0;
        PHIP(hipMalloc((void**)&c->d_buf, bytes + bytes / 4));
        c->cap = bytes + bytes / 4;
    }
    bhrt_particle_k k;
    k.M = bh->mass;
    k.rs = bh->schwarzschild_radius;
    k.a = bh->spin * bh->mass;
    k.r_plus = bh->r_plus;
    k.dt = config->time_step;
    k.spin0 = bh->spin == 0.0;
    PHIP(hipMemcpyAsync(c->d_buf, system->particles, bytes, hipMemcpyHostToDevice, c->stream));
    const int e = bhrt_launch_particles(c->d_buf, n, &k, steps, (void*)c->stream, (void*)c->ev0,
                                        (void*)c->ev1);
    if (e != 0) {
        bhrt_set_err("particle kernel launch failed: %s", hipGetErrorString((hipError_t)e));
        return -1;
    }
    PHIP(hipMemcpyAsync(system->particles, c->d_buf, bytes, hipMemcpyDeviceToHost, c->stream));
    PHIP(hipStreamSynchronize(c->stream));
    if (kernel_ms) {
        float ms = 0.f;
        PHIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
        *kernel_ms = ms;
    }
    return 0;
}

int update_particles(ParticleSystem* system, const BlackHoleParams* bh,
                     const SimulationConfig* config) { /* particle_sim.c:505-566 */
    if (system == NULL || bh == NULL || config == NULL) return -1;
    return bhrt_update_particles_steps(system, bh, config, 1, NULL);
}

/* ======================================================================================= */
/* bh_* particle functions (blackhole_api.c:253-429)                                        */
/* ======================================================================================= */
void* bh_create_particle_system(BHContextHandle context, int capacity) {
    if (context == NULL || capacity <= 0) return NULL;
    ParticleSystem* system = (ParticleSystem*)malloc(sizeof(ParticleSystem));
    if (system == NULL) return NULL;
    if (particle_system_init(system, capacity) != 0) {
        free(system);
        return NULL;
    }
    return system;
}

void bh_destroy_particle_system(BHContextHandle context, void* system) {
    if (context == NULL || system == NULL) return;
    particle_system_cleanup((ParticleSystem*)system);
    free(system);
}

int bh_add_test_particle(BHContextHandle context, void* system, const double position[3],
                         const double velocity[3], double mass) {
    if (context == NULL || system == NULL || position == NULL || velocity == NULL || mass < 0.0)
        return -1;
    const Vector3D pos = {position[0], position[1], position[2]};
    const Vector3D vel = {velocity[0], velocity[1], velocity[2]};
    return add_particle((ParticleSystem*)system, &pos, &vel, mass, PARTICLE_TEST);
}

int bh_create_accretion_disk_particles(BHContextHandle context, void* system,
                                       int num_particles) {
    if (context == NULL || system == NULL || num_particles <= 0) return -1;
    if (!context->disk_enabled) return 0;
    return create_accretion_disk((ParticleSystem*)system, &context->blackhole, &context->disk,
                                 num_particles);
}

int bh_generate_hawking_radiation(BHContextHandle context, void* system, int num_particles) {
    if (context == NULL || system == NULL || num_particles <= 0) return -1;
    return generate_hawking_radiation((ParticleSystem*)system, &context->blackhole, num_particles,
                                      &context->config);
}

BHErrorCode bh_update_particles(BHContextHandle context, void* system) {
    if (context == NULL || system == NULL) return BH_ERROR_INVALID_PARAMETER;
    if (update_particles((ParticleSystem*)system, &context->blackhole, &context->config) != 0)
        return BH_ERROR_SIMULATION;
    return BH_SUCCESS;
}

BHErrorCode bh_get_particle_data(BHContextHandle context, void* system, double* positions,
                                 double* velocities, int* types, int* count) {
    if (context == NULL || system == NULL || positions == NULL || velocities == NULL ||
        types == NULL || count == NULL || *count <= 0)
        return BH_ERROR_INVALID_PARAMETER;
    const ParticleSystem* ps = (const ParticleSystem*)system;
    const int max_count = *count;
    int active = 0;
    for (int i = 0; i < ps->count && active < max_count; i++) {
        const Particle* p = &ps->particles[i];
        if (!p->active) continue;
        positions[active * 3 + 0] = p->position.x;
        positions[active * 3 + 1] = p->position.y;
        positions[active * 3 + 2] = p->position.z;
        velocities[active * 3 + 0] = p->velocity.x;
        velocities[active * 3 + 1] = p->velocity.y;
        velocities[active * 3 + 2] = p->velocity.z;
        types[active] = p->type;
        active++;
    }
    *count = active;
    return BH_SUCCESS;
}
