// particles.hip -- update_particles (src/particle_sim.c:505-566) as a HIP kernel: one lane per
// particle, `steps` updates in registers per launch.
//
// The arithmetic is the reference's, operation for operation and in its evaluation order,
// without FP contraction (the reference's x86-64 build has none): the Euler step of the
// geodesic update (particle_sim.c:232-304) with geodesic_equation's full 4x4x4 Christoffel
// contraction (spacetime.c:95-187, zero entries included, so Inf/NaN velocities propagate as
// they do there), and the Newtonian update (particle_sim.c:306-337). sin/cos/acos/atan2 are
// OCML's (within an ulp or two of glibc).
#include <hip/hip_runtime.h>

#include "bhrt_kernel.h"

#pragma clang fp contract(off)

namespace {

constexpr double kEps = 1.0e-10;                   // BH_EPSILON (math_util.h:21)
constexpr double kTwoPi = 6.28318530717958647692;  // BH_TWO_PI (math_util.h:26-27)

__device__ __forceinline__ double length3(const Vector3D& v) {
    return sqrt((v.x * v.x + v.y * v.y) + v.z * v.z);  // vector3D_length (math_util.c:85-113)
}

// calculate_christoffel_symbols (spacetime.c:95-161) then geodesic_equation (:166-187)
__device__ __forceinline__ void geodesic_accel(double r, double theta, const double v[4],
                                               const bhrt_particle_k& k, double acc[4]) {
    double G[4][4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++)
#pragma unroll
            for (int l = 0; l < 4; l++) G[i][j][l] = 0.0;
    if (k.spin0) {
        const double rs = k.rs;
        if (r <= rs + kEps) r = rs + kEps;
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
    } else {  // the reference's Kerr subset (:126-158)
        const double M = k.M, a = k.a;
        if (r <= k.r_plus + kEps) r = k.r_plus + kEps;
        const double st = sin(theta), ct = cos(theta);
        const double st2 = st * st, ct2 = ct * ct;
        const double Sigma = r * r + a * a * ct2;
        const double Sigma_sq = Sigma * Sigma;
        G[0][0][1] = M * (r * r - a * a * ct2) / Sigma_sq;
        G[0][1][0] = G[0][0][1];
        G[0][1][3] = -a * M * st2 * (r * r - a * a * ct2) / Sigma_sq;
        G[0][3][1] = G[0][1][3];
    }
#pragma unroll
    for (int mu = 0; mu < 4; mu++) {
        double s = 0.0;
#pragma unroll
        for (int al = 0; al < 4; al++)
#pragma unroll
            for (int be = 0; be < 4; be++) s -= G[mu][al][be] * v[al] * v[be];
        acc[mu] = s;
    }
}

// update_particle_geodesic (particle_sim.c:232-304)
__device__ __forceinline__ void step_geodesic(Particle& p, const bhrt_particle_k& k) {
    const double x = p.position.x, y = p.position.y, z = p.position.z;
    const double r = sqrt(x * x + y * y + z * z);  // cartesian_to_spherical (spacetime.c:201-224)
    double theta = 0.0;
    if (r > kEps) theta = acos(z / r);
    double phi = atan2(y, x);
    if (phi < 0.0) phi += kTwoPi;
    double st[8] = {0.0, r, theta, phi, 1.0, 0.0, 0.0, 0.0};
    const double v_mag = length3(p.velocity);
    st[5] = v_mag * cos(theta) * cos(phi);
    st[6] = v_mag * sin(phi);
    st[7] = v_mag * sin(theta) * cos(phi);
    double acc[4];
    const double vel[4] = {st[4], st[5], st[6], st[7]};
    geodesic_accel(st[1], st[2], vel, k, acc);
    const double d[8] = {st[4], st[5], st[6], st[7], acc[0], acc[1], acc[2], acc[3]};
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] += d[i] * k.dt;
    p.position.x = st[1] * sin(st[2]) * cos(st[3]);  // spherical_to_cartesian (spacetime.c:229)
    p.position.y = st[1] * sin(st[2]) * sin(st[3]);
    p.position.z = st[1] * cos(st[2]);
    const double v_r = st[5], v_theta = st[6], v_phi = st[7];
    const double s_t = sin(theta), c_t = cos(theta), s_p = sin(phi), c_p = cos(phi);
    p.velocity.x = v_r * s_t * c_p + r * v_theta * c_t * c_p - r * s_t * v_phi * s_p;
    p.velocity.y = v_r * s_t * s_p + r * v_theta * c_t * s_p + r * s_t * v_phi * c_p;
    p.velocity.z = v_r * c_t - r * v_theta * s_t;
    p.time_dilation = 1.0 / sqrt(1.0 - k.rs / st[1]);  // calculate_time_dilation (:192-196)
}

// update_particle_newtonian (particle_sim.c:306-337)
__device__ __forceinline__ void step_newtonian(Particle& p, const bhrt_particle_k& k) {
    const double r = length3(p.position);
    const double accel_mag = k.M / (r * r);
    const double inv = -1.0 / r;
    const double ax = p.position.x * inv * accel_mag, ay = p.position.y * inv * accel_mag,
                 az = p.position.z * inv * accel_mag;
    p.velocity.x = p.velocity.x + ax * k.dt;
    p.velocity.y = p.velocity.y + ay * k.dt;
    p.velocity.z = p.velocity.z + az * k.dt;
    p.position.x = p.position.x + p.velocity.x * k.dt;
    p.position.y = p.position.y + p.velocity.y * k.dt;
    p.position.z = p.position.z + p.velocity.z * k.dt;
}

__global__ __launch_bounds__(256) void k_update_particles(Particle* ps, int count,
                                                          const bhrt_particle_k k, int steps) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    Particle p = ps[i];
    const double rs20 = 20.0 * k.rs;
    for (int s = 0; s < steps && p.active; s++) {  // update_particles body (:519-562)
        p.age += k.dt;
        const double r = length3(p.position);
        if (p.type == PARTICLE_TEST && r < rs20)
            step_geodesic(p, k);
        else
            step_newtonian(p, k);
        if (length3(p.position) <= k.rs) p.active = 0;
    }
    ps[i] = p;
}

}  // namespace

extern "C" int bhrt_launch_particles(Particle* d, int count, const bhrt_particle_k* k, int steps,
                                     void* stream, void* ev0, void* ev1) {
    hipStream_t st = (hipStream_t)stream;
    if (ev0) (void)hipEventRecord((hipEvent_t)ev0, st);
    if (count > 0 && steps > 0)
        k_update_particles<<<(count + 255) / 256, 256, 0, st>>>(d, count, *k, steps);
    if (ev1) (void)hipEventRecord((hipEvent_t)ev1, st);
    return (int)hipGetLastError();
}
