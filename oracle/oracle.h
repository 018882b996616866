/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference geodesic ray tracer (Klaudiusz321/raytracing-engine-in-c,
 * src/raytracer.c + src/spacetime.c + src/math_util.c), used as the parity checker for the
 * HIP path and as the "port" CPU baseline. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. libbhrt.so never links or calls it.
 *
 * Every symbol is prefixed orc_ so it can share a process with libbhrt.so and with the
 * compiled reference (oracle/_ref/libref.so), which both export the reference names.
 *
 * Pinning: validated against tests/golden/ fixtures produced by the compiled reference
 * (tests/golden/gen_golden.py); integers bit-exact, floats <= 1e-12 relative.
 */
#ifndef BHRT_ORACLE_H
#define BHRT_ORACLE_H

#include "../include/bhrt_api.h" /* types only: the oracle calls nothing in libbhrt */

#ifdef __cplusplus
extern "C" {
#endif

/* literal restatements (reference names with an orc_ prefix) */
RayTraceResult orc_integrate_photon_path(const Vector4D* position, const Vector3D* direction,
                                         const BlackHoleParams* bh, const SimulationConfig* cfg,
                                         IntegrationMethod method, Vector3D* path,
                                         int max_positions, int* num_positions,
                                         RayTraceHit* hit);
RayTraceResult orc_trace_ray(const Ray* ray, const BlackHoleParams* bh,
                             const AccretionDiskParams* disk, const SimulationConfig* cfg,
                             RayTraceHit* hit);
/* trace_ray's structure with a chosen integrator (RKF45 + disk = config C3) */
RayTraceResult orc_trace_ray_method(const Ray* ray, const BlackHoleParams* bh,
                                    const AccretionDiskParams* disk, const SimulationConfig* cfg,
                                    IntegrationMethod method, RayTraceHit* hit);
int orc_check_disk_intersection(const Vector3D* p, const Vector3D* v, const Vector3D* n,
                                const AccretionDiskParams* disk, Vector3D* q);
void orc_calculate_disk_temperature(const Vector3D* p, const BlackHoleParams* bh,
                                    const AccretionDiskParams* disk, double* T, double rgb[3]);
void orc_apply_relativistic_effects(const Vector3D* p, const Vector3D* v,
                                    const BlackHoleParams* bh, double rgb[3], double* dop);
void orc_temperature_to_rgb(double T, double rgb[3]);
double orc_halton_sequence(int index, int base);
void orc_initialize_black_hole_params(BlackHoleParams* bh, double mass, double spin,
                                      double charge);
void orc_camera_ray_direction(int px, int py, double ox, double oy, int W, int H,
                              const bhrt_camera* cam, Vector3D* dir);
void orc_jittered_offset(int sample, int spp, JitterMethod jm, double strength, double* ox,
                         double* oy);

/* frame/batch drivers (OpenMP over rays, nthreads <= 0 = OMP default) */
int orc_render_frame(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                     const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                     const bhrt_rows* rows, IntegrationMethod method, int flags,
                     const bhrt_frame_soa* out, int nthreads);
/* the same frame, plus each ray's knife-edge margin (oracle.c "knife-edge margins") */
int orc_render_frame_margin(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                            const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                            const bhrt_rows* rows, IntegrationMethod method, int flags,
                            const bhrt_frame_soa* out, double* margin, int nthreads);
int orc_trace_rays(const Ray* rays, int n, const BlackHoleParams* bh,
                   const AccretionDiskParams* disk, const SimulationConfig* cfg,
                   IntegrationMethod method, int flags, const bhrt_frame_soa* out, int nthreads);
/* rows of a shard (same rule as bhrt_shard_rows) and local row j -> image row */
/* update_particles (particle_sim.c:505-566) applied `steps` times to ps[0, count) */
void orc_update_particles(Particle* ps, int count, const BlackHoleParams* bh,
                          const SimulationConfig* cfg, int steps);
int orc_shard_rows(int H, const bhrt_rows* rows);
int orc_shard_row(int j, const bhrt_rows* rows);

#ifdef __cplusplus
}
#endif
#endif
