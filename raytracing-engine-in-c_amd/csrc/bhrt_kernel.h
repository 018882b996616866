/*
 * bhrt_kernel.h -- launch parameters shared by the C host layer (bhrt_api.c) and the HIP
 * kernels (geodesic.hip). Plain C, passed by value as the kernel argument block, so every
 * field is wave-uniform and read through the scalar unit.
 *
 * Everything that is the same for all rays of a launch is computed ONCE on the host with
 * the same IEEE operations the reference performs inline (so identical rounding):
 *   - the scene constants (rs*1.5, dt*0.001, ...);
 *   - for a camera frame, the spherical coordinates of the shared origin (glibc acos /
 *     atan2 / sin / cos, exactly the reference's values) and the metric there.
 */
#ifndef BHRT_KERNEL_H
#define BHRT_KERNEL_H

#include "../../include/bhrt_api.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { BHRT_SRC_RAYS = 0, BHRT_SRC_CAMERA = 1 };
enum { BHRT_NUM_COUNTERS = 5 }; /* rays, iterations, stages full/far/kerr */
enum { BHRT_MAX_QUEUE_BITS = 5, BHRT_QUEUE_STRIDE_MAX = 64 }; /* ray queues of k_trace */
enum { BHRT_INIT_FIELDS = 21 }; /* ray arrays: y0..y5, y6, y7, dx, dy, dz, px, py, pz,
                                   far_ok, sin/cos of y1, y2, y3; camera frames use the first
                                   BHRT_INIT_FIELDS_CAMERA rows (the rest is the shared origin) */
enum { BHRT_INIT_FIELDS_CAMERA = 8 }; /* y4, y5, y6, y7, dx, dy, dz, far_ok */

typedef struct {
    /* scene constants (raytracer.c:65-130, 465, 556-571, 652-659; spacetime.c:22) */
    double M, rs, two_m;
    double rs_x1_5, rs_x1_05, rs_x2_5, rs_x5, rs_x15, rs_eps;
    double h_2_5, h_5, h_15, h_far;
    /* the r interval of each step size of the schedule, [h_lo[k], h_hi[k]): k = 0 h_far,
     * 1 h_15, 2 h_5, 3 h_2_5 (an empty interval for a size the select chain never picks) */
    double h_lo[4], h_hi[4];
    double max_dist, tol;
    double disk_in, disk_out, disk_tscale;
    double disk_in_sq, disk_out_sq; /* exact s-bounds of inner <= RN(sqrt(s)) <= outer */
    int max_steps;
    int method;  /* IntegrationMethod */
    int has_disk;
    int flags;   /* BHRT_FLAG_* */
    int spin0;   /* blackhole->spin == 0.0 */
    int far_bounded; /* a state within 2^40 stays below 2^400 over max_steps steps, far-field
                        branch included (bhrt_api.c far_bounded; geodesic.hip repair_at_refill) */
    double rot_vmax; /* zero-acceleration paths: a ray with |state[5]| below this turns state[2]
                        by less than pi/4 per step for every step size (geodesic.hip
                        rotation_trig); a ray at or above it is re-traced by the redo pass */
    int accept_all;  /* RKF45 with 2^-30 <= tol <= 2^300 and finite step sizes: no attempt on the
                        zero-acceleration paths can be rejected (geodesic.hip rkf45_attempt ACC) */
} bhrt_scene_k;

typedef struct {
    /* pixel -> direction (calculate_ray_direction, raytracer.c:999-1039) */
    double fwd[3], right[3], up[3];
    double plane_w, plane_h;
    double off_x, off_y;             /* sub-pixel offset (0.5, 0.5 = centre)   */
    int width, height;
    bhrt_rows rows;
    double inv_width, inv_block;     /* RN(1 / width), RN(1 / rows.row_block)  */
    /* shared origin (integrate_photon_path set-up, raytracer.c:355-466); also filled for ray
     * arrays with one origin (bhrt_kparams.rays_shared) */
    double pos[3];                   /* Cartesian origin                        */
    double r0, th0, ph0;             /* cartesian_to_spherical(origin)          */
    double st_cp, st_sp, ct, ct_cp, ct_sp, st, neg_sp, cp, r_st; /* trig products */
    double g_tt, g_rr, g_hh;         /* calculate_schwarzschild_metric(r0)      */
    double p0[3];                    /* spherical_to_cartesian(r0, th0, ph0)    */
    double sp;                       /* sin(ph0)                                */
    double s_r0, c_r0;               /* sin, cos(r0): state[1] as ray_derivatives' theta */
    int use_approx;                  /* r0 > 15 rs                              */
    int st_tiny;                     /* fabs(sin th0) < BH_EPSILON              */
    /* claim order: the shard's pixels in tiles of 2^tile_w_log2 x 2^tile_h_log2 = 64 pixels
     * (one wavefront), tiles row-major; tiles_per_row == 0: ray id order */
    int tile_w_log2, tile_h_log2, tiles_per_row;
    double inv_tiles_per_row;        /* RN(1 / tiles_per_row)                   */
    int ntiles, tile_stride;         /* tile_stride > 0: the claim order visits tile
                                        (t * tile_stride) mod ntiles at step t (scatter) */
} bhrt_camera_k;

/* Whether the trace kernel writes a scene's colour outputs at each ray's exit, from the state in
 * registers (no separate colour pass re-reading the hits). Since round 6 every scene: the
 * separate pass of a frame could only start once the trace kernel's last wave had ended, by
 * when the next frame's persistent workgroups held every wave slot, so a C2 frame's colour
 * landed ~1 frame late (k_colour dispatches averaged 5.5 ms), and on the
 * current kernels fusing costs nothing (C2 284.5 vs 284.6 Mrays/s same box,
 * profiles/r06/ab_fused_colour.txt; C5 +16%, C1 +9%). Scenes without a disk get the sky / horizon colour
 * alone (geodesic.hip colour_sky). BHRT_FUSE_ALL=0 builds round 5's rule (disk scenes with
 * RKF45 or a != 0; C3, C4) and BHRT_FUSE_COLOUR=0 at run time takes the separate pass (A/B). */
#ifndef BHRT_FUSE_ALL
#define BHRT_FUSE_ALL 1
#endif
#define BHRT_COLOUR_IN_TRACE(method, has_disk, spin)                                        \
    (BHRT_FUSE_ALL ||                                                                       \
     ((has_disk) && ((method) == INTEGRATOR_RKF45 || ((method) == INTEGRATOR_RK4 && (spin)))))

typedef struct {
    bhrt_scene_k sc;
    int src;              /* BHRT_SRC_*                                       */
    int n;                /* rays in this launch                              */
    int refill;           /* refill a wave once >= refill lanes are idle      */
    int claim_min;        /* smallest block of ray ids a wave claims at once (multiple of 64) */
    int claim_div;        /* a claim takes (unclaimed rays) / (waves * claim_div), at least
                             claim_min: large blocks while the queue is full, small at the end */
    const Ray* rays;      /* BHRT_SRC_RAYS: device AoS input                  */
    double* init;         /* [BHRT_INIT_FIELDS][n] initial state (k_init)      */
    int* redo;            /* [n] ids of rays re-traced with the large-argument path */
    bhrt_camera_k cam;    /* BHRT_SRC_CAMERA                                  */
    bhrt_frame_soa out;   /* device SoA outputs; NULL fields skipped          */
    unsigned long long* ctl; /* [1..5] counters, [6] redo count, [7] redo queue head; the
                                launch's slot of the control ring, zero at launch (the ring is
                                filled with zeros on the GPU after each harvest, bhrt_api.c
                                ring_order) */
    unsigned long long* qhead; /* ray-queue heads, queue q at qhead[q * queue_stride]; same slot */
    int queue_bits;       /* 2^queue_bits ray queues (<= BHRT_MAX_QUEUE_BITS)            */
    int queue_stride;     /* u64 words between queue heads (<= BHRT_QUEUE_STRIDE_MAX)     */
    int claim_shift;      /* set by the launcher per launch: a block claim is the queue's
                             remainder >> claim_shift, 2^claim_shift >= waves * claim_div / queues */
    int colour_fused;     /* the trace kernel writes the colour outputs (rgb, rgba32f, rgba8)
                             of each ray at its exit; else a separate colour pass runs */
    const int* order;     /* camera frames: the claim order, queue position -> ray id (a
                             permutation of [0, n)); NULL = ray id order */
    int skip_redo;        /* the redo launch may be left out where no ray can be evicted
                             (geodesic.hip launch_trace_pair); BHRT_SKIP_REDO=0: always launch */
    int no_evict;         /* the host proved that no ray of this launch can be handed to the
                             redo pass (bhrt_api.c origin_no_evict; camera frames and ray
                             arrays with one shared origin) */
    int block_lanes;      /* lanes per workgroup of the hot trace launch (64, 128 or 256) */
    int rays_shared;      /* BHRT_SRC_RAYS whose every origin is cam.pos (the host checked):
                             cam's origin block is filled as for a camera frame, and the
                             trace kernel sets rays up from their directions (no k_init) */
    const double* dirs;   /* rays_shared: ray i's direction at dirs[i * dir_stride + 0..2]
                             (the AoS rays' direction field, stride 6, or packed, stride 3,
                             with rays NULL) */
    int dir_stride;
    int grid_div;         /* > 0: the hot launch takes 1 / grid_div of the resident workgroups */
    int grid_blocks;      /* > 0: at most this many workgroups in the hot launch (A/B knob) */
    int min_tiles;        /* drained-refill launches of fewer 64-ray tiles per resident wave
                             than this take half the grid (0 = off) */
    int diag_slot;        /* the launch's control-block slot (the BHRT_WAVE_STAMPS diagnostic
                             build records per-wave stamps under it; unused otherwise) */
} bhrt_kparams;

/* update_particles (particle_sim.c:505-566) constants, from the BlackHoleParams and
 * SimulationConfig of the call */
typedef struct {
    double M, rs, a, r_plus; /* mass, schwarzschild_radius, spin * mass, r_plus */
    double dt;               /* config->time_step                                 */
    int spin0;               /* blackhole->spin == 0.0                            */
} bhrt_particle_k;

/* particles.hip: `steps` updates of d_particles[0, count) on `stream`, ev0/ev1 (hipEvent_t,
 * may be NULL) recorded around the kernel; returns 0 or a hipError_t value. */
int bhrt_launch_particles(Particle* d_particles, int count, const bhrt_particle_k* k, int steps,
                          void* stream, void* ev0, void* ev1);

/* launch helpers implemented in geodesic.hip; return 0 or a hipError_t value.
 * bhrt_launch_trace records ev0/ev1 (hipEvent_t, may be NULL) around the trace kernel
 * itself, not the set-up or colour passes. */
int bhrt_launch_trace(const bhrt_kparams* kp, void* stream, void* ev0, void* ev1);
/* 1 if bhrt_launch_trace runs kp's RKF45 attempts without the accept test (bhrt_stats) */
int bhrt_trace_untested(const bhrt_kparams* kp);
int bhrt_launch_path(const bhrt_kparams* kp, const double* origin4, const double* dir3,
                     Vector3D* d_path, int max_positions, int* d_num, int num_positions_in,
                     void* stream);

#ifdef __cplusplus
}
#endif
#endif
