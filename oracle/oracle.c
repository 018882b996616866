/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + "port" CPU baseline).
 *
 * A literal CPU restatement of the reference hot path. Each function names the reference
 * lines it follows; the arithmetic keeps the reference's operation order (C evaluates
 * a*b*c as (a*b)*c, a+b+c as (a+b)+c) and is compiled with -ffp-contract=off so that it
 * rounds exactly like the reference build (gcc -O2, x86-64, no FMA).
 *
 * One deliberate convention: ray_derivatives (raytracer.c:44-154) never writes
 * derivatives[6..7], which rk4_integrate (math_util.c:170-174) mallocs uninitialised; the
 * reference therefore integrates heap garbage into state[6..7]. That only reaches
 * RayTraceHit.sky_direction. Here derivatives[6..7] = 0.
 */
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- math_util.c:31-122 vector helpers (SSE2 x,y lanes + scalar z: same rounding) ---- */
static Vector3D v_add(Vector3D a, Vector3D b) { Vector3D r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static Vector3D v_sub(Vector3D a, Vector3D b) { Vector3D r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static Vector3D v_scale(Vector3D v, double s) { Vector3D r = {v.x * s, v.y * s, v.z * s}; return r; }
static double v_dot(Vector3D a, Vector3D b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z); } /* :85-97 */
static Vector3D v_cross(Vector3D a, Vector3D b) {                                               /* :100-109 */
    Vector3D r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    return r;
}
static double v_len(Vector3D v) { return sqrt(v_dot(v, v)); }
static Vector3D v_norm(Vector3D v) { /* :115-122: multiply by the reciprocal */
    double l = v_len(v);
    if (l < BH_EPSILON) { Vector3D z = {0.0, 0.0, 0.0}; return z; }
    return v_scale(v, 1.0 / l);
}
static double orc_clamp(double v, double lo, double hi) { /* math_util.c:505-509 */
    if (v < lo) return lo;
    if (v > hi) return hi;
    return v;
}

/* ---- spacetime.c ---- */
static SchwarzschildMetric schw_metric(double r, const BlackHoleParams* bh) { /* :15-33 */
    SchwarzschildMetric m;
    double rs = bh->schwarzschild_radius;
    if (r <= rs + BH_EPSILON) r = rs + BH_EPSILON;
    m.g_tt = -(1.0 - rs / r);
    m.g_rr = 1.0 / (1.0 - rs / r);
    m.g_thth = r * r;
    m.g_phph = r * r * sin(BH_PI / 2) * sin(BH_PI / 2);
    return m;
}
static double time_dilation(double r, double rs) { return 1.0 / sqrt(1.0 - rs / r); } /* :192-196 */
static void cart2sph(const Vector3D* c, Vector3D* s) { /* :201-224 */
    double r = sqrt(c->x * c->x + c->y * c->y + c->z * c->z);
    double th = 0.0;
    if (r > BH_EPSILON) th = acos(c->z / r);
    double ph = atan2(c->y, c->x);
    if (ph < 0.0) ph += BH_TWO_PI;
    s->x = r; s->y = th; s->z = ph;
}
static void sph2cart(const Vector3D* s, Vector3D* c) { /* :229-237 */
    double r = s->x, th = s->y, ph = s->z;
    c->x = r * sin(th) * cos(ph);
    c->y = r * sin(th) * sin(ph);
    c->z = r * cos(th);
}
static double isco_radius(const BlackHoleParams* bh) { /* :285-308 */
    double M = bh->mass, a = bh->spin * M;
    if (bh->spin == 0.0) return 6.0 * M;
    double Z1 = 1.0 + pow(1.0 - a * a / (M * M), 1.0 / 3.0) *
                          (pow(1.0 + a / (M), 1.0 / 3.0) + pow(1.0 - a / (M), 1.0 / 3.0));
    double Z2 = sqrt(3.0 * a * a / (M * M) + Z1 * Z1);
    return M * (3.0 + Z2 - sqrt((3.0 - Z1) * (3.0 + Z1 + 2.0 * Z2)));
}
void orc_initialize_black_hole_params(BlackHoleParams* bh, double mass, double spin,
                                      double charge) { /* :331-366 */
    bh->mass = mass; bh->spin = spin; bh->charge = charge;
    if (spin == 0.0 && charge == 0.0) {
        bh->schwarzschild_radius = 2.0 * mass;
        bh->r_plus = 2.0 * mass;
        bh->r_minus = 0.0;
        bh->ergosphere_radius = 2.0 * mass;
    } else if (spin > 0.0 && charge == 0.0) {
        double a = spin * mass;
        bh->schwarzschild_radius = 2.0 * mass;
        bh->r_plus = mass + sqrt(mass * mass - a * a);
        bh->r_minus = mass - sqrt(mass * mass - a * a);
        bh->ergosphere_radius = 2.0 * mass;
    } else {
        double a = spin * mass;
        bh->schwarzschild_radius = 2.0 * mass;
        bh->r_plus = mass + sqrt(mass * mass - a * a - charge * charge);
        bh->r_minus = mass - sqrt(mass * mass - a * a - charge * charge);
        bh->ergosphere_radius = 2.0 * mass;
    }
    bh->isco_radius = isco_radius(bh);
}

/* ---- knife-edge margins; off unless orc_render_frame_margin runs ----
 * For every DISCONTINUOUS decision a ray takes (step-size schedule, far-field switch,
 * horizon and distance exits, RKF45 accept, the pole clamp's sign, the disk test's
 * |denominator| threshold, t sign and radii), the relative distance of the tested value from
 * its threshold; a ray's margin is the smallest over the decisions that reach its pinned
 * outputs (for a disk hit at segment i: iterations 1..i and segments 1..i). Continuous clamps
 * (|d| <= 10, r >= 1.5 rs, |sin| >= 0.01) are not decisions in this sense. A ray whose margin
 * is below ~1e-9 can change class or step count under a last-bit difference of its inputs.
 * Tracking never changes a computed value. */
static _Thread_local int g_mg_on;
static _Thread_local double g_mg;       /* running minimum of the current ray */
static _Thread_local double* g_mg_iter; /* [k] = g_mg after the iteration that stored path[k] */
static _Thread_local double g_mg_result;
static void mg_note(double m) {
    if (g_mg_on && m < g_mg) g_mg = m; /* (NaN comparisons decide the same everywhere) */
}
static void mg_rel(double a, double b) {
    if (g_mg_on) mg_note(fabs(a - b) / fabs(b));
}

/* ---- raytracer.c:19-33 integration parameters ---- */
typedef struct {
    const BlackHoleParams* bh;
    double impact_parameter;
    int use_analytic_approx;
    double field_strength_threshold;
} OrcRay;

/* raytracer.c:44-154 -- reads state[0..5] as (r, theta, phi, v_r, v_theta, v_phi) although
 * integrate_photon_path stores (t, r, theta, phi, tdot, rdot, ...): the shift is the
 * reference's and is reproduced. */
static void orc_derivs(const double s[], double d[], const OrcRay* p, int n) {
    double r = s[0], theta = s[1];
    double v_r = s[3], v_theta = s[4], v_phi = s[5];
    d[0] = v_r; d[1] = v_theta; d[2] = v_phi;
    if (n > 6) { d[6] = 0.0; d[7] = 0.0; } /* convention, see file header */
    if (p->use_analytic_approx) mg_rel(r, p->field_strength_threshold);
    if (p->use_analytic_approx && r > p->field_strength_threshold) { /* :65-86 */
        double M = p->bh->mass;
        double deflection_factor = 2.0 * M / (r * r);
        if (p->impact_parameter > 0.0) {
            d[3] = 0.0;
            d[4] = 0.0;
            d[5] = v_phi * deflection_factor;
            return;
        }
    }
    double rs = p->bh->schwarzschild_radius, M = p->bh->mass;
    if (p->bh->spin == 0.0) { /* :92-130 */
        double r_sq = r * r;
        double sin_theta = sin(theta);
        double sin_theta_sq = sin_theta * sin_theta;
        if (r <= rs * 1.5) { r = rs * 1.5; r_sq = r * r; }
        if (fabs(sin_theta) < 0.01) {
            mg_note(fabs(sin_theta)); /* the clamp's sign flips at sin = 0 */
            sin_theta = (sin_theta >= 0.0) ? 0.01 : -0.01;
            sin_theta_sq = sin_theta * sin_theta;
        }
        double term1 = -M / (r_sq * (1.0 - rs / r)) * (1.0 - rs / r);
        double term2 = r * v_theta * v_theta;
        double term3 = r * sin_theta_sq * v_phi * v_phi;
        d[3] = term1 + term2 + term3;
        d[4] = -2.0 * v_r * v_theta / r + sin_theta * cos(theta) * v_phi * v_phi;
        d[5] = -2.0 * v_r * v_phi / r - 2.0 * v_theta * v_phi * cos(theta) / sin_theta;
    } else { /* :131-138 */
        d[3] = d[4] = d[5] = 0.0;
    }
    for (int i = 0; i < 6; i++) /* :141-145 */
        if (isnan(d[i]) || isinf(d[i])) d[i] = 0.0;
    for (int i = 3; i < 6; i++) /* :148-153 */
        if (fabs(d[i]) > 10.0) d[i] = (d[i] > 0) ? 10.0 : -10.0;
}

/* math_util.c:162-207 */
static void orc_rk4(double* y, int n, double h, const OrcRay* p) {
    double k1[8], k2[8], k3[8], k4[8], yt[8];
    orc_derivs(y, k1, p, n);
    for (int i = 0; i < n; i++) yt[i] = y[i] + 0.5 * h * k1[i];
    orc_derivs(yt, k2, p, n);
    for (int i = 0; i < n; i++) yt[i] = y[i] + 0.5 * h * k2[i];
    orc_derivs(yt, k3, p, n);
    for (int i = 0; i < n; i++) yt[i] = y[i] + h * k3[i];
    orc_derivs(yt, k4, p, n);
    for (int i = 0; i < n; i++) y[i] += h * (k1[i] + 2.0 * k2[i] + 2.0 * k3[i] + k4[i]) / 6.0;
}

/* math_util.c:212-457 (debug printing dropped; it does not affect results) */
static int orc_rkf45(double y[], int n, double h, double eps_rel, const OrcRay* p) {
    const double b21 = 1.0 / 4.0;
    const double b31 = 3.0 / 32.0, b32 = 9.0 / 32.0;
    const double b41 = 1932.0 / 2197.0, b42 = -7200.0 / 2197.0, b43 = 7296.0 / 2197.0;
    const double b51 = 439.0 / 216.0, b52 = -8.0, b53 = 3680.0 / 513.0, b54 = -845.0 / 4104.0;
    const double b61 = -8.0 / 27.0, b62 = 2.0, b63 = -3544.0 / 2565.0, b64 = 1859.0 / 4104.0,
                 b65 = -11.0 / 40.0;
    const double c1 = 25.0 / 216.0, c3 = 1408.0 / 2565.0, c4 = 2197.0 / 4104.0, c5 = -1.0 / 5.0;
    const double d1 = 16.0 / 135.0, d3 = 6656.0 / 12825.0, d4 = 28561.0 / 56430.0,
                 d5 = -9.0 / 50.0, d6 = 2.0 / 55.0;
    double yt[8], y4[8], y5[8], k1[8], k2[8], k3[8], k4[8], k5[8], k6[8];
    orc_derivs(y, k1, p, n);
    for (int i = 0; i < n; i++) /* :318-333 */
        if (isnan(k1[i]) || isinf(k1[i])) return 1;
    for (int i = 0; i < n; i++) yt[i] = y[i] + h * b21 * k1[i];
    orc_derivs(yt, k2, p, n);
    for (int i = 0; i < n; i++) yt[i] = y[i] + h * (b31 * k1[i] + b32 * k2[i]);
    orc_derivs(yt, k3, p, n);
    for (int i = 0; i < n; i++) yt[i] = y[i] + h * (b41 * k1[i] + b42 * k2[i] + b43 * k3[i]);
    orc_derivs(yt, k4, p, n);
    for (int i = 0; i < n; i++)
        yt[i] = y[i] + h * (b51 * k1[i] + b52 * k2[i] + b53 * k3[i] + b54 * k4[i]);
    orc_derivs(yt, k5, p, n);
    for (int i = 0; i < n; i++)
        yt[i] = y[i] + h * (b61 * k1[i] + b62 * k2[i] + b63 * k3[i] + b64 * k4[i] + b65 * k5[i]);
    orc_derivs(yt, k6, p, n);
    for (int i = 0; i < n; i++) {
        y4[i] = y[i] + h * (c1 * k1[i] + c3 * k3[i] + c4 * k4[i] + c5 * k5[i]);
        y5[i] = y[i] + h * (d1 * k1[i] + d3 * k3[i] + d4 * k4[i] + d5 * k5[i] + d6 * k6[i]);
    }
    double max_error = 0.0;
    for (int i = 0; i < n; i++) { /* :376-391 */
        double scale = fmax(fabs(y[i]), fabs(y5[i]));
        if (scale < BH_EPSILON) scale = BH_EPSILON;
        double error = fabs(y5[i] - y4[i]) / scale;
        max_error = fmax(max_error, error);
    }
    double error_ratio = max_error / eps_rel;
    mg_rel(error_ratio, 1.0);
    if (error_ratio <= 1.0) { /* :402-434 (t and h_next are not used by the caller) */
        for (int i = 0; i < n; i++) y[i] = y5[i];
        return 0;
    }
    return 1;
}

/* raytracer.c:299-333 */
static void fill_hit_info(RayTraceHit* hit, RayTraceResult result, const Vector3D* pos,
                          double distance, int step_count, double r, double rs,
                          const double* velocity) {
    if (!hit) return;
    hit->result = result;
    hit->hit_position = *pos;
    hit->distance = distance;
    hit->steps = step_count;
    hit->time_dilation = time_dilation(r, rs);
    if (result == RAY_BACKGROUND || result == RAY_MAX_DISTANCE) {
        Vector3D v = {velocity[1], velocity[2], velocity[3]};
        hit->sky_direction = v_norm(v);
    }
}

/* raytracer.c:338-679 */
RayTraceResult orc_integrate_photon_path(const Vector4D* position, const Vector3D* direction,
                                         const BlackHoleParams* bh, const SimulationConfig* cfg,
                                         IntegrationMethod method, Vector3D* path,
                                         int max_positions, int* num_positions,
                                         RayTraceHit* hit) {
    Vector3D nd = v_norm(*direction); /* :355 */
    double state[8];
    Vector3D cp = {position->x, position->y, position->z}, sp;
    cart2sph(&cp, &sp); /* :366 */
    state[0] = position->t; state[1] = sp.x; state[2] = sp.y; state[3] = sp.z;
    double r = sp.x, theta = sp.y, phi = sp.z;
    double dr = sin(theta) * cos(phi) * nd.x + sin(theta) * sin(phi) * nd.y + cos(theta) * nd.z;
    double dtheta = (cos(theta) * cos(phi) * nd.x + cos(theta) * sin(phi) * nd.y -
                     sin(theta) * nd.z) / r;
    double dphi = (-sin(phi) * nd.x + cos(phi) * nd.y) / (r * sin(theta));
    if (fabs(sin(theta)) < BH_EPSILON) dphi = 0.0; /* :402-405 */
    mg_rel(fabs(sin(theta)), BH_EPSILON);
    SchwarzschildMetric m = schw_metric(r, bh); /* :412 */
    double dt_squared = -(m.g_rr * dr * dr + m.g_thth * dtheta * dtheta +
                          m.g_phph * dphi * dphi) / m.g_tt;
    if (dt_squared < 0.0) dt_squared = 0.0;
    double dt = sqrt(dt_squared);
    state[4] = dt; state[5] = dr; state[6] = dtheta; state[7] = dphi;
    double energy = -m.g_tt * dt; /* :437-448 */
    double angular_momentum = m.g_phph * dphi;
    OrcRay rp;
    rp.bh = bh;
    rp.impact_parameter = fabs(angular_momentum / energy);
    rp.field_strength_threshold = bh->schwarzschild_radius * 15.0; /* :465-466 */
    rp.use_analytic_approx = (r > rp.field_strength_threshold) ? 1 : 0;
    mg_rel(r, rp.field_strength_threshold);
    if (rp.use_analytic_approx) mg_note(rp.impact_parameter / r); /* b > 0 selects the branch */

    int step_count = 0;
    double distance_traveled = 0.0;
    Vector3D current_pos, sph0 = {state[1], state[2], state[3]};
    sph2cart(&sph0, &current_pos); /* :501 */
    if (path != NULL && max_positions > 0) { path[0] = current_pos; *num_positions = 1; }
    if (g_mg_iter && path != NULL && max_positions > 0) g_mg_iter[0] = g_mg;
    RayTraceResult result = RAY_MAX_STEPS;
    while (step_count < cfg->max_integration_steps) { /* :517-665 */
        for (int i = 0; i < 8; i++) /* :543-548 */
            if (isnan(state[i]) || isinf(state[i])) state[i] = (i < 4) ? 1.0 : 0.0;
        double h; /* :556-571 */
        if (g_mg_on) { /* the comparisons the chain evaluates */
            const double rs = bh->schwarzschild_radius;
            mg_rel(state[1], rs * 2.5);
            if (!(state[1] < rs * 2.5)) mg_rel(state[1], rs * 5.0);
            if (!(state[1] < rs * 5.0)) mg_rel(state[1], rs * 15.0);
        }
        if (state[1] < bh->schwarzschild_radius * 2.5) h = cfg->time_step * 0.001;
        else if (state[1] < bh->schwarzschild_radius * 5.0) h = cfg->time_step * 0.01;
        else if (state[1] < bh->schwarzschild_radius * 15.0) h = cfg->time_step * 0.1;
        else h = cfg->time_step;
        h = fmin(h, 0.1);
        switch (method) { /* :573-625 */
        case INTEGRATOR_RK4: orc_rk4(state, 8, h, &rp); break;
        case INTEGRATOR_RKF45: (void)orc_rkf45(state, 6, h, cfg->tolerance, &rp); break;
        default: break; /* LEAPFROG / YOSHIDA: "not implemented", state unchanged */
        }
        Vector3D ns = {state[1], state[2], state[3]}, np;
        sph2cart(&ns, &np);
        double step_distance = v_len(v_sub(np, current_pos)); /* :633-640 */
        current_pos = np;
        distance_traveled += step_distance;
        int stored = -1;
        if (path != NULL && *num_positions < max_positions) { /* :643-646 */
            path[*num_positions] = current_pos;
            stored = (*num_positions)++;
        }
        if (g_mg_on) {
            mg_rel(state[1], bh->schwarzschild_radius * 1.05);
            if (!(state[1] <= bh->schwarzschild_radius * 1.05))
                mg_rel(distance_traveled, cfg->max_ray_distance);
            if (g_mg_iter && stored >= 0) g_mg_iter[stored] = g_mg;
        }
        if (state[1] <= bh->schwarzschild_radius * 1.05) { result = RAY_HORIZON; break; }
        if (distance_traveled >= cfg->max_ray_distance) { result = RAY_MAX_DISTANCE; break; }
        step_count++;
    }
    fill_hit_info(hit, result, &current_pos, distance_traveled, step_count, state[1],
                  bh->schwarzschild_radius, &state[4]);
    return result;
}

/* raytracer.c:159-196 (third argument is the previous path point, used as the "normal") */
int orc_check_disk_intersection(const Vector3D* position, const Vector3D* velocity,
                                const Vector3D* disk_normal, const AccretionDiskParams* disk,
                                Vector3D* hit_position) {
    double denom = v_dot(*velocity, *disk_normal);
    if (g_mg_on) {
        const double vn = v_len(*velocity) * v_len(*disk_normal);
        mg_rel(fabs(denom), BH_EPSILON);
        mg_note(fabs(denom) / vn);                                  /* t's sign: den's sign */
        mg_note(fabs(v_dot(*position, *disk_normal)) / (v_len(*position) * v_len(*disk_normal)));
    }
    if (fabs(denom) < BH_EPSILON) return 0;
    double t = -(v_dot(*position, *disk_normal)) / denom;
    if (t < 0.0) return 0;
    *hit_position = v_add(*position, v_scale(*velocity, t));
    double r = sqrt(hit_position->x * hit_position->x + hit_position->y * hit_position->y);
    if (g_mg_on) {
        mg_rel(r, disk->inner_radius);
        if (r >= disk->inner_radius) mg_rel(r, disk->outer_radius);
    }
    return (r >= disk->inner_radius && r <= disk->outer_radius) ? 1 : 0;
}

/* raytracer.c:684-767 with the integrator as a parameter (the reference hard-codes RK4) */
RayTraceResult orc_trace_ray_method(const Ray* ray, const BlackHoleParams* bh,
                                    const AccretionDiskParams* disk, const SimulationConfig* cfg,
                                    IntegrationMethod method, RayTraceHit* hit) {
    Vector4D position = {0.0, ray->origin.x, ray->origin.y, ray->origin.z};
    int max_positions = 0, num_positions = 0;
    Vector3D* path = NULL;
    if (disk != NULL) {
        max_positions = cfg->max_integration_steps;
        path = (Vector3D*)malloc((size_t)(max_positions > 0 ? max_positions : 1) * sizeof(Vector3D));
    }
    if (g_mg_on) {
        g_mg = INFINITY;
        g_mg_iter = path ? (double*)malloc((size_t)(max_positions > 0 ? max_positions : 1) *
                                           sizeof(double)) : NULL;
    }
    RayTraceResult result = orc_integrate_photon_path(&position, &ray->direction, bh, cfg, method,
                                                      path, max_positions, &num_positions, hit);
    const double mg_path = g_mg;
    if (g_mg_on) g_mg = INFINITY; /* from here: the disk tests of the scanned segments */
    int hit_at = 0;
    if (disk != NULL && path != NULL && num_positions > 1) { /* :717-759 */
        for (int i = 1; i < num_positions; i++) {
            Vector3D q;
            if (orc_check_disk_intersection(&path[i], &ray->direction, &path[i - 1], disk, &q)) {
                hit_at = i;
                if (hit != NULL) {
                    hit->result = RAY_DISK;
                    hit->hit_position = q;
                    double dist = 0.0;
                    for (int j = 1; j <= i; j++) dist += v_len(v_sub(path[j], path[j - 1]));
                    dist += v_len(v_sub(q, path[i - 1]));
                    hit->distance = dist;
                    hit->steps = i;
                    hit->time_dilation = time_dilation(v_len(q), bh->schwarzschild_radius);
                }
                result = RAY_DISK;
                break;
            }
        }
    }
    if (g_mg_on) {
        const double m_int = hit_at && g_mg_iter ? g_mg_iter[hit_at] : mg_path;
        g_mg_result = m_int < g_mg ? m_int : g_mg;
        free(g_mg_iter);
        g_mg_iter = NULL;
    }
    free(path);
    return result;
}

RayTraceResult orc_trace_ray(const Ray* ray, const BlackHoleParams* bh,
                             const AccretionDiskParams* disk, const SimulationConfig* cfg,
                             RayTraceHit* hit) {
    return orc_trace_ray_method(ray, bh, disk, cfg, INTEGRATOR_RK4, hit);
}

/* ---- shading: math_util.c:463-503, raytracer.c:201-294 ---- */
void orc_temperature_to_rgb(double temperature, double rgb[3]) {
    temperature = orc_clamp(temperature, 1000.0, 40000.0);
    double t = (temperature - 1000.0) / (40000.0 - 1000.0);
    rgb[0] = (t < 0.5) ? t * 2.0 : 1.0;
    if (t < 0.25) rgb[1] = 0.0;
    else if (t < 0.75) rgb[1] = (t - 0.25) * 2.0;
    else rgb[1] = 1.0;
    rgb[2] = (t < 0.5) ? 0.0 : (t - 0.5) * 2.0;
    double brightness = 0.2 + 0.8 * (t * t);
    rgb[0] *= brightness; rgb[1] *= brightness; rgb[2] *= brightness;
}
void orc_calculate_disk_temperature(const Vector3D* p, const BlackHoleParams* bh,
                                    const AccretionDiskParams* disk, double* T, double rgb[3]) {
    (void)bh;
    double r = sqrt(p->x * p->x + p->y * p->y);
    double nr = (r - disk->inner_radius) / (disk->outer_radius - disk->inner_radius);
    nr = orc_clamp(nr, 0.0, 1.0);
    double temp_factor = pow(1.0 - nr, 0.75);
    *T = disk->temperature_scale * (2000.0 + 18000.0 * temp_factor);
    orc_temperature_to_rgb(*T, rgb);
}
void orc_apply_relativistic_effects(const Vector3D* p, const Vector3D* v,
                                    const BlackHoleParams* bh, double c[3], double* dop_out) {
    double r = sqrt(p->x * p->x + p->y * p->y);
    double phi = atan2(p->y, p->x);
    Vector3D tangent = {-sin(phi), cos(phi), 0.0};
    double doppler = 1.0 + v_dot(*v, tangent) * 0.5;
    double grav = time_dilation(r, bh->schwarzschild_radius);
    double redshift = doppler / grav;
    if (redshift < 1.0) {
        c[2] *= redshift;
        c[0] = fmin(1.0, c[0] * (2.0 - redshift));
    } else {
        c[0] *= 2.0 - redshift;
        c[2] = fmin(1.0, c[2] * redshift);
    }
    double beaming = pow(doppler, 4);
    c[0] *= beaming; c[1] *= beaming; c[2] *= beaming;
    c[0] = orc_clamp(c[0], 0.0, 1.0);
    c[1] = orc_clamp(c[1], 0.0, 1.0);
    c[2] = orc_clamp(c[2], 0.0, 1.0);
    if (dop_out) *dop_out = doppler;
}

/* raytracer.c:852-863 */
double orc_halton_sequence(int index, int base) {
    double result = 0.0, f = 1.0;
    while (index > 0) {
        f /= base;
        result += f * (index % base);
        index /= base;
    }
    return result;
}

/* raytracer.c:868-932 (JITTER_RANDOM uses rand(): unpinned, treated as the pixel centre) */
void orc_jittered_offset(int sample, int spp, JitterMethod jm, double strength, double* ox,
                         double* oy) {
    *ox = 0.5; *oy = 0.5;
    switch (jm) {
    case JITTER_REGULAR_GRID: {
        int g = (int)sqrt((double)spp);
        int x = sample % g, y = sample / g;
        *ox = (x + 0.5) / g;
        *oy = (y + 0.5) / g;
    } break;
    case JITTER_HALTON:
    case JITTER_BLUE_NOISE:
        *ox = orc_halton_sequence(sample, 2);
        *oy = orc_halton_sequence(sample, 3);
        break;
    default: break;
    }
    if (strength != 1.0) {
        *ox = 0.5 + (*ox - 0.5) * strength;
        *oy = 0.5 + (*oy - 0.5) * strength;
    }
}

/* raytracer.c:999-1039 */
void orc_camera_ray_direction(int px, int py, double ox, double oy, int W, int H,
                              const bhrt_camera* cam, Vector3D* dir) {
    double aspect = (double)W / (double)H;
    Vector3D fwd = v_norm(cam->direction);
    Vector3D right = v_norm(v_cross(fwd, cam->up));
    Vector3D up = v_cross(right, fwd);
    double fov_radians = cam->fov_deg * BH_PI / 180.0;
    double plane_h = 2.0 * tan(fov_radians / 2.0);
    double plane_w = plane_h * aspect;
    double ndcX = (2.0 * ((px + ox) / W) - 1.0) * plane_w;
    double ndcY = (1.0 - 2.0 * ((py + oy) / H)) * plane_h;
    Vector3D d = fwd;
    d = v_add(d, v_scale(right, ndcX));
    d = v_add(d, v_scale(up, ndcY));
    *dir = v_norm(d);
}

/* ---- drivers ---- */
/* ---- particle_sim.c: update_particles and its two steppers ---- */
static void christoffel(double r, double theta, const BlackHoleParams* bh, double G[4][4][4]) {
    /* spacetime.c:93-161 */
    memset(G, 0, 4 * 4 * 4 * sizeof(double));
    if (bh->spin == 0.0) {
        double rs = bh->schwarzschild_radius;
        if (r <= rs + BH_EPSILON) r = rs + BH_EPSILON;
        double sin_theta = sin(theta), cos_theta = cos(theta);
        G[0][0][1] = G[0][1][0] = rs / (2.0 * r * (r - rs));
        G[1][0][0] = rs * (r - rs) / (2.0 * r * r * r);
        G[1][1][1] = -rs / (2.0 * r * (r - rs));
        G[1][2][2] = -(r - rs);
        G[1][3][3] = -(r - rs) * sin_theta * sin_theta;
        G[2][1][2] = G[2][2][1] = 1.0 / r;
        G[2][3][3] = -sin_theta * cos_theta;
        G[3][1][3] = G[3][3][1] = 1.0 / r;
        G[3][2][3] = G[3][3][2] = cos_theta / sin_theta;
    } else {
        double M = bh->mass, a = bh->spin * M;
        if (r <= bh->r_plus + BH_EPSILON) r = bh->r_plus + BH_EPSILON;
        double sin_theta = sin(theta), cos_theta = cos(theta);
        double sin_theta_sq = sin_theta * sin_theta, cos_theta_sq = cos_theta * cos_theta;
        double Sigma = r * r + a * a * cos_theta_sq;
        double Sigma_sq = Sigma * Sigma;
        G[0][0][1] = M * (r * r - a * a * cos_theta_sq) / Sigma_sq;
        G[0][1][0] = G[0][0][1];
        G[0][1][3] = -a * M * sin_theta_sq * (r * r - a * a * cos_theta_sq) / Sigma_sq;
        G[0][3][1] = G[0][1][3];
    }
}

static void particle_geodesic(Particle* p, const BlackHoleParams* bh, const SimulationConfig* cfg) {
    /* particle_sim.c:232-304 (particle_derivatives :33-68, geodesic_equation spacetime.c:166-187) */
    Vector3D sph;
    cart2sph(&p->position, &sph);
    double r = sph.x, theta = sph.y, phi = sph.z;
    double state[8] = {0.0, r, theta, phi, 1.0, 0.0, 0.0, 0.0};
    double v_mag = v_len(p->velocity);
    state[5] = v_mag * cos(theta) * cos(phi);
    state[6] = v_mag * sin(phi);
    state[7] = v_mag * sin(theta) * cos(phi);
    double G[4][4][4], acc[4] = {0.0, 0.0, 0.0, 0.0};
    christoffel(state[1], state[2], bh, G);
    for (int mu = 0; mu < 4; mu++)
        for (int al = 0; al < 4; al++)
            for (int be = 0; be < 4; be++) acc[mu] -= G[mu][al][be] * state[4 + al] * state[4 + be];
    double d[8] = {state[4], state[5], state[6], state[7], acc[0], acc[1], acc[2], acc[3]};
    for (int i = 0; i < 8; i++) state[i] += d[i] * cfg->time_step;
    Vector3D ns = {state[1], state[2], state[3]};
    sph2cart(&ns, &p->position);
    double v_r = state[5], v_theta = state[6], v_phi = state[7];
    p->velocity.x = v_r * sin(theta) * cos(phi) + r * v_theta * cos(theta) * cos(phi) - r * sin(theta) * v_phi * sin(phi);
    p->velocity.y = v_r * sin(theta) * sin(phi) + r * v_theta * cos(theta) * sin(phi) + r * sin(theta) * v_phi * cos(phi);
    p->velocity.z = v_r * cos(theta) - r * v_theta * sin(theta);
    p->time_dilation = time_dilation(state[1], bh->schwarzschild_radius);
}

static void particle_newtonian(Particle* p, const BlackHoleParams* bh, const SimulationConfig* cfg) {
    /* particle_sim.c:306-337 */
    double r = v_len(p->position);
    double accel_mag = bh->mass / (r * r);
    Vector3D accel_dir = v_scale(p->position, -1.0 / r);
    Vector3D acceleration = v_scale(accel_dir, accel_mag);
    p->velocity = v_add(p->velocity, v_scale(acceleration, cfg->time_step));
    p->position = v_add(p->position, v_scale(p->velocity, cfg->time_step));
}

void orc_update_particles(Particle* ps, int count, const BlackHoleParams* bh,
                          const SimulationConfig* cfg, int steps) {
    for (int s = 0; s < steps; s++) /* particle_sim.c:505-566, once per step */
        for (int i = 0; i < count; i++) {
            Particle* p = &ps[i];
            if (!p->active) continue;
            p->age += cfg->time_step;
            double r = v_len(p->position);
            if (p->type == PARTICLE_TEST && r < 20.0 * bh->schwarzschild_radius)
                particle_geodesic(p, bh, cfg);
            else
                particle_newtonian(p, bh, cfg);
            r = v_len(p->position);
            if (r <= bh->schwarzschild_radius) p->active = 0;
        }
}

int orc_shard_rows(int H, const bhrt_rows* rows) {
    if (!rows || rows->num_shards <= 1) return H;
    int B = rows->row_block, n = 0;
    for (int b = rows->shard; b * B < H; b += rows->num_shards) {
        int hi = (b + 1) * B;
        n += (hi > H ? H : hi) - b * B;
    }
    return n;
}
int orc_shard_row(int j, const bhrt_rows* rows) {
    if (!rows || rows->num_shards <= 1) return j;
    int B = rows->row_block;
    return ((j / B) * rows->num_shards + rows->shard) * B + j % B;
}

/* frame colour contract: disk -> temperature rgb (+ Doppler/beaming
 * with BHRT_FLAG_DOPPLER), horizon -> black, otherwise the sky gradient of
 * raytracer.c:1150-1157 */
static void frame_colour(int res, const Vector3D* q, const Vector3D* dir,
                         const BlackHoleParams* bh, const AccretionDiskParams* disk, int flags,
                         double rgb[3]) {
    if (res == RAY_DISK) {
        double T;
        orc_calculate_disk_temperature(q, bh, disk, &T, rgb);
        if (flags & BHRT_FLAG_DOPPLER) orc_apply_relativistic_effects(q, dir, bh, rgb, NULL);
    } else if (res == RAY_HORIZON) {
        rgb[0] = rgb[1] = rgb[2] = 0.0;
    } else {
        double t = 0.5 * (dir->y + 1.0);
        rgb[0] = (1.0 - t) * 1.0 + t * 0.5;
        rgb[1] = (1.0 - t) * 1.0 + t * 0.7;
        rgb[2] = (1.0 - t) * 1.0 + t * 1.0;
    }
}

static void store(const bhrt_frame_soa* o, long i, const RayTraceHit* h, const double rgb[3]) {
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
    if (rgb) {
        if (o->rgb_r) o->rgb_r[i] = rgb[0];
        if (o->rgb_g) o->rgb_g[i] = rgb[1];
        if (o->rgb_b) o->rgb_b[i] = rgb[2];
    }
}

static void trace_one(const Ray* ray, const BlackHoleParams* bh, const AccretionDiskParams* disk,
                      const SimulationConfig* cfg, IntegrationMethod method, RayTraceHit* h) {
    memset(h, 0, sizeof(*h));
    orc_trace_ray_method(ray, bh, disk, cfg, method, h); /* disk == NULL: plain integration */
}

static int render_frame(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                        const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                        const bhrt_rows* rows, IntegrationMethod method, int flags,
                        const bhrt_frame_soa* out, double* margin, int nthreads) {
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
        g_mg_on = margin != NULL;
        trace_one(&ray, bh, disk, cfg, method, &h);
        if (margin) margin[i] = g_mg_result;
        g_mg_on = 0;
        double rgb[3];
        frame_colour(h.result, &h.hit_position, &dir, bh, disk, flags, rgb);
        store(out, i, &h, rgb);
    }
    return 0;
}

int orc_render_frame(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                     const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                     const bhrt_rows* rows, IntegrationMethod method, int flags,
                     const bhrt_frame_soa* out, int nthreads) {
    return render_frame(bh, disk, cfg, cam, W, H, rows, method, flags, out, NULL, nthreads);
}

int orc_render_frame_margin(const BlackHoleParams* bh, const AccretionDiskParams* disk,
                            const SimulationConfig* cfg, const bhrt_camera* cam, int W, int H,
                            const bhrt_rows* rows, IntegrationMethod method, int flags,
                            const bhrt_frame_soa* out, double* margin, int nthreads) {
    return render_frame(bh, disk, cfg, cam, W, H, rows, method, flags, out, margin, nthreads);
}

int orc_trace_rays(const Ray* rays, int n, const BlackHoleParams* bh,
                   const AccretionDiskParams* disk, const SimulationConfig* cfg,
                   IntegrationMethod method, int flags, const bhrt_frame_soa* out, int nthreads) {
    if (!rays || !bh || !cfg || !out || n <= 0) return -1;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        RayTraceHit h;
        trace_one(&rays[i], bh, disk, cfg, method, &h);
        double rgb[3]; /* colour sees Ray.direction as given, like the disk test */
        frame_colour(h.result, &h.hit_position, &rays[i].direction, bh, disk, flags, rgb);
        store(out, i, &h, rgb);
    }
    return 0;
}
