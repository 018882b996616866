/*
 * kerr_helpers.c -- the scalar metric helpers of the reference's spacetime.h that no traced
 * ray calls (src/spacetime.c:38-89, 242-263, 314-327, 377-656), for link compatibility of
 * callers written against the reference headers. Host C, the reference's arithmetic in its
 * evaluation order (built without FP contraction, as the reference's x86-64 build).
 */
#include <math.h>
#include <string.h>

#pragma GCC visibility push(default)
#include "../../include/bhrt_api.h"
#pragma GCC visibility pop

KerrMetric calculate_kerr_metric(double r, double theta, const BlackHoleParams* bh) {
    KerrMetric m;
    memset(&m, 0, sizeof m); /* the reference leaves g_thetatheta unset */
    const double M = bh->mass, a = bh->spin * M;
    if (r <= bh->r_plus + BH_EPSILON) r = bh->r_plus + BH_EPSILON;
    const double st = sin(theta);
    const double st2 = st * st;
    const double Sigma = r * r + a * a * st2;
    m.g_tt = -(1.0 - 2.0 * M * r / Sigma);
    m.g_tphi = -2.0 * M * a * r * st2 / Sigma;
    m.g_rr = Sigma / (r * r - 2.0 * M * r + a * a);
    m.g_thth = Sigma;
    m.g_phiphi = (r * r + a * a + 2.0 * M * r * a * a * st2 / Sigma) * st2;
    m.g_phit = m.g_tphi;
    return m;
}

BlackHoleMetric calculate_metric(double r, double theta, const BlackHoleParams* bh) {
    BlackHoleMetric m;
    memset(&m, 0, sizeof m);
    if (bh->spin == 0.0) {
        m.is_kerr = 0;
        m.metric.schwarzschild = calculate_schwarzschild_metric(r, bh);
    } else {
        m.is_kerr = 1;
        m.metric.kerr = calculate_kerr_metric(r, theta, bh);
    }
    return m;
}

double calculate_effective_potential(double r, double l, const BlackHoleParams* bh) {
    if (bh->spin == 0.0) {
        const double rs = bh->schwarzschild_radius;
        if (r <= rs + BH_EPSILON) r = rs + BH_EPSILON;
        return (1.0 - rs / r) * (1.0 + (l * l) / (r * r));
    }
    const double M = bh->mass, a = bh->spin * M, E = 1.0;
    if (r <= bh->r_plus + BH_EPSILON) r = bh->r_plus + BH_EPSILON;
    const double term1 = E * E - 1.0;
    const double term2 = 2.0 * M / r;
    const double term3 = l * l / (r * r);
    const double term4 = -2.0 * M * a * l / (r * r * r);
    return term1 + term2 * (term3 + term4);
}

double calculate_ergosphere_radius(double theta, const BlackHoleParams* bh) {
    const double M = bh->mass, a = bh->spin * M;
    if (a <= BH_EPSILON) return 2.0 * M;
    const double c = cos(theta);
    return M + sqrt(M * M - a * a * c * c);
}

/* sin^2, cos^2 and the Boyer-Lindquist scalars shared by the position[4] helpers */
typedef struct {
    double st, ct, st2, ct2, a2, r2, two_mr, Sigma, Delta;
} bl_terms;

static bl_terms bl(const double position[4], double a, double M) {
    bl_terms t;
    const double r = position[1], theta = position[2];
    t.st = sin(theta);
    t.st2 = t.st * t.st;
    t.ct = cos(theta);
    t.ct2 = t.ct * t.ct;
    t.a2 = a * a;
    t.r2 = r * r;
    t.two_mr = 2.0 * M * r;
    t.Sigma = t.r2 + t.a2 * t.ct2;
    t.Delta = t.r2 - t.two_mr + t.a2;
    return t;
}

int calculate_kerr_metric_bl(const double position[4], double a, double M, KerrMetric* m) {
    if (position == NULL || m == NULL || a < 0 || a >= 1) return -1;
    const bl_terms t = bl(position, a, M);
    m->g_tt = -(1.0 - t.two_mr / t.Sigma);
    m->g_tphi = -t.two_mr * a * t.st2 / t.Sigma;
    m->g_rr = t.Sigma / t.Delta;
    m->g_thetatheta = t.Sigma;
    m->g_phiphi = (t.r2 + t.a2 + t.two_mr * t.a2 * t.st2 / t.Sigma) * t.st2;
    return 0;
}

int calculate_inverse_kerr_metric(const double position[4], double a, double M, KerrMetric* m) {
    if (position == NULL || m == NULL || a < 0 || a >= 1) return -1;
    const bl_terms t = bl(position, a, M);
    m->g_tt = -((t.r2 + t.a2) * (t.r2 + t.a2) - t.Delta * t.a2 * t.st2) / (t.Sigma * t.Delta);
    m->g_tphi = -t.two_mr * a / (t.Sigma * t.Delta);
    m->g_rr = t.Delta / t.Sigma;
    m->g_thetatheta = 1.0 / t.Sigma;
    m->g_phiphi = (t.Delta - t.a2 * t.st2) / (t.Sigma * t.Delta * t.st2);
    return 0;
}

int calculate_kerr_christoffel(const double position[4], double a, double M, double G[4][4][4]) {
    if (position == NULL || G == NULL || a < 0 || a >= 1) return -1;
    memset(G, 0, 4 * 4 * 4 * sizeof(double));
    const double r = position[1], theta = position[2];
    const double st = sin(theta), ct = cos(theta);
    const double a2 = a * a, r2 = r * r, two_mr = 2.0 * M * r;
    const double Sigma = r2 + a2 * ct * ct;
    const double Sigma_sq = Sigma * Sigma;
    const double Delta = r2 - two_mr + a2;
    G[0][0][1] = M * (r2 - a2 * ct * ct) / (Sigma_sq * Delta);
    G[0][0][2] = -2.0 * M * r * a2 * st * ct / Sigma_sq;
    G[1][0][0] = Delta * M * (r2 - a2 * ct * ct) / Sigma_sq;
    G[1][1][1] = (M * (r2 - a2 * ct * ct) - r * Delta) / (Sigma * Delta);
    G[2][2][1] = r / Sigma;
    G[2][2][2] = -a2 * st * ct / Sigma;
    G[3][1][3] = (r * Delta - M * (r2 - a2 * ct * ct)) / (Sigma * Delta);
    G[3][2][3] = 1.0 / tan(theta) - a2 * st * ct / Sigma;
    return 0;
}

double calculate_kerr_isco(double a, double M, bool prograde) {
    const double s = prograde ? a : -a;
    const double Z1 =
        1.0 + pow(1.0 - s * s, 1.0 / 3.0) * (pow(1.0 + s, 1.0 / 3.0) + pow(1.0 - s, 1.0 / 3.0));
    const double Z2 = sqrt(3.0 * s * s + Z1 * Z1);
    return M * (3.0 + Z2 - sqrt((3.0 - Z1) * (3.0 + Z1 + 2.0 * Z2)));
}

double calculate_kerr_event_horizon(double a, double M) { return M * (1.0 + sqrt(1.0 - a * a)); }

double calculate_kerr_ergosphere(double a, double M, double theta) {
    return M * (1.0 + sqrt(1.0 - a * a * cos(theta) * cos(theta)));
}

int calculate_frame_dragging(const double position[4], double a, double M, double velocity[3]) {
    if (position == NULL || velocity == NULL || a < 0 || a >= 1) return -1;
    const double r = position[1], theta = position[2];
    const double st = sin(theta), ct = cos(theta);
    const double Sigma = r * r + a * a * ct * ct;
    const double omega =
        2.0 * M * r * a / (Sigma * (r * r + a * a) + 2.0 * M * r * a * a * st * st);
    velocity[0] = 0.0;
    velocity[1] = 0.0;
    velocity[2] = omega;
    return 0;
}

int calculate_kerr_geodesic(const double position[4], const double velocity[4], double a,
                            double M, double acceleration[4]) {
    if (position == NULL || velocity == NULL || acceleration == NULL || a < 0 || a >= 1)
        return -1;
    double G[4][4][4];
    const int rc = calculate_kerr_christoffel(position, a, M, G);
    if (rc != 0) return rc;
    memset(acceleration, 0, 4 * sizeof(double));
    for (int mu = 0; mu < 4; mu++)
        for (int al = 0; al < 4; al++)
            for (int be = 0; be < 4; be++)
                acceleration[mu] -= G[mu][al][be] * velocity[al] * velocity[be];
    return 0;
}
