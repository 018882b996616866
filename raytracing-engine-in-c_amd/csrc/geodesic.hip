// geodesic.hip -- MI355X (gfx950) kernels of the geodesic ray tracer.
//
// One lane = one ray, FP64 throughout, the integrated state in VGPRs. What each lane
// computes is the reference's integrate_photon_path / trace_ray (src/raytracer.c:338-767,
// with rk4_integrate / rkf45_integrate of src/math_util.c:162-457 inlined), reproduced with
// its quirks: the index-shifted ray_derivatives (raytracer.c:44-154), the clamps, the
// radius step schedule and the zero-acceleration "Kerr" branch. See DESIGN.md section 2.
//
// Restructurings that leave every pinned output unchanged:
//   * trace_ray stores the whole path and scans it for the first disk crossing afterwards
//     (raytracer.c:698-759); here each segment is tested as soon as it exists and the lane
//     stops at the first hit.
//   * RKF45 never adapts h (raytracer.c:556-571 recomputes it from r), so a rejected attempt
//     leaves the state at a fixed point that rejects until max_steps; the lane jumps there.
//   * derivatives[6..7] are never written by the reference (uninitialised malloc); they are 0
//     here, so state[6..7] are per-ray constants.
//
// Divergence: rays live from 1 to max_steps iterations. The grid is persistent; every
// wavefront keeps 64 rays in flight and, once `refill` of its lanes have finished, claims
// that many new ray indices from a global queue with ONE atomic and initialises them in
// the idle lanes (ballot + popcount + lane rank), so a long ray never holds 63 idle lanes.
//
// Arithmetic: FP contraction on; quotients as a * RN(1/b) without the
// generic fdiv scaffolding; sincos specialised for the loop's argument range, shifted by angle
// addition between RK stages and carried from one iteration to the next. The hot
// instantiation contains no call: rays that need a large-argument sincos are re-traced by a
// second launch (k_trace HUGE=true).
//
// This file holds only the shipped variant. The A/B alternatives measured against it (OCML
// sincos, exact quotients, unfolded forms, per-iteration trig, the shift-statistics and
// wave-tail instrumentation) are in git history up to f099035 (tools/build_rev.sh builds any
// revision for a same-box A/B); DESIGN.md section 6 records what each was worth.
#include <hip/hip_runtime.h>

#include <atomic>

#include "bhrt_kernel.h"

#pragma clang fp contract(fast)

namespace {

constexpr double kEps = 1.0e-10;  // BH_EPSILON (math_util.h:21)
constexpr double kTwoPi = 6.28318530717958647692;

using Scene = bhrt_scene_k;

struct Counters {
    unsigned rays = 0, iters = 0, full = 0, far_ = 0, kerr = 0;
    bool huge = false;  // a sincos argument needed the large-argument path (see bhrt_sincos)
};

// Division without the generic fdiv scaffolding.
// rcp_nr is RN(1/b) for b in the normal range: v_rcp_f64 (good to ~2^-24,
// tools/probe/trans_probe.hip) and one cubically convergent step y0 (1 + e + e^2), e^3 ~ 2^-72
// far below the final rounding -- three FMAs instead of the compiler's two Newton steps. One
// reciprocal serves every quotient with the same divisor, and div_nr(a, b, rcp_nr(b)) is
// a * RN(1/b) (<= 1.5 ulp; the same order as the FMA contraction): on every BASELINE config it
// leaves the class and step of every sampled ray equal to the compiled reference's and the hit
// points as close (profiles/r01_bench_all_configs_v6.jsonl), for 7% of C2. Callers keep the
// IEEE a / b for out-of-range operands.
__device__ __forceinline__ double rcp_nr(double b) {
    const double y = __builtin_amdgcn_rcp(b);
    const double e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(y, __builtin_fma(e, e, e), y);
}
__device__ __forceinline__ double div_nr(double a, double /*b*/, double yb) { return a * yb; }

// fma(a, b, c) with c a compile-time coefficient, as ONE v_fma_f64 whose addend is an SGPR
// pair (set up by SALU). Left to itself hipcc copies the coefficient into the destination
// (v_mov_b64) and uses v_fmac_f64: two VALU instructions per Horner step.
__device__ __forceinline__ double fmac_k(double a, double b, double c) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(c));
    return r;
}

// max(a, b) as ONE v_max_f64 (b in SGPRs): fmax would first canonicalize both operands
// (v_max_f64 x, x, x) for its NaN rule; callers pass non-NaN a.
__device__ __forceinline__ double max_raw(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "s"(b));
    return r;
}
// max(|a|, |b|) as ONE v_max_f64 with both abs modifiers (non-NaN a, b)
__device__ __forceinline__ double max_abs_raw(double a, double b) {
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// sin and cos of one argument, for the trace loop. OCML's sincos
// spends ~78 VALU per call on a range reduction valid to 2^30+; every argument here (the
// radius read as an angle by ray_derivatives, theta, phi) stays far below 2^20, where a
// three-constant Cody-Waite reduction with FMA is exact up to a double-double tail. The
// tail feeds the fdlibm kernels (k_sin.c / k_cos.c, FreeBSD form). Measured on 6e7 random
// arguments against glibc (the reference's libm): max 1 ulp, 97% bit-identical.
// |x| >= 2^20 takes OCML's sincos (not inlined: its Payne-Hanek path must not cost registers
// in the loop).
__device__ __attribute__((noinline)) void sincos_ocml(double x, double* s, double* c) {
    sincos(x, s, c);
}

// hc == nullptr: |x| >= 2^20 takes OCML's out-of-line path. Otherwise (the hot trace loop,
// which must contain no call: the call ABI would spill the ray state to scratch) a finite
// |x| >= 2^20 only raises hc->huge and the ray is re-traced by the HUGE instantiation;
// Inf and NaN need no special path (the reduction below turns them into NaN, as glibc does).
__device__ __forceinline__ void bhrt_sincos(double x, double* so, double* co,
                                            Counters* hc = nullptr) {
    if (!(fabs(x) < 1048576.0)) {
        if (!hc) {
            sincos_ocml(x, so, co);
            return;
        }
        if (fabs(x) <= 1.79769313486231570815e+308) hc->huge = true;
    }
    constexpr double kTwoOverPi = 6.36619772367581382433e-01;
    constexpr double P1 = 1.57079632679489655800e+00;   // pi/2 in three parts
    constexpr double P2 = 6.12323399573676603587e-17;
    constexpr double P3 = -1.49738490485916983e-33;
    const double n = rint(x * kTwoOverPi);
    const double r1 = __builtin_fma(-n, P1, x);          // exact for |x| < 2^20
    const double p2 = n * P2;
    const double p2e = __builtin_fma(n, P2, -p2);        // n*P2 = p2 + p2e exactly
    const double hi = r1 - p2;                           // TwoSum(r1, -p2)
    const double t = hi - r1;
    const double e = (r1 - (hi - t)) - (p2 + t);
    const double lo = __builtin_fma(-n, P3, e - p2e);
    const double r = hi + lo;                            // reduced argument r + y
    const double y = (hi - r) + lo;
    constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = r * r, w = z * z;
    const double rs_ = fmac_k(z, fmac_k(z, S4, S3), S2) + z * w * fmac_k(z, S6, S5);
    const double v = z * r;
    const double s = r - ((z * (0.5 * y - v * rs_) - y) - v * S1);
    const double rc = z * fmac_k(z, fmac_k(z, C3, C2), C1) +
                      w * w * fmac_k(z, fmac_k(z, C6, C5), C4);
    const double hz = 0.5 * z, ww = 1.0 - hz;
    const double c = ww + (((1.0 - ww) - hz) + (z * rc - r * y));
    const int q = (int)n;
    double ss = (q & 1) ? c : s;
    double cc = (q & 1) ? s : c;
    *so = (q & 2) ? -ss : ss;
    *co = ((q + 1) & 2) ? -cc : cc;
}

// sin and cos of a + delta from s0 = sin(a), c0 = cos(a), delta in
// [-pi/4, pi/4]: sin(delta) and cos(delta) - 1 from the fdlibm k_sin / k_cos polynomials, and
// the shift adds only small corrections to s0, c0 (error <= the direct value's + 0.5 ulp).
// Returns false, leaving the outputs unset, when delta is outside [-pi/4, pi/4] or when
// a + delta - a would not be exact; the caller then evaluates sincos directly.
__device__ __forceinline__ bool sincos_shift_wide(double a, double s0, double c0, double x,
                                                  double& s, double& c) {
    const double delta = x - a;  // exact when x in [a/2, 2a] (Sterbenz)
    if (!(fabs(delta) <= 0.78539816339744828 && fabs(delta) <= 0.5 * fabs(a))) return false;
    constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double z = delta * delta, w = z * z;
    const double r = fmac_k(z, fmac_k(z, S4, S3), S2) + z * w * fmac_k(z, S6, S5);
    const double sd = delta + (z * delta) * fmac_k(z, r, S1);       // k_sin, tail 0
    const double rc = z * fmac_k(z, fmac_k(z, C3, C2), C1) +
                      w * w * fmac_k(z, fmac_k(z, C6, C5), C4);
    const double cm1 = z * rc - 0.5 * z;                             // k_cos - 1
    s = s0 + (s0 * cm1 + c0 * sd);
    c = c0 + (c0 * cm1 - s0 * sd);
    return true;
}

// sin(delta) and cos(delta) - 1: for |delta| <= 1/16 shift_or_eval's polynomials, above that
// (|delta| <= pi/4) the fdlibm k_sin / k_cos ones of sincos_shift_wide
__device__ __forceinline__ void rotation_coeffs(double delta, double& sd, double& cm1) {
    const double z = delta * delta;
    if (__builtin_expect(fabs(delta) <= 0.0625, 1)) {
        constexpr double S1 = -0.16666666666662605, S2 = 0.00833333327878775,
                         S3 = -0.00019839069723619096;
        constexpr double C1 = 0.04166666666666157, C2 = -0.0013888888827212717,
                         C3 = 2.479927034006378e-05;
        sd = delta + (z * delta) * fmac_k(z, fmac_k(z, S3, S2), S1);
        cm1 = z * __builtin_fma(z, fmac_k(z, fmac_k(z, C3, C2), C1), -0.5);
        return;
    }
    constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                     S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                     S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    constexpr double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
                     C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
                     C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    const double w = z * z;
    const double r = fmac_k(z, fmac_k(z, S4, S3), S2) + z * w * fmac_k(z, S6, S5);
    sd = delta + (z * delta) * fmac_k(z, r, S1);
    const double rc = z * fmac_k(z, fmac_k(z, C3, C2), C1) + w * w * fmac_k(z, fmac_k(z, C6, C5), C4);
    cm1 = z * rc - 0.5 * z;
}

// sin, cos of x given those of a nearby a, as the trace loop needs them: every RK stage after
// the first evaluates ray_derivatives at theta = y1 + delta (the stage increment; |delta| < 0.09
// on a full C2 frame), and the three angles of the state move by one step per iteration.
// Nearly every shift is tiny (on a full C2 frame |x - a| > 0.0625 in < 0.7% of wave
// evaluations at any site), so every lane first runs polynomials fitted to |delta| <= 1/16 --
// three coefficients each for sin(delta) and cos(delta) - 1 instead of fdlibm's six, max error
// 2.4e-19 / 1.0e-21 (tools/shift_poly_fit.py) -- straight-line, and only a lane outside that
// interval then redoes the shift with sincos_shift_wide (|delta| <= pi/4) or evaluates directly.
// The choice is per lane, so a ray's rounding never depends on its wave-mates.
__device__ __forceinline__ void shift_or_eval(double a, double s0, double c0, double x, double& s,
                                              double& c, Counters* hc) {
    const double delta = x - a;  // exact when |delta| <= |a| / 2 (Sterbenz)
    constexpr double S1 = -0.16666666666662605, S2 = 0.00833333327878775,
                     S3 = -0.00019839069723619096;
    constexpr double C1 = 0.04166666666666157, C2 = -0.0013888888827212717,
                     C3 = 2.479927034006378e-05;
    const double z = delta * delta;
    const double sd = delta + (z * delta) * fmac_k(z, fmac_k(z, S3, S2), S1);  // sin(delta)
    const double cm1 = z * __builtin_fma(z, fmac_k(z, fmac_k(z, C3, C2), C1), -0.5);
    // s0 (1 + cm1) + c0 sd as two FMAs (<= 1 ulp)
    s = __builtin_fma(c0, sd, __builtin_fma(s0, cm1, s0));
    c = __builtin_fma(-s0, sd, __builtin_fma(c0, cm1, c0));
    // (delta = x - a is exact for |x - a| <= |a| / 2 (Sterbenz); otherwise -- a near 0 -- it is
    // off by <= ulp(delta) / 2 <= 3.5e-18, well below the polynomials' rounding)
    if (__builtin_expect(!(fabs(delta) <= 0.0625), 0)) {
        if (!sincos_shift_wide(a, s0, c0, x, s, c)) bhrt_sincos(x, &s, &c, hc);
    }
}

// Trig of theta (= y[1]) for one RK stage: stage 1 takes it from the previous iteration
// (carried in Ray_), later stages shift it.
struct Trig1 {
    double a, s, c;  // theta of stage 1 and its sin, cos
};

// ray_derivatives' a = 0 accelerations in the literal form (:92-130, evaluation order as
// written, divisions as div_nr / IEEE), from sin, cos of the unclamped theta.
__device__ __forceinline__ void accel_literal(const double (&y)[6], double (&d)[6], const Scene& sc,
                                              double st, double ct) {
    double r = y[0];
    double rsq = r * r;
    double st2 = st * st;
    if (r <= sc.rs_x1_5) {
        r = sc.rs_x1_5;
        rsq = r * r;
    }
    if (fabs(st) < 0.01) {
        st = (st >= 0.0) ? 0.01 : -0.01;
        st2 = st * st;
    }
    const double term2 = r * y[4] * y[4];
    const double term3 = r * st2 * y[5] * y[5];
    const double n4 = -2.0 * y[3] * y[4];
    const double n5a = -2.0 * y[3] * y[5];
    const double n5b = 2.0 * y[4] * y[5] * ct;
    const double sc4 = st * ct * y[5] * y[5];
    if (r < 1.0e150) {  // r >= 1.5 rs here: every divisor is in the normal range
        const double yr = rcp_nr(r);
        // -M / (r^2 f) * f == -M / r^2 in exact arithmetic
        const double term1 = -(sc.M * yr) * yr;
        d[3] = term1 + term2 + term3;
        d[4] = div_nr(n4, r, yr) + sc4;
        d[5] = div_nr(n5a, r, yr) - div_nr(n5b, st, rcp_nr(st));
    } else {
        const double f = 1.0 - sc.rs / r;
        const double term1 = -sc.M / (rsq * f) * f;
        d[3] = term1 + term2 + term3;
        d[4] = n4 / r + sc4;
        d[5] = n5a / r - n5b / st;
    }
}

// :141-153 -- non-finite -> 0 for all six, then |d[3..5]| <= 10. BOUNDED (k_trace's hot
// instantiations, repair_at_refill): d[0..2] are the stage state's velocities, finite there, so
// only d[3..5] are looked at -- and d[0..2] stay the very registers of the stage state (no copies)
template <bool BOUNDED = false>
__device__ __forceinline__ void repair_clamp(double (&d)[6]) {
#pragma unroll
    for (int i = BOUNDED ? 3 : 0; i < 6; i++)
        if (!isfinite(d[i])) d[i] = 0.0;
#pragma unroll
    for (int i = 3; i < 6; i++) d[i] = fmin(fmax(d[i], -10.0), 10.0);
}

// ray_derivatives (raytracer.c:44-154) for one RK stage. y = (t, r, theta, phi, tdot, rdot)
// of the caller, read -- as the reference does -- as (r, theta, phi, v_r, v_theta, v_phi).
// Stage counters: FAR instantiations count their far-field stages (a lane's branch varies);
// every other stage takes the instantiation's one other branch, and k_trace derives that count
// from the iterations (the HUGE redo, whose RKF45 attempts can stop after stage 1, counts
// every stage).
// Stage-counting build (make DEFS=-DBHRT_COUNT_STAGES=1 -> diag/libbhrt_count.so, built by
// __graft_entry__.build()): every instantiation counts each stage's branch one by one, as the
// FAR && HUGE redo pass always does, instead of deriving the split from the iterations -- the
// GPU test test_stage_counts_are_counted checks that both give the same counters (the FLOP
// credit of bench.py rests on the derived ones) and the same frame.
#ifndef BHRT_COUNT_STAGES
#define BHRT_COUNT_STAGES 0
#endif
template <bool SPIN0, bool FAR, bool HUGE>
__device__ __forceinline__ void rhs(const double (&y)[6], double (&d)[6], const Scene& sc,
                                    bool far_ok, Counters& n, Trig1& tr, bool first) {
    d[0] = y[3];
    d[1] = y[4];
    d[2] = y[5];
    if (FAR && far_ok && y[0] > sc.rs_x15) {  // weak-field branch, no NaN/clamp pass (:65-86)
        d[3] = 0.0;
        d[4] = 0.0;
        d[5] = y[5] * (sc.two_m / (y[0] * y[0]));
        n.far_++;
        return;
    }
    if (SPIN0) {  // :92-130
        double st, ct;
        if (first) {
            st = tr.s;  // carried from the previous iteration (ray_iterate)
            ct = tr.c;
        } else {
            shift_or_eval(tr.a, tr.s, tr.c, y[1], st, ct, HUGE ? nullptr : &n);
        }
        if ((FAR && HUGE) || BHRT_COUNT_STAGES) n.full++;
        // Fast form, straight-line: the same three accelerations with the divisions as one
        // reciprocal and the products regrouped -- d3 = -M/r^2 + r (v_th^2 + (sin th v_ph)^2),
        // d4 = -2 v_r v_th / r + (sin th v_ph)(cos th v_ph),
        // d5 = -2 v_ph (v_r / r + v_th cos th / sin th) -- a few ulp from the literal
        // expressions. y[0] is finite (the state is repaired before
        // the first iteration or at the top of every iteration, and a stage adds a bounded
        // increment), so fmax is the reference's clamp. A lane whose result is not a plain
        // |d| <= 10 value, or whose |sin theta| < 0.01 clamp would bind (never on a C2 frame),
        // recomputes it in the literal form before the repair and clamps.
        const double rc = max_raw(y[0], sc.rs_x1_5);
        // 1/r and 1/sin theta from one reciprocal of the product (r sin theta in [0.03, 1e150]):
        // one v_rcp_f64 + refinement fewer per stage, <= ~2 ulp instead of 1 (+1.7% at 4 waves)
        const double w = rcp_nr(rc * st);
        const double yr = st * w, ys = rc * w;
        const double u = st * y[5];
        const double f3 = rc * __builtin_fma(u, u, y[4] * y[4]);
        d[3] = __builtin_fma(-(sc.M * yr), yr, f3);
        const double p = y[3] * yr;
        d[4] = __builtin_fma(p * -2.0, y[4], u * (ct * y[5]));
        d[5] = (y[5] * -2.0) * __builtin_fma(y[4], ct * ys, p);
        // rc < 1e150 (every divisor of the literal form normal) needs no test in k_trace's hot
        // instantiations: state[0] starts at t = 0 there and moves by h * state[3], whose own
        // derivative is the clamped |d3| <= 10 (or 0), so |state[0]| <= 0.1 * 20 * steps^2;
        // k_path (a caller-given t) and the HUGE redo keep it
        const int plain = (int)(!HUGE ? true : rc < 1.0e150) & (int)(fabs(d[3]) <= 10.0) &
                          (int)(fabs(d[4]) <= 10.0) & (int)(fabs(d[5]) <= 10.0) &
                          (int)(fabs(st) >= 0.01);
        if (__builtin_expect(plain, 1)) return;
        accel_literal(y, d, sc, st, ct);
        repair_clamp<!HUGE>(d);
        return;
    }
    // :131-138
    d[3] = 0.0;
    d[4] = 0.0;
    d[5] = 0.0;
    if ((FAR && HUGE) || BHRT_COUNT_STAGES) n.kerr++;
    // Far-field and Kerr stages: the repair / clamps never change a value here but run as the
    // reference's pass whenever a component is not a plain |d| <= 10 value (NaN and Inf fail
    // the test). d[0..2] = y[3..5] need no test: the iteration starts from a finite state, and
    // a stage state's y[3..5] is that state plus h * (coefficients of |.| <= 8) * k[3..5],
    // which the clamp bounds by 10 -- finite.
    const int plain = (int)(fabs(d[3]) <= 10.0) & (int)(fabs(d[4]) <= 10.0) &
                      (int)(fabs(d[5]) <= 10.0);
    if (plain) return;
    repair_clamp<!HUGE>(d);
}

// Where the loop-top state recovery (raytracer.c:543-548) can only ever act on the first
// iteration, it runs once, at refill (k_trace), and the hot loop drops its 6 VALU per
// iteration. That holds for RK4 and RKF45 without the far-field branch: every acceleration
// the loop feeds back is a plain |d| <= 10 value or comes out of the literal repair and clamps
// (zero on the Kerr branch), so from a finite state a step adds at most h * 10 * (sum of
// |coefficients| <= 18) to state[3..5] -- a finite double plus that rounds to a finite double
// -- and h times stage values of state[3..5] (bounded by the initial velocities, |v| < 2^512
// for any finite set-up, plus 18 per step) to state[0..2], which cannot reach 2^1024 within
// 2^31 steps. For the same reason RKF45's non-finite-k1 reject (math_util.c:318-333) can
// never fire there.
// The far-field branch's acceleration y5 * 2M / y0^2 is unclamped, but it only runs where
// y0 > 15 rs, so its factor is below C = 2M / (15 rs)^2: per step the velocities grow by at
// most a factor 1 + 2 h W C (plus 20 h W), W the step's largest weight sum. The host proves
// from the scene (far_bounded, bhrt_api.c) that a state starting within 2^40 stays below 2^400
// for max_steps steps; far-field instantiations then drop the checks too, and a ray whose
// initial state exceeds 2^40 -- or every ray of a launch the host could not prove bounded --
// is handed to the HUGE redo pass (k_trace's refill), which keeps both checks every iteration.
template <int METHOD, bool FAR, bool HUGE>
constexpr bool repair_at_refill() {
    return (METHOD == INTEGRATOR_RK4 || METHOD == INTEGRATOR_RKF45) && !HUGE;
}

// On the Kerr branch without the far-field one (a != 0, FAR = false) every stage's
// accelerations d[3..5] are the literal 0 (raytracer.c:131-138), so a stage value or update of
// components 3..5 is y + h * (sum of b * 0) = y exactly for the finite state and finite h the
// loop has (only a zero's sign can differ: -0 + +0 = +0). Those components are carried
// unchanged instead of computed (C5: 3 of the 6 components of every RKF45 combination).
template <bool SPIN0, bool FAR>
constexpr bool zero_accel() {
    return !SPIN0 && !FAR;
}

// There, moreover, the stage derivatives of components 0..2 are state[3..5] -- constant over a
// ray's life where the recovery runs once, at refill -- in every stage of every iteration, so
// the weighted stage sums of the step's final combination are per-ray constants: formed once at
// refill (zero_sums, the same expressions on the same values, so bit-identical), and each
// iteration's update of components 0..2 is y + h * sum. RKF45 (C5, two 6-term sums per
// component): +7.5% same-box; RK4 (C4, one 4-term sum, already shared by the iterations of a
// trip) loses 1.5%, so it keeps the inline form (profiles/r02_ab_v24.txt).
template <int METHOD, bool SPIN0, bool FAR, bool HUGE>
constexpr bool hoist_sums() {
    return METHOD == INTEGRATOR_RKF45 && zero_accel<SPIN0, FAR>() &&
           repair_at_refill<METHOD, FAR, HUGE>();
}

// On the same zero-acceleration paths state[2] (theta of the position) advances by a per-ray
// constant times h -- h * (the step's weighted sum of the constant state[5]) -- so within a
// step-size regime the angle turns by the same nominal increment delta every iteration. Its
// sin and cos then follow by a fixed rotation: sin(delta) and cos(delta) - 1 are formed once
// per regime (when h changes, at most three times per ray), and each iteration is the two
// FMA pairs of the shift alone instead of forming delta's polynomials again. The rotation
// tracks the nominal angle, which differs from the rounded state by the states' rounding
// (<= 1 ulp of theta per iteration); the per-iteration shift it replaces carries its own
// rounding the same way.
template <int METHOD, bool SPIN0, bool FAR, bool HUGE>
constexpr bool rotation_trig() {
    return zero_accel<SPIN0, FAR>() && repair_at_refill<METHOD, FAR, HUGE>() &&
           (METHOD == INTEGRATOR_RK4 || METHOD == INTEGRATOR_RKF45);
}

// The step's stage sums (math_util.c:162-207, 367-391), one expression each so that the
// hoisted and the inline forms compile to the same operations.
__device__ __forceinline__ double rk4_acc(double acc, double k) { return acc + 2.0 * k; }
constexpr double kC1 = 25.0 / 216.0, kC3 = 1408.0 / 2565.0, kC4 = 2197.0 / 4104.0,
                 kC5 = -1.0 / 5.0;
constexpr double kD1 = 16.0 / 135.0, kD3 = 6656.0 / 12825.0, kD4 = 28561.0 / 56430.0,
                 kD5 = -9.0 / 50.0, kD6 = 2.0 / 55.0;
__device__ __forceinline__ double rkf45_sum4(double k1, double k3, double k4, double k5) {
    return kC1 * k1 + kC3 * k3 + kC4 * k4 + kC5 * k5;
}
__device__ __forceinline__ double rkf45_sum5(double k1, double k3, double k4, double k5,
                                             double k6) {
    return kD1 * k1 + kD3 * k3 + kD4 * k4 + kD5 * k5 + kD6 * k6;
}

// rk4_integrate (math_util.c:162-207) on the six live components; the running sum
// ((k1 + 2k2) + 2k3) + k4 is the reference's left-to-right evaluation order.
template <bool SPIN0, bool FAR, bool HUGE, bool HS = false>
__device__ __forceinline__ void rk4_step(double (&y)[6], double h, const Scene& sc, bool far_ok,
                                         Counters& n, Trig1& tr, const double* zs = nullptr) {
    constexpr bool Z = zero_accel<SPIN0, FAR>();
    double k[6], acc[6], yt[6];
    const double hh = 0.5 * h;
    const double h6 = h * (1.0 / 6.0);
    rhs<SPIN0, FAR, HUGE>(y, k, sc, far_ok, n, tr, true);
#pragma unroll
    for (int i = 0; i < 6; i++) {
        acc[i] = k[i];
        yt[i] = (Z && i >= 3) ? y[i] : y[i] + hh * k[i];
    }
    rhs<SPIN0, FAR, HUGE>(yt, k, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++) {
        acc[i] = rk4_acc(acc[i], k[i]);
        yt[i] = (Z && i >= 3) ? y[i] : y[i] + hh * k[i];
    }
    rhs<SPIN0, FAR, HUGE>(yt, k, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++) {
        acc[i] = rk4_acc(acc[i], k[i]);
        yt[i] = (Z && i >= 3) ? y[i] : y[i] + h * k[i];
    }
    rhs<SPIN0, FAR, HUGE>(yt, k, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++) {
        // h * (...) / 6 as (h * RN(1/6)) * (...): the increment differs by <= 1 ulp of itself,
        // which is ~h*|k| / |y| ulp of the state
        if (HS && i < 3)
            y[i] = __builtin_fma(h6, zs[i], y[i]);
        else if (!(Z && i >= 3))
            y[i] = __builtin_fma(h6, acc[i] + k[i], y[i]);
    }
}

// RKF45's accept test (math_util.c:367-391, 402-434): accept iff
// RN(max_i RN(err_i / scale_i) / tol) <= 1, scale_i >= 1e-10. For a positive normal (finite)
// tol the outer test is exactly max_error <= tol: x <= t gives x / t <= 1; x > t means
// x >= t + ulp(t), so x / t >= 1 + ulp(t) / t > 1 + 2^-53, the rounding midpoint above 1
// (x = Inf: Inf / t = Inf > 1, also a reject). That is, every component's RN(err / scale) <=
// tol. FAST (where the state is provably bounded, repair_at_refill: |scale| < 2^600) with tol
// in [2^-900, 2^300] decides a component without a division: err <= RN(tol (1 - 2^-40) scale)
// passes, err > RN(tol (1 + 2^-40) scale) rejects, and only an err inside that band (per lane,
// rare) takes the IEEE quotient (v24; v17-v23 formed q = err * rcp(scale) and compared it with
// the same band, 4 more VALU per component; v25 first tries the one-sided test alone, which
// accepts when every component passes it: one product and one compare per component). Otherwise, and for a tol that is <= 0,
// subnormal, Inf or NaN, the literal final quotient decides (wave-uniform branch on tol):
// tol = Inf with max_error = Inf is Inf / Inf = NaN, a reject, where max_error <= tol would
// accept. bhrt_check_rkf45_accept runs both forms on given operands
// (tests/test_gpu_parity.py::test_rkf45_accept_band).
template <bool FAST, int NC = 6>
__device__ __forceinline__ bool rkf45_accept(const double (&err)[6], const double (&scale)[6],
                                             double tol) {
    const bool tol_normal = tol >= 2.2250738585072014e-308 && tol <= 1.79769313486231570815e+308;
    if (FAST && tol >= 0x1p-900 && tol <= 0x1p300) {
        // tol * scale is a normal product here (scale in [1e-10, 2^600]), so RN(lo * scale) and
        // RN(hi * scale) are within 2^-53 of the exact products
        const double lo = tol * (1.0 - 0x1p-40), hi = tol * (1.0 + 0x1p-40);
        // every component clearly inside tol (the usual case): accept with one product and
        // one compare per component; otherwise the two-sided test below
        bool all_pass = true;
#pragma unroll
        for (int i = 0; i < NC; i++) all_pass &= err[i] <= lo * scale[i];
        if (__builtin_expect(all_pass, 1)) return true;
        double near_max = 0.0;
        bool over = false;
#pragma unroll
        for (int i = 0; i < NC; i++) {  // components NC.. have err = 0 (zero_accel)
            // err <= RN(lo s): err / s < tol (1 - 2^-41), so RN(err / s) <= tol;
            // err > RN(hi s): err / s > tol (1 + 2^-41) > tol + ulp(tol) / 2, a reject
            const bool pass = err[i] <= lo * scale[i];
            const bool fail = err[i] > hi * scale[i];
            over |= fail;
            if (__builtin_expect(!pass && !fail, 0)) near_max = fmax(near_max, err[i] / scale[i]);
        }
        return !over && near_max <= tol;
    }
    double max_error = 0.0;
#pragma unroll
    for (int i = 0; i < 6; i++) max_error = fmax(max_error, err[i] / scale[i]);
    return tol_normal ? max_error <= tol : max_error / tol <= 1.0;
}

// Attempts that cannot be rejected (ACC; round 6). Where the stage sums are hoisted (hoist_sums:
// the zero-acceleration paths, C5) every stage derivative of components 0..2 is the ray's
// constant v = state[3..5], so s4 = rkf45_sum4(v, v, v, v) and s5 = rkf45_sum5(v, ..., v) are v
// times weight sums that are exactly 1 in real arithmetic, each within E <= 10u |v| of v (u =
// 2^-53: <= 5 products and sums, partial sums below 1.5 |v|, the weights' own rounding). The
// attempt's a = y5 = RN(y + h s5), b = y4 = RN(y + h s4) and err = RN(|a - b|) then satisfy
//   |a - b| <= |h| |s5 - s4| + u (|a| + |b|)  and  |b| <= |a| + |a - b|,
// so |a - b| <= (|h| |s5 - s4| + 2u |a|) / (1 - u). And scale = max(|y|, |a|, 1e-10) >= |h v| / 2.1
// (if |y| < |h v| / 2, then |a| >= |h v| (1 - E) - |y| - u |a|). Hence err / scale <= 2.1 * 2E
// + 2u (1 + 3u) < 50u < 6e-15 for every component (v = 0: s4 = s5 = 0 and err = 0 exactly;
// tiny v: the absolute rounding is below 2^-1074 against scale >= 1e-10), whatever the state:
// every attempt passes the accept test -- RN(max err / scale) / tol <= 1 -- for any
// tol >= 2^-30 (the host's condition, bhrt_api.c fill_scene: accept_all, with finite step
// sizes and tol <= 2^300). The attempt is then y <- y5 alone: no y4, error, scale or test, and no
// fixed point (C5: ~20 of ~87 VALU per attempt). The state is finite there (repair_at_refill),
// so y + h s5 is too. The redo pass (HUGE) keeps the literal test.
template <bool SPIN0, bool FAR, bool HUGE>
constexpr bool accept_all_ok() {
    return zero_accel<SPIN0, FAR>() && repair_at_refill<INTEGRATOR_RKF45, FAR, HUGE>();
}

// rkf45_integrate (math_util.c:212-457), n = 6. Returns true on accept (y <- y5).
template <bool SPIN0, bool FAR, bool HUGE, bool HS = false, bool ACC = false>
__device__ __forceinline__ bool rkf45_attempt(double (&y)[6], double h, const Scene& sc,
                                              bool far_ok, Counters& n, Trig1& tr,
                                              const double* zs = nullptr) {
    static_assert(!ACC || (HS && accept_all_ok<SPIN0, FAR, HUGE>()), "ACC: hoisted sums only");
    constexpr double b21 = 1.0 / 4.0;
    constexpr double b31 = 3.0 / 32.0, b32 = 9.0 / 32.0;
    constexpr double b41 = 1932.0 / 2197.0, b42 = -7200.0 / 2197.0, b43 = 7296.0 / 2197.0;
    constexpr double b51 = 439.0 / 216.0, b52 = -8.0, b53 = 3680.0 / 513.0,
                     b54 = -845.0 / 4104.0;
    constexpr double b61 = -8.0 / 27.0, b62 = 2.0, b63 = -3544.0 / 2565.0,
                     b64 = 1859.0 / 4104.0, b65 = -11.0 / 40.0;
    double k1[6], k2[6], k3[6], k4[6], k5[6], k6[6], yt[6];
    rhs<SPIN0, FAR, HUGE>(y, k1, sc, far_ok, n, tr, true);
    if (!repair_at_refill<INTEGRATOR_RKF45, FAR, HUGE>()) {
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 6; i++) bad |= !isfinite(k1[i]);  // :318-333
        if (bad) return false;
    }
    const double hb21 = h * b21;
    constexpr bool Z = zero_accel<SPIN0, FAR>();  // components 3..5 stay y (zero_accel)
#pragma unroll
    for (int i = 0; i < 6; i++) yt[i] = (Z && i >= 3) ? y[i] : y[i] + hb21 * k1[i];
    rhs<SPIN0, FAR, HUGE>(yt, k2, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++)
        yt[i] = (Z && i >= 3) ? y[i] : y[i] + h * (b31 * k1[i] + b32 * k2[i]);
    rhs<SPIN0, FAR, HUGE>(yt, k3, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++)
        yt[i] = (Z && i >= 3) ? y[i] : y[i] + h * (b41 * k1[i] + b42 * k2[i] + b43 * k3[i]);
    rhs<SPIN0, FAR, HUGE>(yt, k4, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++)
        yt[i] = (Z && i >= 3) ? y[i]
                              : y[i] + h * (b51 * k1[i] + b52 * k2[i] + b53 * k3[i] + b54 * k4[i]);
    rhs<SPIN0, FAR, HUGE>(yt, k5, sc, far_ok, n, tr, false);
#pragma unroll
    for (int i = 0; i < 6; i++)
        yt[i] = (Z && i >= 3) ? y[i]
                              : y[i] + h * (b61 * k1[i] + b62 * k2[i] + b63 * k3[i] +
                                            b64 * k4[i] + b65 * k5[i]);
    rhs<SPIN0, FAR, HUGE>(yt, k6, sc, far_ok, n, tr, false);
    if constexpr (ACC) {  // never rejected (above): y <- y5, the same expression as below
#pragma unroll
        for (int i = 0; i < 3; i++) y[i] = y[i] + h * zs[3 + i];
        return true;
    }
    double y5[6];
    // :367-391 and :402-434 (rkf45_accept)
    constexpr bool FAST_NORM = repair_at_refill<INTEGRATOR_RKF45, FAR, HUGE>();
    double err[6], scale[6];
#pragma unroll
    for (int i = 0; i < 6; i++) {
        if (Z && i >= 3) {  // y4 = y5 = y: error 0
            y5[i] = y[i];
            scale[i] = fmax(fabs(y[i]), kEps);
            err[i] = 0.0;
            continue;
        }
        const double s4 = HS ? zs[i] : rkf45_sum4(k1[i], k3[i], k4[i], k5[i]);
        const double s5 = HS ? zs[3 + i] : rkf45_sum5(k1[i], k3[i], k4[i], k5[i], k6[i]);
        const double y4 = y[i] + h * s4;
        y5[i] = y[i] + h * s5;
        if (FAST_NORM) {
            // the state is finite and bounded here (repair_at_refill), so y and y5 are not NaN
            // and fmax / the kEps floor are plain maxima: two v_max_f64 instead of five VALU
            scale[i] = max_raw(max_abs_raw(y[i], y5[i]), kEps);
        } else {
            scale[i] = fmax(fabs(y[i]), fabs(y5[i]));
            if (scale[i] < kEps) scale[i] = kEps;
        }
        err[i] = fabs(y5[i] - y4);
    }
    // a zero error passes the fast form's per-component test for any positive normal tol, so
    // the fast form looks at the live components only; the literal form keeps all six (its
    // fmax chain would turn an earlier NaN into the 0 of a later component, as the
    // reference's does)
    const bool accept = rkf45_accept<FAST_NORM, (Z && FAST_NORM) ? 3 : 6>(err, scale, sc.tol);
    if (accept) {
#pragma unroll
        for (int i = 0; i < 6; i++) y[i] = y5[i];
        return true;
    }
    return false;
}

// spherical_to_cartesian (spacetime.c:229-237) from carried sin/cos
__device__ __forceinline__ void sph2cart_t(double r, double st, double ct, double sp, double cp,
                                           double& x, double& y, double& z) {
    x = r * st * cp;
    y = r * st * sp;
    z = r * ct;
}

// sin, cos of x from those of a, the same component one iteration earlier.
// Per ray only (never dependent on which wave runs the ray), so results stay reproducible.
__device__ __forceinline__ void trig_advance(double a, double x, double& s, double& c,
                                             Counters* hc) {
    double s1, c1;
    shift_or_eval(a, s, c, x, s1, c1, hc);
    s = s1;
    c = c1;
}

// sqrt as the compiler's f64 expansion computes it (v_rsq_f64, Goldschmidt refinement, two
// residual corrections) without its denormal scaling and Inf/0 class fix-up, which only
// x < 2^-767 needs -- those lanes take the library sqrt.
__device__ __forceinline__ double sqrt_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double s = x * y, hy = y * 0.5;
    const double r = __builtin_fma(-hy, s, 0.5);
    s = __builtin_fma(s, r, s);
    hy = __builtin_fma(hy, r, hy);
    double e = __builtin_fma(-s, s, x);
    s = __builtin_fma(e, hy, s);
    e = __builtin_fma(-s, s, x);
    s = __builtin_fma(e, hy, s);
    // one rare branch (not an if / else pair of exec-mask regions around both forms)
    if (__builtin_expect(!(x >= 0x1p-767), 0)) s = sqrt(x);
    return s;
}

__device__ __forceinline__ double len3(double x, double y, double z) {
    return sqrt((x * x + y * y) + z * z);  // vector3D_length (math_util.c:85-113)
}
// the per-iteration path length |p - p_prev| of the hot loop
__device__ __forceinline__ double seg_len(double x, double y, double z) {
    return sqrt_nr((x * x + y * y) + z * z);
}

struct Ray_ {
    double y[6];        // (t, r, theta, phi, tdot, rdot)
    double y6, y7;      // (thetadot, phidot): constants, see header
    double dx, dy, dz;  // Ray.direction as given (disk test)
    double px, py, pz;  // current Cartesian position; the disk hit point once T_DISK
    double dist;
    double s1, c1, s2, c2, s3, c3;  // sin, cos of y[1], y[2], y[3] (carried)
    double zs[6];       // per-ray stage sums of components 0..2 (hoist_sums)
    double cd_sd, cd_cm1;        // rotation_trig: sin(delta) and cos(delta) - 1 of the
                                 // increment at the step size h (set with it, hcache)
    double h, h_lo, h_hi;        // hcache: the step size and the r interval it holds on
    int k;              // iterations executed
    bool far_ok;        // use_analytic_approx && impact_parameter > 0
};

// hoist_sums: the stage sums of components 0..2 from the ray's constant state[3..5]
template <int METHOD>
__device__ __forceinline__ void zero_sums(Ray_& R) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const double v = R.y[3 + i];
        if (METHOD == INTEGRATOR_RK4) {
            double a = v;
            a = rk4_acc(a, v);
            a = rk4_acc(a, v);
            R.zs[i] = a + v;
        } else {
            R.zs[i] = rkf45_sum4(v, v, v, v);
            R.zs[3 + i] = rkf45_sum5(v, v, v, v, v);
        }
    }
}

__device__ __forceinline__ void trig_anchor(Ray_& R, Counters* hc = nullptr) {
    bhrt_sincos(R.y[1], &R.s1, &R.c1, hc);
    bhrt_sincos(R.y[2], &R.s2, &R.c2, hc);
    bhrt_sincos(R.y[3], &R.s3, &R.c3, hc);
}

// Trig-free part of integrate_photon_path's set-up (raytracer.c:355-466): the initial
// velocities, dt/dlambda from the null condition, E, L, b. s_* are products of the origin's
// sin/cos, g_* the metric at the origin.
__device__ __forceinline__ void init_velocity(Ray_& R, double nx, double ny, double nz,
                                              double r, double st_cp, double st_sp, double ct,
                                              double ct_cp, double ct_sp, double st,
                                              double neg_sp, double cp, double r_st,
                                              bool st_tiny, double g_tt, double g_rr,
                                              double g_hh, bool use_approx) {
    const double vr = st_cp * nx + st_sp * ny + ct * nz;            // :389-391
    const double vth = (ct_cp * nx + ct_sp * ny - st * nz) / r;     // :394-396
    double vph = (neg_sp * nx + cp * ny) / r_st;                    // :399
    if (st_tiny) vph = 0.0;                                         // :402-405
    double dt2 = -(g_rr * vr * vr + g_hh * vth * vth + g_hh * vph * vph) / g_tt;  // :416-418
    if (dt2 < 0.0) dt2 = 0.0;
    const double vt = sqrt(dt2);
    const double b = fabs((g_hh * vph) / (-g_tt * vt));  // |L / E| (:437-448)
    R.far_ok = use_approx && (b > 0.0);
    R.y[4] = vt;
    R.y[5] = vr;
    R.y6 = isfinite(vth) ? vth : 0.0;  // recovery of :543-548 for the constant components
    R.y7 = isfinite(vph) ? vph : 0.0;
}

__device__ __forceinline__ void normalize3(double x, double y, double z, double& nx, double& ny,
                                           double& nz) {
    const double l = len3(x, y, z);  // vector3D_normalize (math_util.c:115-122)
    if (l < kEps) {
        nx = ny = nz = 0.0;
    } else {
        const double inv = 1.0 / l;
        nx = x * inv;
        ny = y * inv;
        nz = z * inv;
    }
}

// Full per-ray set-up for an arbitrary origin (ray arrays, single-ray path kernel).
__device__ __forceinline__ void ray_init_general(Ray_& R, double t0, double ox, double oy,
                                                 double oz, double dx, double dy, double dz,
                                                 const Scene& sc) {
    R.dx = dx;
    R.dy = dy;
    R.dz = dz;
    double nx, ny, nz;
    normalize3(dx, dy, dz, nx, ny, nz);
    const double r = sqrt(ox * ox + oy * oy + oz * oz);  // cartesian_to_spherical
    const double th = (r > kEps) ? acos(oz / r) : 0.0;
    double ph = atan2(oy, ox);
    if (ph < 0.0) ph += kTwoPi;
    double st, ct, sp, cp;
    sincos(th, &st, &ct);
    sincos(ph, &sp, &cp);
    const double rm = (r <= sc.rs_eps) ? sc.rs_eps : r;  // calculate_schwarzschild_metric
    const double g_tt = -(1.0 - sc.rs / rm);
    const double g_rr = 1.0 / (1.0 - sc.rs / rm);
    const double g_hh = rm * rm;  // g_thth = g_phph (sin^2(pi/2) == 1)
    init_velocity(R, nx, ny, nz, r, st * cp, st * sp, ct, ct * cp, ct * sp, st, -sp, cp, r * st,
                  fabs(st) < kEps, g_tt, g_rr, g_hh, r > sc.rs_x15);
    R.y[0] = t0;
    R.y[1] = r;
    R.y[2] = th;
    R.y[3] = ph;
    R.px = r * st * cp;  // spherical_to_cartesian of the initial state (:498-501)
    R.py = r * st * sp;
    R.pz = r * ct;
    R.dist = 0.0;
    R.k = 0;
}

// floor(a / d) for 0 <= a < 2^31, d >= 1, from inv = RN(1 / d): RN(a * inv) is within 2^-52
// relative of a / d, so its truncation is the quotient or one below it (never above: a / d
// ends at least 1 / d short of the next integer, and d (q + 1) < 2^52), and one test fixes it
// -- a few VALU instead of the ~30 of a 32-bit integer division
__device__ __forceinline__ int div_floor(int a, int d, double inv) {
    int q = (int)((double)a * inv);
    if ((unsigned)(q + 1) * (unsigned)d <= (unsigned)a) q++;
    return q;
}

// calculate_ray_direction (raytracer.c:1013-1038) for pixel-centre ray i of the shard
__device__ __forceinline__ void camera_dir(const bhrt_camera_k& cm, int i, double& dx,
                                           double& dy, double& dz) {
    const int W = cm.width;
    const int j = div_floor(i, W, cm.inv_width), px = i - j * W;
    int py = j;
    if (cm.rows.num_shards > 1) {
        const int B = cm.rows.row_block;
        const int jb = div_floor(j, B, cm.inv_block);
        py = (jb * cm.rows.num_shards + cm.rows.shard) * B + (j - jb * B);
    }
    const double ndcx = (2.0 * ((px + cm.off_x) / W) - 1.0) * cm.plane_w;
    const double ndcy = (1.0 - 2.0 * ((py + cm.off_y) / cm.height)) * cm.plane_h;
    double vx = cm.fwd[0], vy = cm.fwd[1], vz = cm.fwd[2];
    vx = vx + cm.right[0] * ndcx;
    vy = vy + cm.right[1] * ndcx;
    vz = vz + cm.right[2] * ndcx;
    vx = vx + cm.up[0] * ndcy;
    vy = vy + cm.up[1] * ndcy;
    vz = vz + cm.up[2] * ndcy;
    normalize3(vx, vy, vz, dx, dy, dz);
}

// Camera ray set-up: the origin is shared, so only the direction-dependent part runs here.
__device__ __forceinline__ void ray_init_camera(Ray_& R, const bhrt_camera_k& cm, int i) {
    camera_dir(cm, i, R.dx, R.dy, R.dz);
    double nx, ny, nz;
    normalize3(R.dx, R.dy, R.dz, nx, ny, nz);  // integrate_photon_path normalises again
    init_velocity(R, nx, ny, nz, cm.r0, cm.st_cp, cm.st_sp, cm.ct, cm.ct_cp, cm.ct_sp, cm.st,
                  cm.neg_sp, cm.cp, cm.r_st, cm.st_tiny != 0, cm.g_tt, cm.g_rr, cm.g_hh,
                  cm.use_approx != 0);
    R.y[0] = 0.0;
    R.y[1] = cm.r0;
    R.y[2] = cm.th0;
    R.y[3] = cm.ph0;
    R.px = cm.p0[0];
    R.py = cm.p0[1];
    R.pz = cm.p0[2];
    R.dist = 0.0;
    R.k = 0;
}

// A ray of an array whose rays all start at the launch's shared origin (kp.rays_shared): the
// origin part of the set-up is the host's (cm, as for a camera frame); the direction is the
// array's, kept as given for the disk test (Ray.direction) and normalised for the velocities,
// as ray_init_general does.
__device__ __forceinline__ void ray_init_shared(Ray_& R, const bhrt_camera_k& cm,
                                                const double* dirs, int stride, int i) {
    const double* d = dirs + (size_t)i * stride;
    R.dx = d[0];
    R.dy = d[1];
    R.dz = d[2];
    double nx, ny, nz;
    normalize3(R.dx, R.dy, R.dz, nx, ny, nz);
    init_velocity(R, nx, ny, nz, cm.r0, cm.st_cp, cm.st_sp, cm.ct, cm.ct_cp, cm.ct_sp, cm.st,
                  cm.neg_sp, cm.cp, cm.r_st, cm.st_tiny != 0, cm.g_tt, cm.g_rr, cm.g_hh,
                  cm.use_approx != 0);
    R.y[0] = 0.0;
    R.y[1] = cm.r0;
    R.y[2] = cm.th0;
    R.y[3] = cm.ph0;
    R.px = cm.p0[0];
    R.py = cm.p0[1];
    R.pz = cm.p0[2];
    R.dist = 0.0;
    R.k = 0;
}

// check_disk_intersection (raytracer.c:159-196), plane "normal" = previous path point n,
// straight-line: every lane forms t, the candidate point and the radial test, and the four
// rejections are ONE mask (a per-test early return became nested exec-mask regions, ~50 SALU
// per iteration). The radial test compares s = qx^2 + qy^2 against the host's thresholds
// instead of taking sqrt(s) (bhrt_api.c sqrt_lower/upper_bound). t = num * RN(1/den) for
// |den| in [1e-10, 1e150) (a lane whose |den| < 1e-10 is rejected whatever its t); the IEEE
// quotient, in a rare branch, otherwise (NaN den included). A t < 0 by signs (|num| > 0) is
// negative here too, so the reference's rejection order is kept without a sign test.
__device__ __forceinline__ bool disk_hit(const Ray_& R, double nx, double ny, double nz,
                                         const Scene& sc, double big, double& qx, double& qy,
                                         double& qz) {
    const double den = (R.dx * nx + R.dy * ny) + R.dz * nz;
    const double num = -((R.px * nx + R.py * ny) + R.pz * nz);
    double t = div_nr(num, den, rcp_nr(den));
    if (__builtin_expect(!(fabs(den) < big), 0)) t = num / den;  // big = 1e150
    qx = R.px + R.dx * t;
    qy = R.py + R.dy * t;
    qz = R.pz + R.dz * t;
    const double s = qx * qx + qy * qy;
    return !(fabs(den) < kEps) & !(t < 0.0) & (s >= sc.disk_in_sq) & (s <= sc.disk_out_sq);
}

enum Term : int { T_NONE = 0, T_HORIZON, T_DISK, T_MAXDIST, T_MAXSTEPS };

struct HSel {  // the four step sizes of the schedule, hoisted out of the kernel argument block
    double far_, r15, r5, r2_5;
    double big;  // 1e150, the disk test's quotient bound: an SGPR pair set once, outside the
                 // loop (as a literal it was rematerialised by two s_mov in every iteration)
};

// x unchanged, but opaque to the optimiser: the four step sizes stay four register values
// selected by v_cndmask. Left visible as loads, the select chain over them became ONE load at a
// selected address, and the promoted step-size array an LDS table: a ds_read_b64 and an
// lgkmcnt wait at the head of every iteration's dependency chain.
template <bool V>
__device__ __forceinline__ double opaque(double x) {
    if (V)
        asm volatile("" : "+v"(x));
    else
        asm volatile("" : "+s"(x));
    return x;
}
// V: the step sizes in VGPRs (8 more registers; each select is then one v_cndmask per half
// instead of a v_mov from the SGPR and a v_cndmask): where the loop has registers to spare
template <bool V = false>
__device__ __forceinline__ HSel hsel_of(const Scene& sc) {
    return HSel{opaque<V>(sc.h_far), opaque<V>(sc.h_15), opaque<V>(sc.h_5), opaque<V>(sc.h_2_5),
                opaque<false>(1.0e150)};
}

// :543-548, state NaN/Inf recovery at the top of an iteration. One test of the sum
// (non-finite if any component is, or on overflow); the per-component repair runs only then.
// ANCHOR = false: the caller knows state[1..3] are finite, so their sin/cos stay valid.
template <bool ANCHOR = true>
__device__ __forceinline__ void state_repair(Ray_& R, Counters* hc) {
    if (__builtin_expect(
            !isfinite(((R.y[0] + R.y[1]) + (R.y[2] + R.y[3])) + (R.y[4] + R.y[5])), 0)) {
#pragma unroll
        for (int i = 0; i < 6; i++)
            if (!isfinite(R.y[i])) R.y[i] = (i < 4) ? 1.0 : 0.0;
        if (ANCHOR) trig_anchor(R, hc);
    }
}

// every component of the state within +-bound (NaN fails)
__device__ __forceinline__ bool state_within(const Ray_& R, double bound) {
    const double m = fmax(fmax(fmax(fabs(R.y[0]), fabs(R.y[1])), fmax(fabs(R.y[2]), fabs(R.y[3]))),
                          fmax(fabs(R.y[4]), fabs(R.y[5])));
    return m <= bound;
}

// Where the step size is kept per ray with its r interval (ray_iterate): every RK4 path. C4's
// ~80-VALU iteration spent 9 on the select chain: -3.6% kernel time same-box, bit-identical
// (round 3). C2 measured neutral then; with round 6's wave-uniform trip it is +1.1% same-box,
// bit-identical on C1 and C2 full frames (profiles/r06/ab_unroll.txt). RKF45 keeps the chain
// (C3 -1.4%, C5 neutral in round 3); k_path and the HUGE redo always select.
// The zero-acceleration paths (rotation_trig: C4, C5) keep it too, and form the rotation of
// state[2]'s sin, cos for the new step size in the same rare branch: a regime change is then
// one test per iteration instead of two.
template <int METHOD, bool SPIN0, bool FAR, bool HUGE>
constexpr bool hcache() {
    return (METHOD == INTEGRATOR_RK4 && !HUGE) ||
           rotation_trig<METHOD, SPIN0, FAR, HUGE>();
}

// One pass of integrate_photon_path's loop body (raytracer.c:517-665) plus, with DISK, the
// on-the-fly form of trace_ray's segment scan. Returns the termination, or T_NONE.
// hs: the step sizes in registers (k_trace), or NULL to read them from the scene.
template <int METHOD, bool DISK, bool SPIN0, bool FAR, bool HUGE, bool ACC = false>
__device__ __forceinline__ int ray_iterate(Ray_& R, const Scene& sc, Counters& n,
                                           const HSel hs) {
    Counters* const hc = HUGE ? nullptr : &n;
    // Instantiations with repair_at_refill() run the recovery once, when the ray is loaded:
    // there a finite state stays finite.
    if (!repair_at_refill<METHOD, FAR, HUGE>()) state_repair(R, hc);
    // step schedule (:556-571), written as selects so the first true test wins; fmin(h, 0.1)
    // is folded into the values (host)
    const double r = R.y[1];
    double h;
    if constexpr (hcache<METHOD, SPIN0, FAR, HUGE>()) {
        // the size is cached per ray with the r interval it holds on (Scene h_lo / h_hi): a ray
        // changes regime at most three times, so each iteration is two compares instead of the
        // three compares and three 64-bit selects of the chain (NaN r: always re-selected,
        // giving the chain's h_far)
        if (__builtin_expect(!(r >= R.h_lo && r < R.h_hi), 0)) {
            int k = 0;
            k = (r < sc.rs_x15) ? 1 : k;
            k = (r < sc.rs_x5) ? 2 : k;
            k = (r < sc.rs_x2_5) ? 3 : k;
            R.h = k == 0 ? hs.far_ : (k == 1 ? hs.r15 : (k == 2 ? hs.r5 : hs.r2_5));
            // (indexed by the per-lane k these are vector loads from the kernel-argument segment,
            // in this rare branch only; selects of the eight bounds as register values instead
            // measured C4 +-0, C5 -1.5% same-box -- more SGPR spills around the loop --
            // profiles/r05/ab_session_l.txt)
            R.h_lo = sc.h_lo[k];
            R.h_hi = sc.h_hi[k];
            if constexpr (rotation_trig<METHOD, SPIN0, FAR, HUGE>()) {
                // the nominal increment of state[2] at this step size: h/6 * ((v + 2v) + 2v) + v
                // (rk4_step) or h * sum5 (rkf45_attempt), v = state[5] (constant here). |d| <
                // pi/4 for every ray k_trace keeps in these instantiations (|v| <
                // Scene.rot_vmax, checked at refill; any other ray is re-traced by the HUGE
                // pass, which advances its trig directly).
                double d;
                if (METHOD == INTEGRATOR_RK4) {
                    double a = R.y[5];
                    a = rk4_acc(a, R.y[5]);
                    a = rk4_acc(a, R.y[5]);
                    d = (R.h * (1.0 / 6.0)) * (a + R.y[5]);
                } else {
                    d = R.h * R.zs[5];
                }
                rotation_coeffs(d, R.cd_sd, R.cd_cm1);
            }
        }
        h = R.h;
        // h formed at the branch's join: left visible, the compiler sank the step's first uses
        // of h into both arms, and the rare re-select became an if/else diamond (s_xor +
        // s_andn2_saveexec per iteration). C4 SALU 145 -> 137 M per launch, C5 +2%,
        // bit-identical (profiles/r04/session_ad)
        asm volatile("" : "+v"(h));
    } else {
        h = hs.far_;
        h = (r < sc.rs_x15) ? hs.r15 : h;
        h = (r < sc.rs_x5) ? hs.r5 : h;
        h = (r < sc.rs_x2_5) ? hs.r2_5 : h;
    }
    bool moved = true;
    if (METHOD != INTEGRATOR_RK4) n.iters++;  // RK4: counted at termination (k_trace)
    Trig1 tr{R.y[1], R.s1, R.c1};
    const double a2 = R.y[2], a3 = R.y[3];
    constexpr bool HS = hoist_sums<METHOD, SPIN0, FAR, HUGE>();
    if (METHOD == INTEGRATOR_RK4) {
        rk4_step<SPIN0, FAR, HUGE, HS>(R.y, h, sc, R.far_ok, n, tr, R.zs);
    } else if (METHOD == INTEGRATOR_RKF45) {
        moved = rkf45_attempt<SPIN0, FAR, HUGE, HS, ACC>(R.y, h, sc, R.far_ok, n, tr, R.zs);
    } else {
        moved = false;  // LEAPFROG / YOSHIDA: "not implemented", state unchanged (:616-624)
    }
    double x, y, z;
    if (moved) {
        // sin, cos of state[1] feed only the a = 0 accelerations (rhs); the Kerr branch
        // (a != 0, accelerations 0) never reads them, and the compiler keeps a dead
        // loop-carried advance alive otherwise (C5: 45 instructions of the loop)
        if (SPIN0) trig_advance(tr.a, R.y[1], R.s1, R.c1, hc);
        if constexpr (rotation_trig<METHOD, SPIN0, FAR, HUGE>()) {
            // (the rotation for this step size was formed with it, above)
            const double s0 = R.s2, c0 = R.c2;
            R.s2 = __builtin_fma(c0, R.cd_sd, __builtin_fma(s0, R.cd_cm1, s0));
            R.c2 = __builtin_fma(-s0, R.cd_sd, __builtin_fma(c0, R.cd_cm1, c0));
        } else {
            trig_advance(a2, R.y[2], R.s2, R.c2, hc);
        }
        // on the zero-acceleration Kerr paths state[3] never changes (zero_accel): its sin,
        // cos stay as they are
        if (!zero_accel<SPIN0, FAR>()) trig_advance(a3, R.y[3], R.s3, R.c3, hc);
    }
    sph2cart_t(R.y[1], R.s2, R.c2, R.s3, R.c3, x, y, z);
    const double ox = R.px, oy = R.py, oz = R.pz;
    R.dist += seg_len(x - ox, y - oy, z - oz);
    R.px = x;
    R.py = y;
    R.pz = z;
    R.k++;
    if constexpr (!DISK) {
        // exits in the reference's order as early returns (without a disk test they are a
        // short chain of rare branches; the select form below measured -0.9% on C5,
        // profiles/r03_ab_kernel.txt)
        if (R.y[1] <= sc.rs_x1_05) return T_HORIZON;
        if (R.dist >= sc.max_dist) return T_MAXDIST;
        if (!moved) {  // fixed point (below)
            R.k = sc.max_steps;
            return T_MAXSTEPS;
        }
        return R.k >= sc.max_steps ? T_MAXSTEPS : T_NONE;
    } else {
        // the exits as selects (the reference's order: disk, horizon, distance, fixed point,
        // step budget; a disk hit overrides the others below)
        // (as three selects, lowest priority first: the nested form compiled to exec-mask
        // branches)
        int term = (R.k >= sc.max_steps) ? T_MAXSTEPS : T_NONE;
        term = (R.dist >= sc.max_dist) ? T_MAXDIST : term;
        term = (R.y[1] <= sc.rs_x1_05) ? T_HORIZON : term;
        // segment k = (p_k, p_{k-1}) is stored and scanned by trace_ray iff k < max_steps
        double qx, qy, qz;
        if (disk_hit(R, ox, oy, oz, sc, hs.big, qx, qy, qz) & (R.k < sc.max_steps)) {
            // the ray ends here: the hit point replaces the current point, so no extra
            // loop-carried registers hold it (store_hit reads it from R.px..pz; +0.9% on C2)
            R.px = qx;
            R.py = qy;
            R.pz = qz;
            R.dist += seg_len(qx - ox, qy - oy, qz - oz);  // (= len3: sqrt_nr is sqrt here)
            term = T_DISK;
        }
        if (!moved && term == T_NONE) {
            // Fixed point: every later iteration repeats this one with p_j = p_{j-1} = p_k.
            // Only the duplicate segment (p_k, p_k) is new, and only if p_k != p_{k-1}.
            if (R.k + 1 < sc.max_steps && (x != ox || y != oy || z != oz) &&
                disk_hit(R, x, y, z, sc, hs.big, qx, qy, qz)) {
                R.px = qx;
                R.py = qy;
                R.pz = qz;
                R.k++;
                R.dist += len3(qx - x, qy - y, qz - z);
                return T_DISK;
            }
            R.k = sc.max_steps;
            return T_MAXSTEPS;
        }
        return term;
    }
}

// fill_hit_info (raytracer.c:299-333) / the disk branch of trace_ray (:728-753)
__device__ __forceinline__ void store_hit(const bhrt_frame_soa& s, int i, const Ray_& R,
                                          int term, const Scene& sc) {
    int result, steps;
    double hx, hy, hz, tdil, sx = 0.0, sy = 0.0, sz = 0.0;
    if (term == T_DISK) {
        result = RAY_DISK;
        steps = R.k;
        hx = R.px;
        hy = R.py;
        hz = R.pz;
        tdil = 1.0 / sqrt(1.0 - sc.rs / len3(R.px, R.py, R.pz));
    } else {
        result = term == T_HORIZON ? RAY_HORIZON
                                   : (term == T_MAXDIST ? RAY_MAX_DISTANCE : RAY_MAX_STEPS);
        steps = term == T_MAXSTEPS ? R.k : R.k - 1;
        hx = R.px;
        hy = R.py;
        hz = R.pz;
        tdil = 1.0 / sqrt(1.0 - sc.rs / R.y[1]);
        if (term == T_MAXDIST) normalize3(R.y[5], R.y6, R.y7, sx, sy, sz);  // state[5..7]
    }
    if (s.result) s.result[i] = result;
    if (s.steps) s.steps[i] = steps;
    if (s.hit_x) s.hit_x[i] = hx;
    if (s.hit_y) s.hit_y[i] = hy;
    if (s.hit_z) s.hit_z[i] = hz;
    if (s.distance) s.distance[i] = R.dist;
    if (s.time_dilation) s.time_dilation[i] = tdil;
    if (s.sky_x) s.sky_x[i] = sx;
    if (s.sky_y) s.sky_y[i] = sy;
    if (s.sky_z) s.sky_z[i] = sz;
}

// A ray's initial state from the k_init table. A camera frame's table holds only what differs
// between its rays (BHRT_INIT_FIELDS_CAMERA rows: 64 B per ray instead of 168); the shared
// origin -- state[0..3], its Cartesian point and the sin/cos of its angles -- comes from the
// launch's camera block (wave-uniform).
__device__ __forceinline__ void load_init(const bhrt_kparams& kp, int i, Ray_& R) {
    const double* f = kp.init;
    const long n = kp.n;
    if (kp.src == BHRT_SRC_CAMERA) {
        const bhrt_camera_k& cm = kp.cam;
        R.y[0] = 0.0;
        R.y[1] = cm.r0;
        R.y[2] = cm.th0;
        R.y[3] = cm.ph0;
        R.y[4] = f[i];
        R.y[5] = f[n + i];
        R.y6 = f[2 * n + i];
        R.y7 = f[3 * n + i];
        R.dx = f[4 * n + i];
        R.dy = f[5 * n + i];
        R.dz = f[6 * n + i];
        R.far_ok = f[7 * n + i] != 0.0;
        R.px = cm.p0[0];
        R.py = cm.p0[1];
        R.pz = cm.p0[2];
        R.s1 = cm.s_r0;
        R.c1 = cm.c_r0;
        R.s2 = cm.st;
        R.c2 = cm.ct;
        R.s3 = cm.sp;
        R.c3 = cm.cp;
        R.dist = 0.0;
        R.k = 0;
        return;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) R.y[j] = f[j * n + i];
    R.y6 = f[6 * n + i];
    R.y7 = f[7 * n + i];
    R.dx = f[8 * n + i];
    R.dy = f[9 * n + i];
    R.dz = f[10 * n + i];
    R.px = f[11 * n + i];
    R.py = f[12 * n + i];
    R.pz = f[13 * n + i];
    R.far_ok = f[14 * n + i] != 0.0;
    R.s1 = f[15 * n + i];
    R.c1 = f[16 * n + i];
    R.s2 = f[17 * n + i];
    R.c2 = f[18 * n + i];
    R.s3 = f[19 * n + i];
    R.c3 = f[20 * n + i];
    R.dist = 0.0;
    R.k = 0;
}

__device__ __forceinline__ double clampd(double v, double lo, double hi) {
    if (v < lo) return lo;  // math_util.c:505-509 (NaN passes through)
    if (v > hi) return hi;
    return v;
}

// Frame colour contract, one elementwise pass after the trace:
// calculate_disk_temperature + temperature_to_rgb (+ apply_relativistic_effects) for disk
// hits, black for the horizon, the sky gradient of raytracer.c:1150-1157 otherwise.
// (unsigned char)(std::min(1.0f, v) * 255.0f) as the visualizer's x86 build evaluates it:
// std::min keeps 1.0f for NaN, the cast truncates toward zero and keeps the low byte.
__device__ __forceinline__ unsigned to_u8(float v) {
    const float m = (v < 1.0f) ? v : 1.0f;
    return (unsigned)(int)(m * 255.0f) & 0xffu;
}


// Black for the horizon, the sky gradient of raytracer.c:1150-1157 on the ray direction's y
// otherwise (every ray of a scene without a disk)
__device__ __forceinline__ void colour_sky(int res, double dy, double& r, double& g, double& b) {
#pragma clang fp contract(off)
    if (res == RAY_HORIZON) {
        r = g = b = 0.0;
    } else {
        const double t = 0.5 * (dy + 1.0);
        r = (1.0 - t) * 1.0 + t * 0.5;
        g = (1.0 - t) * 1.0 + t * 0.7;
        b = (1.0 - t) * 1.0 + t * 1.0;
    }
}

// The frame colour contract of one ray: calculate_disk_temperature +
// temperature_to_rgb (+ apply_relativistic_effects with BHRT_FLAG_DOPPLER) of a disk hit at
// (hx, hy), black for the horizon, the sky gradient of raytracer.c:1150-1157 on the ray
// direction's y otherwise. Written by the trace kernel at the ray's exit (colour_fused) or by
// the separate k_colour pass.
__device__ __forceinline__ void colour_of(const Scene& sc, int res, double hx, double hy,
                                          double dx, double dy, double dz, double& r,
                                          double& g, double& b) {
    // no FP contraction here: the colour is then the same IEEE operation sequence wherever it
    // is inlined (the trace kernel's exit or the separate k_colour pass), so both colour paths
    // give the same bits (test_display_path_rgba), as the reference's own non-FMA build does
#pragma clang fp contract(off)
    if (res == RAY_DISK) {
        const double rxy = sqrt(hx * hx + hy * hy);  // raytracer.c:201-228
        double nr = (rxy - sc.disk_in) / (sc.disk_out - sc.disk_in);
        nr = clampd(nr, 0.0, 1.0);
        // pow(1 - nr, 0.75) as sqrt(u) * sqrt(sqrt(u)), u in [0, 1] (a few ulp: the colour
        // contract's tolerance is 1e-5)
        const double su = sqrt(1.0 - nr);
        const double T = clampd(sc.disk_tscale * (2000.0 + 18000.0 * (su * sqrt(su))),
                                1000.0, 40000.0);  // math_util.c:463-503
        const double t = (T - 1000.0) / (40000.0 - 1000.0);
        r = (t < 0.5) ? t * 2.0 : 1.0;
        g = (t < 0.25) ? 0.0 : ((t < 0.75) ? (t - 0.25) * 2.0 : 1.0);
        b = (t < 0.5) ? 0.0 : (t - 0.5) * 2.0;
        const double br = 0.2 + 0.8 * (t * t);
        r *= br;
        g *= br;
        b *= br;
        if (sc.flags & BHRT_FLAG_DOPPLER) {  // raytracer.c:233-294
            // sin, cos of atan2(hy, hx) as hy / rxy, hx / rxy (rxy > 0: a disk hit lies at
            // rxy >= disk_in), pow(dop, 4) as two squarings, dop / (1 / sqrt(f)) as
            // dop * sqrt(f): each within a few ulp of the libm forms
            // (rxy = 0 -- a zero inner radius -- is atan2(+-0, +0) = +-0 or atan2(+-0, -0) =
            // +-pi, whose sin, cos are (+-0, 1) and (+-RN(sin pi), -1): selects, no libm call
            // in the trace kernel)
            const double ir = 1.0 / rxy;
            double sp = hy * ir, cp = hx * ir;
            if (!(rxy > 0.0)) {
                const bool neg_x = __builtin_signbit(hx);
                sp = neg_x ? __builtin_copysign(1.2246467991473532e-16, hy) : hy;
                cp = neg_x ? -1.0 : 1.0;
            }
            const double dop = 1.0 + ((dx * -sp + dy * cp) + dz * 0.0) * 0.5;
            const double z = dop * sqrt(1.0 - sc.rs / rxy);
            if (z < 1.0) {
                b *= z;
                r = fmin(1.0, r * (2.0 - z));
            } else {
                r *= 2.0 - z;
                b = fmin(1.0, b * z);
            }
            const double d2 = dop * dop, beam = d2 * d2;
            r = clampd(r * beam, 0.0, 1.0);
            g = clampd(g * beam, 0.0, 1.0);
            b = clampd(b * beam, 0.0, 1.0);
        }
    } else {
        colour_sky(res, dy, r, g, b);
    }
}

__device__ __forceinline__ void store_colour(const bhrt_frame_soa& s, int i, double r, double g,
                                             double b) {
    if (s.rgb_r) {
        s.rgb_r[i] = r;
        s.rgb_g[i] = g;
        s.rgb_b[i] = b;
    }
    if (s.rgba32f || s.rgba8) {  // the display path (renderer.cpp:2090-2125)
        const float fr = (float)r, fg = (float)g, fb = (float)b;
        if (s.rgba32f) reinterpret_cast<float4*>(s.rgba32f)[i] = make_float4(fr, fg, fb, 1.0f);
        if (s.rgba8)
            reinterpret_cast<unsigned*>(s.rgba8)[i] =
                to_u8(fr) | (to_u8(fg) << 8) | (to_u8(fb) << 16) | (to_u8(1.0f) << 24);
    }
}

// store_hit, and where the scene's colour is written in the trace kernel
// (BHRT_COLOUR_IN_TRACE, bhrt_kernel.h; colour_fused) the colour outputs from the exit state in
// registers. Other instantiations do not contain the colour code at all (its registers cost
// more in the loop than the separate pass does).
// The launch parameters as an opaque pointer into the kernel argument segment: the fields read
// through it are loaded (scalar loads) where they are used, instead of being kept live across
// the persistent loop. The refill's camera constants and the store's output pointers held that
// way overflowed the 106 SGPRs into VGPR lanes (v_readlane in every block of the loop).
#ifndef BHRT_COLD_KP
#define BHRT_COLD_KP 1
#endif
#ifndef BHRT_UNIFORM_TRIP  /* 1: every instantiation; 0: none; default: RK4 a = 0 (uniform_trip) */
#define BHRT_UNIFORM_TRIP 2
#endif
#ifndef BHRT_DEFER_STORE
#define BHRT_DEFER_STORE 1
#endif
#ifndef BHRT_FRAME_STAMPS  /* the launch's execution window in ctl[8..10] (bhrt_stats.frame_ms) */
#define BHRT_FRAME_STAMPS 1
#endif
typedef const __attribute__((address_space(4))) bhrt_kparams kparams_as4;
// (k_trace's only argument: it starts the kernel argument segment)
__device__ __forceinline__ const bhrt_kparams& cold(const bhrt_kparams&) {
    kparams_as4* p = (kparams_as4*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const bhrt_kparams*)p;
}

template <int METHOD, bool DISK, bool SPIN0>
__device__ __forceinline__ void store_ray(const bhrt_kparams& kp, int i, const Ray_& R, int term) {
    store_hit(kp.out, i, R, term, kp.sc);
    if (!BHRT_COLOUR_IN_TRACE(METHOD, DISK, !SPIN0)) return;
    if (kp.colour_fused && (kp.out.rgb_r || kp.out.rgba32f || kp.out.rgba8)) {
        const int res = term == T_DISK ? RAY_DISK : (term == T_HORIZON ? RAY_HORIZON : RAY_MAX_STEPS);
        double r, g, b;
        if constexpr (DISK)
            colour_of(kp.sc, res, R.px, R.py, R.dx, R.dy, R.dz, r, g, b);
        else  // (no disk: no disk colour code in the kernel)
            colour_sky(res, R.dy, r, g, b);
        store_colour(kp.out, i, r, g, b);
    }
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned v) {
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    return s;
}

// Queue position -> ray id of a camera launch: the caller's permutation (bhrt_set_claim_order),
// else the shard's pixels tile by tile -- 64-pixel tiles (8x8, 16x4 or 32x2, whichever divides
// the shard; bhrt_api.c claim_tiles), so a wavefront's rays are a compact patch of the image with
// alike lifetimes (its lanes drain together, and a frame's last rays are short tiles, not long
// row segments: claim-order probe, profiles/r03_claim_order_tiles.txt) -- else id order. Which
// lane traces a ray never changes its arithmetic, so the frame is bit-identical in every order.
__device__ __forceinline__ int claim_ray(const bhrt_kparams& kp, int qpos) {
    if (kp.order) return kp.order[qpos];
    const bhrt_camera_k& cm = kp.cam;
    if (cm.tiles_per_row == 0) return qpos;
    int t = qpos >> 6;
    const int w = qpos & 63;
    if (cm.tile_stride > 0)
        t = (int)(((unsigned long long)(unsigned)t * (unsigned)cm.tile_stride) % (unsigned)cm.ntiles);
    const int trow = div_floor(t, cm.tiles_per_row, cm.inv_tiles_per_row);
    const int tcol = t - trow * cm.tiles_per_row;
    const int prow = (trow << cm.tile_h_log2) + (w >> cm.tile_w_log2);
    const int pcol = (tcol << cm.tile_w_log2) + (w & ((1 << cm.tile_w_log2) - 1));
    return prow * cm.width + pcol;
}

// Per-ray set-up pass (integrate_photon_path's prologue, raytracer.c:355-507) into the state
// table the trace kernel refills from ([BHRT_INIT_FIELDS][n] for ray arrays; for a camera frame
// only the BHRT_INIT_FIELDS_CAMERA rows that differ between rays, 64 B per ray). Kept out of the
// persistent loop so that neither the camera uniforms nor acos/atan2 occupy registers there.
template <int SRC>
__global__ __launch_bounds__(256) void k_init(const bhrt_kparams kp) {
    double* f = kp.init;
    const long n = kp.n;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kp.n; i += gridDim.x * blockDim.x) {
        Ray_ R;
        if constexpr (SRC == BHRT_SRC_CAMERA) {  // the per-ray part only (load_init)
            // row i of the table is the i-th ray of the claim order
            ray_init_camera(R, kp.cam, claim_ray(kp, i));
            f[i] = R.y[4];
            f[n + i] = R.y[5];
            f[2 * n + i] = R.y6;
            f[3 * n + i] = R.y7;
            f[4 * n + i] = R.dx;
            f[5 * n + i] = R.dy;
            f[6 * n + i] = R.dz;
            f[7 * n + i] = R.far_ok ? 1.0 : 0.0;
        } else {
            Ray ray;
            if (kp.rays_shared) {  // the origin block's point, the packed or AoS direction
                const double* d = kp.dirs + (size_t)i * kp.dir_stride;
                ray.origin = Vector3D{kp.cam.pos[0], kp.cam.pos[1], kp.cam.pos[2]};
                ray.direction = Vector3D{d[0], d[1], d[2]};
            } else {
                ray = kp.rays[i];
            }
            ray_init_general(R, 0.0, ray.origin.x, ray.origin.y, ray.origin.z, ray.direction.x,
                             ray.direction.y, ray.direction.z, kp.sc);
#pragma unroll
            for (int j = 0; j < 6; j++) f[j * n + i] = R.y[j];
            f[6 * n + i] = R.y6;
            f[7 * n + i] = R.y7;
            f[8 * n + i] = R.dx;
            f[9 * n + i] = R.dy;
            f[10 * n + i] = R.dz;
            f[11 * n + i] = R.px;
            f[12 * n + i] = R.py;
            f[13 * n + i] = R.pz;
            f[14 * n + i] = R.far_ok ? 1.0 : 0.0;
            trig_anchor(R);
            f[15 * n + i] = R.s1;
            f[16 * n + i] = R.c1;
            f[17 * n + i] = R.s2;
            f[18 * n + i] = R.c2;
            f[19 * n + i] = R.s3;
            f[20 * n + i] = R.c3;
        }
    }
}

// Per-instantiation occupancy target (waves per SIMD; 0 = the compiler's choice), same-box
// A/B in profiles/r01_ab_v11_occupancy.txt:
//  * RK4, a = 0 (C1, C2): 4. The straight-line iteration needs <= 123 VGPRs; the register
//    peak (160) sits in the rare-lane blocks (literal accelerations, wide trig shifts,
//    stores). Capped at 128 the allocator spills only inside those blocks -- the hot blocks
//    are instruction-for-instruction the 3-wave code -- so C2 gains the 4th wave (+4.6%).
//  * RKF45, a != 0, no disk (C5): 4. Since v23's two attempts per loop trip, 5 waves spill
//    (96 VGPRs + 156 B scratch) and 4 waves is best: +8.5% over 5, 6 loses 27%
//    (profiles/r02_ab_v23_occupancy.txt).
//  * C3 (RKF45 a = 0 disk): 3 (round 5: 168 VGPRs without spills), with launches of two waves
//    per SIMD (trace_launch_waves). C4 (RK4 Kerr disk) keeps the compiler's choice: 5 waves
//    spill (96 VGPRs + 84 B scratch) and gain nothing even with a capped grid.
// step sizes in VGPRs (hsel_of): the RK4 disk instantiations. C4 (Kerr, ~100 VGPRs) has the
// room; C2 (a = 0, capped at 128) gives its rare-lane blocks a few more spills but its iteration
// loses 7 v_mov_b32 (an SGPR operand of v_cndmask next to VCC exceeds gfx9's one constant-bus
// read, so each select first copied its SGPR half into a VGPR): +1.4% / +2.5% on two boxes,
// bit-identical (profiles/r03_ab/ab_v30a.txt, ab_v30b.txt)
template <int METHOD, bool DISK, bool SPIN0>
constexpr bool hsel_vgpr() {
    return METHOD == INTEGRATOR_RK4 && DISK;
}

template <int METHOD, bool DISK, bool SPIN0>
constexpr int trace_waves() {
    return (METHOD == INTEGRATOR_RKF45 && !DISK && !SPIN0) ? 4
         : (METHOD == INTEGRATOR_RK4 && SPIN0) ? 4
         : 0;
}
// the C3 camera kernel (RKF45, a = 0, disk, in-kernel set-up, near field) at 3 waves per SIMD;
// its other instantiations (ray arrays, far field, the redo pass) keep the compiler's choice
template <int METHOD, bool DISK, bool SPIN0, bool FAR, bool HUGE, int INL>
constexpr bool c3_camera() {
    return METHOD == INTEGRATOR_RKF45 && DISK && SPIN0 && !FAR && !HUGE && INL == 1;
}
// the accept-all attempts (ACC, C5): BHRT_ACC_WAVES per SIMD
#ifndef BHRT_ACC_WAVES
#define BHRT_ACC_WAVES 4
#endif
template <int METHOD, bool DISK, bool SPIN0, bool FAR, bool HUGE, int INL, bool ACC = false>
constexpr int trace_waves_k() {
    return ACC ? BHRT_ACC_WAVES
         : c3_camera<METHOD, DISK, SPIN0, FAR, HUGE, INL>() ? 3 : trace_waves<METHOD, DISK, SPIN0>();
}
// Waves per SIMD ONE hot launch takes (0: every resident slot). C3 is resident at 3 waves per
// SIMD (168 VGPRs, no spills) but launches 2 per SIMD's worth: the frames in flight fill the third
// slot. A full 3-wave grid deals each wave ~10 blocks in its first (static) claim and loses 10%
// against the 2-wave kernel; the 2-of-3 grid keeps ~16 blocks per wave and gains 11.6% (C3 13.1
// -> 14.6 Grays/s same-box; 448 / 576 blocks +8% / -6%, profiles/r05/ab_occupancy_grid.txt).
// The accept-all kernel (C5) launches 3 of its 4 resident waves per SIMD: +0.5...2.5% same-box
// over three sessions at 16 attempts per trip (2, 2.5 and 3.5 waves per SIMD alike, C4 -2% at 3;
// profiles/r06/ab_kernel_knobs.txt).
#ifndef BHRT_ACC_LAUNCH_WAVES
#define BHRT_ACC_LAUNCH_WAVES 3
#endif
template <int METHOD, bool DISK, bool SPIN0, bool FAR, int INL, bool ACC = false>
constexpr int trace_launch_waves() {
    return c3_camera<METHOD, DISK, SPIN0, FAR, false, INL>() ? 2 : ACC ? BHRT_ACC_LAUNCH_WAVES : 0;}
constexpr int BHRT_TRACE_WAVES_PER_BLOCK = 4;

// Ray queues of k_trace: 64-id block b of the launch belongs to queue b mod 2^qbits; queue q's
// j-th id and its length.
__device__ __forceinline__ unsigned queue_ray(unsigned qbits, unsigned q, unsigned j) {
    return ((j >> 6) << (6u + qbits)) | (q << 6) | (j & 63u);
}
__device__ __forceinline__ unsigned queue_size(unsigned ntotal, unsigned qbits, unsigned q) {
    const unsigned nb = ntotal >> 6, last = nb & ((1u << qbits) - 1u);
    return (((nb >> qbits) + (q < last ? 1u : 0u)) << 6) + (q == last ? (ntotal & 63u) : 0u);
}  // k_trace launches 256-lane workgroups
#define BHRT_TRACE_BOUNDS __attribute__((amdgpu_flat_work_group_size(1, 256), \
                                         amdgpu_waves_per_eu(trace_waves_k<METHOD, DISK, SPIN0, FAR, HUGE, INL, ACC>() > 0 ? trace_waves_k<METHOD, DISK, SPIN0, FAR, HUGE, INL, ACC>() : 1)))

// Diagnostic build only (make DEFS=-DBHRT_WAVE_STAMPS=1, tools/wave_stamps.py): every wave of a
// hot k_trace launch records, under the launch's control-block slot, its start and end on the
// constant 100 MHz clock, its CU, and its trips, refills, lane-iterations and rays. The shipped
// build has none of it.
#ifndef BHRT_WAVE_STAMPS
#define BHRT_WAVE_STAMPS 0
#endif
#if BHRT_WAVE_STAMPS
constexpr int kStampSlots = 64, kStampWaves = 8192, kStampWords = 8;
__device__ unsigned long long g_stamps[kStampSlots * kStampWaves * kStampWords];
#endif

// Loop iterations per trip of the persistent loop (the HUGE redo pass keeps one): RKF45 with the
// accept test 2, from same-box sweeps of 1..8 (round 2); RK4 a = 0 4 under a wave-uniform guard
// (uniform_trip; predicated, 10 measured C2 +0.3…0.5%, C1 +0.5…1% against round 2's 6 and 12 / 16
// no better, profiles/r06/ab_unroll.txt). The zero-acceleration
// paths' short iterations -- C4's RK4 step (~80 VALU) and C5's untested attempt (ACC, ~55) --
// pay the trip's own cost (the live ballot, the refill test and its scalar loads) for fewer
// instructions each: 16 per trip, C4 +2.2%, C5 +14.5% same-box against 6 / 2; the sweeps
// flatten from 12 (C5) / 16 (C4) up to 24 / 32 (profiles/r06/ab_unroll.txt).
#ifndef BHRT_UNROLL_ZA
#define BHRT_UNROLL_ZA 16
#endif
#ifndef BHRT_UNROLL_A0
#define BHRT_UNROLL_A0 4
#endif
// The trip's later iterations under a wave-uniform guard (k_trace): RK4 a = 0 (C1, C2), whose
// predicated form copies ~12 carried values (v_mov_b64) at the end of every iteration for the
// lanes that stopped. 8 per trip gave C1 +1.2%, C2 +0.4% against the predicated 10 same-box (10
// spill: 416 B scratch, C2 -65%); with the per-ray step-size cache (hcache) shallower trips win:
// 4 per trip, C2 +1.1%, C1 +4% against 8. The zero-acceleration paths stay predicated (uniform:
// C4 -1%, C5 +-0; profiles/r06/ab_unroll.txt).
template <int METHOD, bool SPIN0>
constexpr bool uniform_trip() {
    return BHRT_UNIFORM_TRIP == 1 ||
           (BHRT_UNIFORM_TRIP == 2 && METHOD == INTEGRATOR_RK4 && SPIN0);
}
template <int METHOD, bool SPIN0, bool FAR, bool HUGE, bool ACC = false>
constexpr int unroll_n() {
    return HUGE                      ? 1
         : METHOD == INTEGRATOR_RK4  ? (zero_accel<SPIN0, FAR>() ? BHRT_UNROLL_ZA : BHRT_UNROLL_A0)
         : ACC                       ? BHRT_UNROLL_ZA
                                     : 2;
}

// Persistent trace kernel: grid = what is resident; each wave refills idle lanes from the
// global queue kp.ctl[0] (one returning atomic per refill).
// FAR: some ray may take ray_derivatives' weak-field branch (origin beyond 15 rs). A camera
// frame knows this once for all its rays (shared origin); ray arrays always assume it.
// HUGE = false: the hot instantiation, rays [0, kp.n) from the queues kp.qhead. A ray that
// needs a large-argument sincos (bhrt_sincos) is dropped and its id appended to kp.redo
// (count ctl[6]). HUGE = true: re-traces kp.redo[0, ctl[6]) from queue head ctl[7].
// INL: rays set up here, at refill, instead of being loaded from k_init's table: 1 = camera
// launch (ray_init_camera), 2 = ray array with one shared origin (ray_init_shared: the origin's
// set-up from the host, the direction from the array). Used where rays are short-lived (Kerr,
// RKF45), so refills are frequent and each table load stalls its wave on HBM latency, and on the
// a = 0 RK4 disk path; ray arrays from trace_rays_batch take 2, so a chunk's
// trace depends on its upload alone (no set-up kernel queued behind the previous chunk's).
// The sin/cos anchors of the shared origin are the same for every ray: computed once per wave.
template <int METHOD, bool DISK, bool SPIN0, bool FAR, bool HUGE, int INL = 0, bool ACC = false>
__global__ BHRT_TRACE_BOUNDS void k_trace(const bhrt_kparams kp) {
    const unsigned long long total =
        HUGE ? *(volatile unsigned long long*)(kp.ctl + 6) : (unsigned long long)kp.n;
    if (total == 0) return;
    // sin, cos of the origin state's angles (r0, th0, ph0): the host's libm values
    const double as1 = kp.cam.s_r0, ac1 = kp.cam.c_r0, as2 = kp.cam.st, ac2 = kp.cam.ct,
                 as3 = kp.cam.sp, ac3 = kp.cam.cp;
    const int lane = threadIdx.x & 63;
    // the launch's execution window on the constant-rate wall clock (bhrt_stats.frame_ms:
    // first wave's start to the last wave's end, or the colour pass's end): ctl[8] holds the
    // complement of the start -- stamped by the first workgroup's first wave alone (workgroups
    // are dispatched in order; one atomic per wave at the launch's start would serialise 4096
    // atomics on one word) -- and ctl[9] the latest end
    if (!HUGE && BHRT_FRAME_STAMPS && blockIdx.x == 0 && threadIdx.x == 0)
        atomicMax(kp.ctl + 8, ~(unsigned long long)wall_clock64());
#if BHRT_WAVE_STAMPS
    const unsigned long long st_t0 = (unsigned long long)wall_clock64();
    unsigned st_trips = 0, st_refills = 0, st_claims = 0;
    unsigned long long st_claim_t = 0, st_first = 0;  // time in claim round trips; the first's
#endif
    const unsigned long long below = (1ull << lane) - 1ull;
    Counters n;
    Ray_ R;
    int rid = 0;
    bool live = false;
    // Ray queues. The rays are dealt, in blocks of 64 consecutive ids, round
    // robin over Q = 2^queue_bits queues, each with its own head word: every claim is a
    // returning device-scope atomic, and claims on ONE word serialise at the memory side
    // (~65 M/s: short-lived scenes -- C3 -- were bound by exactly that rate with one queue).
    // A wave starts on queue (its index mod Q) and moves on to the next queue when its own
    // runs dry, never back (a dry queue stays dry). A claim takes the lanes' need; with
    // claim_div > 0 it takes a block (the queue's unclaimed remainder / (waves * claim_div),
    // at least claim_min, guided scheduling) that the wave hands out over its next refills.
    // Per-wave state in LDS (touched only at refill, so it holds no registers across the
    // loop): [lo, hi) = claimed ids not yet handed out, cur = queue, moves = queues left behind.
    // The RK4 a = 0 path (C1, C2) keeps ONE queue and claims exactly the idle lanes: its rays
    // live up to max_steps iterations, so claims are rare (~30 M/s on C2) and the multi-queue
    // refill block measured -2% there (its registers perturb the 4-wave hot loop; same-box
    // A/B, profiles/r02_claim_sweep.txt).
    constexpr bool MULTIQ = !(METHOD == INTEGRATOR_RK4 && SPIN0);
    __shared__ unsigned s_q[BHRT_TRACE_WAVES_PER_BLOCK][4];
    const unsigned ntotal = (unsigned)total;
    const unsigned qbits = HUGE ? 0u : (unsigned)kp.queue_bits;
    const unsigned nq = 1u << qbits;
    unsigned long long* const heads = HUGE ? kp.ctl + 7 : kp.qhead;
    const unsigned qstride = HUGE ? 0u : (unsigned)kp.queue_stride;
    // claim = remainder >> shift (no division in the loop; claim_shift from the launcher)
    const unsigned shift = (unsigned)kp.claim_shift;
    const int wv = threadIdx.x >> 6;
    if (MULTIQ && lane == 0) {
        s_q[wv][0] = 0u;
        s_q[wv][1] = 0u;
        s_q[wv][2] = (blockIdx.x * (blockDim.x >> 6) + wv) & (nq - 1u);
        s_q[wv][3] = 0u;
    }
    constexpr bool COLD = BHRT_COLD_KP;
    // Deferred stores (drained-refill instantiations): a ray that finishes keeps its final state
    // in its lane's registers (the lane takes no new ray before the wave's next refill) and is
    // stored AT that refill, together with every other lane that finished meanwhile -- where a
    // wave refills only once drained (C3, C4, C5), all 64 lanes store at once, full lines of
    // every field, instead of a few lanes per trip (partial lines, written to HBM more than once:
    // C3's traffic was 1.40x its output) -- and the trip loop has no store code in it.
    constexpr bool DEFER = MULTIQ && !HUGE && BHRT_DEFER_STORE;
    int pterm = T_NONE;  // DEFER: how this lane's finished ray ended (T_NONE: nothing pending)
    bool exhausted = false;  // no ids left to claim or hand out; wave-uniform
    const HSel hsel = hsel_of<hsel_vgpr<METHOD, DISK, SPIN0>()>(kp.sc);
    for (;;) {
        // (re-laundered at the top of every trip, in wave-uniform control flow)
        const bhrt_kparams& kc = COLD ? cold(kp) : kp;
        const unsigned long long live_mask = __ballot(live);
        int n_live = __popcll(live_mask);
        if (!exhausted && (64 - n_live >= kp.refill || n_live == 0)) {
#if BHRT_WAVE_STAMPS
            st_refills++;
#endif
            if constexpr (DEFER) {
                if (pterm != T_NONE) store_ray<METHOD, DISK, SPIN0>(kc, rid, R, pterm);
                pterm = T_NONE;
            }
            bool ok;
            unsigned long long id;
            if constexpr (MULTIQ) {
                const unsigned need = 64u - (unsigned)n_live;
                unsigned lo = __builtin_amdgcn_readfirstlane(s_q[wv][0]);
                unsigned hi = __builtin_amdgcn_readfirstlane(s_q[wv][1]);
                unsigned cur = __builtin_amdgcn_readfirstlane(s_q[wv][2]);
                unsigned moves = __builtin_amdgcn_readfirstlane(s_q[wv][3]);
                const unsigned avail = hi - lo;
                const unsigned rank = (unsigned)__popcll(~live_mask & below);
                unsigned q = cur, j = lo + rank;  // lanes beyond the block take ids of the new claim
                ok = rank < avail;
                if (avail >= need || moves >= nq) {
                    lo += avail >= need ? need : avail;
                } else {
                    const unsigned want = need - avail;
                    unsigned b = 0, e = 0;
                    bool hopped = false;
                    for (;;) {  // wave-uniform; ends once a claim lands or every queue is dry
                        const unsigned size = queue_size(ntotal, qbits, cur);
                        unsigned long long* const hp = heads + (size_t)cur * qstride;
                        unsigned c = want;
                        if (kp.claim_div > 0 && !hopped) {
                            c = ((size - hi) >> shift) + 63u & ~63u;
                            if (c < (unsigned)kp.claim_min) c = (unsigned)kp.claim_min;
                            if (c < want) c = want;
                        }
                        unsigned long long base = 0;
#if BHRT_WAVE_STAMPS
                        const unsigned long long tq0 = (unsigned long long)wall_clock64();
#endif
                        if (lane == 0) base = atomicAdd(hp, (unsigned long long)c);
                        base = __shfl(base, 0);
#if BHRT_WAVE_STAMPS
                        {
                            const unsigned long long dtq = (unsigned long long)wall_clock64() - tq0;
                            st_claim_t += dtq;
                            if (st_claims++ == 0) st_first = dtq;
                        }
#endif
                        if (base < size) {
                            b = (unsigned)base;
                            e = base + c < size ? (unsigned)(base + c) : size;
                            break;
                        }
                        // Queue `cur` is dry. The queues not yet left behind are looked at in
                        // ONE round trip -- lane k reads the head of queue cur + 1 + k -- and
                        // the wave moves to the first with ids left (a dry queue stays dry).
                        // Hopping one queue per round trip had cost a wave up to 15 serial
                        // atomic round trips (~30 us) at the end of every launch: a quarter of a
                        // strong-scaled C4 shard's wave lifetime (tools/wave_stamps.py).
                        const unsigned left = nq - 1u - moves;
                        bool room = false;
                        if ((unsigned)lane < left) {
                            const unsigned qk = (cur + 1u + (unsigned)lane) & (nq - 1u);
                            room = __hip_atomic_load(heads + (size_t)qk * qstride, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) <
                                   (unsigned long long)queue_size(ntotal, qbits, qk);
                        }
                        const unsigned long long rm = __ballot(room);
                        if (rm == 0ull) {
                            moves = nq;
                            break;
                        }
                        const unsigned k = (unsigned)__builtin_ctzll(rm);
                        moves += k + 1u;
                        cur = (cur + 1u + k) & (nq - 1u);
                        hi = 0u;
                        hopped = true;
                    }
                    if (!ok) {
                        q = cur;
                        j = b + (rank - avail);
                        ok = j < e;
                    }
                    lo = b + want < e ? b + want : e;
                    hi = e;
                }
                exhausted = moves >= nq && lo >= hi;
                if (lane == 0) {
                    s_q[wv][0] = lo;
                    s_q[wv][1] = hi;
                    s_q[wv][2] = cur;
                    s_q[wv][3] = moves;
                }
                id = queue_ray(qbits, q, j);
            } else {
                const int need = 64 - n_live;
                unsigned long long base = 0;
                if (lane == 0) base = atomicAdd(heads, (unsigned long long)need);
                base = __shfl(base, 0);
                exhausted = base + (unsigned long long)need >= total;
                id = base + __popcll(~live_mask & below);
                ok = id < total;
            }
            if (!live) {
                if (ok) {
                    // queue position -> ray id; the k_init table is in queue order
                    const int qpos = (int)id;
                    rid = HUGE ? kp.redo[id] : (kp.src == BHRT_SRC_CAMERA ? claim_ray(kc, qpos) : qpos);
                    // (the redo list holds ray ids; the k_init table is in claim order)
                    if (INL || (HUGE && (kp.order || kp.cam.tiles_per_row))) {
                        if constexpr (INL == 2)
                            ray_init_shared(R, kc.cam, kc.dirs, kc.dir_stride, rid);
                        else
                            ray_init_camera(R, kc.cam, rid);
                        R.s1 = as1;
                        R.c1 = ac1;
                        R.s2 = as2;
                        R.c2 = ac2;
                        R.s3 = as3;
                        R.c3 = ac3;
                    } else {
                        load_init(kp, HUGE ? rid : qpos, R);
                    }
                    // the first iteration's state recovery (the loop is skipped at max_steps <= 0);
                    // an in-kernel camera set-up has a finite origin (|r0| < 2^20, host-checked),
                    // so only the velocities can need it and the origin's sin/cos stay valid
                    if (repair_at_refill<METHOD, FAR, HUGE>() && kp.sc.max_steps > 0)
                        state_repair<!INL>(R, &n);
                    if (hoist_sums<METHOD, SPIN0, FAR, HUGE>()) zero_sums<METHOD>(R);
                    if (hcache<METHOD, SPIN0, FAR, HUGE>()) R.h_lo = R.h_hi = __builtin_nan("");  // select on entry
                    // the far-field bound (repair_at_refill) not proven for this ray: it is handed
                    // to the HUGE redo pass after its first trip, like a large-argument ray (the
                    // trip's one iteration is discarded; a branch here would cost spills at
                    // every refill)
                    if (FAR && !HUGE && !(kp.sc.far_bounded && state_within(R, 0x1p40)))
                        n.huge = true;
                    // the rotation of state[2]'s sin, cos needs |h state[5]| < pi/4 (rotation_trig)
                    if (rotation_trig<METHOD, SPIN0, FAR, HUGE>() && !(fabs(R.y[5]) < kp.sc.rot_vmax))
                        n.huge = true;
                    n.rays++;
                    live = true;
                    if (kp.sc.max_steps <= 0) {  // loop never runs: MAX_STEPS, steps 0
                        store_ray<METHOD, DISK, SPIN0>(kc, rid, R, T_MAXSTEPS);
                        live = false;
                        n.huge = false;
                    }
                }
            }
            n_live = __popcll(__ballot(live));
        }
        if (n_live == 0) {
            if (exhausted) {
                if constexpr (DEFER) {
                    if (pterm != T_NONE) store_ray<METHOD, DISK, SPIN0>(kc, rid, R, pterm);
                }
                break;
            }
            continue;
        }
#if BHRT_WAVE_STAMPS
        st_trips++;
#endif
        if (live) {
            int term = ray_iterate<METHOD, DISK, SPIN0, FAR, HUGE, ACC>(R, kp.sc, n, hsel);
            // further iterations in the same trip for rays that go on: the loop's hand-over
            // copies between iterations (state, point, distance, carried sin/cos) fold away. A
            // lane's iterations are the same either way; only its refill point moves.
            if constexpr (uniform_trip<METHOD, SPIN0>()) {
                // wave-uniform guard: the trip goes on only while EVERY live lane does, so the
                // next iteration runs on the same exec mask -- no per-lane region around it, and
                // no copies of the values a lane that stopped must keep (they are copied once, on
                // the trip's exit edge, instead of after every iteration)
#pragma unroll
                for (int u = 1; u < unroll_n<METHOD, SPIN0, FAR, HUGE, ACC>(); u++) {
                    if (__ballot(term != T_NONE || n.huge) != 0ull) break;
                    term = ray_iterate<METHOD, DISK, SPIN0, FAR, HUGE, ACC>(R, kp.sc, n, hsel);
                }
            } else {
#pragma unroll
                for (int u = 1; u < unroll_n<METHOD, SPIN0, FAR, HUGE, ACC>(); u++)
                    if (term == T_NONE && !n.huge)
                        term = ray_iterate<METHOD, DISK, SPIN0, FAR, HUGE, ACC>(R, kp.sc, n, hsel);
            }
            if (METHOD == INTEGRATOR_RK4 && (term != T_NONE || (!HUGE && n.huge)))
                n.iters += R.k;  // every RK4 iteration moves, so R.k = iterations executed
            if (!HUGE && n.huge) {  // hand the ray to the HUGE instantiation
                n.huge = false;
                n.rays--;
                kp.redo[atomicAdd(kp.ctl + 6, 1ull)] = rid;
                // no redo pass follows a launch the host proved eviction-free: if that proof
                // was wrong for this scene, the ray is marked, never left stale (the host's
                // harvest reports the count as an error, bhrt_api.c)
                if (kc.no_evict && kc.skip_redo && kc.out.result) kc.out.result[rid] = RAY_ERROR;
                live = false;
            } else if (term != T_NONE) {
                if constexpr (DEFER)
                    pterm = term;
                else
                    store_ray<METHOD, DISK, SPIN0>(kc, rid, R, term);
                live = false;
            }
        }
    }
    const unsigned long long s0 = wave_sum(n.rays), s1 = wave_sum(n.iters),
                             s3 = wave_sum(n.far_);
    unsigned long long s2, s4;
    if ((FAR && HUGE) || BHRT_COUNT_STAGES) {  // stages counted one by one
        s2 = wave_sum(n.full);
        s4 = wave_sum(n.kerr);
    } else {  // every stage that was not a far-field one took the instantiation's branch
        const unsigned long long st =
            s1 * (METHOD == INTEGRATOR_RK4 ? 4ull : (METHOD == INTEGRATOR_RKF45 ? 6ull : 0ull)) -
            (FAR ? s3 : 0ull);
        s2 = SPIN0 ? st : 0ull;
        s4 = SPIN0 ? 0ull : st;
    }
#if BHRT_WAVE_STAMPS
    if (!HUGE && lane == 0 && kp.diag_slot >= 0 && kp.diag_slot < kStampSlots) {
        const unsigned w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
        if (w < (unsigned)kStampWaves) {
            unsigned long long* p =
                g_stamps + ((size_t)kp.diag_slot * kStampWaves + w) * kStampWords;
            p[0] = st_t0;
            p[1] = (unsigned long long)wall_clock64();
            p[2] = (unsigned long long)__smid();
            p[3] = (unsigned long long)st_trips | ((unsigned long long)st_refills << 32);
            p[4] = s1;
            p[5] = s0;
            p[6] = st_claim_t | ((unsigned long long)st_claims << 48);
            p[7] = st_first;
        }
    }
#endif
    if (lane == 0) {
        if (BHRT_FRAME_STAMPS) atomicMax(kp.ctl + 9, (unsigned long long)wall_clock64());
        if (s0) atomicAdd(kp.ctl + 1, s0);
        if (s1) atomicAdd(kp.ctl + 2, s1);
        if (s2) atomicAdd(kp.ctl + 3, s2);
        if (s3) atomicAdd(kp.ctl + 4, s3);
        if (s4) atomicAdd(kp.ctl + 5, s4);
    }
}

template <int SRC>
__global__ __launch_bounds__(256) void k_colour(const bhrt_kparams kp) {
    const bhrt_frame_soa& s = kp.out;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kp.n; i += gridDim.x * blockDim.x) {
        double dx, dy, dz;
        if (SRC == BHRT_SRC_CAMERA) {
            camera_dir(kp.cam, i, dx, dy, dz);
        } else if (kp.rays_shared) {
            const double* d = kp.dirs + (size_t)i * kp.dir_stride;
            dx = d[0];
            dy = d[1];
            dz = d[2];
        } else {
            dx = kp.rays[i].direction.x;
            dy = kp.rays[i].direction.y;
            dz = kp.rays[i].direction.z;
        }
        const int res = s.result[i];
        double r, g, b;
        colour_of(kp.sc, res, res == RAY_DISK ? s.hit_x[i] : 0.0,
                  res == RAY_DISK ? s.hit_y[i] : 0.0, dx, dy, dz, r, g, b);
        store_colour(s, i, r, g, b);
    }
    if (BHRT_FRAME_STAMPS) {
        __syncthreads();  // the frame is complete once the last workgroup's stores are (ctl[10])
        if (threadIdx.x == 0) atomicMax(kp.ctl + 10, (unsigned long long)wall_clock64());
    }
}

// integrate_photon_path with a recorded path (one ray, one lane). The output hit goes to
// element 0 of kp.out; the path and the stored-point count to path / d_num.
template <int METHOD, bool SPIN0>
__global__ void k_path(const bhrt_kparams kp, double t0, double ox, double oy, double oz,
                       double dx, double dy, double dz, Vector3D* path, int max_positions,
                       int* d_num, int num_in) {
    if (blockIdx.x != 0 || threadIdx.x != 0) return;
    Counters n;
    Ray_ R;
    ray_init_general(R, t0, ox, oy, oz, dx, dy, dz, kp.sc);
    trig_anchor(R);
    int num = num_in;
    if (path && max_positions > 0) {  // :504-507
        path[0].x = R.px;
        path[0].y = R.py;
        path[0].z = R.pz;
        num = 1;
    }
    int term = T_MAXSTEPS;
    if (kp.sc.max_steps > 0) {
        for (;;) {
            const int k_before = R.k;
            term = ray_iterate<METHOD, false, SPIN0, true, true>(R, kp.sc, n, hsel_of(kp.sc));
            // positions of the iterations executed (a fixed-point jump repeats p_k)
            for (int j = k_before; j < R.k && path && num >= 0 && num < max_positions; j++) {
                path[num].x = R.px;
                path[num].y = R.py;
                path[num].z = R.pz;
                num++;
            }
            if (term != T_NONE) break;
        }
    }
    if (d_num) *d_num = num;
    store_hit(kp.out, 0, R, term, kp.sc);
}

// Both forms of the RKF45 accept test (rkf45_accept) on given operands: case i has six
// components err[6i..6i+5], scale[6i..6i+5] and tolerance tol[i]; out[2i] = the fast form's
// decision, out[2i+1] = the literal quotient's.
__global__ void k_check_accept(const double* err, const double* scale, const double* tol, int n,
                               int* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double e[6], s[6];
#pragma unroll
    for (int c = 0; c < 6; c++) {
        e[c] = err[6 * i + c];
        s[c] = scale[6 * i + c];
    }
    out[2 * i] = rkf45_accept<true>(e, s, tol[i]);
    out[2 * i + 1] = rkf45_accept<false>(e, s, tol[i]);
}

// ---- launch plumbing --------------------------------------------------------------------
// Launch geometry is cached per device: a process may drive several devices (bhrt_render_frame
// splits a frame over every visible one) from several host threads. Every cached value is a
// pure function of (device, kernel), so concurrent first calls may both compute it and store
// the same value; the atomics make that race-free without a lock on the launch path.
constexpr int kMaxDev = 64;
std::atomic<int> g_cus[kMaxDev];

int current_device() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) dev = 0;
    return dev;
}

int device_cus(int dev) {
    int cus = g_cus[dev].load(std::memory_order_relaxed);
    if (cus == 0) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            cus <= 0)
            cus = 256;
        g_cus[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}

// resident workgroups of `lanes` lanes of kernel fn on device dev (the persistent grid)
int resident_blocks(const void* fn, int dev, int lanes = 256) {
    int per_cu = 0;
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, lanes, 0);
    if (per_cu <= 0) per_cu = 1;
    return device_cus(dev) * per_cu;
}

// grid of a grid-stride elementwise kernel over n items (at most one resident wave of blocks)
int grid_for(const void* fn, int n) {
    long blocks = ((long)n + 255) / 256;
    const long cap = resident_blocks(fn, current_device());
    if (blocks > cap) blocks = cap;
    return blocks < 1 ? 1 : (int)blocks;
}

// smallest shift with 2^shift >= (waves * claim_div) / 2^queue_bits, at least 1 (a grid of
// fewer waves than queues claims half a queue's remainder at a time); 0 = exact claims
int claim_shift(int blocks, int claim_div, int queue_bits, int lanes = 256) {
    if (claim_div <= 0) return 0;
    const unsigned long long wq =
        ((unsigned long long)blocks * (unsigned)(lanes / 64) * (unsigned)claim_div) >> queue_bits;
    int shift = 1;
    while (shift < 31 && (1ull << shift) < wq) shift++;
    return shift;
}

template <int METHOD, bool DISK, bool SPIN0, bool FAR, int INL, bool ACC = false>
void launch_trace_pair(const bhrt_kparams& kp, hipStream_t st) {
    // resident workgroups of the two instantiations, per device (and per hot block size:
    // kp.block_lanes, 64/128/256 lanes -- a workgroup's slot frees only once ALL its waves
    // have drained, so small launches prefer one wave per workgroup)
    static std::atomic<int> grid_cap[kMaxDev][3], grid_huge[kMaxDev];
    const int dev = current_device();
    const int lanes = kp.block_lanes == 64 || kp.block_lanes == 128 ? kp.block_lanes : 256;
    const int bi = lanes == 64 ? 0 : lanes == 128 ? 1 : 2;
    int cap = grid_cap[dev][bi].load(std::memory_order_relaxed);
    int cap_huge = grid_huge[dev].load(std::memory_order_relaxed);
    if (cap == 0 || cap_huge == 0) {
        cap = resident_blocks(
            reinterpret_cast<const void*>(&k_trace<METHOD, DISK, SPIN0, FAR, false, INL, ACC>), dev,
            lanes);
        cap_huge = resident_blocks(
            reinterpret_cast<const void*>(&k_trace<METHOD, DISK, SPIN0, FAR, true, INL>), dev);
        grid_cap[dev][bi].store(cap, std::memory_order_relaxed);
        grid_huge[dev].store(cap_huge, std::memory_order_relaxed);
    }
    int blocks = (kp.n + lanes - 1) / lanes;
    // Waves of a drained-refill launch (C3, C4, C5) get their work in guided blocks whose first
    // claim is the queue's size / its waves, so a launch of few tiles per wave is partitioned
    // almost statically at its start and ends with the waves that drew the costliest tiles
    // (a strong-scaled C4 shard: ~4 tiles per wave, trips per wave from 12 to 46,
    // profiles/r05/c4_shard_wave_stamps.txt). Such a launch -- fewer than min_tiles 64-ray
    // tiles per wave on the resident grid -- takes half the grid and shares the chip with the
    // next frames' launches: C4 8-GPU shard 0.146 -> 0.127 ms, 4-GPU shard +3.6% same-box,
    // while launches of >= 16 tiles per wave lose 6-7% at half the grid (C3, C4 full, C5) and a
    // quarter grid loses against a half (profiles/r05/ab_grid_fraction.txt, ab_min_tiles.txt).
    // kp.grid_div > 0 overrides (BHRT_GRID_DIV).
    if (trace_launch_waves<METHOD, DISK, SPIN0, FAR, INL, ACC>() > 0 && kp.grid_blocks <= 0) {
        const int lw = device_cus(dev) * trace_launch_waves<METHOD, DISK, SPIN0, FAR, INL, ACC>() * 4 / (lanes / 64);
        if (lw > 0 && lw < cap) cap = lw;
    }
    if (kp.grid_blocks > 0) {  // (A/B: an absolute grid, BHRT_GRID_BLOCKS)
        cap = kp.grid_blocks < cap ? kp.grid_blocks : cap;
    } else if (kp.grid_div > 0) {
        cap = cap / kp.grid_div > 0 ? cap / kp.grid_div : 1;
    } else if (!(METHOD == INTEGRATOR_RK4 && SPIN0) && kp.min_tiles > 0 &&  // (MULTIQ)
               (long)kp.n < 64L * kp.min_tiles * (long)cap * (lanes / 64)) {
        cap = (cap + 1) / 2;
    }
    if (blocks > cap) blocks = cap;
    if (blocks < 1) blocks = 1;
    bhrt_kparams k = kp;
    k.claim_shift = claim_shift(blocks, kp.claim_div, kp.queue_bits, lanes);
    k_trace<METHOD, DISK, SPIN0, FAR, false, INL, ACC><<<blocks, lanes, 0, st>>>(k);
    // A launch the host proved eviction-free (bhrt_api.c origin_no_evict: every ray starts at
    // one origin, and every state the loop can reach keeps its sincos arguments below 2^20 --
    // C1, C2, C3 -- or, on the zero-acceleration paths, C4 and C5, the loop has no sincos and
    // the one refill-time test |state[5]| < rot_vmax holds for every unit direction) hands no
    // ray over: no redo launch follows, one dispatch less per frame, and the frame's end no
    // longer waits behind the next frame's persistent workgroups for a wave slot
    if (kp.no_evict && kp.skip_redo) return;
    // rays evicted by the large-argument check (normally none: every wave exits at once). 64
    // workgroups: the evicted rays are rare, and a full-chip grid of waves that only read the
    // count and exit costs ~15 us per frame (C3 +8.5% same-box, profiles/r02_ab_v24.txt)
    // A far-field launch the host could not prove bounded hands every ray over: full grid.
    int redo_blocks = (FAR && !kp.sc.far_bounded) ? blocks : (blocks < 64 ? blocks : 64);
    if (redo_blocks > cap_huge) redo_blocks = cap_huge;
    k.claim_shift = claim_shift(redo_blocks, kp.claim_div, 0);  // (the redo list is one queue)
    k_trace<METHOD, DISK, SPIN0, FAR, true, INL><<<redo_blocks, 256, 0, st>>>(k);
}

template <int METHOD, bool DISK, bool SPIN0, bool FAR>
int launch_t(const bhrt_kparams& kp, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    // camera rays set up inside k_trace (no k_init table, no table load at refill): scenes with
    // a disk (most rays end on it within tens of iterations: C4 +6.6%, C3 +16.5%; the a = 0 RK4
    // path since v31, whose in-kernel set-up now fits the 4-wave 128-VGPR cap with spills only
    // in rare-lane blocks: C2 +1.2% same-box, profiles/r03_ab/ab_c2inl.txt), and the Kerr RKF45
    // path without a disk (C5: 51 attempts per ray since v21's cheaper attempts, so k_init's
    // 168-byte table -- 0.7 GB written and read per 8K shard -- outweighs the set-up: +1.5%
    // same-box, profiles/r02_ab_v20_occupancy.txt; it lost 5% on round 1's 193-attempt slab,
    // r01_ab_v10.txt).
    // Ray arrays with one shared origin (kp.rays_shared) the same way where a camera frame
    // would (mode 2: the direction from the array).
    constexpr bool CAN_INL = DISK ? true : (METHOD == INTEGRATOR_RKF45 && !SPIN0);
    const int inl = !CAN_INL || !(fabs(kp.cam.r0) < 1048576.0) ? 0
                  : kp.src == BHRT_SRC_CAMERA                  ? 1
                  : kp.rays_shared                             ? 2
                                                               : 0;
    if (inl)
        ;
    else if (kp.src == BHRT_SRC_CAMERA)
        k_init<BHRT_SRC_CAMERA><<<grid_for(reinterpret_cast<const void*>(&k_init<BHRT_SRC_CAMERA>),
                                           kp.n), 256, 0, st>>>(kp);
    else
        k_init<BHRT_SRC_RAYS><<<grid_for(reinterpret_cast<const void*>(&k_init<BHRT_SRC_RAYS>),
                                         kp.n), 256, 0, st>>>(kp);
    if (ev0) (void)hipEventRecord(ev0, st);
    // attempts that cannot be rejected (rkf45_attempt ACC): the zero-acceleration RKF45
    // instantiations with the host's accept_all (C5)
    constexpr bool CAN_ACC = METHOD == INTEGRATOR_RKF45 && accept_all_ok<SPIN0, FAR, false>();
    if constexpr (CAN_ACC && CAN_INL) {
        if (kp.sc.accept_all && inl == 1)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 1, true>(kp, st);
        else if (kp.sc.accept_all && inl == 2)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 2, true>(kp, st);
        else if (kp.sc.accept_all)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 0, true>(kp, st);
        else if (inl == 1)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 1>(kp, st);
        else if (inl == 2)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 2>(kp, st);
        else
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 0>(kp, st);
    } else if constexpr (CAN_INL) {
        if (inl == 1)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 1>(kp, st);
        else if (inl == 2)
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 2>(kp, st);
        else
            launch_trace_pair<METHOD, DISK, SPIN0, FAR, 0>(kp, st);
    } else {
        launch_trace_pair<METHOD, DISK, SPIN0, FAR, 0>(kp, st);
    }
    if (ev1) (void)hipEventRecord(ev1, st);
    if (!kp.colour_fused && (kp.out.rgb_r || kp.out.rgba32f || kp.out.rgba8)) {
        if (kp.src == BHRT_SRC_CAMERA)
            k_colour<BHRT_SRC_CAMERA><<<grid_for(reinterpret_cast<const void*>(&k_colour<BHRT_SRC_CAMERA>),
                                                 kp.n), 256, 0, st>>>(kp);
        else
            k_colour<BHRT_SRC_RAYS><<<grid_for(reinterpret_cast<const void*>(&k_colour<BHRT_SRC_RAYS>),
                                               kp.n), 256, 0, st>>>(kp);
    }
    return (int)hipGetLastError();
}

template <int METHOD, bool DISK, bool SPIN0>
int dispatch_far(const bhrt_kparams& kp, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    // a camera frame, or a ray array with one shared origin, knows from the host whether its
    // origin is beyond 15 rs (use_analytic_approx); other ray arrays assume some ray may be
    const bool far = (kp.src == BHRT_SRC_CAMERA || kp.rays_shared) ? kp.cam.use_approx != 0 : true;
    return far ? launch_t<METHOD, DISK, SPIN0, true>(kp, st, e0, e1)
               : launch_t<METHOD, DISK, SPIN0, false>(kp, st, e0, e1);
}

template <int METHOD, bool DISK>
int dispatch_spin(const bhrt_kparams& kp, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    return kp.sc.spin0 ? dispatch_far<METHOD, DISK, true>(kp, st, e0, e1)
                       : dispatch_far<METHOD, DISK, false>(kp, st, e0, e1);
}

template <int METHOD>
int dispatch_disk(const bhrt_kparams& kp, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    return kp.sc.has_disk ? dispatch_spin<METHOD, true>(kp, st, e0, e1)
                          : dispatch_spin<METHOD, false>(kp, st, e0, e1);
}

template <int METHOD>
void launch_path(const bhrt_kparams& kp, const double* o4, const double* d3, Vector3D* d_path,
                 int max_positions, int* d_num, int num_in, hipStream_t st) {
    if (kp.sc.spin0)
        k_path<METHOD, true><<<1, 64, 0, st>>>(kp, o4[0], o4[1], o4[2], o4[3], d3[0], d3[1], d3[2],
                                               d_path, max_positions, d_num, num_in);
    else
        k_path<METHOD, false><<<1, 64, 0, st>>>(kp, o4[0], o4[1], o4[2], o4[3], d3[0], d3[1],
                                                d3[2], d_path, max_positions, d_num, num_in);
}

}  // namespace

extern "C" int bhrt_launch_trace(const bhrt_kparams* kp, void* stream, void* ev0, void* ev1) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    hipEvent_t e0 = static_cast<hipEvent_t>(ev0), e1 = static_cast<hipEvent_t>(ev1);
    switch (kp->sc.method) {
    case INTEGRATOR_RK4: return dispatch_disk<INTEGRATOR_RK4>(*kp, st, e0, e1);
    case INTEGRATOR_RKF45: return dispatch_disk<INTEGRATOR_RKF45>(*kp, st, e0, e1);
    default: return dispatch_disk<INTEGRATOR_LEAPFROG>(*kp, st, e0, e1);  // no-op integrators
    }
}

// whether bhrt_launch_trace runs this launch's RKF45 attempts without the accept test (the
// ACC instantiations above: the host's accept_all on a zero-acceleration path), for the
// statistics' attempts_untested
extern "C" int bhrt_trace_untested(const bhrt_kparams* kp) {
    if (kp->sc.method != INTEGRATOR_RKF45 || !kp->sc.accept_all) return 0;
    const bool far = (kp->src == BHRT_SRC_CAMERA || kp->rays_shared) ? kp->cam.use_approx != 0 : true;
    if (kp->sc.spin0)
        return far ? accept_all_ok<true, true, false>() : accept_all_ok<true, false, false>();
    return far ? accept_all_ok<false, true, false>() : accept_all_ok<false, false, false>();
}

extern "C" __attribute__((visibility("default"))) int bhrt_check_rkf45_accept(
    const double* d_err, const double* d_scale, const double* d_tol, int n, int* d_out,
    void* stream) {
    if (n <= 0) return 0;
    k_check_accept<<<(n + 255) / 256, 256, 0, static_cast<hipStream_t>(stream)>>>(
        d_err, d_scale, d_tol, n, d_out);
    return (int)hipGetLastError();
}

extern "C" int bhrt_launch_path(const bhrt_kparams* kp, const double* o4, const double* d3,
                                Vector3D* d_path, int max_positions, int* d_num, int num_in,
                                void* stream) {
    hipStream_t st = static_cast<hipStream_t>(stream);
    switch (kp->sc.method) {
    case INTEGRATOR_RK4:
        launch_path<INTEGRATOR_RK4>(*kp, o4, d3, d_path, max_positions, d_num, num_in, st);
        break;
    case INTEGRATOR_RKF45:
        launch_path<INTEGRATOR_RKF45>(*kp, o4, d3, d_path, max_positions, d_num, num_in, st);
        break;
    default:
        launch_path<INTEGRATOR_LEAPFROG>(*kp, o4, d3, d_path, max_positions, d_num, num_in, st);
        break;
    }
    return (int)hipGetLastError();
}

#if BHRT_WAVE_STAMPS
// Diagnostic build: copy the per-wave stamps to host memory dst (kStampSlots x kStampWaves x
// kStampWords u64; NULL = do not copy) and, with reset, zero them. Synchronises the device.
extern "C" __attribute__((visibility("default"))) long bhrt_diag_stamps(void* dst, int reset) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (dst && hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), sizeof g_stamps) != hipSuccess)
        return -1;
    if (reset) {
        void* p = nullptr;
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps)) != hipSuccess ||
            hipMemset(p, 0, sizeof g_stamps) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
            return -1;
    }
    return (long)sizeof g_stamps;
}
#endif
