// Accuracy of the raw f64 transcendental instructions on gfx950 (v_rcp_f64, v_rsq_f64,
// v_sqrt_f64) and of v_rcp_f64 + one / two Newton steps, against correctly rounded host
// values, over random doubles spread across [2^-20, 2^20). Diagnostic only.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

__global__ void k(const double* x, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double v = x[i];
    double r = __builtin_amdgcn_rcp(v);
    double e = __builtin_fma(-v, r, 1.0);
    double r1 = __builtin_fma(r, e, r);
    double e2 = __builtin_fma(-v, r1, 1.0);
    double r2 = __builtin_fma(r1, e2, r1);
    out[6 * i + 0] = r;
    out[6 * i + 1] = r1;
    out[6 * i + 2] = r2;
    out[6 * i + 3] = __builtin_amdgcn_rsq(v);
    out[6 * i + 4] = __builtin_amdgcn_sqrt(v);
    out[6 * i + 5] = sqrt(v);
}

static double ulps(double got, long double want) {
    double w = (double)want;
    double u = nextafter(fabs(w), INFINITY) - fabs(w);
    return (double)(fabsl((long double)got - want) / u);
}

int main() {
    const int n = 1 << 22;
    std::vector<double> x(n), out(6 * (size_t)n);
    uint64_t s = 0x9e3779b97f4a7c15ull;
    for (int i = 0; i < n; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        double m = 1.0 + (double)(s >> 11) * 0x1.0p-53;
        int ex = (int)((s >> 3) % 40) - 20;
        x[i] = ldexp(m, ex);
    }
    double *dx, *dout;
    hipMalloc(&dx, n * sizeof(double));
    hipMalloc(&dout, 6 * (size_t)n * sizeof(double));
    hipMemcpy(dx, x.data(), n * sizeof(double), hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, dout, n);
    hipMemcpy(out.data(), dout, 6 * (size_t)n * sizeof(double), hipMemcpyDeviceToHost);
    double mx[6] = {0};
    long exact[6] = {0};
    for (int i = 0; i < n; i++) {
        long double xv = x[i];
        long double want[6] = {1.0L / xv, 1.0L / xv, 1.0L / xv, 1.0L / sqrtl(xv), sqrtl(xv), sqrtl(xv)};
        for (int j = 0; j < 6; j++) {
            double u = ulps(out[6 * (size_t)i + j], want[j]);
            if (u > mx[j]) mx[j] = u;
            if (out[6 * (size_t)i + j] == (double)want[j]) exact[j]++;
        }
    }
    const char* names[6] = {"v_rcp_f64", "rcp+1NR", "rcp+2NR", "v_rsq_f64", "v_sqrt_f64", "sqrt()"};
    for (int j = 0; j < 6; j++)
        printf("%-11s max %.3g ulp, correctly rounded %.4f\n", names[j], mx[j], (double)exact[j] / n);
    return 0;
}
