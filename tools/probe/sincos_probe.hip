// Probe: OCML sincos / sin / cos on the device for arguments around 2^20, written to a file
// the host compares with glibc.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const double* x, double* s, double* c, double* s2, double* c2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a, b;
    sincos(x[i], &a, &b);
    s[i] = a;
    c[i] = b;
    s2[i] = sin(x[i]);
    c2[i] = cos(x[i]);
}

int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), s(n), c(n), s2(n), c2(n);
    for (int i = 0; i < n; i++) x[i] = 1048576.0 - 64.0 + 128.0 * i / n;
    double *dx, *ds, *dc, *ds2, *dc2;
    hipMalloc(&dx, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dc, n * 8);
    hipMalloc(&ds2, n * 8); hipMalloc(&dc2, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, ds, dc, ds2, dc2, n);
    hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(s2.data(), ds2, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c2.data(), dc2, n * 8, hipMemcpyDeviceToHost);
    double worst[4] = {0, 0, 0, 0}, wx[4] = {0, 0, 0, 0};
    long bad[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        double ref[4] = {std::sin(x[i]), std::cos(x[i]), std::sin(x[i]), std::cos(x[i])};
        double got[4] = {s[i], c[i], s2[i], c2[i]};
        for (int j = 0; j < 4; j++) {
            double e = std::fabs(got[j] - ref[j]);
            if (e > 1e-15) bad[j]++;
            if (e > worst[j]) { worst[j] = e; wx[j] = x[i]; }
        }
    }
    const char* nm[4] = {"sincos.s", "sincos.c", "sin", "cos"};
    for (int j = 0; j < 4; j++)
        printf("%-9s abs err > 1e-15: %ld of %d, worst %.3e at x = %.17g\n", nm[j], bad[j], n,
               worst[j], wx[j]);
    return 0;
}
