// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp) and of 1 / 2 Newton steps,
// in ulps of the correctly rounded 1/d, over random d in [2^-40, 2^40].
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

__global__ void k(const double *d, double *r0, double *r1, double *r2, int n)
{
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double r = __builtin_amdgcn_rcp(x);
    r0[i] = r;
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    r1[i] = r;
    e = fma(-x, r, 1.0);
    r2[i] = fma(r, e, r);
}

static double ulps(double a, double b)
{
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    return std::fabs((double)(ia - ib));
}

int main()
{
    const int n = 1 << 22;
    double *h = new double[n], *o0 = new double[n], *o1 = new double[n], *o2 = new double[n];
    uint64_t s = 0x12345;
    for (int i = 0; i < n; i++) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        double u = (double)(s >> 11) / 9007199254740992.0;
        h[i] = std::ldexp(1.0 + u, (int)((s >> 3) % 81) - 40);
    }
    double *d, *a, *b, *c;
    hipMalloc(&d, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8);
    hipMemcpy(d, h, n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, d, a, b, c, n);
    hipMemcpy(o0, a, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(o1, b, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(o2, c, n * 8, hipMemcpyDeviceToHost);
    double m0 = 0, m1 = 0, m2 = 0;
    for (int i = 0; i < n; i++) {
        const double ref = 1.0 / h[i];
        m0 = std::fmax(m0, ulps(o0[i], ref));
        m1 = std::fmax(m1, ulps(o1[i], ref));
        m2 = std::fmax(m2, ulps(o2[i], ref));
    }
    printf("v_rcp_f64 max error %.0f ulp; +1 Newton %.0f ulp; +2 Newton %.0f ulp (n = %d)\n", m0, m1, m2, n);
    return 0;
}
