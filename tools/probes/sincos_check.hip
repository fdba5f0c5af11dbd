// Probe: ocml sincos(x) returns exactly sin(x) and cos(x) (bitwise), over the
// argument range the cosine-PDF generate uses (phi = 2*pi*u, u = k * 2^-32).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(unsigned long long n, unsigned long long* bad) {
    for (unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x; i < n;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const double u = (double)(unsigned)(i * 2654435761ull + (i >> 7)) * (1.0 / 4294967296.0);
        const double phi = 2.0 * 3.141592653589793 * u;
        double s, c;
        sincos(phi, &s, &c);
        if (__double_as_longlong(s) != __double_as_longlong(sin(phi)) ||
            __double_as_longlong(c) != __double_as_longlong(cos(phi)))
            atomicAdd(bad, 1ull);
        float sf, cf;
        const float pf = (float)phi;
        sincosf(pf, &sf, &cf);
        if (__float_as_int(sf) != __float_as_int(sinf(pf)) || __float_as_int(cf) != __float_as_int(cosf(pf)))
            atomicAdd(bad + 1, 1ull);
    }
}
int main() {
    unsigned long long* d;
    hipMalloc(&d, 16);
    hipMemset(d, 0, 16);
    const unsigned long long n = 1ull << 32;
    hipLaunchKernelGGL(k, dim3(8192), dim3(256), 0, 0, n, d);
    unsigned long long h[2];
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("sincos_check n=%llu f64_mismatch=%llu f32_mismatch=%llu\n", n, h[0], h[1]);
    return (h[0] || h[1]) ? 1 : 0;
}
