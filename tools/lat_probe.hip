// Diagnostic: dependent-chain latency (shader cycles, s_memtime) of FP64
// ops for one wave alone on a CU.  hipcc --offload-arch=gfx950 -O3 tools/lat_probe.hip -o build/lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void k(double* out, long long* cyc, double seed, int n)
{
    double x = seed + threadIdx.x * 1e-9, y = 1.0000001;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < n; ++i) {
        if (OP == 0) x = fma(x, y, 1e-7);
        if (OP == 1) x = rsqrt(x) + 1.0;
        if (OP == 2) x = __builtin_amdgcn_rsq(x) + 1.0;
        if (OP == 3) x = 1.0 / x + 1.0;
        if (OP == 4) x = sqrt(x) + 1.0;
        if (OP == 5) x = x * y;
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main()
{
    double* out; long long* cyc; long long h;
    hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
    const int n = 4096;
    const char* names[] = {"fma", "rsqrt(ocml)", "v_rsq_f64", "1/x", "sqrt", "mul"};
    for (int op = 0; op < 6; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (op) {
                case 0: k<0><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 1: k<1><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 2: k<2><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 3: k<3><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 4: k<4><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 5: k<5><<<1, 64>>>(out, cyc, 1.5, n); break;
            }
            hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
        }
        printf("%-12s %.1f cycles per dependent op\n", names[op], double(h) / n);
    }
    // wall-clock check of the s_memtime rate
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k<0><<<1, 64>>>(out, cyc, 1.5, 1 << 22);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("fma chain 4M: %lld cycles in %.3f ms -> %.0f MHz counter\n", h, ms, h / (ms * 1e3));
    return 0;
}
