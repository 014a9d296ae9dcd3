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
        if (OP == 6) x = __builtin_amdgcn_rcp(x) + 1.0;
        if (OP == 7) {  // a lane-varying branch on the chain's value
            x = fma(x, y, 1e-7);
            if (x > 2.0 + threadIdx.x * 1e-3) x *= 0.5;
        }
        if (OP == 8) {  // the same select without a branch
            x = fma(x, y, 1e-7);
            x = (x > 2.0 + threadIdx.x * 1e-3) ? x * 0.5 : x;
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

// max relative error of v_rcp_f64 against the IEEE quotient
__global__ void rcp_err(double* out, int n)
{
    double worst = 0.0;
    for (int i = 0; i < n; ++i) {
        const double x = 1.0 + (threadIdx.x * 7919.0 + i * 104729.0) * 1.1102230246251565e-12 * 37.0;
        const double r = __builtin_amdgcn_rcp(x), q = 1.0 / x;
        worst = fmax(worst, fabs(r - q) / q);
    }
    out[threadIdx.x] = worst;
}

int main()
{
    double* out; long long* cyc; long long h;
    hipMalloc(&out, 64 * 8); hipMalloc(&cyc, 8);
    const int n = 4096;
    const char* names[] = {"fma", "rsqrt(ocml)", "v_rsq_f64", "1/x", "sqrt", "mul", "v_rcp_f64", "fma+branch",
                           "fma+select"};
    for (int op = 0; op < 9; ++op) {
        for (int rep = 0; rep < 2; ++rep) {
            switch (op) {
                case 0: k<0><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 1: k<1><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 2: k<2><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 3: k<3><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 4: k<4><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 5: k<5><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 6: k<6><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 7: k<7><<<1, 64>>>(out, cyc, 1.5, n); break;
                case 8: k<8><<<1, 64>>>(out, cyc, 1.5, n); break;
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
    rcp_err<<<1, 64>>>(out, 1 << 16);
    double hw[64];
    hipMemcpy(hw, out, 64 * 8, hipMemcpyDeviceToHost);
    double w = 0.0;
    for (double v : hw) w = v > w ? v : w;
    printf("v_rcp_f64 max relative error %.3g (%.2f ulp of 1)\n", w, w / 2.220446049250313e-16);
    return 0;
}
