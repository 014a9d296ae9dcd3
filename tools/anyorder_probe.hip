// anyorder_probe.hip -- does hipExtAnyOrderLaunch let two consecutive
// kernels of one stream overlap on gfx950?  Kernel A and kernel B each keep
// one workgroup busy for ~T us (s_memrealtime, 100 MHz); with the flag on B
// the pair should take ~T instead of ~2T.  Also: a consumer that spins on a
// flag written by the producer kernel (bounded spin: gives up after ~20 ms).
// Tooling only.  hipcc --offload-arch=gfx950 -O2 tools/anyorder_probe.hip -o build/anyorder_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void busy(unsigned long long ticks, unsigned long long* out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0) out[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
}

__global__ void producer(unsigned long long ticks, int* flag, double* data)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    data[threadIdx.x] = 1.0 + threadIdx.x;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void consumer(const int* flag, const double* data, double* out, unsigned long long* spins)
{
    __shared__ int ok;
    if (threadIdx.x == 0) {
        unsigned long long n = 0;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0) {
            ++n;
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) break;  // 20 ms: give up
        }
        ok = __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        spins[0] = n;
    }
    __syncthreads();
    out[threadIdx.x] = ok ? data[threadIdx.x] : -1.0;
}

int main()
{
    unsigned long long* d;
    int* flag;
    double *data, *out;
    unsigned long long* spins;
    hipMalloc(&d, 64 * sizeof(unsigned long long));
    hipMalloc(&flag, sizeof(int));
    hipMalloc(&data, 64 * sizeof(double));
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&spins, sizeof(unsigned long long));
    hipStream_t s;
    hipStreamCreate(&s);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const unsigned long long T = 5000;  // 50 us at 100 MHz
    for (int flags = 0; flags < 2; ++flags) {
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0, s);
            hipExtLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, nullptr, nullptr, 0, T, d);
            hipExtLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, nullptr, nullptr, flags, T, d + 1);
            hipExtLaunchKernelGGL(busy, dim3(1), dim3(64), 0, s, nullptr, nullptr, flags, T, d + 2);
            hipEventRecord(e1, s);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            std::printf("three 50-us kernels, flags %d: %.1f us\n", flags, ms * 1e3);
        }
    }
    for (int rep = 0; rep < 3; ++rep) {
        hipMemsetAsync(flag, 0, sizeof(int), s);
        hipMemsetAsync(data, 0, 64 * sizeof(double), s);
        hipEventRecord(e0, s);
        hipExtLaunchKernelGGL(producer, dim3(1), dim3(64), 0, s, nullptr, nullptr, 0, T, flag, data);
        hipExtLaunchKernelGGL(consumer, dim3(1), dim3(64), 0, s, nullptr, nullptr, 1, (const int*)flag,
                              (const double*)data, out, spins);
        hipEventRecord(e1, s);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double h[64];
        unsigned long long n;
        hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
        hipMemcpy(&n, spins, sizeof(n), hipMemcpyDeviceToHost);
        bool good = true;
        for (int i = 0; i < 64; ++i) good = good && h[i] == 1.0 + i;
        std::printf("producer -> spinning consumer (any order): %.1f us, spins %llu, data %s\n", ms * 1e3, n,
                    good ? "ok" : "WRONG");
    }
    return 0;
}
