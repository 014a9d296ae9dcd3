// Diagnostic: resident blocks per CU of the lfg kernels (occupancy API) and
// of probe kernels that isolate the LDS and VGPR limits.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include tools/occupancy.hip -o build/occupancy
#include "../lfit_python_amd/csrc/lfg.hip"
#include <cstdio>

template <int LDS_BYTES>
__global__ __launch_bounds__(512) void probe_lds(double* out)
{
    __shared__ double buf[LDS_BYTES / 8];
    buf[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[blockIdx.x * 512 + threadIdx.x] = buf[(threadIdx.x + 1) % 512];
}

template <typename K>
static void report(const char* name, K kern, int threads, size_t dyn = 0)
{
    int nb = -1;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, threads, dyn);
    hipFuncAttributes a{};
    (void)hipFuncGetAttributes(&a, reinterpret_cast<const void*>(kern));
    printf("%-22s threads %4d  blocks/CU %2d (%s)  vgpr-ish numRegs %3d  lds %6zu  scratch %zu\n", name, threads,
           nb, hipGetErrorString(e), a.numRegs, a.sharedSizeBytes, a.localSizeBytes);
}

int main()
{
    hipDeviceProp_t p;
    (void)hipGetDeviceProperties(&p, 0);
    printf("%s: %d CUs, LDS/block max %zu, LDS/CU %zu, regs/block %d\n", p.gcnArchName, p.multiProcessorCount,
           p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor, p.regsPerBlock);
    report("k_setup", k_setup, SETUP_BLOCK);
    report("k_elements", k_elements, ELEM_BLOCK);
    report("k_lnlike<0>", k_lnlike<0>, LIKE_THREADS);
    report("k_lnlike<1>", k_lnlike<1>, LIKE_THREADS);
    report("k_lnlike<2>", k_lnlike<2>, LIKE_THREADS);
    report("probe_lds<32768>", probe_lds<32768>, 512);
    report("probe_lds<65536>", probe_lds<65536>, 512);
    report("probe_lds<67248>", probe_lds<67248>, 512);
    report("probe_lds<81920>", probe_lds<81920>, 512);
    return 0;
}
