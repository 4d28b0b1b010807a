// Probe: resident one-wave workgroups per CU vs LDS bytes per workgroup on this GPU
// (hipOccupancyMaxActiveBlocksPerMultiprocessor with dynamic LDS), to find the LDS allocation
// granularity behind the paired kernel's occupancy (12 workgroups of <= 13.6 KB fit 160 KB).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(64, 3) void k64(unsigned* out) {
    extern __shared__ unsigned lds[];
    lds[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[blockIdx.x] = lds[(threadIdx.x + 1) & 63];
}

int main() {
    int dev = 0, lds = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    printf("LDS per CU %d bytes, %d CUs\n", lds, cus);
    int prev = -1;
    for (int b = 9000; b <= 16384; b += 64) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k64, 64, b) != hipSuccess) return 1;
        if (n != prev) printf("bytes %6d -> %d workgroups/CU\n", b, n);
        prev = n;
    }
    return 0;
}
