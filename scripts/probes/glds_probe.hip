// Probe: layout of __builtin_amdgcn_global_load_lds with size 1 (ubyte) and 4 on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void probe(const uint8_t* src, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[512];
    for (int i = threadIdx.x; i < 512; i += 64) lds[i] = 0xDEADBEEF;
    __syncthreads();
    const int l = threadIdx.x;
    __builtin_amdgcn_global_load_lds(src + 3 * l + 1, lds, 1, 0, 0);        // ubyte, lds base 0
    __builtin_amdgcn_global_load_lds(src + 4 * l, lds + 256, 4, 0, 0);     // dword, lds base 1024 B
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 512; i += 64) out[i] = lds[i];
}

int main() {
    uint8_t h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t* d; uint32_t* o;
    hipMalloc(&d, 1024); hipMalloc(&o, 2048);
    hipMemcpy(d, h, 1024, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(d, o);
    uint32_t r[512];
    hipMemcpy(r, o, 2048, hipMemcpyDeviceToHost);
    int ok1 = 1, ok4 = 1;
    for (int l = 0; l < 64; ++l) if (r[l] != h[3 * l + 1]) ok1 = 0;
    for (int l = 0; l < 64; ++l) {
        uint32_t w = h[4*l] | h[4*l+1] << 8 | h[4*l+2] << 16 | (uint32_t)h[4*l+3] << 24;
        if (r[256 + l] != w) ok4 = 0;
    }
    printf("ubyte->dword-per-lane: %s  (lds[0..4] = %08x %08x %08x %08x, expect %02x %02x ...)\n",
           ok1 ? "YES" : "NO", r[0], r[1], r[2], r[3], h[1], h[4]);
    printf("lds[64..67] = %08x %08x %08x %08x\n", r[64], r[65], r[66], r[67]);
    printf("dword: %s\n", ok4 ? "YES" : "NO");
    return 0;
}
