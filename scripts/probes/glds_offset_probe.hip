// Probe: does the immediate offset of global_load_lds_ubyte (saddr form) move
// the LDS destination as well as the global address on gfx950?  One M0 value,
// three DMAs with offset:0 / 256 / 512, global voffset pre-compensated.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__global__ void probe(const uint8_t* src, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = 0xDEADBEEF;
    __syncthreads();
    const uint32_t lane = threadIdx.x;
    const uint32_t base = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)lds;
    // DMA i: global byte lane + 64 i + 1000 (from voff = lane + 64 i + 1000 - 256 i, imm 256 i)
    const uint32_t v0 = lane + 1000, v1 = lane + 64 + 1000 - 256, v2 = lane + 128 + 1000 - 512;
    asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\t"
                 "global_load_lds_ubyte %0, %4\n\t"
                 "global_load_lds_ubyte %1, %4 offset:256\n\t"
                 "global_load_lds_ubyte %2, %4 offset:512\n\t"
                 "s_waitcnt vmcnt(0)"
                 :: "v"(v0), "v"(v1), "v"(v2), "s"(base), "s"(src) : "memory", "m0");
    __syncthreads();
    for (int i = threadIdx.x; i < 1024; i += 64) out[i] = lds[i];
}

int main() {
    static uint8_t h[4096];
    for (int i = 0; i < 4096; ++i) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t* d; uint32_t* o;
    hipMalloc(&d, 4096); hipMalloc(&o, 4096);
    hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o);
    static uint32_t r[1024];
    hipMemcpy(r, o, 4096, hipMemcpyDeviceToHost);
    // expectation if the offset moves both: lds[64 i + l] = h[1000 + 64 i + l]
    int both = 1, global_only = 1;
    for (int i = 0; i < 3; ++i)
        for (int l = 0; l < 64; ++l) {
            if (r[64 * i + l] != h[1000 + 64 * i + l]) both = 0;
        }
    // expectation if the offset moves only the global address: lds[l] written three times (last wins)
    for (int l = 0; l < 64; ++l) if (r[l] != h[1000 + 128 + l]) global_only = 0;
    printf("offset moves LDS and global: %s; global only: %s\n", both ? "YES" : "no", global_only ? "YES" : "no");
    printf("lds[0..3] %08x %08x %08x %08x | lds[64..65] %08x %08x | lds[128] %08x | lds[256] %08x\n",
           r[0], r[1], r[2], r[3], r[64], r[65], r[128], r[256]);
    printf("h[1000] %02x h[1064] %02x h[1128] %02x\n", h[1000], h[1064], h[1128]);
    return 0;
}
