// Probe: calibrate rocprofv3 FETCH_SIZE against a known byte count for the load forms the block-match
// kernels use (round 4).  Each kernel reads every byte of a 64 MiB buffer exactly
// once; before each launch a 512 MiB write evicts the L2s and the 256 MiB Infinity Cache, so every byte
// comes from HBM.  Run under `rocprofv3 --pmc FETCH_SIZE` (and a WRITE_SIZE pass) and divide the
// per-dispatch counter (KiB) by the 64 MiB read: the factor per form goes into profiles/counters.json.
//   rd_vload_x4      global_load_dwordx4 into VGPRs (16 B per lane; the guide's reference form)
//   rd_glds_x4       global_load_lds_dwordx4 (16 B per lane into LDS: the distance-table staging)
//   rd_glds_ubyte    global_load_lds_ubyte (1 B per lane, 64 consecutive bytes per wave instruction)
//   rd_buf_ubyte     buffer_load_ubyte ... lds (the steady-state R-row DMA form, soffset rows)
//   rd_sload_x8      s_load_dwordx8 (32 B per wave instruction: the L-row segment form)
//   wr_store_x4      global_store_dwordx4 (16 B per lane; WRITE_SIZE reference)
//   wr_store_b64     global_store_dwordx2 (8 B per lane: the disparity flush store)
// Prints the bytes each kernel moved; the counters come from rocprofv3.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = 64ull << 20;
constexpr size_t kFlush = 512ull << 20;
constexpr int kBlock = 256;

__global__ __launch_bounds__(kBlock) void flush_l2(uint4* p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        p[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ __launch_bounds__(kBlock) void rd_vload_x4(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

__global__ __launch_bounds__(kBlock) void rd_glds_x4(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4 * 1024];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_addr(lds + w * 256));
    // wave-instruction = 1 KiB contiguous
    for (size_t c = ((size_t)blockIdx.x * 4 + w) * 1024; c < n; c += (size_t)gridDim.x * 4 * 1024) {
        const uint8_t* q = p + c;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %2" ::"v"((uint32_t)lane * 16u),
                     "s"(m0), "s"(q) : "memory", "m0");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lds[threadIdx.x] == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(kBlock) void rd_glds_ubyte(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4 * 64];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_addr(lds + w * 64));
    for (size_t c = ((size_t)blockIdx.x * 4 + w) * 64; c < n; c += (size_t)gridDim.x * 4 * 64) {
        const uint8_t* q = p + c;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %2" ::"v"((uint32_t)lane), "s"(m0),
                     "s"(q) : "memory", "m0");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lds[threadIdx.x] == 0x12345678u) out[0] = 1;
}

__global__ __launch_bounds__(kBlock) void rd_buf_ubyte(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4 * 64];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_addr(lds + w * 64));
    typedef uint32_t su4 __attribute__((ext_vector_type(4)));
    su4 rsrc;
    const uint64_t base = reinterpret_cast<uint64_t>(p);
    rsrc[0] = (uint32_t)base;
    rsrc[1] = (uint32_t)(base >> 32);
    rsrc[2] = 0xFFFFFFFFu;
    rsrc[3] = 0x00020000u;
    // soffset = the 64-byte chunk (< 2^32: the buffer is 64 MiB)
    for (size_t c = ((size_t)blockIdx.x * 4 + w) * 64; c < n; c += (size_t)gridDim.x * 4 * 64) {
        const uint32_t soff = (uint32_t)c;
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_ubyte %0, %2, %3 offen lds" ::"v"((uint32_t)lane),
                     "s"(m0), "s"(rsrc), "s"(soff) : "memory", "m0");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lds[threadIdx.x] == 0x12345678u) out[0] = 1;
}

// each wave reads its own contiguous 4 KiB chunks (no 128-B line shared by two XCDs' L2s)
__global__ __launch_bounds__(64) void rd_sload_x8(const uint8_t* __restrict__ p, size_t n, uint32_t* out) {
    typedef uint32_t su8 __attribute__((ext_vector_type(8)));
    uint32_t acc = 0;
    for (size_t c = (size_t)blockIdx.x * 4096; c < n; c += (size_t)gridDim.x * 4096)
    for (size_t k = 0; k < 4096; k += 32) {
        const size_t cc = c + k;
        su8 v;
        asm volatile("s_load_dwordx8 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p + cc) : "memory");
        acc ^= v[0] ^ v[7];
    }
    if (acc == 0x12345678u && threadIdx.x == 0) out[0] = acc;
}

__global__ __launch_bounds__(kBlock) void wr_store_x4(uint4* __restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        p[i] = make_uint4((uint32_t)i, 7, 8, 9);
}

__global__ __launch_bounds__(kBlock) void wr_store_b64(uint2* __restrict__ p, size_t n) {
    for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (size_t)gridDim.x * kBlock)
        p[i] = make_uint2((uint32_t)i, 7);
}

#define CHECK(x)                                                                \
    do {                                                                        \
        if ((x) != hipSuccess) {                                                \
            fprintf(stderr, "HIP error at %s:%d\n", __FILE__, __LINE__);        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main() {
    uint8_t *buf = nullptr, *fl = nullptr;
    uint32_t* out = nullptr;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&fl, kFlush));
    CHECK(hipMalloc(&out, 64));
    CHECK(hipMemset(buf, 1, kBytes));
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const dim3 grid(cus * 8), blk(kBlock);
    auto flush = [&]() {
        hipLaunchKernelGGL(flush_l2, dim3(cus * 8), blk, 0, 0, reinterpret_cast<uint4*>(fl), kFlush / 16);
        return hipDeviceSynchronize();
    };
    for (int rep = 0; rep < 3; ++rep) {
        CHECK(flush());
        hipLaunchKernelGGL(rd_vload_x4, grid, blk, 0, 0, reinterpret_cast<const uint4*>(buf), kBytes / 16, out);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(rd_glds_x4, grid, blk, 0, 0, buf, kBytes, out);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(rd_glds_ubyte, grid, blk, 0, 0, buf, kBytes, out);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(rd_buf_ubyte, grid, blk, 0, 0, buf, kBytes, out);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(rd_sload_x8, dim3(cus * 16), dim3(64), 0, 0, buf, kBytes, out);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(wr_store_x4, grid, blk, 0, 0, reinterpret_cast<uint4*>(buf), kBytes / 16);
        CHECK(hipDeviceSynchronize());
        CHECK(flush());
        hipLaunchKernelGGL(wr_store_b64, grid, blk, 0, 0, reinterpret_cast<uint2*>(buf), kBytes / 8);
        CHECK(hipDeviceSynchronize());
    }
    printf("each probe kernel moved %zu bytes (%.1f KiB); flush kernel wrote %zu bytes before each\n", kBytes,
           kBytes / 1024.0, kFlush);
    return 0;
}
