// Probe (round 5): gfx950 LDS / LDS-DMA behaviour at byte-unaligned addresses.
//   1. ds_read_b128 / ds_read_b64 / ds_read_b32 at a per-lane byte offset (lane + s): values, and cycles per
//      wave-instruction (one wave per SIMD, 4 per CU, back-to-back reads) against the aligned forms
//   2. global_load_lds_dword from byte-unaligned global addresses: which bytes land in LDS
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

template <int W>
__device__ __forceinline__ void rd(uint32_t (&v)[4], uint32_t addr) {
    if constexpr (W == 16) {
        u4 t;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(addr) : "memory");
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else if constexpr (W == 8) {
        u2 t;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(addr) : "memory");
        v[0] = t.x; v[1] = t.y; v[2] = v[3] = 0;
    } else {
        uint32_t t;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(t) : "v"(addr) : "memory");
        v[0] = t; v[1] = v[2] = v[3] = 0;
    }
}

// values: lane l reads W bytes at byte (STRIDE * l + s)
template <int W>
__global__ void values(uint32_t* out, int s, int stride) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096];
    for (int i = threadIdx.x; i < 4096; i += 64) lds[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    uint32_t v[4];
    rd<W>(v, (uint32_t)(uintptr_t)lds + (uint32_t)(stride * threadIdx.x + s));
    for (int i = 0; i < 4; ++i) out[threadIdx.x * 4 + i] = v[i];
}

// timing: N reads per lane, addresses lane * STRIDE + s (+ 512 per iteration), in flight 8 at a time
template <int W>
__global__ void timing(uint32_t* out, int s, int stride, long long* cyc) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[16384];
    for (int i = threadIdx.x; i < 16384; i += 64) lds[i] = (uint8_t)i;
    __syncthreads();
    const uint32_t base = (uint32_t)(uintptr_t)lds + (uint32_t)(stride * threadIdx.x + s);
    uint32_t acc = 0;
    const long long t0 = clock64();
    for (int it = 0; it < 64; ++it) {
        u4 a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t addr = base + (uint32_t)(((it * 8 + k) & 15) * 1024);
            if constexpr (W == 16) asm volatile("ds_read_b128 %0, %1" : "=v"(a[k]) : "v"(addr) : "memory");
            else if constexpr (W == 8) { u2 t; asm volatile("ds_read_b64 %0, %1" : "=v"(t) : "v"(addr) : "memory"); a[k] = u4{t.x, t.y, 0, 0}; }
            else { uint32_t t; asm volatile("ds_read_b32 %0, %1" : "=v"(t) : "v"(addr) : "memory"); a[k] = u4{t, 0, 0, 0}; }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += a[k].x ^ a[k].y ^ a[k].z ^ a[k].w;
    }
    const long long t1 = clock64();
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void dma(const uint8_t* src, uint32_t* out, int s) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[256];
    for (int i = threadIdx.x; i < 256; i += 64) lds[i] = 0xDEADBEEFu;
    __syncthreads();
    __builtin_amdgcn_global_load_lds(src + 4 * threadIdx.x + s, lds, 4, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int i = threadIdx.x; i < 64; i += 64) out[i] = lds[i];
}

template <int W>
void check(uint32_t* d, int s, int stride) {
    values<W><<<1, 64>>>(d, s, stride);
    std::vector<uint32_t> r(256);
    hipMemcpy(r.data(), d, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int i = 0; i < W / 4; ++i) {
            uint32_t e = 0;
            for (int b = 0; b < 4; ++b) {
                const int a = stride * l + s + 4 * i + b;
                e |= (uint32_t)(uint8_t)(a * 7 + 3) << (8 * b);
            }
            if (r[l * 4 + i] != e) ++bad;
        }
    printf("ds_read_b%d at byte stride*lane + %d (stride %d): %s (%d wrong dwords)\n", 8 * W, s, stride,
           bad ? "WRONG" : "exact", bad);
}

template <int W>
void timeit(uint32_t* d, long long* c, int s, int stride) {
    const int blocks = 1024;  // 4 per CU: one wave per SIMD
    timing<W><<<blocks, 64>>>(d, s, stride, c);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    for (int i = 0; i < 20; ++i) timing<W><<<blocks, 64>>>(d, s, stride, c);
    hipEventRecord(b);
    hipEventSynchronize(b);
    std::vector<long long> h(blocks);
    hipMemcpy(h.data(), c, blocks * 8, hipMemcpyDeviceToHost);
    long long sum = 0;
    for (auto x : h) sum += x;
    printf("ds_read_b%d offset %d stride %d: %.1f cycles per wave-instruction (median-ish mean over waves)\n", 8 * W,
           s, stride, (double)sum / blocks / (64 * 8));
}

int main() {
    uint32_t* d; long long* c; uint8_t* src;
    hipMalloc(&d, 1024 * 64 * 4); hipMalloc(&c, 1024 * 8); hipMalloc(&src, 1024);
    std::vector<uint8_t> h(1024);
    for (int i = 0; i < 1024; ++i) h[i] = (uint8_t)(i * 13 + 1);
    hipMemcpy(src, h.data(), 1024, hipMemcpyHostToDevice);
    for (int s : {0, 1, 2, 3, 5}) {
        check<16>(d, s, 16); check<16>(d, s, 1); check<8>(d, s, 8); check<8>(d, s, 1); check<4>(d, s, 4);
    }
    for (int s : {0, 1, 4, 8}) { timeit<16>(d, c, s, 16); }
    for (int s : {0, 1}) { timeit<16>(d, c, s, 1); timeit<8>(d, c, s, 8); timeit<8>(d, c, s, 1); timeit<4>(d, c, s, 4); }
    for (int s : {0, 1, 2, 3}) {
        dma<<<1, 64>>>(src, d, s);
        std::vector<uint32_t> r(64);
        hipMemcpy(r.data(), d, 256, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l) {
            uint32_t e = 0;
            for (int b = 0; b < 4; ++b) e |= (uint32_t)h[4 * l + s + b] << (8 * b);
            if (r[l] != e) ++bad;
        }
        printf("global_load_lds_dword at byte 4*lane + %d: %s (lane0 %08x lane1 %08x)\n", s, bad ? "WRONG" : "exact",
               r[0], r[1]);
    }
    return 0;
}
