// Probe (round 5): V = max(B, G, R) histogram of a 1920x1080 BGR frame, LDS strategies on gfx950.
//   mode 0: one 256-bin copy per wave, ds_add_u32 per pixel (the product's v_hist_kernel)
//   mode 1: 32 copies per block, bin b of copy c at dword 32 b + c, c = lane & 31: every lane of a 32-lane
//           LDS group on its own bank
//   mode 2: as 1 with two bins per dword (u16 halves)
//   mode 3: 64 copies per block (dword 64 b + lane)
//   mode 9: no histogram at all (the loads and V only: the floor)
// Each block adds its bins into one of 8 global copies.  Prints us per launch (HIP events, 200 launches).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int W = 1920, H = 1080, NQ = W * H / 4;  // quads of 4 pixels = 12 bytes

template <int MODE, int QPT>
__global__ __launch_bounds__(256) void hist(const uint8_t* __restrict__ bgr, uint32_t* __restrict__ out) {
    constexpr int WORDS = MODE == 0 ? 4 * 256 : MODE == 1 ? 256 * 32 : MODE == 2 ? 128 * 32 : MODE == 3 ? 256 * 64 : 1;
    __shared__ uint32_t lh[WORDS];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    for (int i = t; i < WORDS; i += 256) lh[i] = 0;
    uint32_t q[QPT][3];
    const int base = blockIdx.x * 256 * QPT + t;
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
        const int qi = base + u * 256;
        if (qi < NQ) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(bgr + 12 * (size_t)qi);
            q[u][0] = p[0]; q[u][1] = p[1]; q[u][2] = p[2];
        } else {
            q[u][0] = q[u][1] = q[u][2] = 0;
        }
    }
    __syncthreads();
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
        if (base + u * 256 >= NQ) break;
        uint8_t c[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) c[i] = (q[u][i >> 2] >> (8 * (i & 3))) & 0xFF;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t v = max(max(c[3 * k], c[3 * k + 1]), c[3 * k + 2]);
            if constexpr (MODE == 0) atomicAdd(&lh[wv * 256 + v], 1u);
            else if constexpr (MODE == 1) atomicAdd(&lh[v * 32 + (lane & 31)], 1u);
            else if constexpr (MODE == 2) atomicAdd(&lh[(v >> 1) * 32 + (lane & 31)], 1u << (16 * (v & 1)));
            else if constexpr (MODE == 3) atomicAdd(&lh[v * 64 + lane], 1u);
            else acc += v;
        }
    }
    __syncthreads();
    uint32_t sum = 0;
    if constexpr (MODE == 0) {
        for (int w = 0; w < 4; ++w) sum += lh[w * 256 + t];
    } else if constexpr (MODE == 1) {
        const uint4* r = reinterpret_cast<const uint4*>(lh + t * 32);
#pragma unroll
        for (int i = 0; i < 8; ++i) { const uint4 x = r[i]; sum += x.x + x.y + x.z + x.w; }
    } else if constexpr (MODE == 2) {
        const uint4* r = reinterpret_cast<const uint4*>(lh + (t >> 1) * 32);
        uint32_t s2 = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) { const uint4 x = r[i]; s2 += x.x + x.y + x.z + x.w; }
        sum = (t & 1) ? (s2 >> 16) : (s2 & 0xFFFF);
    } else if constexpr (MODE == 3) {
        const uint4* r = reinterpret_cast<const uint4*>(lh + t * 64);
#pragma unroll
        for (int i = 0; i < 16; ++i) { const uint4 x = r[i]; sum += x.x + x.y + x.z + x.w; }
    } else {
        sum = acc & 1;
    }
    if (sum) atomicAdd(&out[(blockIdx.x & 7) * 256 + t], sum);
}

template <int MODE, int QPT>
float run(const uint8_t* d, uint32_t* o, std::vector<uint32_t>& h) {
    const int blocks = (NQ + 256 * QPT - 1) / (256 * QPT);
    hipMemset(o, 0, 8 * 256 * 4);
    hist<MODE, QPT><<<blocks, 256>>>(d, o);
    std::vector<uint32_t> r(8 * 256);
    hipMemcpy(r.data(), o, r.size() * 4, hipMemcpyDeviceToHost);
    h.assign(256, 0);
    for (int c = 0; c < 8; ++c) for (int b = 0; b < 256; ++b) h[b] += r[c * 256 + b];
    for (int i = 0; i < 50; ++i) hist<MODE, QPT><<<blocks, 256>>>(d, o);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    for (int i = 0; i < 200; ++i) hist<MODE, QPT><<<blocks, 256>>>(d, o);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / 200;
}

int main() {
    std::vector<uint8_t> img(3 * (size_t)W * H);
    uint32_t s = 12345;
    for (auto& x : img) { s = s * 1664525u + 1013904223u; x = (uint8_t)(s >> 24); }
    std::vector<uint32_t> ref(256, 0);
    for (int p = 0; p < W * H; ++p) ++ref[std::max(std::max(img[3 * p], img[3 * p + 1]), img[3 * p + 2])];
    uint8_t* d; uint32_t* o;
    hipMalloc(&d, img.size()); hipMalloc(&o, 8 * 256 * 4);
    hipMemcpy(d, img.data(), img.size(), hipMemcpyHostToDevice);
    std::vector<uint32_t> h;
#define R(M, Q) { float us = run<M, Q>(d, o, h); printf("mode %d quads/thread %d: %7.2f us  %s\n", M, Q, us, \
                                                         M == 9 ? "(floor)" : (h == ref ? "ok" : "MISMATCH")); }
    R(0, 2) R(0, 4) R(0, 8)
    R(1, 2) R(1, 4) R(1, 8)
    R(2, 2) R(2, 4) R(2, 8)
    R(3, 2) R(3, 4) R(3, 8)
    R(9, 2) R(9, 4)
    return 0;
}
