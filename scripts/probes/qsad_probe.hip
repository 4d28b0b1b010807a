// Probe: v_qsad_pk_u16_u8 / v_mqsad_pk_u16_u8 / v_mqsad_u32_u8 on gfx950 --
// (1) semantics on fixed operands (which bytes pair with which, which operand
// the mask reads), (2) issue rate with 1..4 waves per SIMD (independent
// accumulators), against v_sad_u8 as the yardstick.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void sem(uint64_t* out, uint64_t s0, uint32_t s1, uint64_t s2) {
    if (threadIdx.x) return;
    out[0] = __builtin_amdgcn_qsad_pk_u16_u8(s0, s1, s2);
    out[1] = __builtin_amdgcn_mqsad_pk_u16_u8(s0, s1, s2);
    using u4 = uint32_t __attribute__((ext_vector_type(4)));
    u4 acc = {1000u, 2000u, 3000u, 4000u};
    u4 r = __builtin_amdgcn_mqsad_u32_u8(s0, s1, acc);
    out[2] = r.x | ((uint64_t)r.y << 32);
    out[3] = r.z | ((uint64_t)r.w << 32);
}

constexpr int ITER = 1024;
#define Q(A) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(A) : "v"(b), "v"(c));
#define MQ(A) asm volatile("v_mqsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(A) : "v"(b), "v"(c));
#define S(A) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(A) : "v"(c), "v"(c2));
#define X8(M) M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#define PROBE(NAME, T, BODY)                                                              \
    __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint64_t* cyc) {          \
        T a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, \
          a6 = a0 + 6, a7 = a0 + 7;                                                        \
        uint64_t b = threadIdx.x * 0x0102030405060708ull;                                  \
        uint32_t c = threadIdx.x ^ 0x55u, c2 = threadIdx.x * 7u;                           \
        const int w = threadIdx.x / 64;                                                    \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                        \
        for (int i = 0; i < ITER; ++i) { BODY BODY }                                       \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7); \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;                    \
    }
PROBE(p_qsad, uint64_t, X8(Q))
PROBE(p_mqsad, uint64_t, X8(MQ))
PROBE(p_sad, uint32_t, X8(S))

int main() {
    uint64_t* d;
    hipMalloc(&d, 64);
    // s0 bytes 0..7 = 10,20,...,80 ; s1 bytes = 15,0,35,100 ; s2 = 0
    const uint64_t s0 = 0x504030201E140A00ull + 0x0A0A0A0A0A0A0A0Aull;  // 10,20,30,40,50,60,70,80
    const uint32_t s1 = 0x6423000Fu;  // 15, 0, 35, 100
    hipLaunchKernelGGL(sem, dim3(1), dim3(64), 0, 0, d, s0, s1, 0x0004000300020001ull);
    uint64_t h[4];
    hipMemcpy(h, d, 32, hipMemcpyDeviceToHost);
    printf("s0=%016llx s1=%08x s2=(1,2,3,4)\n", (unsigned long long)s0, s1);
    printf("qsad_pk   : %u %u %u %u\n", (unsigned)(h[0] & 0xFFFF), (unsigned)(h[0] >> 16 & 0xFFFF),
           (unsigned)(h[0] >> 32 & 0xFFFF), (unsigned)(h[0] >> 48));
    printf("mqsad_pk  : %u %u %u %u\n", (unsigned)(h[1] & 0xFFFF), (unsigned)(h[1] >> 16 & 0xFFFF),
           (unsigned)(h[1] >> 32 & 0xFFFF), (unsigned)(h[1] >> 48));
    printf("mqsad_u32 : %u %u %u %u (acc 1000..4000)\n", (unsigned)h[2], (unsigned)(h[2] >> 32),
           (unsigned)h[3], (unsigned)(h[3] >> 32));
    // host expectations: result i = acc_i + sum_k |s0.b[i+k] - s1.b[k]| (masked: skip s1.b[k]==0)
    for (int m = 0; m < 2; ++m) {
        printf("expect %s:", m ? "masked" : "plain ");
        for (int i = 0; i < 4; ++i) {
            unsigned s = 0;
            for (int k = 0; k < 4; ++k) {
                int a = (s0 >> (8 * (i + k))) & 0xFF, r = (s1 >> (8 * k)) & 0xFF;
                if (m && r == 0) continue;
                s += a > r ? a - r : r - a;
            }
            printf(" %u", s);
        }
        printf("  (+acc)\n");
    }
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint64_t *out, *cyc;
    hipMalloc(&out, 8 << 20);
    hipMalloc(&cyc, 1 << 20);
    struct P { const char* n; void (*k)(uint64_t*, uint64_t*); } ps[] = {
        {"16 v_qsad_pk", p_qsad}, {"16 v_mqsad_pk", p_mqsad}, {"16 v_sad_u8", p_sad}};
    printf("cycles per wave-instruction per SIMD (median wave / waves per SIMD)\n");
    for (auto& p : ps) {
        printf("%-16s", p.n);
        for (int wps : {1, 2, 3, 4}) {
            const int blocks = cus * wps;
            std::vector<uint64_t> c(blocks * 4);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            if (hipDeviceSynchronize() != hipSuccess) { printf(" error\n"); return 1; }
            hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
            std::nth_element(c.begin(), c.begin() + c.size() / 2, c.end());
            printf(" %8.2f", (double)c[c.size() / 2] / ITER / 16 / wps);
        }
        printf("\n");
    }
    return 0;
}
