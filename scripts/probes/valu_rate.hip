// Probe: sustained issue rate of the VALU instructions the SAD kernel uses, on
// gfx950, with WPS waves per SIMD.  Each lane runs ITER x 16 independent
// instructions (8 accumulators, inline asm so nothing is folded).  Output:
// cycles per wave-instruction per SIMD, from s_memtime around the loop
// (median wave) and from the kernel wall time at the measured clock.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int ITER = 2048;

#define BODY8(INSN)                                                                     \
    asm volatile(INSN : "+v"(a0) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a1) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a2) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a3) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a4) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a5) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a6) : "v"(b), "v"(c));                                     \
    asm volatile(INSN : "+v"(a7) : "v"(b), "v"(c));

#define PROBE(NAME, INSN)                                                               \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint64_t* cyc) {        \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                \
        uint32_t b = threadIdx.x * 3u + 1u, c = threadIdx.x ^ 0x55u;                    \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                     \
        for (int i = 0; i < ITER; ++i) { BODY8(INSN) BODY8(INSN) }                     \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7; \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }

PROBE(p_fma_f32, "v_fma_f32 %0, %1, %2, %0")
PROBE(p_add_u32, "v_add_u32 %0, %1, %0")
PROBE(p_sad_u8, "v_sad_u8 %0, %1, %2, %0")
PROBE(p_sad_hi_u8, "v_sad_hi_u8 %0, %1, %2, %0")
PROBE(p_pk_add_u16, "v_pk_add_u16 %0, %1, %0")
PROBE(p_pk_sub_u16, "v_pk_sub_u16 %0, %0, %1")
PROBE(p_pk_min_u16, "v_pk_min_u16 %0, %1, %0")
PROBE(p_perm_b32, "v_perm_b32 %0, %1, %2, %0")
PROBE(p_min_u32, "v_min_u32 %0, %1, %0")
PROBE(p_min3_u32, "v_min3_u32 %0, %1, %2, %0")
PROBE(p_cndmask, "v_cndmask_b32 %0, %1, %0, vcc")
PROBE(p_lshl_or, "v_lshl_or_b32 %0, %1, 8, %0")
PROBE(p_mov_dpp, "v_min_u32_dpp %0, %1, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf")
PROBE(p_permlane32, "v_permlane32_swap_b32 %0, %1")
PROBE(p_dot4_u8, "v_dot4_u32_u8 %0, %1, %2, %0")
PROBE(p_msad_u8, "v_msad_u8 %0, %1, %2, %0")
PROBE(p_bfe_u32, "v_bfe_u32 %0, %1, 8, 8")
PROBE(p_max3_u32, "v_max3_u32 %0, %1, %2, %0")
PROBE(p_pk_mad_u16, "v_pk_mad_u16 %0, %1, %2, %0")

using K = void (*)(uint32_t*, uint64_t*);
struct P { const char* name; K k; };

int main() {
    const P probes[] = {{"v_fma_f32", p_fma_f32},         {"v_add_u32", p_add_u32},
                        {"v_sad_u8", p_sad_u8},           {"v_sad_hi_u8", p_sad_hi_u8},
                        {"v_pk_add_u16", p_pk_add_u16},   {"v_pk_sub_u16", p_pk_sub_u16},
                        {"v_pk_min_u16", p_pk_min_u16},   {"v_perm_b32", p_perm_b32},
                        {"v_min_u32", p_min_u32},         {"v_min3_u32", p_min3_u32},
                        {"v_cndmask_b32", p_cndmask},     {"v_lshl_or_b32", p_lshl_or},
                        {"v_min_u32_dpp", p_mov_dpp},     {"v_permlane32_swap", p_permlane32},
                        {"v_dot4_u32_u8", p_dot4_u8},
                        {"v_msad_u8", p_msad_u8},         {"v_bfe_u32", p_bfe_u32},
                        {"v_max3_u32", p_max3_u32},       {"v_pk_mad_u16", p_pk_mad_u16}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    uint64_t* cyc;
    hipMalloc(&out, 4 << 20);
    hipMalloc(&cyc, 1 << 20);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double insn_per_wave = ITER * 16.0;
    printf("CUs %d; cycles per wave-instruction per SIMD (median wave s_memtime / waves-per-SIMD)\n", cus);
    printf("%-20s %8s %8s %8s\n", "insn", "1w/SIMD", "2w/SIMD", "4w/SIMD");
    for (const P& p : probes) {
        printf("%-20s", p.name);
        for (int wps : {1, 2, 4}) {
            const int blocks = cus * wps;  // 256 threads = 4 waves = one per SIMD
            std::vector<uint64_t> c(blocks * 4);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            hipEventRecord(e0);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
            std::nth_element(c.begin(), c.begin() + c.size() / 2, c.end());
            const double med = (double)c[c.size() / 2];
            // one wave's loop spans med cycles; wps waves share the SIMD
            printf(" %8.2f", med / insn_per_wave / wps);
        }
        printf("\n");
    }
    return 0;
}
