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
PROBE(p_sad_u32, "v_sad_u32 %0, %1, %2, %0")
PROBE(p_sad_u16, "v_sad_u16 %0, %1, %2, %0")
PROBE(p_add3_u32, "v_add3_u32 %0, %1, %2, %0")
PROBE(p_sub_u32, "v_sub_u32 %0, %0, %1")
PROBE(p_or_b32, "v_or_b32 %0, %1, %0")
PROBE(p_lshl_add, "v_lshl_add_u32 %0, %1, 8, %0")
PROBE(p_mad_u24, "v_mad_u32_u24 %0, %1, %2, %0")
PROBE(p_mul_u24, "v_mul_u32_u24 %0, %1, %0")
PROBE(p_mul_lo, "v_mul_lo_u32 %0, %1, %0")
PROBE(p_alignbyte, "v_alignbyte_b32 %0, %1, %0, 1")
PROBE(p_and_or, "v_and_or_b32 %0, %1, %2, %0")
PROBE(p_xad, "v_xad_u32 %0, %1, %2, %0")

// Mixed streams: cycles per loop iteration (16 VALU [+ 16 or 8 SALU]) per SIMD.
#define SBODY8                                                                          \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s2) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s3) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s4) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s5) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s6) : "s"(sb) : "scc");                \
    asm volatile("s_add_u32 %0, %0, %1" : "+s"(s7) : "s"(sb) : "scc");
#define MIXPROBE(NAME, BODY)                                                            \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint64_t* cyc) {        \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                \
        uint32_t b = threadIdx.x * 3u + 1u, c = threadIdx.x ^ 0x55u;                    \
        uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4,  \
                 s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7, sb = blockIdx.x * 7 + 1;        \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                     \
        for (int i = 0; i < ITER; ++i) { BODY }                                         \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 \
            ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7;                                    \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    }
// VALU with an SGPR source operand, cndmask with a real mask, DPP move
#define SBODY_V8(INSN)                                                                  \
    asm volatile(INSN : "+v"(a0) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a1) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a2) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a3) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a4) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a5) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a6) : "s"(sb), "v"(c));                                    \
    asm volatile(INSN : "+v"(a7) : "s"(sb), "v"(c));
MIXPROBE(m_sad_sgpr, SBODY_V8("v_sad_u8 %0, %1, %2, %0") SBODY_V8("v_sad_u8 %0, %1, %2, %0"))
MIXPROBE(m_cnd_mask, asm volatile("v_cmp_gt_u32 vcc, %0, %1" :: "v"(b), "v"(c) : "vcc");
         BODY8("v_cndmask_b32 %0, %1, %0, vcc") BODY8("v_cndmask_b32 %0, %1, %0, vcc"))
MIXPROBE(m_cnd_e64, asm volatile("v_cmp_gt_u32 s[40:41], %0, %1" :: "v"(b), "v"(c) : "s40", "s41");
         BODY8("v_cndmask_b32_e64 %0, %1, %0, s[40:41]") BODY8("v_cndmask_b32_e64 %0, %1, %0, s[40:41]"))
MIXPROBE(m_mov_dpp, BODY8("v_mov_b32_dpp %0, %1 row_mirror row_mask:0xf bank_mask:0xf")
         BODY8("v_mov_b32_dpp %0, %1 row_mirror row_mask:0xf bank_mask:0xf"))
MIXPROBE(m_valu16, BODY8("v_sad_u8 %0, %1, %2, %0") BODY8("v_sad_u8 %0, %1, %2, %0"))
MIXPROBE(m_salu16, SBODY8 SBODY8)
MIXPROBE(m_v16_s16, BODY8("v_sad_u8 %0, %1, %2, %0") SBODY8 BODY8("v_sad_u8 %0, %1, %2, %0") SBODY8)
MIXPROBE(m_v16_s8, BODY8("v_sad_u8 %0, %1, %2, %0") SBODY8 BODY8("v_sad_u8 %0, %1, %2, %0"))
MIXPROBE(m_add16_s16, BODY8("v_add_u32 %0, %1, %0") SBODY8 BODY8("v_add_u32 %0, %1, %0") SBODY8)

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
                        {"v_max3_u32", p_max3_u32},       {"v_pk_mad_u16", p_pk_mad_u16},
                        {"v_sad_u32", p_sad_u32},         {"v_sad_u16", p_sad_u16},
                        {"v_add3_u32", p_add3_u32},       {"v_sub_u32", p_sub_u32},
                        {"v_or_b32", p_or_b32},           {"v_lshl_add_u32", p_lshl_add},
                        {"v_mad_u32_u24", p_mad_u24},     {"v_mul_u32_u24", p_mul_u24},
                        {"v_mul_lo_u32", p_mul_lo},       {"v_alignbyte_b32", p_alignbyte},
                        {"v_and_or_b32", p_and_or},       {"v_xad_u32", p_xad}};
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
    const P mixes[] = {{"16 sad", m_valu16}, {"16 s_add", m_salu16}, {"16 sad+16 s_add", m_v16_s16},
                       {"16 sad+8 s_add", m_v16_s8}, {"16 v_add+16 s_add", m_add16_s16}, {"16 sad(sgpr src)", m_sad_sgpr},
                       {"16 cndmask vcc", m_cnd_mask}, {"16 cndmask sgpr", m_cnd_e64}, {"16 mov_dpp", m_mov_dpp}};
    printf("\nmixed streams: cycles per loop iteration per SIMD\n");
    for (const P& p : mixes) {
        printf("%-20s", p.name);
        for (int wps : {1, 2, 3, 4}) {
            const int blocks = cus * wps;
            std::vector<uint64_t> c(blocks * 4);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc);
            hipDeviceSynchronize();
            hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
            std::nth_element(c.begin(), c.begin() + c.size() / 2, c.end());
            printf(" %8.2f", (double)c[c.size() / 2] / ITER / wps);
        }
        printf("\n");
    }
    return 0;
}
