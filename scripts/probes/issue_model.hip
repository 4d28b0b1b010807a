// Probe: the issue model the SAD kernel lives in, on gfx950.  Per loop
// iteration each wave runs a fixed instruction mix; output is cycles per
// iteration per SIMD (median wave's s_memtime span / waves per SIMD), for
// 1..4 waves per SIMD.  Questions it answers:
//   * dependent v_sad chains: the latency a single accumulator chain exposes;
//   * VALU + SALU from different waves: do they co-issue?
//   * ds_read_b64 and LDS-DMA (global_load_lds_ubyte) issue/throughput cost.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr int ITER = 1024;

#define V(INSN, A) asm volatile(INSN : "+v"(A) : "v"(b), "v"(c));
#define CHAIN16(A) V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) \
    V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) \
    V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) \
    V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) \
    V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A) \
    V("v_sad_u8 %0, %1, %2, %0", A) V("v_sad_u8 %0, %1, %2, %0", A)
#define IND8(INSN) V(INSN, a0) V(INSN, a1) V(INSN, a2) V(INSN, a3) V(INSN, a4) V(INSN, a5) V(INSN, a6) V(INSN, a7)
#define S1(INSN, X) asm volatile(INSN : "+s"(X) : "s"(sb) : "scc");
#define SALU8(INSN) S1(INSN, s0) S1(INSN, s1) S1(INSN, s2) S1(INSN, s3) S1(INSN, s4) S1(INSN, s5) S1(INSN, s6) S1(INSN, s7)
#define DSR(OFF) asm volatile("ds_read_b64 %0, %1 offset:" #OFF : "=v"(q) : "v"(la) : "memory"); acc ^= q.x;
#define DSR8 DSR(0) DSR(512) DSR(1024) DSR(1536) DSR(2048) DSR(2560) DSR(3072) DSR(3584)
#define DMA1(OFF) asm volatile("s_add_u32 m0, %1, " #OFF "\n\ts_nop 0\n\tglobal_load_lds_ubyte %0, %2" :: "v"(voff), "s"(lbase), "s"(gp) : "memory", "m0", "scc");
#define DMA4 DMA1(0) DMA1(256) DMA1(512) DMA1(768)

#define PL32(A, B) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(A), "+v"(B));
#define PL16(A, B) asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(A), "+v"(B));
#define DPPMIN(A) asm volatile("v_min_u32_dpp %0, %1, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(A) : "v"(b));
#define CND(A) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(A) : "v"(b), "s"(msk));
#define PERM(A) asm volatile("v_perm_b32 %0, %1, %2, %3" : "+v"(A) : "v"(b), "v"(c), "s"(sb));
#define VMIN(A) asm volatile("v_min_u32 %0, %1, %0" : "+v"(A) : "v"(b));
#define VMIN3(A) asm volatile("v_min3_u32 %0, %1, %2, %0" : "+v"(A) : "v"(b), "v"(c));
#define X8(M) M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7)
#define P8(M) M(a0, a1) M(a2, a3) M(a4, a5) M(a6, a7) M(a1, a2) M(a3, a4) M(a5, a6) M(a7, a0)
#define PROBE(NAME, BODY)                                                                   \
    __global__ __launch_bounds__(256) void NAME(uint32_t* out, uint64_t* cyc, const uint8_t* g) { \
        __shared__ uint32_t lds[4 * 1024];                                                  \
        uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,     \
                 a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                    \
        uint32_t b = threadIdx.x * 3u + 1u, c = threadIdx.x ^ 0x55u, acc = 0;               \
        uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3, s4 = s0 + 4,      \
                 s5 = s0 + 5, s6 = s0 + 6, s7 = s0 + 7, sb = blockIdx.x * 7 + 1;            \
        const int w = threadIdx.x >> 6;                                                     \
        uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(lds + w * 1024) + (threadIdx.x & 63) * 8; \
        uint32_t lbase = __builtin_amdgcn_readfirstlane(la - (threadIdx.x & 63) * 8);       \
        uint32_t voff = threadIdx.x & 63;                                                   \
        const uint8_t* gp = g + blockIdx.x * 256;                                           \
        uint2 q;                                                                            \
        const uint64_t msk = 0xFF00FF00FF00FF00ull ^ blockIdx.x;                            \
        lds[threadIdx.x] = threadIdx.x;                                                     \
        __syncthreads();                                                                    \
        uint64_t t0 = __builtin_amdgcn_s_memtime();                                         \
        for (int i = 0; i < ITER; ++i) { BODY }                                             \
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                          \
        uint64_t t1 = __builtin_amdgcn_s_memtime();                                         \
        out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ acc \
            ^ s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7 ^ lds[(threadIdx.x * 7) & 4095];           \
        if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + w] = t1 - t0;                     \
    }

PROBE(p_ind16, IND8("v_sad_u8 %0, %1, %2, %0") IND8("v_sad_u8 %0, %1, %2, %0"))
PROBE(p_chain16x1, CHAIN16(a0))
PROBE(p_chain16x2, CHAIN16(a0) CHAIN16(a1))  // 32 insns: two chains back to back
PROBE(p_chain2il, V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1)
                  V("v_sad_u8 %0, %1, %2, %0", a0) V("v_sad_u8 %0, %1, %2, %0", a1))
PROBE(p_salu16, SALU8("s_add_u32 %0, %0, %1") SALU8("s_add_u32 %0, %0, %1"))
PROBE(p_bfe16, SALU8("s_bfe_u32 %0, %0, %1") SALU8("s_bfe_u32 %0, %0, %1"))
PROBE(p_v16s16, IND8("v_sad_u8 %0, %1, %2, %0") SALU8("s_add_u32 %0, %0, %1")
                IND8("v_sad_u8 %0, %1, %2, %0") SALU8("s_add_u32 %0, %0, %1"))
PROBE(p_v16s8, IND8("v_sad_u8 %0, %1, %2, %0") SALU8("s_add_u32 %0, %0, %1") IND8("v_sad_u8 %0, %1, %2, %0"))
PROBE(p_ds8, DSR8 asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");)
PROBE(p_ds8_v16, DSR8 IND8("v_sad_u8 %0, %1, %2, %0") IND8("v_sad_u8 %0, %1, %2, %0") asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");)
PROBE(p_dma4, DMA4 asm volatile("s_waitcnt vmcnt(8)" ::: "memory");)
PROBE(p_dma4_v16, DMA4 IND8("v_sad_u8 %0, %1, %2, %0") IND8("v_sad_u8 %0, %1, %2, %0") asm volatile("s_waitcnt vmcnt(8)" ::: "memory");)
PROBE(p_nop16, asm volatile("s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\t"
                            "s_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0\n\ts_nop 0");)

PROBE(p_pl32, P8(PL32) P8(PL32))
PROBE(p_pl16, P8(PL16) P8(PL16))
PROBE(p_dppmin, X8(DPPMIN) X8(DPPMIN))
PROBE(p_cnd, X8(CND) X8(CND))
PROBE(p_perm, X8(PERM) X8(PERM))
PROBE(p_vmin, X8(VMIN) X8(VMIN))
PROBE(p_vmin3, X8(VMIN3) X8(VMIN3))

using K = void (*)(uint32_t*, uint64_t*, const uint8_t*);
struct P { const char* name; K k; };

int main() {
    const P probes[] = {{"16 ind sad", p_ind16},          {"16 chain sad", p_chain16x1},
                        {"2x16 chain seq", p_chain16x2},  {"2 chains interl16", p_chain2il},
                        {"16 s_add", p_salu16},           {"16 s_bfe", p_bfe16},
                        {"16 sad+16 s_add", p_v16s16},    {"16 sad+8 s_add", p_v16s8},
                        {"8 ds_read_b64", p_ds8},         {"8 ds_rd+16 sad", p_ds8_v16},
                        {"4 dma ubyte", p_dma4},          {"4 dma+16 sad", p_dma4_v16},
                        {"16 s_nop 0", p_nop16},          {"16 permlane32_swap", p_pl32},
                        {"16 permlane16_swap", p_pl16},   {"16 v_min_dpp", p_dppmin},
                        {"16 cndmask_e64", p_cnd},        {"16 v_perm", p_perm},
                        {"16 v_min", p_vmin},             {"16 v_min3", p_vmin3}};
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    uint64_t* cyc;
    uint8_t* g;
    hipMalloc(&out, 8 << 20);
    hipMalloc(&cyc, 1 << 20);
    hipMalloc(&g, 8 << 20);
    hipMemset(g, 1, 8 << 20);
    printf("CUs %d; cycles per loop iteration per SIMD (median wave / waves per SIMD)\n", cus);
    printf("%-20s %8s %8s %8s %8s\n", "mix", "1w/SIMD", "2w/SIMD", "3w/SIMD", "4w/SIMD");
    for (const P& p : probes) {
        printf("%-20s", p.name);
        for (int wps : {1, 2, 3, 4}) {
            const int blocks = cus * wps;  // 256 threads = 4 waves, one per SIMD
            std::vector<uint64_t> c(blocks * 4);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc, g);
            hipLaunchKernelGGL(p.k, dim3(blocks), dim3(256), 0, 0, out, cyc, g);
            if (hipDeviceSynchronize() != hipSuccess) { printf(" error\n"); return 1; }
            hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
            std::nth_element(c.begin(), c.begin() + c.size() / 2, c.end());
            printf(" %8.1f", (double)c[c.size() / 2] / ITER / wps);
        }
        printf("\n");
        fflush(stdout);
    }
    return 0;
}
