// Probe (round 5): the A / B operand lane maps of v_mfma_i32_32x32x32_i8 and v_mfma_i32_16x16x64_i8 on gfx950,
// tested with random i8 matrices against a host matmul, for candidate maps (16 bytes per lane, 4 VGPRs):
//   H0: lane l holds A[i = l % M][k = (K/ (64/M)) * (l / M) + e]              (contiguous k per lane group)
//   H1: element e < 8: k = 8 (l / M) + e;  e >= 8: k = K/2 + 8 (l / M) + e - 8  (two half-K passes)
// and the same with A <-> B roles (B[k][j = l % N]).  C/D: 32x32: col = l & 31, row = (r & 3) + 8 (r >> 2) + 4 (l >> 5);
// 16x16: col = l & 15, row = 4 (l >> 4) + r.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

__global__ void k32(const int8_t* a, const int8_t* b, int* d) {  // a, b: 64 lanes x 16 bytes, d: 64 x 16
    const int l = threadIdx.x;
    i32x4 av = reinterpret_cast<const i32x4*>(a)[l];
    i32x4 bv = reinterpret_cast<const i32x4*>(b)[l];
    i32x16 c = {};
    c = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = c[r];
}
__global__ void k16(const int8_t* a, const int8_t* b, int* d) {
    const int l = threadIdx.x;
    i32x4 av = reinterpret_cast<const i32x4*>(a)[l];
    i32x4 bv = reinterpret_cast<const i32x4*>(b)[l];
    i32x4 c = {};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}

static int kmap(int hyp, int l, int e, int M, int K) {
    const int g = l / M, groups = 64 / M;
    if (hyp == 0) return (K / groups) * g + e;
    return e < 8 ? 8 * g + e : K / 2 + 8 * g + e - 8;
}

static void test(int M) {
    const int K = M == 32 ? 32 : 64;
    std::vector<int8_t> A(M * K), B(K * M);
    for (auto& x : A) x = (int8_t)(rand() % 256 - 128);
    for (auto& x : B) x = (int8_t)(rand() % 256 - 128);
    std::vector<long> ref(M * M, 0);
    for (int i = 0; i < M; ++i)
        for (int j = 0; j < M; ++j)
            for (int k = 0; k < K; ++k) ref[i * M + j] += (long)A[i * K + k] * B[k * M + j];
    int8_t *da, *db; int* dd;
    hipMalloc(&da, 1024); hipMalloc(&db, 1024); hipMalloc(&dd, 64 * 16 * 4);
    for (int hyp = 0; hyp < 2; ++hyp) {
        std::vector<int8_t> pa(1024), pb(1024);
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 16; ++e) {
                const int k = kmap(hyp, l, e, M, K);
                pa[l * 16 + e] = A[(l % M) * K + k];
                pb[l * 16 + e] = B[k * M + (l % M)];
            }
        hipMemcpy(da, pa.data(), 1024, hipMemcpyHostToDevice);
        hipMemcpy(db, pb.data(), 1024, hipMemcpyHostToDevice);
        const int nreg = M == 32 ? 16 : 4;
        if (M == 32) k32<<<1, 64>>>(da, db, dd); else k16<<<1, 64>>>(da, db, dd);
        std::vector<int> d(64 * 16);
        hipMemcpy(d.data(), dd, 64 * nreg * 4, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < nreg; ++r) {
                const int col = M == 32 ? (l & 31) : (l & 15);
                const int row = M == 32 ? (r & 3) + 8 * (r >> 2) + 4 * (l >> 5) : 4 * (l >> 4) + r;
                if (d[l * nreg + r] != ref[row * M + col]) ++bad;
            }
        printf("%dx%dx%d i8 hypothesis H%d: %d / %d outputs wrong\n", M, M, K, hyp, bad, 64 * nreg);
    }
}

int main() {
    srand(7);
    test(32);
    test(16);
    return 0;
}
