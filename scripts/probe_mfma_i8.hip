// Determine the operand lane maps of the gfx950 int8 MFMAs with exact random
// data (cdna_hip_programming.md: "check the map with exact integer data").
//   hipcc --offload-arch=gfx950 -O3 scripts/probe_mfma_i8.hip -o scripts/probe_mfma_i8
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

typedef int32_t i32x4 __attribute__((ext_vector_type(4)));
typedef int32_t i32x16 __attribute__((ext_vector_type(16)));

__global__ void k16(const int32_t *a, const int32_t *b, int32_t *d) {
    const int l = threadIdx.x;
    i32x4 A = {a[l * 4], a[l * 4 + 1], a[l * 4 + 2], a[l * 4 + 3]};
    i32x4 B = {b[l * 4], b[l * 4 + 1], b[l * 4 + 2], b[l * 4 + 3]};
    i32x4 C = {0, 0, 0, 0};
    i32x4 D = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B, C, 0, 0, 0);
    for (int r = 0; r < 4; ++r) d[l * 4 + r] = D[r];
}

__global__ void k32(const int32_t *a, const int32_t *b, int32_t *d) {
    const int l = threadIdx.x;
    i32x4 A = {a[l * 4], a[l * 4 + 1], a[l * 4 + 2], a[l * 4 + 3]};
    i32x4 B = {b[l * 4], b[l * 4 + 1], b[l * 4 + 2], b[l * 4 + 3]};
    i32x16 C = {};
    i32x16 D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, C, 0, 0, 0);
    for (int r = 0; r < 16; ++r) d[l * 16 + r] = D[r];
}

static int8_t A8[64][16], B8[64][16];

// candidate k of element e of lane l: 0 = contiguous 16 per lane group, 1 = two 8-runs
static int kmap(int cand, int l, int e, int groups) {
    const int g = l / (64 / groups);
    if (cand == 0) return 16 * g + e;
    return 8 * g + (e & 7) + 8 * groups * (e >> 3);
}

int main() {
    srand(7);
    for (int l = 0; l < 64; ++l)
        for (int e = 0; e < 16; ++e) { A8[l][e] = (int8_t)(rand() & 0xff); B8[l][e] = (int8_t)(rand() & 0xff); }
    int32_t *da, *db, *dd;
    hipMalloc(&da, 1024); hipMalloc(&db, 1024); hipMalloc(&dd, 64 * 16 * 4);
    hipMemcpy(da, A8, 1024, hipMemcpyHostToDevice);
    hipMemcpy(db, B8, 1024, hipMemcpyHostToDevice);
    int32_t D[64 * 16];
    // 16x16x64
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, da, db, dd);
    hipMemcpy(D, dd, 64 * 4 * 4, hipMemcpyDeviceToHost);
    for (int ca = 0; ca < 2; ++ca) for (int cb = 0; cb < 2; ++cb) {
        int A[16][64] = {}, B[64][16] = {};
        for (int l = 0; l < 64; ++l) for (int e = 0; e < 16; ++e) {
            A[l & 15][kmap(ca, l, e, 4)] = A8[l][e];
            B[kmap(cb, l, e, 4)][l & 15] = B8[l][e];
        }
        int bad = 0;
        for (int l = 0; l < 64; ++l) for (int r = 0; r < 4; ++r) {
            int row = (l >> 4) * 4 + r, col = l & 15, s = 0;
            for (int k = 0; k < 64; ++k) s += A[row][k] * B[k][col];
            bad += s != D[l * 4 + r];
        }
        printf("16x16x64 candA=%d candB=%d mismatches=%d\n", ca, cb, bad);
    }
    // 32x32x32
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, da, db, dd);
    hipMemcpy(D, dd, 64 * 16 * 4, hipMemcpyDeviceToHost);
    for (int ca = 0; ca < 2; ++ca) for (int cb = 0; cb < 2; ++cb) {
        int A[32][32] = {}, B[32][32] = {};
        for (int l = 0; l < 64; ++l) for (int e = 0; e < 16; ++e) {
            A[l & 31][kmap(ca, l, e, 2)] = A8[l][e];
            B[kmap(cb, l, e, 2)][l & 31] = B8[l][e];
        }
        int bad = 0;
        for (int l = 0; l < 64; ++l) for (int r = 0; r < 16; ++r) {
            int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), col = l & 31, s = 0;
            for (int k = 0; k < 32; ++k) s += A[row][k] * B[k][col];
            bad += s != D[l * 16 + r];
        }
        printf("32x32x32 candA=%d candB=%d mismatches=%d\n", ca, cb, bad);
    }
    return 0;
}
