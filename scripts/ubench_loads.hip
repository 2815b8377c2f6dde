// Request shape of the first-pass MAC's sector loads:
// the same 32 KiB per wave (64 blocks x 512 B, S = 16, 256-bit sectors) read
// with four lane -> address mappings, each its own kernel so that rocprofv3
// --kernel-trace / --pmc split them:
//   mac32  the shipped shape (hb_mfma_block_acc, v_mfma_i32_32x32x32_i8 B
//          operand): lane (h, n) reads 16 B at block n + 32 j + 16 h; each
//          128-B line of a block is touched by 4 instructions, 32 B each
//   mac16  the v_mfma_i32_16x16x64_i8 B operand: lane (q, n), q = l >> 4,
//          reads 16 B at block n + 64 jj + 16 q; 2 instructions per line,
//          64 B each, from lanes n, n+16, n+32, n+48
//   line   8 consecutive lanes read one block's whole 128-B line
//   stream 64 consecutive lanes read 1 KiB contiguous
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_loads.hip -o scripts/ubench_loads
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef unsigned int u32;
typedef unsigned long long u64;
typedef int32_t i32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// one wave per 32 KiB chunk, grid-stride over chunks; 4 loads in flight per batch
template <int P>
__global__ __launch_bounds__(256) void ld_kernel(const unsigned char *data, u64 nchunks, u32 *out) {
    const u32 l = threadIdx.x & 63u;
    const u64 wave = ((u64)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const u64 nwaves = ((u64)gridDim.x * blockDim.x) >> 6;
    i32x4 acc = {0, 0, 0, 0};
    for (u64 ch = wave; ch < nchunks; ch += nwaves) {
        const unsigned char *base = data + ch * 32768ull;
        if constexpr (P == 0) {          // mac32
            const u32 h = l >> 5, n = l & 31u;
#pragma unroll
            for (u32 g = 0; g < 2; ++g) {
                const i32x4 *src = reinterpret_cast<const i32x4 *>(base + (32u * g + n) * 512u + 16u * h);
#pragma unroll
                for (u32 j0 = 0; j0 < 16; j0 += 4) {
                    i32x4 b[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) b[jj] = src[2 * (j0 + jj)];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) acc ^= b[jj];
                }
            }
        } else if constexpr (P == 1) {   // mac16
            const u32 q = l >> 4, n = l & 15u;
#pragma unroll
            for (u32 g = 0; g < 4; ++g) {
                const i32x4 *src = reinterpret_cast<const i32x4 *>(base + (16u * g + n) * 512u + 16u * q);
#pragma unroll
                for (u32 j0 = 0; j0 < 8; j0 += 4) {
                    i32x4 b[4];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) b[jj] = src[4 * (j0 + jj)];
#pragma unroll
                    for (int jj = 0; jj < 4; ++jj) acc ^= b[jj];
                }
            }
        } else if constexpr (P == 2) {   // line: lanes 8m..8m+7 -> block m's line
            const u32 m = l >> 3, q = l & 7u;
#pragma unroll
            for (u32 i = 0; i < 8; ++i) {
                const i32x4 *src = reinterpret_cast<const i32x4 *>(base + (8u * i + m) * 512u + 16u * q);
                i32x4 b[4];
#pragma unroll
                for (int ll = 0; ll < 4; ++ll) b[ll] = src[8 * ll];
#pragma unroll
                for (int ll = 0; ll < 4; ++ll) acc ^= b[ll];
            }
        } else {                         // stream
            const i32x4 *src = reinterpret_cast<const i32x4 *>(base + 16u * l);
#pragma unroll
            for (u32 k0 = 0; k0 < 32; k0 += 4) {
                i32x4 b[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) b[kk] = src[64 * (k0 + kk)];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) acc ^= b[kk];
            }
        }
    }
    const u32 v = (u32)(acc[0] ^ acc[1] ^ acc[2] ^ acc[3]);
    if (v == 0x9e3779b9u) out[0] = v;   // keeps the loads live; practically never stores
}

int main(int argc, char **argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const u64 bytes = (u64)(gib * (1ull << 30)) / 32768ull * 32768ull;
    const u64 nchunks = bytes / 32768ull;
    unsigned char *d;
    u32 *out;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&out, 4));
    CK(hipMemset(d, 0x5a, bytes));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    // 16 waves per CU resident, as in the encode, x 8 rounds
    const int grid = prop.multiProcessorCount * 4 * 8;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const char *names[4] = {"mac32", "mac16", "line", "stream"};
    for (int p = 0; p < 4; ++p) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(a));
            if (p == 0) ld_kernel<0><<<grid, 256>>>(d, nchunks, out);
            if (p == 1) ld_kernel<1><<<grid, 256>>>(d, nchunks, out);
            if (p == 2) ld_kernel<2><<<grid, 256>>>(d, nchunks, out);
            if (p == 3) ld_kernel<3><<<grid, 256>>>(d, nchunks, out);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        printf("%-7s %.3f ms  %.1f GB/s  (%.2f GiB, best of %d)\n", names[p], best, bytes / (best * 1e-3) / 1e9,
               bytes / (double)(1ull << 30), reps);
    }
    CK(hipFree(d));
    return 0;
}
