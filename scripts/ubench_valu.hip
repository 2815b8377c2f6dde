// VALU issue rate per instruction form on gfx950 (inline asm, 16 independent
// chains per lane), in lane-ops per clock per CU (the VALU's 128/clk nominal).
// Drives the cost model of the bitsliced AES engine and the T-table address
// arithmetic.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_valu.hip -o scripts/ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef unsigned int u32;
#define CK(x) (void)(x)

#define OP_XOR      "v_xor_b32 %0, %1, %0"
#define OP_XOR64    "v_xor_b32_e64 %0, %1, %0"
#define OP_AND      "v_and_b32 %0, %1, %0"
#define OP_LSHL     "v_lshlrev_b32 %0, 3, %0"
#define OP_BITOP3   "v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96"
#define OP_BITOP3_2 "v_bitop3_b32 %0, %1, %0, %0 bitop3:0x96"
#define OP_BITOP3_S "v_bitop3_b32 %0, %1, %0, s0 bitop3:0x96"
#define OP_PERM     "v_perm_b32 %0, %1, %2, %0"
#define OP_PERM_S   "v_perm_b32 %0, %0, %1, s0"
#define OP_ADD3     "v_add3_u32 %0, %1, %2, %0"
#define OP_XOR3     "v_xad_u32 %0, %1, %2, %0"
#define OP_FMA      "v_fma_f32 %0, %1, %2, %0"
#define OP_SDWA     "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2"
#define OP_DPP      "v_mov_b32_dpp %0, %1 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
#define OP_XORDPP   "v_xor_b32_dpp %0, %1, %0 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
#define OP_CND      "v_cndmask_b32 %0, %1, %0, vcc"
#define OP_ALIGN    "v_alignbit_b32 %0, %1, %0, 8"

template <int K>
__device__ __forceinline__ void op(u32 &x, u32 a, u32 b) {
    if constexpr (K == 0) asm volatile(OP_XOR : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 1) asm volatile(OP_XOR64 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 2) asm volatile(OP_AND : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 3) asm volatile(OP_LSHL : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 4) asm volatile(OP_BITOP3 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 5) asm volatile(OP_BITOP3_2 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 6) asm volatile(OP_BITOP3_S : "+v"(x) : "v"(a), "v"(b) : "s0");
    else if constexpr (K == 7) asm volatile(OP_PERM : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 8) asm volatile(OP_PERM_S : "+v"(x) : "v"(a), "v"(b) : "s0");
    else if constexpr (K == 9) asm volatile(OP_ADD3 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 10) asm volatile(OP_XOR3 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 11) asm volatile(OP_FMA : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 12) asm volatile(OP_SDWA : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 13) asm volatile(OP_DPP : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 14) asm volatile(OP_XORDPP : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 15) asm volatile(OP_CND : "+v"(x) : "v"(a), "v"(b) : "vcc");
    else if constexpr (K == 16) asm volatile(OP_ALIGN : "+v"(x) : "v"(a), "v"(b));
}

template <int K>
__global__ __launch_bounds__(256) void kv(u32 *out, u32 iters) {
    u32 v[16], c0 = threadIdx.x * 7u, c1 = threadIdx.x * 13u + 5u;
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 0x9E3779B1u + i * 0x85EBCA77u;
    asm volatile("s_mov_b32 s0, 0x05040100\n s_mov_b64 vcc, -1" ::: "s0", "vcc");
    for (u32 it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int i = 0; i < 16; ++i) op<K>(v[i], c0, c1);
    }
    u32 acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= v[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char *names[] = {"v_xor_b32 (VOP2)", "v_xor_b32_e64 (VOP3)", "v_and_b32", "v_lshlrev_b32 imm",
                              "v_bitop3 3 vgpr", "v_bitop3 2 vgpr", "v_bitop3 2 vgpr+sgpr", "v_perm 3 vgpr",
                              "v_perm 2 vgpr+sgpr", "v_add3_u32", "v_xad_u32", "v_fma_f32", "v_mov_sdwa byte",
                              "v_mov_b32_dpp", "v_xor_b32_dpp", "v_cndmask_b32", "v_alignbit_b32"};

template <int K>
static void run(u32 *out, int ncu, int wpc, double ghz) {
    const u32 iters = 2048;
    const int grid = ncu * wpc / 4;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(kv<K>, dim3(grid), dim3(256), 0, 0, out, iters);
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(kv<K>, dim3(grid), dim3(256), 0, 0, out, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)grid * 256 * iters * 8 * 16;
    printf("%-24s %2d waves/CU: %6.1f lane-ops/clk/CU\n", names[K], wpc, ops / (ms * 1e-3) / (ghz * 1e9) / ncu);
}

template <int K>
static void all(u32 *out, int ncu, double ghz) {
    run<K>(out, ncu, 8, ghz);
    run<K>(out, ncu, 16, ghz);
    if constexpr (K + 1 <= 16) all<K + 1>(out, ncu, ghz);
}

int main() {
    hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
    int clk; CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    u32 *out; CK(hipMalloc(&out, 256 * 4 * 256 * 16));
    all<0>(out, p.multiProcessorCount, clk / 1e6);
    return 0;
}
