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
#define OP_XOR_S    "v_xor_b32 %0, s0, %0"
#define OP_BITOP3_I "v_bitop3_b32 %0, %1, %0, 1 bitop3:0xea"
#define OP_ANDOR    "v_and_or_b32 %0, %0, %1, %2"
#define OP_OR3      "v_or3_b32 %0, %0, %1, %2"
#define OP_ADD      "v_add_u32 %0, %1, %0"
#define OP_MUL24    "v_mul_u32_u24 %0, %1, %0"
#define OP_MAD24    "v_mad_u32_u24 %0, %1, %2, %0"
#define OP_LSHLOR   "v_lshl_or_b32 %0, %0, 8, %1"
#define OP_BFE      "v_bfe_u32 %0, %0, 8, 8"
#define OP_CVTUB    "v_cvt_f32_ubyte1 %0, %0"
#define OP_PKADD    "v_pk_add_u16 %0, %1, %0"
#define OP_LSHR     "v_lshrrev_b32 %0, 8, %0"
#define OP_AND_S    "v_and_b32 %0, s0, %0"
#define OP_AND_L    "v_and_b32 %0, 0xff00, %0"
#define OP_BITOP3_M "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xea"
#define OP_MAD64    "v_mad_u64_u32 v[40:41], vcc, %0, %1, 0"
#define OP_LSHLADD  "v_lshl_add_u32 %0, %0, 2, %1"
#define OP_XOR_I    "v_xor_b32 %0, 7, %0"
#define OP_PKMAD    "v_pk_mad_u16 %0, %0, %1, %2 op_sel:[1,0,0] op_sel_hi:[1,0,1]"
#define OP_PKMUL    "v_pk_mul_lo_u16 %0, %0, %1"
#define OP_PKLSHR   "v_pk_lshrrev_b16 %0, %1, %0"
#define OP_BITOP3_D "v_bitop3_b32 %0, %0, %1, %2 bitop3:0xea"
#define OP_BITOP3_SI "v_bitop3_b32 %0, %0, s0, %1 bitop3:0xea"

template <int K>
__device__ __forceinline__ void op(u32 &x, u32 a, u32 b, u32 y1 = 0, u32 y2 = 0) {
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
    else if constexpr (K == 17) asm volatile(OP_XOR_S : "+v"(x) : "v"(a), "v"(b) : "s0");
    else if constexpr (K == 18) asm volatile(OP_BITOP3_I : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 19) asm volatile(OP_ANDOR : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 20) asm volatile(OP_OR3 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 21) asm volatile(OP_ADD : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 22) asm volatile(OP_MUL24 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 23) asm volatile(OP_MAD24 : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 24) asm volatile(OP_LSHLOR : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 25) asm volatile(OP_BFE : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 26) asm volatile(OP_CVTUB : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 27) asm volatile(OP_PKADD : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 28) asm volatile(OP_LSHR : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 29) asm volatile(OP_AND_S : "+v"(x) : "v"(a), "v"(b) : "s0");
    else if constexpr (K == 30) asm volatile(OP_AND_L : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 31) asm volatile(OP_BITOP3_M : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 32) asm volatile(OP_MAD64 : "+v"(x) : "v"(a), "v"(b) : "v40", "v41", "vcc");
    else if constexpr (K == 33) asm volatile(OP_LSHLADD : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 34) asm volatile(OP_XOR_I : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 35) asm volatile(OP_BITOP3_SI : "+v"(x) : "v"(a), "v"(b) : "s0");
    else if constexpr (K == 36) asm volatile(OP_PKMAD : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 37) asm volatile(OP_PKMUL : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 38) asm volatile(OP_PKLSHR : "+v"(x) : "v"(a), "v"(b));
    else if constexpr (K == 39) asm volatile(OP_BITOP3_D : "+v"(x) : "v"(y1), "v"(y2));
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
            for (int i = 0; i < 16; ++i) op<K>(v[i], c0, c1, v[(i + 5) & 15], v[(i + 11) & 15]);
    }
    u32 acc = 0;
    for (int i = 0; i < 16; ++i) acc ^= v[i];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

static const char *names[] = {"v_xor_b32 (VOP2)", "v_xor_b32_e64 (VOP3)", "v_and_b32", "v_lshlrev_b32 imm",
                              "v_bitop3 3 vgpr", "v_bitop3 2 vgpr", "v_bitop3 2 vgpr+sgpr", "v_perm 3 vgpr",
                              "v_perm 2 vgpr+sgpr", "v_add3_u32", "v_xad_u32", "v_fma_f32", "v_mov_sdwa byte",
                              "v_mov_b32_dpp", "v_xor_b32_dpp", "v_cndmask_b32", "v_alignbit_b32",
                              "v_xor_b32 vop2 sgpr", "v_bitop3 inline const", "v_and_or_b32 3 vgpr", "v_or3_b32 3 vgpr", "v_add_u32 vop2", "v_mul_u32_u24", "v_mad_u32_u24", "v_lshl_or_b32 imm", "v_bfe_u32 imm", "v_cvt_f32_ubyte1", "v_pk_add_u16", "v_lshrrev_b32 imm", "v_and_b32 vop2 sgpr", "v_and_b32 literal", "v_bitop3 andor 3 vgpr", "v_mad_u64_u32", "v_lshl_add_u32 imm", "v_xor_b32 inline", "v_bitop3 andor sgpr", "v_pk_mad_u16 opsel", "v_pk_mul_lo_u16", "v_pk_lshrrev_b16", "v_bitop3 andor chains"};

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

#ifndef HB_FIRST_OP
#define HB_FIRST_OP 0
#endif
template <int K>
static void all(u32 *out, int ncu, double ghz) {
    run<K>(out, ncu, 8, ghz);
    run<K>(out, ncu, 16, ghz);
    if constexpr (K + 1 <= 39) all<K + 1>(out, ncu, ghz);
}

int main() {
    hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
    int clk; CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    u32 *out; CK(hipMalloc(&out, 256 * 4 * 256 * 16));
    all<HB_FIRST_OP>(out, p.multiProcessorCount, clk / 1e6);
    return 0;
}
