// ubench_latency.hip -- dependent-chain latencies of the instructions the
// prove's quad PRF engine chains (one wave, nothing else on the GPU):
// ds_read_b32 behind a v_perm address, DPP moves, v_bitop3, a whole quad
// T-table round and a whole quad CFB-8 step.  Experiment code, not shipped.
//   hipcc --offload-arch=gfx950 -O3 -I heartbeat_amd/csrc scripts/ubench_latency.hip -o /tmp/ubl
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include "hb_kernels.hpp"
thread_local bool hb_load_only = false;

#define N_IT 4096
#define QP(a, b, c, d) ((a) | ((b) << 2) | ((c) << 4) | ((d) << 6))

template <int CTRL>
__device__ __forceinline__ u32 qdpp(u32 x) { return hb_qdpp<CTRL>(x); }

__device__ __forceinline__ u32 quad_round(const LaneTab &L, u32 w, u32 rk) {
    const u32 a = hb_t<0, 0>(L, w), b = hb_t<1, 1>(L, w), c = hb_t<2, 2>(L, w), d = hb_t<3, 3>(L, w);
    const u32 x = hb_xor3(a, rk, qdpp<QP(1, 2, 3, 0)>(b));
    return hb_xor3(x, qdpp<QP(2, 3, 0, 1)>(c), qdpp<QP(3, 0, 1, 2)>(d));
}

// variant: one lookup per lane chain but the three DPP gathers done as
// one xor tree level (a^b' and c'^d' in parallel)
__device__ __forceinline__ u32 quad_round2(const LaneTab &L, u32 w, u32 rk) {
    const u32 a = hb_t<0, 0>(L, w), b = hb_t<1, 1>(L, w), c = hb_t<2, 2>(L, w), d = hb_t<3, 3>(L, w);
    const u32 bc = qdpp<QP(1, 2, 3, 0)>(b), cc = qdpp<QP(2, 3, 0, 1)>(c), dc = qdpp<QP(3, 0, 1, 2)>(d);
    return hb_xor3(a ^ rk, bc, cc ^ dc);
}

__global__ __launch_bounds__(1024) void k_bench(const u32 *init, u32 *out, unsigned long long *cyc, int which) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_TAB_BYTES / 4];
    for (int i = threadIdx.x; i < HB_TAB_BYTES / 4; i += blockDim.x) lds[i] = init[i & 4095] ^ (u32)i * 2654435761u;
    __syncthreads();
    const u32 lane = threadIdx.x & 63;
    LaneTab L;
    L.tab = (const char *)lds;
    for (int t = 0; t < 4; ++t) L.lb[t] = ((u32)(t >> 1) << 16) | ((u32)(t & 1) * 128u) | ((lane & 31u) * 4u);
    u32 x = init[lane], y = init[64 + lane];
    const u32 rk = init[128];
    __builtin_amdgcn_s_barrier();
    const unsigned long long c0 = __builtin_readcyclecounter();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    switch (which) {
    case 0:   // v_perm address + ds_read_b32
        for (int i = 0; i < N_IT; ++i) x = hb_t<1, 0>(L, x);
        break;
    case 1:   // ds_read_b32 pointer chase (address = value & mask, one v_and)
        for (int i = 0; i < N_IT; ++i) x = hb_tab_ld(L.tab, x & 0x1fffcu);
        break;
    case 2:   // mov_dpp quad_perm, dependent
        for (int i = 0; i < N_IT; ++i) x = qdpp<QP(1, 2, 3, 0)>(x) + 1u;
        break;
    case 3:   // v_bitop3 dependent
        for (int i = 0; i < N_IT; ++i) x = hb_xor3(x, y, (u32)i);
        break;
    case 4:   // quad round
        for (int i = 0; i < N_IT; ++i) x = quad_round(L, x, rk);
        break;
    case 5:   // quad round, flatter xor tree
        for (int i = 0; i < N_IT; ++i) x = quad_round2(L, x, rk);
        break;
    case 6:   // 4 independent lookups then xor (no dpp): LDS issue of 4 + latency
        for (int i = 0; i < N_IT; ++i) {
            const u32 a = hb_t<0, 0>(L, x), b = hb_t<1, 1>(L, x), c = hb_t<2, 2>(L, x), d = hb_t<3, 3>(L, x);
            x = hb_xor3(a, b, c ^ d);
        }
        break;
    case 7:   // ds_bpermute chain
        for (int i = 0; i < N_IT; ++i) x = (u32)__builtin_amdgcn_ds_bpermute((int)((x & 63u) << 2), (int)x) + 1u;
        break;
    case 9: {   // quad CFB-8 step (AES-256), the prove's v chain
        const QuadLane Q = hb_quad_lane(L);
        u32 rkv[60], rkq[15];
        for (int i = 0; i < 60; ++i) rkv[i] = __builtin_amdgcn_readfirstlane(init[200 + i]);
        const u32 q = lane & 3u;
        for (int r = 0; r <= 14; ++r) rkq[r] = rkv[4 * r + q];
        u32 sr = x;
        for (int i = 0; i < N_IT / 16; ++i) hb_quad_cfb8_step<14>(Q, rkq, rkv, sr, y + (u32)i);
        x = sr;
        break;
    }
    case 8:   // 16 independent lookups then xor (lane engine round shape)
        for (int i = 0; i < N_IT; ++i) {
            u32 acc = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const u32 w = x + (u32)k * 0x01010101u;
                acc ^= hb_xor3(hb_t<0, 0>(L, w), hb_t<1, 1>(L, w), hb_t<2, 2>(L, w) ^ hb_t<3, 3>(L, w));
            }
            x = acc;
        }
        break;
    }
    const unsigned long long c1 = __builtin_readcyclecounter();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    out[threadIdx.x] = x;
    if (threadIdx.x == 0) {
        cyc[0] = c1 - c0;
        cyc[1] = r1 - r0;
    }
    if (threadIdx.x == blockDim.x - 64) {
        cyc[2] = c1 - c0;
    }
}

int main() {
    u32 *init, *out;
    unsigned long long *cyc;
    hipMalloc(&init, 4096 * 4);
    hipMalloc(&out, 1024 * 4);
    hipMalloc(&cyc, 32);
    u32 h[4096];
    srand(7);
    for (int i = 0; i < 4096; ++i) h[i] = ((u32)rand() << 16) ^ (u32)rand();
    hipMemcpy(init, h, sizeof h, hipMemcpyHostToDevice);
    const char *names[] = {"perm+ds_read", "ds_read chase", "mov_dpp+add", "bitop3", "quad_round",
                           "quad_round2", "4 lookups+xor", "ds_bpermute+add", "16 lookups+xor",
                           "quad cfb8 step/16"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int w = 0; w < 10; ++w) {
            hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, init, out, cyc, w);
            unsigned long long c[2];
            hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
            const double ns = c[1] * 10.0;   // s_memrealtime: 100 MHz
            printf("%-16s %8.1f clk/it %8.2f ns/it  (clock %.0f MHz)\n", names[w], (double)c[0] / N_IT, ns / N_IT,
                   c[0] / (ns * 1e-3));
        }
    }
    // the CFB-8 step with 1..4 waves per SIMD (a workgroup's waves are spread
    // over the CU's four SIMDs)
    for (int nw = 1; nw <= 16; nw *= 2) {
        hipLaunchKernelGGL(k_bench, dim3(1), dim3(64 * nw), 0, 0, init, out, cyc, 9);
        unsigned long long c[3];
        hipMemcpy(c, cyc, 24, hipMemcpyDeviceToHost);
        printf("cfb8 step, %2d waves: %8.1f clk/step (first wave) %8.1f (last wave)\n", nw, (double)c[0] * 16 / N_IT,
               (double)c[2] * 16 / N_IT);
    }
    return 0;
}
