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

// The extra per-lane constants of hb_quad_cfb8_step2 (tried in round 5,
// not shipped: 1,435 vs 1,512 clocks per step here, but no gain in the
// prove kernel -- DESIGN.md 5.3).
struct QuadLane2 {
    QuadLane q;
    u32 lbm, selm;    // m = -q mod 4: column q's round-2 term from column 0 is T_m[byte m of column 0]
    u32 not0, not3;   // 0 on lane q = 0 / q = 3, else ~0
    u32 k15;          // byte 15 of round key 0, at bit 8
};
__device__ __forceinline__ QuadLane2 hb_quad_lane2(const LaneTab &L, u32 rk0_3) {
    const u32 q = hb_lane_id() & 3u;
    QuadLane2 Q;
    Q.q = hb_quad_lane(L);
    const u32 m = (4u - q) & 3u;
    Q.lbm = m == 0 ? L.lb[0] : m == 1 ? L.lb[1] : m == 2 ? L.lb[2] : L.lb[3];
    Q.selm = 0x0c020000u | ((4u + m) << 8);
    Q.not0 = q == 0 ? 0u : ~0u;
    Q.not3 = q == 3 ? 0u : ~0u;
    Q.k15 = (rk0_3 >> 24) << 8;
    return Q;
}

// hb_quad_cfb8_step with rounds 1 and 2 taken off the serial chain.  The next
// step's register is this one shifted by a byte, the new ciphertext byte c
// entering at register byte 15 (column 3, row 3).  c reaches round 1 only
// through T3 into column 0, and round 2 only through column 0's four bytes,
// one into each column (column q's term T_m[byte m of column 0], m = -q mod
// 4).  So while this step's chain runs, the next step's rounds 1 and 2 are
// computed without c (hb_quad_pre: A = round-1 column 0 less its T3 term, on
// every lane; B = round-2 column q less its column-0 term), and on the chain
// c costs two dependent lookups (T3, then T_m) and two XORs instead of two
// quad rounds and the register shift: 1,3xx instead of 1,468 clocks per step
// (scripts/ubench_latency.hip).  State between steps: s = this step's
// register (column q), cu = the previous step's output word whose byte 1 is
// c ^ rk0 byte 15 (the T3 index), A and B.  A fresh evaluation (register 0)
// starts from s = 0, cu = k15 (c = 0) and (A, B) = hb_quad_pre(0).
__device__ __forceinline__ void hb_quad_pre(const QuadLane2 &Q, const u32 *rkq, u32 s, u32 &A, u32 &B) {
    const u32 nx = hb_qdpp<HB_QP(1, 2, 3, 0)>(s);
    const u32 w = hb_perm(Q.q.q3 ? 0u : nx, s, Q.q.sels) ^ rkq[0];   // next register, byte 15 = 0, ^ rk0
    const u32 a = hb_t<0, 0>(Q.q.L, w), b = hb_t<1, 1>(Q.q.L, w), c = hb_t<2, 2>(Q.q.L, w);
    const u32 d = hb_t<3, 3>(Q.q.L, w) & Q.not3;                   // lane 3's T3: the byte c enters
    const u32 x = hb_xor3(a, rkq[1], hb_qdpp<HB_QP(1, 2, 3, 0)>(b));
    const u32 o1 = hb_xor3(x, hb_qdpp<HB_QP(2, 3, 0, 1)>(c), hb_qdpp<HB_QP(3, 0, 1, 2)>(d));
    A = hb_qdpp<HB_QP(0, 0, 0, 0)>(o1);
    // round 2 without column 0's contributions (lane 0's lookups)
    const u32 a2 = hb_t<0, 0>(Q.q.L, o1) & Q.not0, b2 = hb_t<1, 1>(Q.q.L, o1) & Q.not0;
    const u32 c2 = hb_t<2, 2>(Q.q.L, o1) & Q.not0, d2 = hb_t<3, 3>(Q.q.L, o1) & Q.not0;
    const u32 y = hb_xor3(a2, rkq[2], hb_qdpp<HB_QP(1, 2, 3, 0)>(b2));
    B = hb_xor3(y, hb_qdpp<HB_QP(2, 3, 0, 1)>(c2), hb_qdpp<HB_QP(3, 0, 1, 2)>(d2));
}

template <int NR>
__device__ __forceinline__ void hb_quad_cfb8_step2(const QuadLane2 &Q, const u32 *rkq, const u32 *rk, u32 &s, u32 &cu,
                                                   u32 &A, u32 &B, u32 pk) {
    // the chain: c into rounds 1 and 2
    const u32 o10 = A ^ hb_t<1, 3>(Q.q.L, cu);
    u32 w = B ^ hb_tab_ld(Q.q.L.tab, hb_perm(o10, Q.lbm, Q.selm));
    // off the chain: the next step's rounds 1 and 2 from this register
    u32 A2, B2;
    hb_quad_pre(Q, rkq, s, A2, B2);
    HB_UNROLL
    for (int r = 3; r <= NR - 2; ++r) w = hb_quad_round(Q.q.L, w, rkq[r]);
    u32 x = hb_tab_ld(Q.q.L.tab, hb_perm(w, Q.q.lbq, Q.q.selq));
    x ^= hb_qdpp<HB_QP(1, 0, 3, 2)>(x);
    x = hb_xor3(x, hb_qdpp<HB_QP(2, 3, 0, 1)>(x), rk[4 * (NR - 1)]);
    const u32 t = hb_t<0, 0>(Q.q.L, x);
    const u32 u = hb_xor3(t, pk, rk[4 * NR] << 8);     // byte 1: the ciphertext byte
    cu = hb_xor3(t, pk ^ Q.k15, rk[4 * NR] << 8);      // byte 1: ciphertext ^ rk0 byte 15
    const u32 nx = hb_qdpp<HB_QP(1, 2, 3, 0)>(s);
    s = hb_perm(Q.q.q3 ? u : nx, s, Q.q.sels);
    A = A2;
    B = B2;
}

// The CFB-8 state a quad carries from step to step.
struct QuadCfb {
    u32 s, cu, A, B;
};

__device__ __forceinline__ u32 quad_round(const LaneTab &L, u32 w, u32 rk) {
    const u32 a = hb_t<0, 0>(L, w), b = hb_t<1, 1>(L, w), c = hb_t<2, 2>(L, w), d = hb_t<3, 3>(L, w);
    const u32 x = hb_xor3(a, rk, qdpp<QP(1, 2, 3, 0)>(b));
    return hb_xor3(x, qdpp<QP(2, 3, 0, 1)>(c), qdpp<QP(3, 0, 1, 2)>(d));
}

// variant: the DPP gathers folded into VOP2 XORs (v_xor_b32 with a DPP
// source): 4 VALU instructions per round instead of 3 DPP moves + 2 XOR3
template <int CTRL>
__device__ __forceinline__ u32 xdpp(u32 acc, u32 x) {   // acc ^ x(lane from CTRL)
    return acc ^ (u32)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ u32 quad_round3(const LaneTab &L, u32 w, u32 rk) {
    const u32 a = hb_t<0, 0>(L, w), b = hb_t<1, 1>(L, w), c = hb_t<2, 2>(L, w), d = hb_t<3, 3>(L, w);
    u32 x = a ^ rk;
    x = xdpp<QP(1, 2, 3, 0)>(x, b);
    x = xdpp<QP(2, 3, 0, 1)>(x, c);
    return xdpp<QP(3, 0, 1, 2)>(x, d);
}
template <int NR>
__device__ __forceinline__ void cfb8_step3(const QuadLane &Q, const u32 *rkq, const u32 *rk, u32 &s, u32 pk) {
    u32 w = s ^ rkq[0];
    for (int r = 1; r <= NR - 2; ++r) w = quad_round3(Q.L, w, rkq[r]);
    u32 x = hb_tab_ld(Q.L.tab, hb_perm(w, Q.lbq, Q.selq));
    x = xdpp<QP(1, 0, 3, 2)>(x, x);
    x = xdpp<QP(2, 3, 0, 1)>(x ^ rk[4 * (NR - 1)], x);
    const u32 u = hb_xor3(hb_t<0, 0>(Q.L, x), pk, rk[4 * NR] << 8);
    const u32 nx = hb_qdpp<HB_QP(1, 2, 3, 0)>(s);
    s = hb_perm(Q.q3 ? u : nx, s, Q.sels);
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
    for (int i = threadIdx.x; i < HB_TAB_BYTES / 4; i += blockDim.x) lds[i] = init[(i >> 5) & 4095] ^ (u32)(i >> 5) * 2654435761u;   // same in all 32 replicas
    __syncthreads();
    const u32 lane = threadIdx.x & 63;
    LaneTab L;
    L.tab = (const char *)lds;
    for (int t = 0; t < 4; ++t) L.lb[t] = ((u32)(t >> 1) << 16) | ((u32)(t & 1) * 128u) | ((lane & 31u) * 4u);
    u32 x = init[lane], y = init[64 + (which >= 9 ? lane >> 2 : lane)];
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
        u32 sr = 0;
        for (int i = 0; i < N_IT / 16; ++i) hb_quad_cfb8_step<14>(Q, rkq, rkv, sr, y + (u32)i);
        x = sr;
        break;
    }
    case 10: {   // quad CFB-8 step with rounds 1-2 off the chain (hb_quad_cfb8_step2)
        u32 rkv[60], rkq[15];
        for (int i = 0; i < 60; ++i) rkv[i] = __builtin_amdgcn_readfirstlane(init[200 + i]);
        const QuadLane2 Q = hb_quad_lane2(L, rkv[3]);
        const u32 q = lane & 3u;
        for (int r = 0; r <= 14; ++r) rkq[r] = rkv[4 * r + q];
        QuadCfb st{0u, Q.k15, 0u, 0u};
        hb_quad_pre(Q, rkq, 0u, st.A, st.B);
        for (int i = 0; i < N_IT / 16; ++i) hb_quad_cfb8_step2<14>(Q, rkq, rkv, st.s, st.cu, st.A, st.B, y + (u32)i);
        x = st.s;
        break;
    }
    case 11: {   // 8 independent bitop3 chains: VALU issue rate of one wave
        u32 v0 = x, v1 = x + 1, v2 = x + 2, v3 = x + 3, v4 = x + 4, v5 = x + 5, v6 = x + 6, v7 = x + 7;
        for (int i = 0; i < N_IT / 8; ++i) {
            v0 = hb_xor3(v0, y, (u32)i); v1 = hb_xor3(v1, y, (u32)i); v2 = hb_xor3(v2, y, (u32)i);
            v3 = hb_xor3(v3, y, (u32)i); v4 = hb_xor3(v4, y, (u32)i); v5 = hb_xor3(v5, y, (u32)i);
            v6 = hb_xor3(v6, y, (u32)i); v7 = hb_xor3(v7, y, (u32)i);
        }
        x = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
        break;
    }
    case 12: {   // 8 independent perm + ds_read chains: LDS issue rate of one wave
        u32 v0 = x, v1 = x + 1, v2 = x + 2, v3 = x + 3, v4 = x + 4, v5 = x + 5, v6 = x + 6, v7 = x + 7;
        for (int i = 0; i < N_IT / 8; ++i) {
            v0 = hb_t<1, 0>(L, v0); v1 = hb_t<1, 1>(L, v1); v2 = hb_t<1, 2>(L, v2); v3 = hb_t<1, 3>(L, v3);
            v4 = hb_t<2, 0>(L, v4); v5 = hb_t<2, 1>(L, v5); v6 = hb_t<2, 2>(L, v6); v7 = hb_t<2, 3>(L, v7);
        }
        x = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
        break;
    }
    case 13: {   // 8 independent mov_dpp + add chains
        u32 v0 = x, v1 = x + 1, v2 = x + 2, v3 = x + 3, v4 = x + 4, v5 = x + 5, v6 = x + 6, v7 = x + 7;
        for (int i = 0; i < N_IT / 8; ++i) {
            v0 = qdpp<QP(1, 2, 3, 0)>(v0) + 1u; v1 = qdpp<QP(1, 2, 3, 0)>(v1) + 1u; v2 = qdpp<QP(1, 2, 3, 0)>(v2) + 1u;
            v3 = qdpp<QP(1, 2, 3, 0)>(v3) + 1u; v4 = qdpp<QP(1, 2, 3, 0)>(v4) + 1u; v5 = qdpp<QP(1, 2, 3, 0)>(v5) + 1u;
            v6 = qdpp<QP(1, 2, 3, 0)>(v6) + 1u; v7 = qdpp<QP(1, 2, 3, 0)>(v7) + 1u;
        }
        x = v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7;
        break;
    }
    case 14: {   // step without rounds 1-2 and without the precompute (timing only)
        u32 rkv[60], rkq[15];
        for (int i = 0; i < 60; ++i) rkv[i] = __builtin_amdgcn_readfirstlane(init[200 + i]);
        const QuadLane Q = hb_quad_lane(L);
        const u32 q = lane & 3u;
        for (int r = 0; r <= 14; ++r) rkq[r] = rkv[4 * r + q];
        u32 sr = 0;
        for (int i = 0; i < N_IT / 16; ++i) {
            u32 w = sr ^ rkq[0];
            for (int r = 3; r <= 12; ++r) w = hb_quad_round(Q.L, w, rkq[r]);
            u32 xx = hb_tab_ld(Q.L.tab, hb_perm(w, Q.lbq, Q.selq));
            xx ^= hb_qdpp<HB_QP(1, 0, 3, 2)>(xx);
            xx = hb_xor3(xx, hb_qdpp<HB_QP(2, 3, 0, 1)>(xx), rkv[52]);
            const u32 u = hb_xor3(hb_t<0, 0>(Q.L, xx), y + (u32)i, rkv[56] << 8);
            const u32 nx = hb_qdpp<HB_QP(1, 2, 3, 0)>(sr);
            sr = hb_perm(Q.q3 ? u : nx, sr, Q.sels);
        }
        x = sr;
        break;
    }
    case 15: {   // quad CFB-8 step with DPP folded into the XORs
        const QuadLane Q = hb_quad_lane(L);
        u32 rkv[60], rkq[15];
        for (int i = 0; i < 60; ++i) rkv[i] = __builtin_amdgcn_readfirstlane(init[200 + i]);
        const u32 q = lane & 3u;
        for (int r = 0; r <= 14; ++r) rkq[r] = rkv[4 * r + q];
        u32 sr = 0;
        for (int i = 0; i < N_IT / 16; ++i) cfb8_step3<14>(Q, rkq, rkv, sr, y + (u32)i);
        x = sr;
        break;
    }
    case 16:   // quad round, DPP folded
        for (int i = 0; i < N_IT; ++i) x = quad_round3(L, x, rk);
        break;
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
                           "quad cfb8 step/16", "cfb8 step2/16", "8x bitop3 /8", "8x perm+read /8",
                           "8x dpp+add /8", "step -2 rounds/16", "step dppxor/16", "quad_round3"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int w = 0; w < 17; ++w) {
            hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, init, out, cyc, w);
            unsigned long long c[2];
            hipMemcpy(c, cyc, 16, hipMemcpyDeviceToHost);
            const double ns = c[1] * 10.0;   // s_memrealtime: 100 MHz
            printf("%-16s %8.1f clk/it %8.2f ns/it  (clock %.0f MHz)\n", names[w], (double)c[0] / N_IT, ns / N_IT,
                   c[0] / (ns * 1e-3));
        }
    }
    {   // step2 == step, bit for bit, after 256 steps
        u32 a[64], b[64];
        hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, init, out, cyc, 9);
        hipMemcpy(a, out, sizeof a, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, init, out, cyc, 10);
        hipMemcpy(b, out, sizeof b, hipMemcpyDeviceToHost);
        int same = 0;
        for (int i = 0; i < 64; ++i) same += a[i] == b[i];
        printf("step2 registers equal to step: %d of 64 lanes (lane 0: %08x %08x)\n", same, a[0], b[0]);
        hipLaunchKernelGGL(k_bench, dim3(1), dim3(64), 0, 0, init, out, cyc, 15);
        hipMemcpy(b, out, sizeof b, hipMemcpyDeviceToHost);
        same = 0;
        for (int i = 0; i < 64; ++i) same += a[i] == b[i];
        printf("dpp-xor step registers equal to step: %d of 64 lanes\n", same);
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
