// Does the vector L1 add lookup throughput beside the LDS?  The byte-0
// T-table AES-256 of hb_lane.hpp (CFB-8-like chains, 16 waves/CU, one chain
// per lane as in the encode) with G of each full round's 16 lookups served by
// global loads of a 1 KiB T0 table (L1-resident: T0[w_c byte 0], the a_c
// terms of hb_aes_round) instead of the LDS image.  Reports byte-0 AES per
// second per CU for G = 0..4; G > 0 pays only if the L1 path's lookups come on
// top of the LDS array's instead of slowing it.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_aes_l1.hip -o /tmp/ubench_aes_l1
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../heartbeat_amd/csrc/hb_lane.hpp"

#define HB_LDS_WORDS (HB_TAB_BYTES / 4)

__device__ __forceinline__ void fill_lds(u32 *lds, const u32 *t0) {
    for (u32 g = threadIdx.x; g < HB_LDS_WORDS / 4; g += blockDim.x) {
        const u32 off = g * 16u;
        const u32 e = (off >> 8) & 0xffu, t = ((off >> 16) << 1) | ((off >> 7) & 1u);
        u32 v = t0[e];
        if (t) v = (v << (8 * t)) | (v >> (32 - 8 * t));
        reinterpret_cast<uint4 *>(lds)[g] = make_uint4(v, v, v, v);
    }
    __syncthreads();
}

struct Args {
    u32 rk[60];
    const u32 *t0;
    u32 *out;
    u32 iters;
};

template <int G>
__device__ __forceinline__ u32 ta(const LaneTab &L, const u32 *__restrict__ gt, u32 w, int c) {
    if (c < G) return gt[w & 0xffu];
    return hb_t<0, 0>(L, w);
}

template <int G>
__device__ __forceinline__ void round_g(const LaneTab &L, const u32 *__restrict__ gt, const u32 *rk, u32 &w0, u32 &w1,
                                        u32 &w2, u32 &w3) {
    // global lookups first in program order so their latency overlaps the LDS ones
    u32 a0 = ta<G>(L, gt, w0, 0), a1 = ta<G>(L, gt, w1, 2), a2 = ta<G>(L, gt, w2, 1), a3 = ta<G>(L, gt, w3, 3);
    u32 b0 = hb_t<1, 1>(L, w1), c0 = hb_t<2, 2>(L, w2), d0 = hb_t<3, 3>(L, w3);
    u32 b1 = hb_t<1, 1>(L, w2), c1 = hb_t<2, 2>(L, w3), d1 = hb_t<3, 3>(L, w0);
    u32 b2 = hb_t<1, 1>(L, w3), c2 = hb_t<2, 2>(L, w0), d2 = hb_t<3, 3>(L, w1);
    u32 b3 = hb_t<1, 1>(L, w0), c3 = hb_t<2, 2>(L, w1), d3 = hb_t<3, 3>(L, w2);
    w0 = hb_xor3(hb_xor3(a0, b0, c0), d0, rk[0]);
    w1 = hb_xor3(hb_xor3(a1, b1, c1), d1, rk[1]);
    w2 = hb_xor3(hb_xor3(a2, b2, c2), d2, rk[2]);
    w3 = hb_xor3(hb_xor3(a3, b3, c3), d3, rk[3]);
}

template <int G, int WG, int OCC>
__global__ __launch_bounds__(WG, OCC) void kaes(Args A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    fill_lds(lds, A.t0);
    const u32 r4 = (threadIdx.x & 31u) * 4u;
    const LaneTab L{(const char *)lds, {r4, 128u + r4, 0x10000u | r4, 0x10000u | (128u + r4)}};
    const u32 *__restrict__ gt = A.t0;
    const u32 gid = blockIdx.x * WG + threadIdx.x;
    u32 s0 = gid * 2654435761u, s1 = 7u, s2 = gid, s3 = 0x12345678u;
    for (u32 it = 0; it < A.iters; ++it) {
        u32 w0 = s0 ^ A.rk[0], w1 = s1 ^ A.rk[1], w2 = s2 ^ A.rk[2], w3 = s3 ^ A.rk[3];
#pragma unroll
        for (int r = 1; r <= 12; ++r) round_g<G>(L, gt, A.rk + 4 * r, w0, w1, w2, w3);
        u32 a = hb_t<0, 0>(L, w0), b = hb_t<1, 1>(L, w1), c = hb_t<2, 2>(L, w2), d = hb_t<3, 3>(L, w3);
        u32 x = hb_xor3(hb_xor3(a, b, c), d, A.rk[52]) & 0xffu;
        u32 o = ((hb_t<0, 0>(L, x) >> 8) ^ A.rk[56]) & 0xffu;
        s0 = hb_alignbit(s1, s0, 8);
        s1 = hb_alignbit(s2, s1, 8);
        s2 = hb_alignbit(s3, s2, 8);
        s3 = (s3 >> 8) | (o << 24);
    }
    A.out[gid] = s3 ^ s0;
}

static u32 T0[256];
static void make_t0() {
    unsigned char sbox[256];
    auto xt = [](unsigned x) { return ((x << 1) ^ ((x & 0x80) ? 0x1b : 0)) & 0xff; };
    auto mul = [&](unsigned a, unsigned b) { unsigned r = 0; while (b) { if (b & 1) r ^= a; a = xt(a); b >>= 1; } return r; };
    for (int x = 0; x < 256; ++x) {
        unsigned inv = 0;
        if (x) for (unsigned y = 1; y < 256; ++y) if (mul(x, y) == 1) { inv = y; break; }
        unsigned s = inv, r = inv;
        for (int i = 0; i < 4; ++i) { r = ((r << 1) | (r >> 7)) & 0xff; s ^= r; }
        sbox[x] = (unsigned char)(s ^ 0x63);
    }
    for (int x = 0; x < 256; ++x) {
        unsigned s = sbox[x], s2 = xt(s), s3 = s2 ^ s;
        T0[x] = s2 | (s << 8) | (s << 16) | (s3 << 24);
    }
}

static u32 ref_G0 = 0;

template <int G>
static void run(Args A, int grid, int ncu, u32 *host) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((kaes<G, 1024, 4>), dim3(grid), dim3(1024), 0, 0, A);
    (void)hipEventRecord(e0, 0);
    for (int rep = 0; rep < 5; ++rep) hipLaunchKernelGGL((kaes<G, 1024, 4>), dim3(grid), dim3(1024), 0, 0, A);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    (void)hipMemcpy(host, A.out, (size_t)grid * 1024 * 4, hipMemcpyDeviceToHost);
    u32 h = 0;
    for (int i = 0; i < grid * 1024; ++i) h = h * 31u + host[i];
    if (G == 0) ref_G0 = h;
    const double aes = (double)grid * 1024 * A.iters;
    printf("G=%d global lookups/round  ms=%8.3f  AES/s/CU=%.4e  rel=%.4f  checksum %s\n", G, ms, aes / (ms * 1e-3) / ncu,
           0.0, h == ref_G0 ? "ok" : "MISMATCH");
}

int main() {
    make_t0();
    u32 *t0, *out;
    (void)hipMalloc(&t0, 1024);
    (void)hipMemcpy(t0, T0, 1024, hipMemcpyHostToDevice);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    (void)hipMalloc(&out, (size_t)ncu * 1024 * 4);
    u32 *host = (u32 *)malloc((size_t)ncu * 1024 * 4);
    Args A;
    for (int i = 0; i < 60; ++i) A.rk[i] = 0x9e3779b9u * (i + 1);
    A.t0 = t0;
    A.out = out;
    A.iters = 4096;
    for (int pass = 0; pass < 2; ++pass) {
        run<0>(A, ncu, ncu, host);
        run<1>(A, ncu, ncu, host);
        run<2>(A, ncu, ncu, host);
        run<3>(A, ncu, ncu, host);
        run<4>(A, ncu, ncu, host);
    }
    return 0;
}
