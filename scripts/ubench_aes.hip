// LDS-lookup throughput of the byte-0 T-table AES-256 (hb_lane.hpp) on gfx950
// as a function of independent AES chains per lane (N) and waves per CU.
// Each lane runs CFB-8-like chains: the next input is the register shifted by
// one byte with the output byte inserted.  Reports LDS lookups per clock per
// CU against the ds_read_b32 peak (32 lane-lookups / clk / CU).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_aes.hip -o /tmp/ubench_aes
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

template <int N, int WG, int OCC>
__global__ __launch_bounds__(WG, OCC) void kaes(Args A) {
    __shared__ __attribute__((aligned(16))) u32 lds[HB_LDS_WORDS];
    fill_lds(lds, A.t0);
    const u32 r4 = (threadIdx.x & 31u) * 4u;
    const LaneTab L{(const char *)lds, {r4, 128u + r4, 0x10000u | r4, 0x10000u | (128u + r4)}};
    u32 s[N][4];
    const u32 gid = blockIdx.x * WG + threadIdx.x;
    for (int n = 0; n < N; ++n) {
        s[n][0] = gid * 2654435761u + n;
        s[n][1] = n * 7u;
        s[n][2] = gid;
        s[n][3] = 0x12345678u ^ n;
    }
    for (u32 it = 0; it < A.iters; ++it) {
        u32 o[N];
        hb_aes_byte0_n<14, N>(L, A.rk, s, o);
        for (int n = 0; n < N; ++n) {
            s[n][0] = hb_alignbit(s[n][1], s[n][0], 8);
            s[n][1] = hb_alignbit(s[n][2], s[n][1], 8);
            s[n][2] = hb_alignbit(s[n][3], s[n][2], 8);
            s[n][3] = (s[n][3] >> 8) | (o[n] << 24);
        }
    }
    u32 acc = 0;
    for (int n = 0; n < N; ++n) acc ^= s[n][3];
    A.out[gid] = acc;
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

template <int N, int WG, int OCC>
static void run(const char *name, Args A, int grid, int ncu) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((kaes<N, WG, OCC>), dim3(grid), dim3(WG), 0, 0, A);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((kaes<N, WG, OCC>), dim3(grid), dim3(WG), 0, 0, A);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    double lookups = (double)grid * WG * N * A.iters * 197.0;
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    double per_clk_cu = lookups / (ms * 1e-3) / (clk * 1e3) / ncu;
    printf("%-28s grid=%5d ms=%8.3f lookups/s=%.3e  per clk/CU=%.2f (%.1f%% of 32 @ %d MHz)\n", name, grid, ms,
           lookups / (ms * 1e-3), per_clk_cu, 100.0 * per_clk_cu / 32.0, clk / 1000);
}

int main() {
    make_t0();
    u32 *t0, *out;
    (void)hipMalloc(&t0, 1024);
    (void)hipMemcpy(t0, T0, 1024, hipMemcpyHostToDevice);
    (void)hipMalloc(&out, 256 * 1024 * 4 * 4);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    Args A;
    for (int i = 0; i < 60; ++i) A.rk[i] = 0x9e3779b9u * (i + 1);
    A.t0 = t0;
    A.out = out;
    A.iters = 2048;
    run<1, 1024, 4>("N=1 wg=1024 (16 waves/CU)", A, ncu, ncu);
    run<2, 1024, 4>("N=2 wg=1024 (16 waves/CU)", A, ncu, ncu);
    A.iters = 1024;
    run<2, 768, 3>("N=2 wg=768 (12 waves/CU)", A, ncu, ncu);
    run<2, 512, 2>("N=2 wg=512 (8 waves/CU)", A, ncu, ncu);
    run<4, 512, 2>("N=4 wg=512 (8 waves/CU)", A, ncu, ncu);
    run<4, 1024, 4>("N=4 wg=1024 (16 waves/CU)", A, ncu, ncu);
    run<3, 1024, 4>("N=3 wg=1024 (16 waves/CU)", A, ncu, ncu);
    return 0;
}
