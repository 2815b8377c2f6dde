// Bitsliced AES-CFB8 engine (hb_bitslice.hpp) on gfx950: correctness against
// the host AES-CFB8 (hb_aes_host.hpp), then throughput in byte-0 AES per
// clock per CU -- alone, and co-resident with T-table waves (hb_lane.hpp) in
// one workgroup, each wave role running for a fixed wall-clock time.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/bitslice/ubench_bs.hip -o scripts/bitslice/ubench_bs
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "hb_bitslice.hpp"
#include "../../heartbeat_amd/csrc/hb_aes_host.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)
#define HB_LDS_WORDS (HB_TAB_BYTES / 4)

HB_BOTH u32 init_byte(u32 B, u32 b) {
    u32 x = B * 0x9E3779B1u ^ (b * 0x85EBCA77u + 0x1234567u);
    x ^= x >> 15; x *= 0x2C1B3C6Du; x ^= x >> 12; x *= 0x297A2D39u; x ^= x >> 15;
    return x & 0xffu;
}
HB_BOTH u32 pt_byte(u32 B, u32 t) { return init_byte(B ^ 0x55555555u, t + 1000u); }

struct Args {
    u32 keytab[HB_BS_KEYTAB_WORDS];
    u32 rk[60];
    const u32 *t0;
    unsigned char *out;
    unsigned long long *count;   // [0] T-table AES, [1] bitsliced AES
    u32 iters;
    unsigned long long ticks;    // wall-clock ticks (100 MHz) per wave
};

__device__ __forceinline__ void fill_t(u32 *lds, const u32 *t0) {
    for (u32 g = threadIdx.x; g < HB_LDS_WORDS / 4; g += blockDim.x) {
        const u32 off = g * 16u;
        const u32 e = (off >> 8) & 0xffu, t = ((off >> 16) << 1) | ((off >> 7) & 1u);
        u32 v = t0[e];
        if (t) v = (v << (8 * t)) | (v >> (32 - 8 * t));
        reinterpret_cast<uint4 *>(lds)[g] = make_uint4(v, v, v, v);
    }
}

// ---------------------------------------------------------------- check
__global__ __launch_bounds__(256) void kcheck(Args A) {
    __shared__ __attribute__((aligned(16))) u32 kt[HB_BS_KEYTAB_WORDS];
    for (u32 i = threadIdx.x; i < HB_BS_KEYTAB_WORDS; i += blockDim.x) kt[i] = A.keytab[i];
    __syncthreads();
    const u32 gl = blockIdx.x * blockDim.x + threadIdx.x, quad = gl >> 2, q = gl & 3u;
    BsLane Q(kt, q);
    u32 reg[4][8];
    for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 8; ++i) {
            u32 w = 0;
            for (u32 l = 0; l < 32; ++l) w |= ((init_byte(quad * 32 + l, 4 * q + j) >> (7 - i)) & 1u) << l;
            reg[j][i] = w;
        }
    for (u32 t = 0; t < A.iters; ++t) {
        u32 d[8], c[8];
        for (int i = 0; i < 8; ++i) {
            u32 w = 0;
            for (u32 l = 0; l < 32; ++l) w |= ((pt_byte(quad * 32 + l, t) >> (7 - i)) & 1u) << l;
            d[i] = w;
        }
        hb_bs_cfb8_step<u32>(Q, reg, d, c);
    }
    for (u32 l = 0; l < 32; ++l)
        for (int j = 0; j < 4; ++j) {
            u32 byte = 0;
            for (int i = 0; i < 8; ++i) byte |= ((reg[j][i] >> l) & 1u) << (7 - i);
            A.out[(size_t)(quad * 32 + l) * 16 + 4 * q + j] = (unsigned char)byte;
        }
}

// ---------------------------------------------------------------- throughput
// Waves 0 .. NT-1 of the workgroup run T-table byte-0 AES chains, the others
// the bitsliced engine, each until its wall-clock budget is spent.
template <int WG, int NT, int OCC, int TPRIO = 0>
__global__ __launch_bounds__(WG, OCC) void kmix(Args A) {
    constexpr u32 TW = NT > 0 ? HB_LDS_WORDS : 4;
    __shared__ __attribute__((aligned(16))) u32 lds[TW + HB_BS_KEYTAB_WORDS];
    u32 *kt = lds + TW;
    for (u32 i = threadIdx.x; i < HB_BS_KEYTAB_WORDS; i += blockDim.x) kt[i] = A.keytab[i];
    if (NT > 0) fill_t(lds, A.t0);
    __syncthreads();
    const u32 wave = threadIdx.x >> 6;
    const u32 gl = blockIdx.x * WG + threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    unsigned long long n = 0;
    if ((int)wave < NT) {
        // latency-bound LDS chains first in VALU issue arbitration
        if (TPRIO) __builtin_amdgcn_s_setprio(TPRIO);
        const u32 r4 = (threadIdx.x & 31u) * 4u;
        const LaneTab L{(const char *)lds, {r4, 128u + r4, 0x10000u | r4, 0x10000u | (128u + r4)}};
        u32 s0 = gl * 2654435761u, s1 = gl, s2 = 7u, s3 = 0x12345678u;
        while (wall_clock64() - t0 < A.ticks) {
            for (int k = 0; k < 16; ++k) {
                const u32 o = hb_aes_byte0<14>(L, A.rk, s0, s1, s2, s3);
                s0 = hb_alignbit(s1, s0, 8); s1 = hb_alignbit(s2, s1, 8); s2 = hb_alignbit(s3, s2, 8);
                s3 = (s3 >> 8) | (o << 24);
            }
            n += 16;
        }
        if (s3 == 0x9u && s0 == 0x1u) A.out[gl] = 1;   // keep the chain live
        if ((threadIdx.x & 63u) == 0) atomicAdd(A.count, n * 64ull);
    } else {
        BsLane Q(kt, threadIdx.x);
        u32 reg[4][8];
        for (int j = 0; j < 4; ++j)
            for (int i = 0; i < 8; ++i) reg[j][i] = gl * 0x9E3779B1u + (u32)(8 * j + i) * 0x85EBCA77u;
        u32 d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        while (wall_clock64() - t0 < A.ticks) {
            u32 c[8];
            hb_bs_cfb8_step<u32>(Q, reg, d, c);
            d[0] ^= c[3];
            ++n;
        }
        if (d[0] == 0x9u && reg[0][0] == 0x1u) A.out[gl] = 1;
        // 32 evaluations per quad = 8 per lane-step
        if ((threadIdx.x & 63u) == 0) atomicAdd(A.count + 1, n * 512ull);
    }
}

static const int kCheckBlocks = 64 * 32;   // 64 quads x 32 evaluations

template <int WG, int NT, int OCC, int TPRIO = 0>
static void run(const char *name, Args &A, Args *dA, int grid, int ncu, double clk_ghz) {
    // HB_BS_ONLY: run only the configurations whose name contains it
    const char *only = getenv("HB_BS_ONLY");
    if (only && !strstr(name, only)) return;
    CK(hipMemset(A.count, 0, 16));
    hipLaunchKernelGGL((kmix<WG, NT, OCC, TPRIO>), dim3(grid), dim3(WG), 0, 0, A);
    CK(hipDeviceSynchronize());
    unsigned long long c[2];
    CK(hipMemcpy(c, A.count, 16, hipMemcpyDeviceToHost));
    const double secs = (double)A.ticks / 1e8;
    const double tt = c[0] / secs, bs = c[1] / secs;
    const double per = 1e9 * clk_ghz * ncu;
    printf("%-34s AES/s T-table %.3e + bitsliced %.3e = %.3e | per clk/CU: %.4f + %.4f = %.4f\n", name, tt, bs,
           tt + bs, tt / per, bs / per, (tt + bs) / per);
    fflush(stdout);
    (void)dA;
}

int main(int argc, char **argv) {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    int clk = 0;
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0));
    const double clk_ghz = clk / 1e6;
    printf("%s, %d CUs, %.2f GHz\n", prop.name, ncu, clk_ghz);

    const hbhost::AesTables &T = hbhost::aes_tables();
    uint8_t key[32];
    for (int i = 0; i < 32; ++i) key[i] = (uint8_t)(i * 37 + 11);
    hbhost::AesKey K;
    hbhost::aes_expand(key, 32, K);
    static Args A;
    memcpy(A.rk, K.rk, sizeof(A.rk));
    hb_bs_key_table(K.rk, A.keytab);
    u32 *t0;
    CK(hipMalloc(&t0, 1024));
    CK(hipMemcpy(t0, T.t0, 1024, hipMemcpyHostToDevice));
    A.t0 = t0;
    CK(hipMalloc(&A.out, (size_t)kCheckBlocks * 16 + (1 << 22)));
    CK(hipMalloc(&A.count, 16));

    // ---- correctness
    A.iters = 40;
    hipLaunchKernelGGL(kcheck, dim3(kCheckBlocks / 32 * 4 / 256), dim3(256), 0, 0, A);
    CK(hipDeviceSynchronize());
    std::vector<unsigned char> got((size_t)kCheckBlocks * 16);
    CK(hipMemcpy(got.data(), A.out, got.size(), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int B = 0; B < kCheckBlocks; ++B) {
        uint8_t iv[16], pt[64], ct[64];
        for (int b = 0; b < 16; ++b) iv[b] = (uint8_t)init_byte(B, b);
        for (u32 t = 0; t < A.iters; ++t) pt[t] = (uint8_t)pt_byte(B, t);
        hbhost::aes_cfb8(K, iv, pt, ct, A.iters, true);
        if (memcmp(got.data() + (size_t)B * 16, ct + A.iters - 16, 16) != 0) {
            if (bad < 4) {
                printf("block %d mismatch: got", B);
                for (int b = 0; b < 16; ++b) printf(" %02x", got[(size_t)B * 16 + b]);
                printf("\n             want");
                for (int b = 0; b < 16; ++b) printf(" %02x", ct[A.iters - 16 + b]);
                printf("\n");
            }
            ++bad;
        }
    }
    printf("bitsliced CFB-8 check: %d / %d blocks wrong (%u steps)\n", bad, kCheckBlocks, A.iters);
    if (bad) return 1;
    if (argc > 1 && !strcmp(argv[1], "check")) return 0;

    // ---- throughput: 0.2 s per configuration
    A.ticks = 20000000ull;
    // HB_BS_SECONDS: longer runs per configuration (power sampling)
    if (getenv("HB_BS_SECONDS")) A.ticks = (unsigned long long)(atof(getenv("HB_BS_SECONDS")) * 1e8);
    run<256, 0, 1>("bitsliced 4 waves/CU", A, nullptr, ncu, ncu, clk_ghz);
    run<256, 0, 2>("bitsliced 8 waves/CU", A, nullptr, 2 * ncu, ncu, clk_ghz);
    run<256, 0, 3>("bitsliced 12 waves/CU", A, nullptr, 3 * ncu, ncu, clk_ghz);
    run<256, 0, 4>("bitsliced 16 waves/CU", A, nullptr, 4 * ncu, ncu, clk_ghz);
    run<1024, 16, 4>("T-table 16 waves/CU", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 12, 4>("mixed 12 T + 4 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 10, 4>("mixed 10 T + 6 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 8, 4>("mixed 8 T + 8 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 6, 4>("mixed 6 T + 10 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 4, 4>("mixed 4 T + 12 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<512, 4, 2>("mixed 4 T + 4 bitsliced (8 w)", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 12, 4, 3>("prio3 12 T + 4 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 10, 4, 3>("prio3 10 T + 6 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 8, 4, 3>("prio3 8 T + 8 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    run<1024, 6, 4, 3>("prio3 6 T + 10 bitsliced", A, nullptr, ncu, ncu, clk_ghz);
    return 0;
}
