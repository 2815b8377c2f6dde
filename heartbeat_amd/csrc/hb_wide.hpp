// hb_wide.hpp -- the split wide-prime encode's MAC kernels (primes above 256
// bits): the device-built int8 digit table (hb_wtab_kernel) and the MFMA MAC
// that turns the PRF passes' F into tags (hb_wmac_kernel; the short last
// block goes through hb_mac_split_kernel / hb_mac_kernel, hb_runtime.cpp).  Instantiated by hb_kern_wide.hip only, so that these
// kernels build apart from the PRF engine's translation units.
#pragma once
#include "hb_kernels.hpp"
#include "hb_wide_args.hpp"

// ------------------------------------------------------------------ split wide-prime MAC
// Primes above 256 bits (hb_args.hpp, WtabArgs / WmacArgs): the PRF passes
// (ALIGN = 0) store F, the MAC runs here on the int8 matrix cores.  With the
// MAC inside the PRF kernels (the ALIGN = 1/16 path) a 1024-bit block costs
// S x 32 x 32 VALU multiply-adds next to ~233 AES, run by the accepting lanes
// of a wave only, and its 65-limb accumulator halves the PRF kernels'
// occupancy (512-thread workgroups).

// The digit table: thread x < 64 nslices forms r_x = alpha_j 256^(ss-1-k) mod
// p (x = j ss + k; zero past the block), its representative r'_x (r_x, or
// r_x - p above `half`) and the D balanced base-256 digits of r'_x, written
// to the A fragments; thread 64 nslices forms kz = (sum_j alpha_j) 128 G mod
// p + p 2^w.
template <int NL>
__global__ __launch_bounds__(256) void hb_wtab_kernel(WtabArgs<NL> A) {
    const u32 x = blockIdx.x * blockDim.x + threadIdx.x;
    const u32 K = 64u * A.nslices;
    if (x > K) return;
    if (x == K) {
        u32 s[NL];   // sum_j alpha_j R mod p
        HB_UNROLL
        for (int t = 0; t < NL; ++t) s[t] = 0;
        for (u32 j = 0; j < A.S; ++j) hb_add_mod<NL>(s, A.alpha_mont + (u64)j * NL, A.mod);
        u32 acc[2 * NL + 1], v[NL + 1], r[NL];
        HB_UNROLL
        for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
        hb_mac<NL>(acc, A.g128, s);   // REDC: (sum_j alpha_j) 128 G mod p
        hb_redc<NL>(acc, A.mod, v);
        hb_reduce_small<NL>(v, A.mod, r);
        u64 c = 0;
        HB_UNROLL
        for (int t = 0; t <= NL; ++t) {
            c += (u64)A.p2w[t] + (t < NL ? r[t] : 0u);
            A.kz[t] = (u32)c;
            c >>= 32;
        }
        return;
    }
    u32 r[NL];
    bool neg = false;
    if (x < A.C) {
        const u32 j = x / A.ss, e = A.ss - 1u - (x - j * A.ss);
        u32 acc[2 * NL + 1], v[NL + 1];
        HB_UNROLL
        for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
        hb_mac<NL>(acc, A.alpha_mont + (u64)j * NL, A.pw + (u64)e * NL);   // REDC: alpha_j 256^e
        hb_redc<NL>(acc, A.mod, v);
        hb_reduce_small<NL>(v, A.mod, r);
        // r > half: take r - p (two's complement over NL limbs)
        u32 gt = 0, decided = 0;
        HB_UNROLL
        for (int t = NL - 1; t >= 0; --t) {
            const bool d = !decided && r[t] != A.half[t];
            gt = d ? (r[t] > A.half[t] ? 1u : 0u) : gt;
            decided |= d ? 1u : 0u;
        }
        neg = gt != 0;
        if (neg) {
            u32 br = 0;
            HB_UNROLL
            for (int t = 0; t < NL; ++t) {
                const u64 d = (u64)r[t] - A.mod.p[t] - br;
                r[t] = (u32)d;
                br = (u32)(d >> 63);
            }
        }
    } else {
        HB_UNROLL
        for (int t = 0; t < NL; ++t) r[t] = 0;
    }
    const u32 q = x >> 6, g = (x >> 4) & 3u, e = x & 15u;
    int8_t *dst = A.afrag + ((u64)q * A.Mt * 64u + 16u * g) * 16u + e;
    u32 carry = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t)
        HB_UNROLL
        for (int b = 0; b < 4; ++b) {
            const u32 c = 4u * (u32)t + (u32)b;
            if (c < 16u * A.Mt) {
                int dg = 0;
                if (c < A.D) {
                    const u32 vb = ((r[t] >> (8 * b)) & 0xffu) + carry;
                    carry = vb >= 128u ? 1u : 0u;
                    dg = (int)vb - 256 * (int)carry;
                }
                // tile c / 16, row c % 16: lane 16 g + c % 16, byte e
                dst[((u64)(c >> 4) * 64u + (c & 15u)) * 16u] = (int8_t)dg;
            }
        }
    // exact iff the digits' carry out is the sign (0 for r' >= 0, 1 for r' < 0)
    if (carry != (neg ? 1u : 0u)) atomicOr(A.status, 1u);
}

// v (NL+1 limbs, v < 2^32 p) -> v mod p in place (limbs 0..NL-1), as
// hb_reduce_small but without its second NL+1-limb array: the comparison
// with p runs first and the subtraction in place (registers of the MAC
// kernel's finish, which set its occupancy)
template <int NL>
__device__ __forceinline__ void hb_reduce_small_lean(u32 v[NL + 1], const ModP<NL> &P) {
    constexpr int T0 = NL - 2 - 31 > 0 ? NL - 2 - 31 : 0;
    double vd = 0.0, sc = HbScale<NL, T0>::v;
    HB_UNROLL
    for (int t = T0; t <= NL; ++t) {
        vd += (double)v[t] * sc;
        sc *= 4294967296.0;
    }
    const double qd = vd * P.inv_scaled;
    const u32 q = qd >= 2.0 ? (u32)qd - 1u : 0u;   // floor(qd) - 1 <= true quotient
    u64 carry = 0;
    u32 borrow = 0;
    HB_UNROLL
    for (int t = 0; t <= NL; ++t) {
        const u64 pr = (u64)q * (t < NL ? P.p[t] : 0u) + carry;
        carry = pr >> 32;
        const u64 d = (u64)v[t] - (u32)pr - borrow;
        v[t] = (u32)d;
        borrow = (u32)(d >> 63);
    }
    for (;;) {   // at most a few iterations: v >= p ?
        bool ge = v[NL] != 0, decided = ge;
        HB_UNROLL
        for (int t = NL - 1; t >= 0; --t) {
            const bool d = !decided && v[t] != P.p[t];
            ge = d ? v[t] > P.p[t] : ge;
            decided = decided || d;
        }
        if (decided && !ge) break;   // v < p; otherwise v >= p (all limbs equal: v == p)
        u32 br = 0;
        HB_UNROLL
        for (int t = 0; t <= NL; ++t) {
            const u64 d = (u64)v[t] - (t < NL ? P.p[t] : 0u) - br;
            v[t] = (u32)d;
            br = (u32)(d >> 63);
        }
    }
}

// tag = (F + sum_j alpha_j m_j) mod p for the blocks [0, nfull) of a launch
// that lie wholly inside the data.  A workgroup of HB_WMAC_WAVES waves takes
// 16 NG consecutive blocks, NG groups of 16 (group g: the B columns of a
// v_mfma_i32_16x16x64_i8), and its waves split the Mt digit tiles (wave v:
// tiles v TW .. v TW + TW - 1), so a wave holds 16 NG TW accumulator
// registers.  The blocks' bytes go through LDS once per workgroup, one 64-byte
// K slice of every block at a time, double-buffered: the workgroup's threads
// load slice s + 1 (four threads per 64-byte piece, coalesced) while the waves
// run slice s's MFMAs from LDS; each A fragment (global, L2-resident) serves
// the NG groups.  Every 16-byte piece is read from HBM once and every A
// fragment once per 16 NG blocks per wave (with the blocks read by every wave
// straight from global memory and 4 groups, the kernel took 5.7 ms for 8 GiB
// at 1024 bits, profiles/r06/c; with one wave holding all Mt tiles, 9.0 ms
// at one wave per SIMD, profiles/r06/b).  At NL = 64 (16 tiles) a workgroup
// is 8 waves x 128 blocks, 2 tiles per wave: half the A-fragment traffic per
// block of 4 waves x 64 (7.99 vs 8.36 ms per 8 GiB, profiles/r06/r6v).
// Tile t's result at lane (q, n) is
// digits 16 t + 4 q .. + 3 of block 16 g + n, i.e. limb 4 t + q; a 4 x 4
// transpose of (group within a quad of groups, lane row) --
// v_permlane32_swap, v_permlane16_swap -- leaves lane l with limbs 4 t ..
// 4 t + 3 of block 64 h + l of group quad h, written to the LDS limb table
// ([limb][block]: conflict-free), which reuses the slice buffers.  One lane
// per block then folds the limbs into T = sum_c col_c 256^c + kz in limb
// order, adds F and reduces.
#ifndef HB_WMAC_WAVES
#define HB_WMAC_WAVES 4
#endif
#ifndef HB_WMAC_WPE
#define HB_WMAC_WPE 3
#endif
#ifndef HB_WMAC_WAVES64
#define HB_WMAC_WAVES64 8
#endif
#ifndef HB_WMAC_NG64
#define HB_WMAC_NG64 8
#endif
// K slices in flight from global memory per thread (registers)
#ifndef HB_WMAC_PF
#define HB_WMAC_PF 3
#endif
#ifndef HB_WMAC_NG
#define HB_WMAC_NG 8
#endif
template <int NL>
struct HbWmac {
    static constexpr int WAVES = NL >= 64 ? HB_WMAC_WAVES64 : HB_WMAC_WAVES;     // waves per workgroup
    static constexpr int NG = NL >= 64 ? HB_WMAC_NG64 : HB_WMAC_NG;              // groups of 16 blocks
    static constexpr int NB = 16 * NG;                                          // blocks per workgroup
    static constexpr int TW = (NL / 4 + WAVES - 1) / WAVES;                      // tiles per wave (D <= 4 NL)
    // LDS: two slice buffers (NB x 64 bytes each), or the limb table (NL x NB x 8 bytes);
    // then the finish's staging of F and the tags, [NL words][NB blocks] with
    // a row pitch of NB + 64 / NL words (conflict-free both ways, see below)
    static constexpr int LIMB_BYTES = 2 * NB * 64 > NL * NB * 8 ? 2 * NB * 64 : NL * NB * 8;
    // (NL = 64 keeps the per-lane F loads and tag stores: with the staging its
    // finish spilled more, 12.3 vs 9.0 ms per 8 GiB at 2048 bits, profiles/r06/r6u)
    static constexpr bool CO = NL <= 32;
    static constexpr int PITCH = NB + 64 / NL;
    static constexpr int LDS_BYTES = LIMB_BYTES + (CO ? NL * PITCH * 4 : 0);
    // the default waves-per-SIMD bound: HB_WMAC_WPE; NL = 64 the compiler's
    // choice (8 waves x 128 blocks: 7.28 ms per 8 GiB at 2048 bits against
    // 8.1 with WPE 3, whose 168 VGPRs spill 388 bytes; profiles/r06/r6w)
    static constexpr int WPE = NL >= 64 ? 0 : HB_WMAC_WPE;
};

// One block's T + F, reduced, out: F from the staging array (co) or from
// fsrc, the tag into the staging array as big-endian words (co) or to tags.
template <int NL>
__device__ __forceinline__ void hb_wmac_finish(const WmacArgs<NL> &A, const long long *lim, u32 *stg, bool co,
                                               u32 bi, u64 blk) {
    constexpr int NB = HbWmac<NL>::NB, PITCH = HbWmac<NL>::PITCH;
    // v = T + F, T = sum_i lim_i 2^(32 i) + kz (limbs past the tiles' digits: kz and the carry)
    const u32 lt = 4u * A.Mt;
    const u32 *fp = A.fsrc + blk * NL;
    u32 v[NL + 1];
    long long carry = 0;
    u64 c = 0;
#pragma unroll
    for (int t = 0; t < NL; t += 4) {
        u32 F4[4];
        if (co) {
#pragma unroll
            for (int k = 0; k < 4; ++k) F4[k] = stg[(t + k) * PITCH + bi];
        } else {
            const uint4 f = *reinterpret_cast<const uint4 *>(fp + t);
            F4[0] = f.x;
            F4[1] = f.y;
            F4[2] = f.z;
            F4[3] = f.w;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const u32 i = (u32)(t + k);
            const long long xv = (long long)A.kz[i] + (i < lt ? lim[i * NB + bi] : 0ll) + carry;
            carry = xv >> 32;
            c += (u64)(u32)xv + F4[k];
            v[t + k] = (u32)c;
            c >>= 32;
        }
    }
    v[NL] = (u32)((long long)A.kz[NL] + carry) + (u32)c;
    hb_reduce_small_lean<NL>(v, A.mod);
    if (co) {   // word NL - 1 - t of the big-endian tag is limb t
#pragma unroll
        for (int t = 0; t < NL; ++t) stg[(NL - 1 - t) * PITCH + bi] = hb_bswap(v[t]);
    } else {
        hb_store_be<NL>(A.tags + blk * (u64)A.tw, A.tw, v);
    }
}

// WPE: waves per SIMD the register allocator is held to; 0 = the compiler's
// choice.  The launcher takes HB_WMAC_WPE unless WmacArgs::wpe (test switch
// $HB_WMAC_WPE, A/B) names another instantiated value.
template <int WPE>
struct HbWpe { static constexpr int v = WPE > 0 ? WPE : 1; };
template <int NL, int WPE>
__global__ __launch_bounds__(64 * HbWmac<NL>::WAVES) __attribute__((amdgpu_waves_per_eu(HbWpe<WPE>::v)))
void hb_wmac_kernel(WmacArgs<NL> A) {
    constexpr int NG = HbWmac<NL>::NG, NB = HbWmac<NL>::NB, TW = HbWmac<NL>::TW;
    constexpr int NT = 64 * HbWmac<NL>::WAVES;
    __shared__ __attribute__((aligned(16))) unsigned char lds[HbWmac<NL>::LDS_BYTES];
    const u32 l = hb_lane_id(), wv = threadIdx.x >> 6;
    const u64 w0 = (u64)blockIdx.x * NB;
    // slice loads: thread i fills LDS unit u = r NT + i (16 bytes at 16 u),
    // unit u = (g 4 + q) 16 + n holding bytes 16 q .. + 15 of the slice of
    // block 16 g + n -- lane (q, n) of a wave reads unit (g, q, n), and the
    // stores of consecutive lanes land on consecutive 16 bytes (no bank
    // conflicts; with one thread per 64-byte piece 48 % of the LDS cycles
    // were conflicts, profiles/r06/r6m).  A wave's load still covers 16
    // blocks x 64 contiguous bytes.
    constexpr int LR = NB * 4 / NT;   // 16-byte pieces per thread per slice
    const unsigned char *src[LR];
    bool okp[LR];
    u32 qof[LR];
#pragma unroll
    for (int r = 0; r < LR; ++r) {
        const u32 u = (u32)r * NT + threadIdx.x, b = ((u >> 6) << 4) | (u & 15u), qq = (u >> 4) & 3u;
        const u64 blk = w0 + b;
        okp[r] = blk < A.nfull;
        qof[r] = 16u * qq;
        src[r] = A.data + (okp[r] ? blk : w0) * A.C + 16u * qq;
    }
    auto gload = [&](u32 s, hb_i32x4 v[LR]) {
#pragma unroll
        for (int r = 0; r < LR; ++r) {
            const bool in = okp[r] && 64u * s + qof[r] < A.C;
            v[r] = in ? *reinterpret_cast<const hb_i32x4 *>(src[r] + 64u * s) : hb_i32x4{0, 0, 0, 0};
        }
    };
    auto lstore = [&](u32 buf, const hb_i32x4 v[LR]) {
#pragma unroll
        for (int r = 0; r < LR; ++r)
            *reinterpret_cast<hb_i32x4 *>(lds + buf * (NB * 64) + 16u * ((u32)r * NT + threadIdx.x)) =
                v[r] ^ (int32_t)0x80808080;
    };
    const u32 t0 = wv * (u32)TW;
    const bool mine = t0 < A.Mt;   // wave-uniform: this wave has tiles
    hb_i32x4 acc[TW][NG];
#pragma unroll
    for (int t = 0; t < TW; ++t)
#pragma unroll
        for (int g = 0; g < NG; ++g) acc[t][g] = hb_i32x4{0, 0, 0, 0};
    const hb_i32x4 *afr = reinterpret_cast<const hb_i32x4 *>(A.afrag) + (u64)t0 * 64u + l;
    // slices go global -> registers HB_WMAC_PF slices ahead (slot x % PF
    // holds slice x), registers -> LDS one slice ahead (double buffer)
    constexpr int PF = HB_WMAC_PF;
    hb_i32x4 pv[PF][LR];
#pragma unroll
    for (int k = 0; k < PF; ++k)
        if ((u32)k < A.nslices) gload((u32)k, pv[k]);
    lstore(0, pv[0]);
    if ((u32)PF < A.nslices) gload((u32)PF, pv[0]);
    __syncthreads();
    // this wave's A fragments of the slice, one slice ahead
    auto aload = [&](u32 s, hb_i32x4 a[TW]) {
#pragma unroll
        for (int t = 0; t < TW; ++t)
            a[t] = mine && t0 + (u32)t < A.Mt ? afr[((u64)s * A.Mt + (u32)t) * 64u] : hb_i32x4{0, 0, 0, 0};
    };
    hb_i32x4 an[TW];
    aload(0, an);
    for (u32 s0 = 0; s0 < A.nslices; s0 += PF) {
#pragma unroll
        for (int k = 0; k < PF; ++k) {
            const u32 s = s0 + (u32)k;
            if (s >= A.nslices) break;   // uniform
            const u32 cur = s & 1u;
            hb_i32x4 a[TW];
#pragma unroll
            for (int t = 0; t < TW; ++t) a[t] = an[t];
            if (s + 1 < A.nslices) aload(s + 1, an);
            if (mine) {
                const unsigned char *bb = lds + cur * (NB * 64) + l * 16u;
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const hb_i32x4 b = *reinterpret_cast<const hb_i32x4 *>(bb + (u32)g * 1024u);
#pragma unroll
                    for (int t = 0; t < TW; ++t)
                        acc[t][g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[t], b, acc[t][g], 0, 0, 0);
                }
            }
            const int nx = (k + 1) % PF;   // the slot of slice s + 1 (static once unrolled)
            if (s + 1 < A.nslices) {
                lstore(cur ^ 1u, pv[nx]);
                if (s + 1 + PF < A.nslices) gload(s + 1 + PF, pv[nx]);
            }
            __syncthreads();
        }
    }
    // Tags exactly NL words wide (16-byte aligned): the workgroup's F and tags
    // are contiguous 4 NB NL-byte runs, moved by all threads in coalesced
    // 16-byte pieces through the staging array -- word w of block b at
    // stg[w PITCH + b]; a piece (b, q) is words 4 q .. 4 q + 3, and the pitch
    // puts the 64 lanes of a piece access (64 / (NL / 4) blocks x NL / 4
    // pieces) and a finish lane's word access on distinct banks.  (One lane
    // per block reading its 4 NL bytes and writing them back as NL dword
    // stores 4 NL bytes apart took 1.06 of the kernel's 3.13 ms at 1024 bits:
    // 64 cache lines per store instruction, profiles/r06/r6t3.)
    constexpr int PITCH = HbWmac<NL>::PITCH, NQ = NL / 4, NP = NB * NQ, PPT = (NP + NT - 1) / NT;
    u32 *stg = reinterpret_cast<u32 *>(lds + HbWmac<NL>::LIMB_BYTES);
    const bool co = HbWmac<NL>::CO && A.tw == 4u * NL && ((uintptr_t)A.tags & 15u) == 0 && ((uintptr_t)A.fsrc & 15u) == 0;
    const u64 nvalid = A.nfull - w0 < (u64)NB ? A.nfull - w0 : (u64)NB;
    uint4 fv[PPT];
    if (co) {   // F in flight while the accumulators go to the limb table
        const uint4 *fq = reinterpret_cast<const uint4 *>(A.fsrc + w0 * NL);
#pragma unroll
        for (int r = 0; r < PPT; ++r) {
            const u32 u = (u32)r * NT + threadIdx.x;
            if (u < (u32)NP && u / NQ < nvalid) fv[r] = fq[u];
        }
    }
    // the slice buffers are free (every wave passed the last barrier): limb table
    long long *lim = reinterpret_cast<long long *>(lds);
    if (mine) {
#pragma unroll
        for (int t = 0; t < TW; ++t) {
            if (t0 + (u32)t < A.Mt) {
#pragma unroll
                for (int h = 0; h < NG / 4; ++h) {
                    u32 X[4][2];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const hb_i32x4 &a = acc[t][4 * h + g];
                        const long long v = (long long)a[0] + ((long long)a[1] << 8) + ((long long)a[2] << 16) +
                                            ((long long)a[3] << 24);
                        X[g][0] = (u32)v;
                        X[g][1] = (u32)((u64)v >> 32);
                    }
#pragma unroll
                    for (int d = 0; d < 2; ++d) {
                        const auto s02 = __builtin_amdgcn_permlane32_swap((int)X[0][d], (int)X[2][d], false, false);
                        const auto s13 = __builtin_amdgcn_permlane32_swap((int)X[1][d], (int)X[3][d], false, false);
                        const auto s01 = __builtin_amdgcn_permlane16_swap((int)s02[0], (int)s13[0], false, false);
                        const auto s23 = __builtin_amdgcn_permlane16_swap((int)s02[1], (int)s13[1], false, false);
                        X[0][d] = (u32)s01[0];
                        X[1][d] = (u32)s01[1];
                        X[2][d] = (u32)s23[0];
                        X[3][d] = (u32)s23[1];
                    }
                    // X[s]: limb 4 (t0 + t) + s of block 64 h + l
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4) {
                        const u32 i = 4u * (t0 + (u32)t) + (u32)s4;
                        if (i < (u32)NL) lim[i * NB + 64u * h + l] = (long long)(((u64)X[s4][1] << 32) | X[s4][0]);
                    }
                }
            }
        }
    }
    if (co) {
#pragma unroll
        for (int r = 0; r < PPT; ++r) {
            const u32 u = (u32)r * NT + threadIdx.x, b = u / NQ, q = u % NQ;
            if (u < (u32)NP && b < nvalid) {
                stg[(4 * q) * PITCH + b] = fv[r].x;
                stg[(4 * q + 1) * PITCH + b] = fv[r].y;
                stg[(4 * q + 2) * PITCH + b] = fv[r].z;
                stg[(4 * q + 3) * PITCH + b] = fv[r].w;
            }
        }
    }
    __syncthreads();
    const u32 bi = threadIdx.x;   // block of this lane
    if (bi < (u32)NB && bi < nvalid) hb_wmac_finish<NL>(A, lim, stg, co, bi, w0 + bi);
    if (!co) return;
    __syncthreads();
    unsigned char *tq = A.tags + w0 * (u64)(4 * NL);
#pragma unroll
    for (int r = 0; r < PPT; ++r) {
        const u32 u = (u32)r * NT + threadIdx.x, b = u / NQ, q = u % NQ;
        if (u < (u32)NP && b < nvalid) {
            uint4 t;
            t.x = stg[(4 * q) * PITCH + b];
            t.y = stg[(4 * q + 1) * PITCH + b];
            t.z = stg[(4 * q + 2) * PITCH + b];
            t.w = stg[(4 * q + 3) * PITCH + b];
            *reinterpret_cast<uint4 *>(tq + 16u * u) = t;
        }
    }
}

// ------------------------------------------------------------------ launchers
template <int NL>
hipError_t hb_launch_wtab(const WtabArgs<NL> &A, hipStream_t s) {
    const u32 n = 64u * A.nslices + 1u;
    HB_LAUNCH((hb_wtab_kernel<NL>), dim3((n + 255u) / 256u), dim3(256), s, A);
    return hipGetLastError();
}

template <int NL>
hipError_t hb_launch_wmac(const WmacArgs<NL> &A, hipStream_t s) {
    if (hb_load_only) {
        hb_load_kernel(&hb_wmac_kernel<NL, HbWmac<NL>::WPE>);
        return hipSuccess;
    }
    if (A.nfull) {
        const dim3 g((u32)((A.nfull + HbWmac<NL>::NB - 1) / HbWmac<NL>::NB)), b(64 * HbWmac<NL>::WAVES);
        if (A.wpe == 3) HB_LAUNCH((hb_wmac_kernel<NL, 3>), g, b, s, A);
        else if (A.wpe == 4) HB_LAUNCH((hb_wmac_kernel<NL, 4>), g, b, s, A);
        else if (A.wpe == 5) HB_LAUNCH((hb_wmac_kernel<NL, 5>), g, b, s, A);
        else if (A.wpe == 1) HB_LAUNCH((hb_wmac_kernel<NL, 0>), g, b, s, A);
        else HB_LAUNCH((hb_wmac_kernel<NL, HbWmac<NL>::WPE>), g, b, s, A);
    }
    return hipGetLastError();
}

#define HB_INST_WIDE(NL)                                                           \
    template hipError_t hb_launch_wtab<NL>(const WtabArgs<NL> &, hipStream_t);     \
    template hipError_t hb_launch_wmac<NL>(const WmacArgs<NL> &, hipStream_t);
