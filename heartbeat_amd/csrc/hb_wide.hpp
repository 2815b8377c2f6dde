// hb_wide.hpp -- the split wide-prime encode's MAC kernels (primes above 256
// bits): the device-built int8 digit table (hb_wtab_kernel) and the MFMA MAC
// that turns the PRF passes' F into tags (hb_wmac_kernel, the VALU tail
// hb_wmac_tail_kernel).  Instantiated by hb_kern_wide.hip only, so that these
// kernels build apart from the PRF engine's translation units.
#pragma once
#include "hb_kernels.hpp"

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

// tag = (F + sum_j alpha_j m_j) mod p for the blocks [0, nfull) of a launch
// that lie wholly inside the data.  A wave takes 64 consecutive blocks, four
// groups of 16 (group g: blocks 16 g .. 16 g + 15, the B columns of a
// v_mfma_i32_16x16x64_i8); per 64-byte K slice of the blocks lane (q, n)
// loads bytes 16 q .. 16 q + 15 of block 16 g + n for each group (the four
// lanes n, n+16, n+32, n+48 read one contiguous 64-byte piece) and every A
// tile of the slice is applied to the four groups.  Tile t's result at lane
// (q, n) is digits 16 t + 4 q .. + 3 of block 16 g + n, i.e. limb 4 t + q; a
// 4 x 4 transpose of (group, lane row) -- v_permlane32_swap and
// v_permlane16_swap -- leaves lane l with limbs 4 t .. 4 t + 3 of its own
// block l, and the lane folds them into T = sum_c col_c 256^c + kz in limb
// order.  At most 8 tiles are held at once (128 accumulator registers);
// 2048-bit primes (16 tiles) take two passes over the K slices.
template <int NL>
struct HbWmac {
    static constexpr int MTP = NL / 4 < 8 ? NL / 4 : 8;   // tiles per pass
    static constexpr int NP = (NL / 4 + MTP - 1) / MTP;    // passes for D = 4 NL
};

template <int NL>
__global__ __launch_bounds__(256) void hb_wmac_kernel(WmacArgs<NL> A) {
    constexpr int MTP = HbWmac<NL>::MTP, NP = HbWmac<NL>::NP;
    const u32 l = hb_lane_id(), q = l >> 4, n = l & 15u;
    const u64 w0 = ((u64)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 64u;
    if (w0 >= A.nfull) return;   // wave-uniform
    const unsigned char *bp[4];
    bool okg[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const u64 b = w0 + 16u * (u32)g + n;
        okg[g] = b < A.nfull;
        bp[g] = A.data + (okg[g] ? b : w0) * A.C + 16u * q;
    }
    const hb_i32x4 *afr = reinterpret_cast<const hb_i32x4 *>(A.afrag);
    u32 T[NL + 1];
    long long carry = 0;
#pragma unroll
    for (int P = 0; P < NP; ++P) {
        const u32 t0 = (u32)(P * MTP);
        if (t0 < A.Mt) {   // uniform
            hb_i32x4 acc[MTP][4];
#pragma unroll
            for (int t = 0; t < MTP; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) acc[t][g] = hb_i32x4{0, 0, 0, 0};
            for (u32 s = 0; s < A.nslices; ++s) {
                const bool in = 64u * s + 16u * q < A.C;   // 16-byte pieces past the block: zero
                hb_i32x4 b[4];
#pragma unroll
                for (int g = 0; g < 4; ++g)
                    b[g] = okg[g] && in ? *reinterpret_cast<const hb_i32x4 *>(bp[g] + 64u * s) : hb_i32x4{0, 0, 0, 0};
#pragma unroll
                for (int g = 0; g < 4; ++g) b[g] ^= (int32_t)0x80808080;
                const hb_i32x4 *as = afr + ((u64)s * A.Mt + t0) * 64u + l;
#pragma unroll
                for (int t = 0; t < MTP; ++t) {
                    if (t0 + (u32)t < A.Mt) {
                        const hb_i32x4 a = as[(u64)t * 64u];
#pragma unroll
                        for (int g = 0; g < 4; ++g)
                            acc[t][g] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b[g], acc[t][g], 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < MTP; ++t) {
                if (t0 + (u32)t < A.Mt) {
                    u32 X[4][2];
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const hb_i32x4 &a = acc[t][g];
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
                    // X[s]: limb 4 (t0 + t) + s of this lane's block
#pragma unroll
                    for (int s4 = 0; s4 < 4; ++s4) {
                        const int i = 4 * (P * MTP + t) + s4;
                        if (i < NL) {
                            const long long L = (long long)(((u64)X[s4][1] << 32) | X[s4][0]);
                            const long long xv = (long long)A.kz[i] + L + carry;
                            T[i] = (u32)xv;
                            carry = xv >> 32;
                        }
                    }
                }
            }
        }
    }
    // limbs above the tiles' digits: kz and the carry only
#pragma unroll
    for (int i = 0; i <= NL; ++i) {
        if ((u32)i >= 4u * A.Mt) {
            const long long xv = (long long)A.kz[i] + carry;
            T[i] = (u32)xv;
            carry = xv >> 32;
        }
    }
    const u64 blk = w0 + l;
    if (blk >= A.nfull) return;
    u32 F[NL], v[NL + 1], tag[NL];
    const u32 *fp = A.fsrc + blk * NL;
#pragma unroll
    for (int t = 0; t < NL; t += 4) {
        const uint4 f = *reinterpret_cast<const uint4 *>(fp + t);
        F[t] = f.x; F[t + 1] = f.y; F[t + 2] = f.z; F[t + 3] = f.w;
    }
    u64 c = 0;
#pragma unroll
    for (int t = 0; t < NL; ++t) {
        c += (u64)T[t] + F[t];
        v[t] = (u32)c;
        c >>= 32;
    }
    v[NL] = T[NL] + (u32)c;
    hb_reduce_small<NL>(v, A.mod, tag);
    hb_store_be<NL>(A.tags + blk * (u64)A.tw, A.tw, tag);
}

// The blocks [nfull, nblocks) of a split encode (the short last block and any
// past the end of the data): one lane each, the VALU MAC (hb_block_tag).
template <int NL>
__global__ __launch_bounds__(64) void hb_wmac_tail_kernel(WmacArgs<NL> A) {
    const u64 blk = A.nfull + (u64)blockIdx.x * blockDim.x + threadIdx.x;
    if (blk >= A.nblocks) return;
    u32 F[NL], tag[NL];
    for (int t = 0; t < NL; ++t) F[t] = A.fsrc[blk * NL + t];
    hb_block_tag<NL, 1>(A.data, A.len, blk, A.C, A.ss, A.S, A.alpha_mont, A.mod, F, tag);
    hb_store_be<NL>(A.tags + blk * (u64)A.tw, A.tw, tag);
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
        hb_load_kernel(&hb_wmac_kernel<NL>);
        hb_load_kernel(&hb_wmac_tail_kernel<NL>);
        return hipSuccess;
    }
    if (A.nfull) {
        const u64 waves = (A.nfull + 63) / 64;
        HB_LAUNCH((hb_wmac_kernel<NL>), dim3((u32)((waves + 3) / 4)), dim3(256), s, A);
    }
    if (A.nblocks > A.nfull) {
        const u64 n = A.nblocks - A.nfull;
        HB_LAUNCH((hb_wmac_tail_kernel<NL>), dim3((u32)((n + 63) / 64)), dim3(64), s, A);
    }
    return hipGetLastError();
}

#define HB_INST_WIDE(NL)                                                           \
    template hipError_t hb_launch_wtab<NL>(const WtabArgs<NL> &, hipStream_t);     \
    template hipError_t hb_launch_wmac<NL>(const WmacArgs<NL> &, hipStream_t);
