// hb_wide_args.hpp -- argument blocks of the split wide-prime encode's MAC
// kernels (hb_wide.hpp), shared with the host runtime.  Apart from
// hb_args.hpp so that the MAC kernels' unit rebuilds alone.
#pragma once
#include "hb_args.hpp"

// Split wide-prime encode (primes above 256 bits; hb_runtime.cpp, wide_*):
// the PRF passes store F per block, then hb_wmac_kernel forms
//     tag = (F + sum_j alpha_j m_j) mod p
// with the sector MAC on the int8 matrix cores.  A block is C = S ss bytes
// u_x (x = j ss + k), sector j = sum_k u_x 256^(ss-1-k), so
//     sum_j alpha_j m_j = sum_x u_x r_x (mod p),  r_x = alpha_j 256^(ss-1-k) mod p.
// Each r_x is taken as the representative r'_x in the range of D = tw signed
// base-256 digits (r_x or r_x - p) and split into its digits d_x[c]; the
// MFMA forms the D column sums col_c = sum_x d_x[c] (u_x - 128) of each
// block, and
//     T = sum_c col_c 256^c + kz,  kz = (128 sum_x r_x mod p) + p 2^w
// is == sum_j alpha_j m_j (mod p), 0 < T < 3 p 2^w (w: hb_runtime.cpp,
// wide_plan).  sum_x r_x = G sum_j alpha_j with G = sum_{e<ss} 256^e mod p.
// The digit table is built on the device (hb_wtab_kernel) from alpha_j R mod p.
// A fragments: [slice q < Kp/64][tile t < Mt][lane][16 bytes], the
// v_mfma_i32_16x16x64_i8 A operand: lane (g, m) = (l >> 4, l & 15) byte e
// holds d_x[c] for x = 64 q + 16 g + e, c = 16 t + m.
#define HB_WIDE_MAX_C 32768u      // bytes per block the MFMA MAC takes (i32 column sums, w <= 29)
template <int NL>
struct WtabArgs {
    ModP<NL> mod;
    const u32 *alpha_mont;        // S x NL: alpha_j R mod p
    const u32 *pw;                // ss x NL: 256^e mod p (plain)
    u32 g128[NL];                 // 128 G mod p (plain)
    u32 half[NL];                 // the largest representative: D bytes of 0x7f
    u32 p2w[NL + 1];              // p 2^w
    u32 C, ss, S, D, Mt, nslices;
    int8_t *afrag;                // nslices x Mt x 64 x 16 bytes
    u32 *kz;                      // NL + 1 limbs
    unsigned int *status;         // bit 0: a digit expansion did not close (internal error)
};

template <int NL>
struct WmacArgs {
    ModP<NL> mod;
    const unsigned char *data;    // block k of this launch at data[k C]
    u64 len;
    u64 nfull;                    // blocks [0, nfull): wholly inside the data (the rest: hb_mac_*_kernel)
    u64 C;
    u32 ss, S, tw, Mt, nslices;
    const int8_t *afrag;
    const u32 *kz;                // NL + 1 limbs (device)
    const u32 *fsrc;              // F per block, NL limbs
    unsigned char *tags;          // tw big-endian bytes per block
    u32 wpe;                      // A/B: hb_wmac_kernel's waves-per-SIMD bound (0: the default)
};

