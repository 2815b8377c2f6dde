// hb_lane.hpp -- per-lane arithmetic of the Swizzle hot path.
//
// Everything a single lane does for one block lives here:
//   * SHA-256 of the decimal block index          (heartbeat/util.py:91)
//   * AES-CFB8 keystream with byte-0-only output   (heartbeat/util.py:88-93)
//     using a bank-replicated T0..T3 LDS image (128 KiB)
//   * the rejection test num < R                    (heartbeat/util.py:94)
//   * the fixed-width Montgomery multiply-accumulate and reduction of
//     tag = F(i) + sum_j alpha_j m_ij mod p        (PySwizzle.py:297-307)
//
// The header compiles as HIP device code (inlined into the kernels of
// hb_kernels.hpp) and as plain C++ (tests/emul), so the lane logic can be
// checked against the CPU oracle without a GPU.  Wave-level work distribution
// (job queue, ballots) is in hb_kernels.hpp, not here.
#pragma once
#include <stdint.h>

#if defined(__HIP__)
#define HB_HD __device__ __forceinline__
#define HB_HHD __host__ __device__ inline
#else
#define HB_HD static inline
#define HB_HHD static inline
#endif

#if defined(__HIP_DEVICE_COMPILE__)
#define HB_UNROLL _Pragma("unroll")
#define HB_NOUNROLL _Pragma("unroll 1")
#else
#define HB_UNROLL
#define HB_NOUNROLL
#endif

typedef uint32_t u32;
typedef uint64_t u64;

// Instruction-count experiments (scripts/build_variant.sh) that make the
// kernels emit WRONG tags.  They compile only together with
// HB_EXPERIMENT_BUILD, which the product Makefile refuses for
// libhbswizzle.so and which makes the library report itself as an experiment
// build (hb_build_flags), so heartbeat_amd refuses it unless HB_LIB_PATH
// selects it explicitly.
#if (defined(HB_EXP_NO_SHA) || defined(HB_EXP_MAC_NOLOAD) || defined(HB_EXP_NO_MAC) || \
     defined(HB_EXP_NO_FINISH) || defined(HB_EXP_NO_MFMA) || defined(HB_EXP_MFMA_NOLOAD)) && \
    !defined(HB_EXPERIMENT_BUILD)
#error "HB_EXP_* switches produce wrong tags: experiment builds only (scripts/build_variant.sh)"
#endif

// ------------------------------------------------------------------ intrinsics
HB_HD u32 hb_perm(u32 s0, u32 s1, u32 sel) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_perm(s0, s1, sel);
#else
    // v_perm_b32: selector byte b picks byte b of {s0:s1} (0-3 = s1, 4-7 = s0),
    // 12 = 0x00, >= 13 = 0xff (8-11, sign replication, unused here).
    u64 v = ((u64)s0 << 32) | s1;
    u32 r = 0;
    HB_UNROLL
    for (int i = 0; i < 4; ++i) {
        u32 b = (sel >> (8 * i)) & 0xffu, o;
        if (b < 8) o = (u32)(v >> (8 * b)) & 0xffu;
        else if (b == 12) o = 0;
        else o = 0xffu;
        r |= o << (8 * i);
    }
    return r;
#endif
}

// ({hi,lo} >> sh)[31:0], sh in [0,31]
HB_HD u32 hb_alignbit(u32 hi, u32 lo, u32 sh) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_alignbit(hi, lo, sh);
#else
    return (u32)((((u64)hi << 32) | lo) >> (sh & 31));
#endif
}

HB_HD u32 hb_rotl16(u32 x) { return hb_alignbit(x, x, 16); }
HB_HD u32 hb_xor3(u32 a, u32 b, u32 c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // v_bitop3_b32: a ^ b ^ c
#else
    return a ^ b ^ c;
#endif
}
HB_HD u32 hb_bswap(u32 x) { return hb_perm(x, x, 0x00010203u); }

// ------------------------------------------------------------------ AES
// LDS image of the four T tables, 128 KiB.  Entry e of table t (Tt =
// rotl(8t) of T0) replica r (0..31) is the u32 at byte
//     (t >> 1) * 65536 + e * 256 + (t & 1) * 128 + r * 4.
// Lane l reads replica (l & 31), so the 32 lanes of each ds_read_b32 half-wave
// hit 32 distinct banks (bank = (addr/4) mod 32) whatever the indices: no bank
// conflicts.  The address of Tt[byte k of x] is ONE v_perm_b32:
//     {0, lb_t.byte2, x.byte[k], lb_t.byte0},  lb_t = (t>>1) << 16 | (t&1)*128 + (l&31)*4.
// A column of a round is then 4 lookups and two 3-input XORs (v_bitop3).
#define HB_TAB_BYTES 131072

struct LaneTab {
    const char *tab;       // LDS image base (generic pointer; LDS after inlining)
    u32 lb[4];             // lane bases of T0..T3
};

HB_HD u32 hb_tab_ld(const char *tab, u32 addr) {
    return *(const u32 *)(tab + addr);
}

template <int K, int T>
HB_HD u32 hb_t(const LaneTab &L, u32 x) {
    u32 addr = hb_perm(x, L.lb[T], 0x0c020000u | ((4u + K) << 8));
    return hb_tab_ld(L.tab, addr);
}

// One full AES round on little-endian column words (byte r of w_c = row r):
// col_c = T0[w_c.0] ^ T1[w_(c+1).1] ^ T2[w_(c+2).2] ^ T3[w_(c+3).3] ^ rk_c.
HB_HD void hb_aes_round(const LaneTab &L, const u32 *rk, u32 &w0, u32 &w1, u32 &w2, u32 &w3) {
    u32 a0 = hb_t<0, 0>(L, w0), b0 = hb_t<1, 1>(L, w1), c0 = hb_t<2, 2>(L, w2), d0 = hb_t<3, 3>(L, w3);
    u32 a1 = hb_t<0, 0>(L, w1), b1 = hb_t<1, 1>(L, w2), c1 = hb_t<2, 2>(L, w3), d1 = hb_t<3, 3>(L, w0);
    u32 a2 = hb_t<0, 0>(L, w2), b2 = hb_t<1, 1>(L, w3), c2 = hb_t<2, 2>(L, w0), d2 = hb_t<3, 3>(L, w1);
    u32 a3 = hb_t<0, 0>(L, w3), b3 = hb_t<1, 1>(L, w0), c3 = hb_t<2, 2>(L, w1), d3 = hb_t<3, 3>(L, w2);
    w0 = hb_xor3(hb_xor3(a0, b0, c0), d0, rk[0]);
    w1 = hb_xor3(hb_xor3(a1, b1, c1), d1, rk[1]);
    w2 = hb_xor3(hb_xor3(a2, b2, c2), d2, rk[2]);
    w3 = hb_xor3(hb_xor3(a3, b3, c3), d3, rk[3]);
}

// Byte 0 of AES_k(state).  CFB-8 consumes only that byte, so round NR-1
// computes one byte of column 0 (4 lookups) and the last round one S-box
// lookup (S[x] = byte 1 of T0[x]): 16*(NR-2) + 5 lookups per block.
template <int NR>
HB_HD u32 hb_aes_byte0(const LaneTab &L, const u32 *rk, u32 s0, u32 s1, u32 s2, u32 s3) {
    u32 w0 = s0 ^ rk[0], w1 = s1 ^ rk[1], w2 = s2 ^ rk[2], w3 = s3 ^ rk[3];
    HB_UNROLL
    for (int r = 1; r <= NR - 2; ++r) hb_aes_round(L, rk + 4 * r, w0, w1, w2, w3);
    u32 a = hb_t<0, 0>(L, w0), b = hb_t<1, 1>(L, w1), c = hb_t<2, 2>(L, w2), d = hb_t<3, 3>(L, w3);
    u32 s = hb_xor3(hb_xor3(a, b, c), d, rk[4 * (NR - 1)]) & 0xffu;
    u32 o = hb_t<0, 0>(L, s) >> 8;
    return (o ^ rk[4 * NR]) & 0xffu;
}

// hb_aes_byte0 for N independent states at once (s[n][0..3] -> o[n]): the N
// states' lookups of a round are independent, so a wave keeps up to 16 N
// ds_read_b32 in flight per round instead of 16.
template <int NR, int N>
HB_HD void hb_aes_byte0_n(const LaneTab &L, const u32 *rk, const u32 s[N][4], u32 o[N]) {
    u32 w[N][4];
    HB_UNROLL
    for (int n = 0; n < N; ++n)
        HB_UNROLL
        for (int c = 0; c < 4; ++c) w[n][c] = s[n][c] ^ rk[c];
    HB_UNROLL
    for (int r = 1; r <= NR - 2; ++r)
        HB_UNROLL
        for (int n = 0; n < N; ++n) hb_aes_round(L, rk + 4 * r, w[n][0], w[n][1], w[n][2], w[n][3]);
    HB_UNROLL
    for (int n = 0; n < N; ++n) {
        u32 a = hb_t<0, 0>(L, w[n][0]), b = hb_t<1, 1>(L, w[n][1]), c = hb_t<2, 2>(L, w[n][2]),
            d = hb_t<3, 3>(L, w[n][3]);
        u32 x = hb_xor3(hb_xor3(a, b, c), d, rk[4 * (NR - 1)]) & 0xffu;
        o[n] = ((hb_t<0, 0>(L, x) >> 8) ^ rk[4 * NR]) & 0xffu;
    }
}

// ------------------------------------------------------------------ SHA-256
HB_HD u32 hb_rotr(u32 x, u32 n) { return hb_alignbit(x, x, n); }

// One SHA-256 compression of the message block W (16 big-endian words,
// clobbered) into the chaining state st (8 words).
HB_HD void hb_sha256_compress(u32 st[8], u32 W[16]) {
    const u32 K[64] = {
        0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
        0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
        0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
        0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
        0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
        0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
        0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
        0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
        0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
        0xc67178f2u};
    u32 a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    HB_UNROLL
    for (int t = 0; t < 64; ++t) {
        u32 w;
        if (t < 16) {
            w = W[t];
        } else {
            u32 w15 = W[(t - 15) & 15], w2 = W[(t - 2) & 15];
            u32 s0 = hb_xor3(hb_rotr(w15, 7), hb_rotr(w15, 18), w15 >> 3);
            u32 s1 = hb_xor3(hb_rotr(w2, 17), hb_rotr(w2, 19), w2 >> 10);
            w = W[t & 15] + s0 + W[(t - 7) & 15] + s1;
            W[t & 15] = w;
        }
        // three-input XORs (v_bitop3): the compiler does not fuse rotr ^ rotr ^ rotr
        u32 S1 = hb_xor3(hb_rotr(e, 6), hb_rotr(e, 11), hb_rotr(e, 25));
        u32 ch = (e & f) ^ (~e & g);
        u32 t1 = h + S1 + ch + K[t] + w;
        u32 S0 = hb_xor3(hb_rotr(a, 2), hb_rotr(a, 13), hb_rotr(a, 22));
        u32 mj = (a & b) ^ (a & c) ^ (b & c);
        u32 t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1;
        d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

HB_HD void hb_sha256_init(u32 st[8]) {
    st[0] = 0x6a09e667u; st[1] = 0xbb67ae85u; st[2] = 0x3c6ef372u; st[3] = 0xa54ff53au;
    st[4] = 0x510e527fu; st[5] = 0x9b05688cu; st[6] = 0x1f83d9abu; st[7] = 0x5be0cd19u;
}

// One SHA-256 compression from the initial state over the padded message
// block W (16 big-endian words, clobbered).  Digest as 8 big-endian words.
HB_HD void hb_sha256_block(u32 W[16], u32 H[8]) {
    hb_sha256_init(H);
    hb_sha256_compress(H, W);
}

// SHA-256 of ASCII decimal(x) (str(x).encode(), util.py:91); one compression
// since len <= 20 < 56.  Digest as 8 big-endian words.
HB_HD void hb_sha256_decimal(u64 x, u32 H[8]) {
#if defined(HB_EXP_NO_SHA)   // instruction-count experiment only (wrong digests)
    for (int t = 0; t < 8; ++t) H[t] = (u32)x * 2654435761u + (u32)t * 40503u;
    return;
#endif
    // Build the message right-to-left: shifting a 24-byte big-endian register
    // right by one byte per digit and inserting the digit at the top leaves
    // the decimal string left-aligned with the 0x80 pad byte right behind it.
    u32 R0 = 0x80000000u, R1 = 0, R2 = 0, R3 = 0, R4 = 0, R5 = 0;
    u32 n = 0;
    auto push = [&](u32 dgt) {
        R5 = hb_alignbit(R4, R5, 8);
        R4 = hb_alignbit(R3, R4, 8);
        R3 = hb_alignbit(R2, R3, 8);
        R2 = hb_alignbit(R1, R2, 8);
        R1 = hb_alignbit(R0, R1, 8);
        R0 = (R0 >> 8) | ((0x30u + dgt) << 24);
        ++n;
    };
    // 64-bit divisions only while x needs them; the (common) rest in 32 bits
    while (x >> 32) {
        const u64 q = x / 10u;
        push((u32)(x - q * 10u));
        x = q;
    }
    u32 y = (u32)x;
    do {
        const u32 q = y / 10u;
        push(y - q * 10u);
        y = q;
    } while (y != 0);
    u32 W[16] = {R0, R1, R2, R3, R4, R5, 0, 0, 0, 0, 0, 0, 0, 0, 0, n * 8u};
    hb_sha256_block(W, H);
}

// SHA-256 of the 4 raw bytes of a 32-bit unsigned int in x86 (little-endian)
// order: the cxx prf's message (cxx/prf.hxx:174, (unsigned char*)&i).
HB_HD void hb_sha256_le32(u32 x, u32 H[8]) {
    u32 W[16] = {hb_bswap(x), 0x80000000u, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 32u};
    hb_sha256_block(W, H);
}

// ------------------------------------------------------------------ PRF try
// Parameters of one KeyedPRF instance (util.py:66-81): AES key schedule and
// the range R.  R is little-endian in NL u32 limbs; nb = ceil(bitlen(R)/8)
// keystream bytes per try; topmask masks the most significant output byte.
template <int NL>
struct PrfParams {
    u32 rk[60];
    u32 R[NL];
    u32 nb;
    u32 topmask;
    // Round-1 constants of a first try's CFB-8 steps whose shift register
    // starts with z = 1..3 zero words (hb_aes_round1_z): r1z[4 (z - 1) + c] =
    // round key 1 word c ^ the lookups of column c that read those words.
    u32 r1z[12];
};

// Round 1 (hb_aes_round) when register words 0 .. z-1 are zero, z = 1..3, so
// that w_c = rk[c] for c < z: every lookup of such a word is a constant of the
// key, and k = r1z + 4 (z - 1) holds, per output column, round key 1 XOR those
// constants (host: hbhost::aes_round1_zero_consts).  z is a compile-time
// constant at every call (hb_cfb8_step's ZC).
HB_HD void hb_aes_round1_z(const LaneTab &L, const u32 *r1z, u32 z, u32 &w0, u32 &w1, u32 &w2, u32 &w3) {
    if (z == 3) {
        const u32 *k = r1z + 8;
        const u32 n0 = hb_t<3, 3>(L, w3) ^ k[0], n1 = hb_t<2, 2>(L, w3) ^ k[1];
        const u32 n2 = hb_t<1, 1>(L, w3) ^ k[2], n3 = hb_t<0, 0>(L, w3) ^ k[3];
        w0 = n0; w1 = n1; w2 = n2; w3 = n3;
    } else if (z == 2) {
        const u32 *k = r1z + 4;
        const u32 n0 = hb_xor3(hb_t<2, 2>(L, w2), hb_t<3, 3>(L, w3), k[0]);
        const u32 n1 = hb_xor3(hb_t<1, 1>(L, w2), hb_t<2, 2>(L, w3), k[1]);
        const u32 n2 = hb_xor3(hb_t<0, 0>(L, w2), hb_t<1, 1>(L, w3), k[2]);
        const u32 n3 = hb_xor3(hb_t<0, 0>(L, w3), hb_t<3, 3>(L, w2), k[3]);
        w0 = n0; w1 = n1; w2 = n2; w3 = n3;
    } else {
        const u32 *k = r1z;
        const u32 n0 = hb_xor3(hb_t<1, 1>(L, w1), hb_t<2, 2>(L, w2), hb_t<3, 3>(L, w3)) ^ k[0];
        const u32 n1 = hb_xor3(hb_t<0, 0>(L, w1), hb_t<1, 1>(L, w2), hb_t<2, 2>(L, w3)) ^ k[1];
        const u32 n2 = hb_xor3(hb_t<0, 0>(L, w2), hb_t<1, 1>(L, w3), hb_t<3, 3>(L, w1)) ^ k[2];
        const u32 n3 = hb_xor3(hb_t<0, 0>(L, w3), hb_t<2, 2>(L, w1), hb_t<3, 3>(L, w2)) ^ k[3];
        w0 = n0; w1 = n1; w2 = n2; w3 = n3;
    }
}

// One CFB-8 step on the shift register s0..s3 (little-endian words of the 16
// register bytes): AES it, ciphertext byte c = byte 0 of the output ^ the
// plaintext byte, shift c in at the top.  The plaintext byte is byte 1 of pk
// (the other bytes of pk are ignored).  The last round is one S-box lookup,
// S[x] = byte 1 of T0[x]; XORing pk and the last round key's byte (shifted to
// byte 1) into that word and picking its byte 1 with the same v_perm that
// shifts s3 makes the step's bookkeeping 1 v_bitop3 + 1 v_perm + 3 v_alignbit.
//
// ZC > 0: the number of leading register words s0 .. s_{ZC-1} known to be
// zero (only a first try's steps 4-12 have them).  Their round-1 lookups are
// then key constants (PrfParams::r1z) and round 1 reads only the other words:
// 4 (ZC = 3), 8 or 12 lookups instead of 16.
template <int NR, int ZC = 0>
HB_HD void hb_cfb8_step(const LaneTab &L, const u32 *rk, u32 &s0, u32 &s1, u32 &s2, u32 &s3, u32 pk,
                        const u32 *r1z = nullptr) {
    u32 w0 = s0 ^ rk[0], w1 = s1 ^ rk[1], w2 = s2 ^ rk[2], w3 = s3 ^ rk[3];
    if constexpr (ZC != 0) hb_aes_round1_z(L, r1z, ZC, w0, w1, w2, w3);
    else hb_aes_round(L, rk + 4, w0, w1, w2, w3);
    HB_UNROLL
    for (int r = 2; r <= NR - 2; ++r) hb_aes_round(L, rk + 4 * r, w0, w1, w2, w3);
    // byte 0 of round NR-1's column 0 (the other bytes of x are not used)
    const u32 x = hb_xor3(hb_xor3(hb_t<0, 0>(L, w0), hb_t<1, 1>(L, w1), hb_t<2, 2>(L, w2)), hb_t<3, 3>(L, w3),
                          rk[4 * (NR - 1)]);
    const u32 u = hb_xor3(hb_t<0, 0>(L, x), pk, rk[4 * NR] << 8);
    s0 = hb_alignbit(s1, s0, 8);
    s1 = hb_alignbit(s2, s1, 8);
    s2 = hb_alignbit(s3, s2, 8);
    s3 = hb_perm(u, s3, 0x05030201u);   // {u.1, s3.3, s3.2, s3.1}
}

// Four CFB-8 steps over the big-endian plaintext word d; returns the four
// ciphertext bytes as a big-endian word (they are s3 afterwards, oldest lowest).
// Z0 / Z1: leading zero register words before the first / the other three
// steps (hb_cfb8_step, ZC).
template <int NR, int Z0 = 0, int Z1 = 0>
HB_HD u32 hb_cfb8_word(const LaneTab &L, const u32 *rk, u32 &s0, u32 &s1, u32 &s2, u32 &s3, u32 d,
                       const u32 *r1z = nullptr) {
    hb_cfb8_step<NR, Z0>(L, rk, s0, s1, s2, s3, d >> 16, r1z);
    hb_cfb8_step<NR, Z1>(L, rk, s0, s1, s2, s3, d >> 8, r1z);
    hb_cfb8_step<NR, Z1>(L, rk, s0, s1, s2, s3, d, r1z);
    hb_cfb8_step<NR, Z1>(L, rk, s0, s1, s2, s3, d << 8, r1z);
    return hb_bswap(s3);
}

// One rejection-sampling try of KeyedPRF.eval: nb CFB-8 steps continuing the
// stream held in the shift register sr[0..3] (little-endian words of the 16
// register bytes).  dig: SHA-256 digest (big-endian words) -- the padded
// plaintext is dig bytes then zeros (KeyedPRF.pad).  out = mask & BE(ct).
// Returns 1 if out < R (accepted).
//
// FIRST = 1: the first output word (keystream bytes 0-3 of a fresh eval) is
// already in out[0] and sr (hb_prf_prefix); the try continues at byte 4.
template <int NL, int NR, int FIRST>
HB_HD u32 hb_prf_try_from(const LaneTab &L, const PrfParams<NL> &P, u32 sr[4], const u32 dig[8],
                          u32 out[NL]) {
    u32 dq[8];
    HB_UNROLL
    for (int t = 0; t < 8; ++t) dq[t] = t + FIRST < 8 ? dig[t + FIRST] : 0u;
    HB_UNROLL
    for (int t = FIRST; t < NL; ++t) out[t] = 0;
    const u32 nw = P.nb >> 2, tail = P.nb & 3u;
    u32 s0 = sr[0], s1 = sr[1], s2 = sr[2], s3 = sr[3];
    // mask of the try's first output byte (the top byte of the first word)
    u32 top = FIRST ? 0xffffffffu : (P.topmask << 24) | 0xffffffu;
    auto emit = [&](u32 word) {
        HB_UNROLL
        for (int t = 0; t < 7; ++t) dq[t] = dq[t + 1];
        dq[7] = 0;
        HB_UNROLL
        for (int t = NL - 1; t > 0; --t) out[t] = out[t - 1];
        out[0] = word;
    };
    u32 wi = FIRST;
    // A first try enters word 1 with register words 0-2 zero (the prefix
    // image's four steps shifted in 4 bytes): steps 4-7 start with 3, 2, 2, 2
    // zero words, so that word is peeled with its round 1 on the key
    // constants (36 of its 788 lookups go).  Peeling word 2 as well (steps
    // 8-11: 2, 1, 1, 1 zero words, 20 more) measured slower (code size);
    // word 1 alone: +0.9 % at configs[2] (same-box A/B, profiles/r03/s3).
    // The rest of the word loop stays rolled: unrolled (no register rotation
    // of dq / out, 116 instead of 128 VGPRs, no scratch) it measured -1.8 %
    // (profiles/r04/j).
    if constexpr (FIRST != 0) {
        if (wi < nw) {
            emit(hb_cfb8_word<NR, 3, 2>(L, P.rk, s0, s1, s2, s3, dq[0], P.r1z));
            ++wi;
        }
    }
    HB_NOUNROLL
    for (; wi < nw; ++wi) {
        emit(hb_cfb8_word<NR>(L, P.rk, s0, s1, s2, s3, dq[0]) & top);
        top = 0xffffffffu;
    }
    if (tail) {
        // 1-3 more bytes (nb % 4): plaintext bytes 0..tail-1 of dq[0]
        const u32 d = dq[0];
        for (u32 bi = 0; bi < tail; ++bi) hb_cfb8_step<NR>(L, P.rk, s0, s1, s2, s3, d >> (16 - 8 * bi));
        const u32 sh = 32 - 8 * tail;   // shift out left by 8*tail bits
        u32 word = hb_bswap(s3) & (0xffffffffu >> sh);
        if (!FIRST && nw == 0) word &= (P.topmask << (24 - sh)) | (0xffffffu >> sh);
        HB_UNROLL
        for (int t = NL - 1; t > 0; --t) out[t] = hb_alignbit(out[t], out[t - 1], sh);
        out[0] = hb_alignbit(out[0], word << sh, sh);
    }
    sr[0] = s0; sr[1] = s1; sr[2] = s2; sr[3] = s3;
    // out < R  <=>  out - R borrows
    u32 borrow = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        u64 d = (u64)out[t] - (u64)P.R[t] - (u64)borrow;
        borrow = (u32)(d >> 63);
    }
    return borrow;
}

template <int NL, int NR>
HB_HD u32 hb_prf_try(const LaneTab &L, const PrfParams<NL> &P, u32 sr[4], const u32 dig[8],
                     u32 out[NL]) {
    return hb_prf_try_from<NL, NR, 0>(L, P, sr, dig, out);
}

// ------------------------------------------------------------------ cxx prf
// The cxx Swizzle extension's PRF F' (cxx/prf.hxx:125-176), a different
// function from KeyedPRF: one Crypto++ CFB_Mode<AES> (full 16-byte feedback,
// IV = 0^16) resynchronised once per evaluate (:132); every try
// (rand_buf, :170-176) encrypts buf = SHA256(LE32(i)) zero-padded (or
// truncated) to limit_sz = ByteCount(limit) bytes, the stream continuing
// across tries; a = BE(buf) with the top byte masked to the bit length of the
// limit's top byte (set_limit :97-116, clz.h:36-48: 32-bit clz of a positive
// int, so the mask is 2^bitlen(b) - 1 = KeyedPRF's topmask); accepted when
// a < limit, or unconditionally after 81 tries (`count++ < 80`, :135-142).
#define HB_CXX_MAX_TRIES 81u

// All 16 output bytes of AES_k(w) in place (little-endian column words).  The
// last round's S[x] is byte k of T_{(k+2)&3}[x]: T0 = (2S, S, S, 3S),
// T1 = (3S, 2S, S, S), T2 = (S, 3S, 2S, S), T3 = (S, S, 3S, 2S).
template <int NR>
HB_HD void hb_aes_full(const LaneTab &L, const u32 *rk, u32 &w0, u32 &w1, u32 &w2, u32 &w3) {
    w0 ^= rk[0]; w1 ^= rk[1]; w2 ^= rk[2]; w3 ^= rk[3];
    HB_UNROLL
    for (int r = 1; r <= NR - 1; ++r) hb_aes_round(L, rk + 4 * r, w0, w1, w2, w3);
    const u32 *k = rk + 4 * NR;
    const u32 o0 = (hb_t<0, 2>(L, w0) & 0xffu) | (hb_t<1, 3>(L, w1) & 0xff00u) |
                   (hb_t<2, 0>(L, w2) & 0xff0000u) | (hb_t<3, 1>(L, w3) & 0xff000000u);
    const u32 o1 = (hb_t<0, 2>(L, w1) & 0xffu) | (hb_t<1, 3>(L, w2) & 0xff00u) |
                   (hb_t<2, 0>(L, w3) & 0xff0000u) | (hb_t<3, 1>(L, w0) & 0xff000000u);
    const u32 o2 = (hb_t<0, 2>(L, w2) & 0xffu) | (hb_t<1, 3>(L, w3) & 0xff00u) |
                   (hb_t<2, 0>(L, w0) & 0xff0000u) | (hb_t<3, 1>(L, w1) & 0xff000000u);
    const u32 o3 = (hb_t<0, 2>(L, w3) & 0xffu) | (hb_t<1, 3>(L, w0) & 0xff00u) |
                   (hb_t<2, 0>(L, w1) & 0xff0000u) | (hb_t<3, 1>(L, w2) & 0xff000000u);
    w0 = o0 ^ k[0]; w1 = o1 ^ k[1]; w2 = o2 ^ k[2]; w3 = o3 ^ k[3];
}

// One try of F': nb / 16 CFB-128 blocks (P.nb = limit_sz, a multiple of 16,
// <= 4 NL -- checked on the host) continuing from the feedback register sr
// (the previous ciphertext block, little-endian words; 0 = the IV).
// dig: SHA256(LE32(i)) as big-endian words; plaintext = dig then zeros.
// out = masked BE(ciphertext) in NL little-endian limbs; returns out < limit.
template <int NL, int NR>
HB_HD u32 hb_cxx_try(const LaneTab &L, const PrfParams<NL> &P, u32 sr[4], const u32 dig[8],
                     u32 out[NL]) {
    static_assert(NL >= 4, "cxx prf limits are at least 16 bytes");
    HB_UNROLL
    for (int t = 0; t < NL; ++t) out[t] = 0;
    u32 r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3];
    const u32 nblk = P.nb >> 4;
    HB_NOUNROLL
    for (u32 k = 0; k < nblk; ++k) {
        hb_aes_full<NR>(L, P.rk, r0, r1, r2, r3);
        // plaintext words of block k (bytes 16k..16k+15 of dig || 0...)
        const u32 p0 = k == 0 ? dig[0] : k == 1 ? dig[4] : 0u, p1 = k == 0 ? dig[1] : k == 1 ? dig[5] : 0u;
        const u32 p2 = k == 0 ? dig[2] : k == 1 ? dig[6] : 0u, p3 = k == 0 ? dig[3] : k == 1 ? dig[7] : 0u;
        r0 ^= hb_bswap(p0); r1 ^= hb_bswap(p1); r2 ^= hb_bswap(p2); r3 ^= hb_bswap(p3);
        // ciphertext block k = the next feedback register; append it to out
        // (big-endian words, the first block ends up most significant)
        u32 b0 = hb_bswap(r0);
        if (k == 0) b0 &= (P.topmask << 24) | 0xffffffu;
        HB_UNROLL
        for (int t = NL - 1; t >= 4; --t) out[t] = out[t - 4];
        out[3] = b0; out[2] = hb_bswap(r1); out[1] = hb_bswap(r2); out[0] = hb_bswap(r3);
    }
    sr[0] = r0; sr[1] = r1; sr[2] = r2; sr[3] = r3;
    u32 borrow = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        u64 d = (u64)out[t] - (u64)P.R[t] - (u64)borrow;
        borrow = (u32)(d >> 63);
    }
    return borrow;
}

// One try of F' for any limit_sz (P.nb = ByteCount(limit) <= 4 NL, not
// necessarily a multiple of 16: the cxx prove's indexer, limit = #tags).  The
// stream continues across tries at byte granularity, so try `ntry` (0-based)
// of an evaluation starts at byte (ntry * nb) mod 16 of the current CFB-128
// block.  sr holds the register the way OpenSSL's CRYPTO_cfb128_encrypt keeps
// ivec: at byte position 0 it is replaced by its encryption, then byte pos of
// it is XORed with the plaintext and becomes the ciphertext byte.  With
// nb % 16 == 0 this is hb_cxx_try.  Not on the encode hot path.
template <int NL, int NR>
HB_HD u32 hb_cxx_try_bytes(const LaneTab &L, const PrfParams<NL> &P, u32 sr[4], const u32 dig[8],
                           u32 out[NL], u32 ntry) {
    HB_UNROLL
    for (int t = 0; t < NL; ++t) out[t] = 0;
    u32 r0 = sr[0], r1 = sr[1], r2 = sr[2], r3 = sr[3];
    const u32 nb = P.nb;
    u32 pos = (ntry * nb) & 15u;
    HB_NOUNROLL
    for (u32 b = 0; b < nb; ++b) {
        if (pos == 0) hb_aes_full<NR>(L, P.rk, r0, r1, r2, r3);
        // plaintext byte b of dig || 0... (dig holds big-endian words)
        const u32 pt = b < 32 ? (dig[b >> 2] >> (24 - 8 * (b & 3))) & 0xffu : 0u;
        const u32 sh = 8 * (pos & 3), wsel = pos >> 2;
        const u32 x = (pt << sh);
        r0 ^= wsel == 0 ? x : 0u; r1 ^= wsel == 1 ? x : 0u;
        r2 ^= wsel == 2 ? x : 0u; r3 ^= wsel == 3 ? x : 0u;
        const u32 w = wsel == 0 ? r0 : wsel == 1 ? r1 : wsel == 2 ? r2 : r3;
        u32 cb = (w >> sh) & 0xffu;
        if (b == 0) cb &= P.topmask;
        // ciphertext byte b is byte nb-1-b of the big-endian result
        const u32 at = nb - 1 - b, ti = at >> 2, tsh = 8 * (at & 3);
        HB_UNROLL
        for (int t = 0; t < NL; ++t) out[t] |= (u32)t == ti ? cb << tsh : 0u;
        pos = (pos + 1) & 15u;
    }
    sr[0] = r0; sr[1] = r1; sr[2] = r2; sr[3] = r3;
    u32 borrow = 0;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        u64 d = (u64)out[t] - (u64)P.R[t] - (u64)borrow;
        borrow = (u32)(d >> 63);
    }
    return borrow;
}

// ------------------------------------------------------------------ CFB prefix
// Every eval starts a fresh cipher with IV = 0 (util.py:88), so the first four
// AES inputs of the first try are 0^16, 0^15 c0, 0^14 c0 c1 and 0^13 c0 c1 c2:
// for a fixed key the first four keystream bytes are o0 = E(0)[0] (a
// constant) and byte 0 of E(...) as a function of the first one, two and three
// ciphertext bytes.  The prefix image holds those three functions,
//   P1[c0]                         at HB_PFX_P1 (256 B)
//   P2[c0 | c1 << 8]               at HB_PFX_P2 (64 KiB)
//   P3[c0 | c1 << 8 | c2 << 16]    at HB_PFX_P3 (16 MiB),
// indexed by the register bytes in little-endian order so that the AES input
// word s3 of an entry is its index shifted left (hb_pfx_s3).  Built once per
// key (hb_prefix_kernel: 2^24 + 2^16 + 2^8 byte-0 AES, ~0.3 % of a 64 GiB
// encode); each first try then runs nb - 4 AES instead of nb.
#define HB_PFX_P1 0u
#define HB_PFX_P2 256u
#define HB_PFX_P3 65792u
#define HB_PFX_BYTES (65792u + (1u << 24))

// AES input word 3 (register bytes 12..15) of prefix image entry i; words 0-2 are 0.
HB_HD u32 hb_pfx_s3(u32 i) {
    if (i < HB_PFX_P2) return i << 24;
    if (i < HB_PFX_P3) return (i - HB_PFX_P2) << 16;
    return (i - HB_PFX_P3) << 8;
}

// First four CFB-8 steps of a fresh eval (nb >= 4) from the prefix image:
// d = digest word 0 (plaintext bytes 0-3, big-endian).  Leaves the shift
// register in sr and the first output word (top byte masked) in out[0].
template <int NL>
HB_HD void hb_prf_prefix(const unsigned char *pfx, u32 o0, const PrfParams<NL> &P, u32 d, u32 sr[4],
                         u32 out[NL]) {
    const u32 c0 = ((d >> 24) ^ o0) & 0xffu;
    const u32 c1 = ((d >> 16) ^ pfx[HB_PFX_P1 + c0]) & 0xffu;
    u32 x = c0 | (c1 << 8);
    const u32 c2 = ((d >> 8) ^ pfx[HB_PFX_P2 + x]) & 0xffu;
    x |= c2 << 16;
    const u32 c3 = (d ^ pfx[HB_PFX_P3 + x]) & 0xffu;
    sr[0] = sr[1] = sr[2] = 0;
    sr[3] = x | (c3 << 24);
    out[0] = ((c0 & P.topmask) << 24) | (c1 << 16) | (c2 << 8) | c3;
}

// Top 32 bits of R in the nb-byte frame of a PRF output (P.nb >= 4).  A try
// whose first output word (hb_prf_prefix's out[0], top byte masked) exceeds it
// is rejected whatever its other bytes are: out >= out[0] 2^(8nb-32) >
// (top + 1) 2^(8nb-32) - 1 >= R.  (The encode's early retry listing,
// HB_RETRY_DIGEST; checked by tests/emul.)
template <int NL>
HB_HHD u32 hb_range_top(const PrfParams<NL> &P) {
    const u32 sh = 8 * P.nb - 32, wi = sh / 32, off = sh % 32;
    u32 top = P.R[wi] >> off;
    if (off && wi + 1 < (u32)NL) top |= P.R[wi + 1] << (32 - off);
    return top;
}

// The first try of a fresh eval through the prefix image (P.nb >= 4).
template <int NL, int NR>
HB_HD u32 hb_prf_first_try(const LaneTab &L, const PrfParams<NL> &P, const unsigned char *pfx, u32 o0,
                           u32 sr[4], const u32 dig[8], u32 out[NL]) {
    hb_prf_prefix<NL>(pfx, o0, P, dig[0], sr, out);
    return hb_prf_try_from<NL, NR, 1>(L, P, sr, dig, out);
}

// ------------------------------------------------------------------ Merkle chunks
// heartbeat/Merkle/Merkle.py:481-515 (MerkleHelper.get_chunk_hash): the chunk
// of a seed starts at KeyedPRF(seed, filesz - chunksz + 1).eval(0) and its
// leaf is HMAC-SHA256(seed, chunk).  Every seed is its own AES key, so a lane
// expands its key schedule itself (below) instead of taking uniform round keys.

// S-box of each byte of w in place: S[x] is byte 1 of T0[x], i.e. byte k of
// T_{(k+3)&3}[x].
HB_HD u32 hb_subword(const LaneTab &L, u32 w) {
    return (hb_t<0, 3>(L, w) & 0xffu) | (hb_t<1, 0>(L, w) & 0xff00u) | (hb_t<2, 1>(L, w) & 0xff0000u) |
           (hb_t<3, 2>(L, w) & 0xff000000u);
}

// FIPS-197 key expansion in the kernels' word order (little-endian column
// words, as hbhost::aes_expand): key = NK = NR - 6 words, rk = 4 (NR + 1).
template <int NR>
HB_HD void hb_aes_expand_lane(const LaneTab &L, const u32 *key, u32 *rk) {
    constexpr int NK = NR - 6;
    const u32 rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40, 0x80, 0x1b, 0x36};
    HB_UNROLL
    for (int i = 0; i < NK; ++i) rk[i] = key[i];
    HB_UNROLL
    for (int i = NK; i < 4 * (NR + 1); ++i) {
        u32 t = rk[i - 1];
        if (i % NK == 0) t = hb_subword(L, (t >> 8) | (t << 24)) ^ rcon[i / NK - 1];
        else if (NK > 6 && i % NK == 4) t = hb_subword(L, t);
        rk[i] = rk[i - NK] ^ t;
    }
}

// HMAC-SHA256 (RFC 2104) of msg = data[off .. off + n) under a key of
// klen <= 64 bytes given as 16 big-endian words kw (zero padded).  len: bytes
// readable at data (whole-block word loads are used where they stay inside).
HB_HD void hb_hmac_sha256(const u32 kw[16], const unsigned char *data, u64 len, u64 off, u64 n, u32 out[8]) {
    u32 st[8], W[16];
    hb_sha256_init(st);
    HB_UNROLL
    for (int t = 0; t < 16; ++t) W[t] = kw[t] ^ 0x36363636u;
    hb_sha256_compress(st, W);
    // inner message: (64 + n) bytes hashed so far + padding
    const u64 total = n + 9;                       // msg, 0x80, 8-byte length
    const u64 nblk = (total + 63) / 64;
    const u64 bits = (64 + n) * 8;
    for (u64 b = 0; b < nblk; ++b) {
        const u64 p0 = 64 * b;                     // message position of this block
        const u64 base = off + p0;
        if (p0 + 64 <= n && (base & ~3ull) + 68 <= len) {
            // whole block inside the message: 17 aligned dword loads, funnel-shifted
            const u64 a = base & ~3ull;
            const u32 sh = 8u * (u32)(base & 3u);
            const u32 *q = (const u32 *)(data + a);
            u32 prev = q[0];
            HB_UNROLL
            for (int t = 0; t < 16; ++t) {
                const u32 nx = q[t + 1];
                W[t] = hb_bswap(sh ? hb_alignbit(nx, prev, sh) : prev);
                prev = nx;
            }
        } else {
            HB_UNROLL
            for (int t = 0; t < 16; ++t) {
                u32 w = 0;
                for (int k = 0; k < 4; ++k) {
                    const u64 p = p0 + 4 * (u64)t + (u64)k;
                    u32 byte = p < n ? data[off + p] : (p == n ? 0x80u : 0u);
                    w = (w << 8) | byte;
                }
                W[t] = w;
            }
            if (b == nblk - 1) {
                W[14] |= (u32)(bits >> 32);
                W[15] |= (u32)bits;
            }
        }
        hb_sha256_compress(st, W);
    }
    u32 inner[8];
    HB_UNROLL
    for (int t = 0; t < 8; ++t) inner[t] = st[t];
    hb_sha256_init(st);
    HB_UNROLL
    for (int t = 0; t < 16; ++t) W[t] = kw[t] ^ 0x5c5c5c5cu;
    hb_sha256_compress(st, W);
    HB_UNROLL
    for (int t = 0; t < 8; ++t) W[t] = inner[t];
    W[8] = 0x80000000u;
    HB_UNROLL
    for (int t = 9; t < 15; ++t) W[t] = 0;
    W[15] = (64 + 32) * 8;
    hb_sha256_compress(st, W);
    HB_UNROLL
    for (int t = 0; t < 8; ++t) out[t] = st[t];
}

// ------------------------------------------------------------------ mod p
// p as NL little-endian limbs, Montgomery R = 2^(32 NL), pinv = -p^-1 mod 2^32,
// inv_scaled = 2^(32 (NL-2)) / p (double) for the final quotient estimate.
template <int NL>
struct ModP {
    u32 p[NL];
    u32 pinv;
    u32 pad_;
    double inv_scaled;
};

// acc (2NL+1 limbs) += a * b  (a, b: NL limbs).  Product scanning with a
// 96-bit column accumulator.
// (hi:lo) += a * b with lo 64-bit, hi 32-bit.  On gfx950 v_mad_u64_u32 has a
// carry-out, so one product-accumulate is 2 instructions (the generic C form
// compiles to a 64-bit add + compare + select per product).
HB_HD void hb_madc(u64 &lo, u32 &hi, u32 a, u32 b) {
#if defined(__HIP_DEVICE_COMPILE__)
    u64 cy;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\t"
        "v_addc_co_u32_e64 %1, %2, %1, 0, %2"
        : "+v"(lo), "+v"(hi), "=&s"(cy)
        : "v"(a), "v"(b));
#else
    u64 pr = (u64)a * b;
    u64 y = lo + pr;
    hi += (u32)(y < lo);
    lo = y;
#endif
}

// acc (2NL+1 limbs) += a * b  (a, b: NL limbs).  Product scanning with a
// 96-bit column accumulator (hi:lo).
template <int NL>
HB_HD void hb_mac(u32 acc[2 * NL + 1], const u32 *a, const u32 b[NL]) {
    u64 lo = 0;
    u32 hi = 0;
    HB_UNROLL
    for (int t = 0; t < 2 * NL - 1; ++t) {
        u64 x = lo + acc[t];
        hi += (u32)(x < lo);
        lo = x;
        const int a0 = t < NL ? 0 : t - NL + 1, a1 = t < NL ? t : NL - 1;
        HB_UNROLL
        for (int i = a0; i <= a1; ++i) hb_madc(lo, hi, a[i], b[t - i]);
        acc[t] = (u32)lo;
        lo = (lo >> 32) | ((u64)hi << 32);
        hi = 0;
    }
    // lo < (NL + 1) 2^32 here: adding one limb cannot wrap 64 bits.
    u64 x = lo + acc[2 * NL - 1];
    acc[2 * NL - 1] = (u32)x;
    acc[2 * NL] += (u32)(x >> 32);
}

// Montgomery reduction of acc (2NL+1 limbs, value T): v = (T + M p) / R with
// v < T/R + p, NL+1 limbs.
template <int NL>
HB_HD void hb_redc_row(u32 *acc, const ModP<NL> &P, int i, u32 &extra) {
    u32 q = acc[i] * P.pinv;
    u64 carry = 0;
    HB_UNROLL
    for (int b = 0; b < NL; ++b) {
        u64 t = (u64)q * P.p[b] + acc[i + b] + carry;
        acc[i + b] = (u32)t;
        carry = t >> 32;
    }
    u64 t = (u64)acc[i + NL] + carry + extra;
    acc[i + NL] = (u32)t;
    extra = (u32)(t >> 32);
}

// Rows I.. of the reduction with compile-time row indices: at NL = 32 the
// compiler leaves a plain outer loop rolled (32 x 32 MACs is past its unroll
// budget), which indexes acc dynamically and moves it to scratch.
template <int NL, int I>
HB_HD void hb_redc_rows(u32 *acc, const ModP<NL> &P, u32 &extra) {
    if constexpr (I < NL) {
        hb_redc_row<NL>(acc, P, I, extra);
        hb_redc_rows<NL, I + 1>(acc, P, extra);
    }
}

template <int NL>
HB_HD void hb_redc(u32 acc[2 * NL + 1], const ModP<NL> &P, u32 v[NL + 1]) {
    u32 extra = 0;
    if constexpr (NL <= 32) {
        hb_redc_rows<NL, 0>(acc, P, extra);
    } else {   // NL = 64 does not fit the register file either way
        for (int i = 0; i < NL; ++i) hb_redc_row<NL>(acc, P, i, extra);
    }
    acc[2 * NL] += extra;
    HB_UNROLL
    for (int t = 0; t <= NL; ++t) v[t] = acc[NL + t];
}

template <int E>
struct HbPow2 {   // 2^(32 E), E >= 0, as a compile-time double
    static constexpr double v = HbPow2<E - 1>::v * 4294967296.0;
};
template <>
struct HbPow2<0> { static constexpr double v = 1.0; };

// 2^(32 (T - (NL - 2))): limb T of a value scaled so that NL+1 limbs stay
// inside the double exponent range.  Limbs more than 31 limbs below the top
// (NL = 64 only) are dropped: they move the quotient estimate by < 2^-960
// relative, and the estimate is corrected by exact subtractions anyway.
template <int NL, int T>
struct HbScale {
    static constexpr int E = T - (NL - 2);
    static constexpr double v = E >= 0 ? HbPow2<(E >= 0 ? E : 0)>::v
                              : E < -31 ? 0.0 : 1.0 / HbPow2<(E < 0 && E >= -31 ? -E : 0)>::v;
};

// v (NL+1 limbs, v < 2^32 p) -> v mod p in out (NL limbs).
template <int NL>
HB_HD void hb_reduce_small(u32 v[NL + 1], const ModP<NL> &P, u32 out[NL]) {
    constexpr int T0 = NL - 2 - 31 > 0 ? NL - 2 - 31 : 0;   // lowest limb HbScale keeps
    double vd = 0.0, sc = HbScale<NL, T0>::v;
    HB_UNROLL
    for (int t = T0; t <= NL; ++t) {
        vd += (double)v[t] * sc;
        sc *= 4294967296.0;
    }
    double qd = vd * P.inv_scaled;
    u32 q = qd >= 2.0 ? (u32)qd - 1u : 0u;   // floor(qd) - 1 <= true quotient
    if (q) {
        u64 carry = 0;
        u32 borrow = 0;
        HB_UNROLL
        for (int t = 0; t <= NL; ++t) {
            u64 pr = (u64)q * (t < NL ? P.p[t] : 0u) + carry;
            carry = pr >> 32;
            u64 d = (u64)v[t] - (u32)pr - borrow;
            v[t] = (u32)d;
            borrow = (u32)(d >> 63);
        }
    }
    for (;;) {   // at most a few iterations
        u32 borrow = 0;
        u32 d[NL + 1];
        HB_UNROLL
        for (int t = 0; t <= NL; ++t) {
            u64 x = (u64)v[t] - (t < NL ? P.p[t] : 0u) - borrow;
            d[t] = (u32)x;
            borrow = (u32)(x >> 63);
        }
        if (borrow) break;   // v < p
        HB_UNROLL
        for (int t = 0; t <= NL; ++t) v[t] = d[t];
    }
    HB_UNROLL
    for (int t = 0; t < NL; ++t) out[t] = v[t];
}

// ------------------------------------------------------------------ sectors
// Little-endian limbs of the big-endian integer data[off .. off+r) (r <= 4 NL),
// byte by byte: used for tail sectors and unaligned sector sizes.
template <int NL>
HB_HD void hb_load_be_bytes(const unsigned char *data, u64 off, u32 r, u32 m[NL]) {
    HB_UNROLL
    for (int t = 0; t < NL; ++t) m[t] = 0;
    for (u32 k = 0; k < r; ++k) {
        u32 byte = data[off + k];
        HB_UNROLL
        for (int t = NL - 1; t > 0; --t) m[t] = hb_alignbit(m[t], m[t - 1], 24);
        m[0] = (m[0] << 8) | byte;
    }
}

// Whole sector, ss % 4 == 0 and data + off 4-byte aligned.
template <int NL>
HB_HD void hb_load_be_words(const unsigned char *data, u64 off, u32 ss, u32 m[NL]) {
    const u32 nw = ss >> 2;
    HB_UNROLL
    for (int t = 0; t < NL; ++t) {
        m[t] = 0;
        if ((u32)t < nw) m[t] = hb_bswap(*(const u32 *)(data + off + ss - 4u * (u32)(t + 1)));
    }
}

// Store v (NL limbs) as tw big-endian bytes at dst.
template <int NL>
HB_HD void hb_store_be(unsigned char *dst, u32 tw, const u32 v[NL]) {
    if ((tw & 3u) == 0) {
        HB_UNROLL
        for (int t = 0; t < NL; ++t)
            if (4u * (u32)(t + 1) <= tw) *(u32 *)(dst + tw - 4u * (u32)(t + 1)) = hb_bswap(v[t]);
    } else {
        HB_UNROLL
        for (int t = 0; t < NL; ++t)
            HB_UNROLL
            for (int b = 0; b < 4; ++b) {
                u32 pos = 4u * (u32)t + (u32)b;   // byte index from the least significant end
                if (pos < tw) dst[tw - 1 - pos] = (unsigned char)(v[t] >> (8 * b));
            }
    }
}

// hb_store_be for the kernels' sector-alignment class: ALIGN = 16 implies
// ss == 4 NL, i.e. a prime of exactly 32 NL bits and tw == 4 NL -- NL
// unconditional dword stores, none of the generic width's byte stores (whose
// offsets would otherwise stay live in registers).
template <int NL, int ALIGN>
HB_HD void hb_store_tag(unsigned char *dst, u32 tw, const u32 v[NL]) {
#if defined(HB_EXP_GENERIC_TAG_STORE)   // A/B: the generic store everywhere
    if (0) {
#else
    if (ALIGN == 16) {
#endif
        HB_UNROLL
        for (int t = 0; t < NL; ++t) *(u32 *)(dst + 4u * (u32)(NL - 1 - t)) = hb_bswap(v[t]);
    } else {
        hb_store_be<NL>(dst, tw, v);
    }
}

// ------------------------------------------------------------------ block tag
// Sector loads of a whole block.  ALIGN = 16: full-width sectors (ss == 4 NL,
// e.g. a 256-bit prime with 32-byte sectors), ss, C and the data base all
// 16-byte aligned: each sector is NL/4 unconditional 16-byte loads, issued for
// a batch of HB_GROUP(NL) sectors before any of them is consumed.  Any other
// shape (ALIGN = 1): byte loads.
template <int NL>
HB_HD void hb_load_full16(const unsigned char *data, u64 off, u32 m[NL]) {
#if defined(HB_EXP_MAC_NOLOAD)
    HB_UNROLL
    for (int t = 0; t < NL; ++t) m[t] = (u32)off * 2654435761u + (u32)t;
    return;
#endif
    HB_UNROLL
    for (int u = 0; u < NL / 4; ++u) {
        const u32 *q = (const u32 *)(data + off + 4u * NL - 16u * (u32)(u + 1));
#if defined(__HIP_DEVICE_COMPILE__)
        uint4 v = *(const uint4 *)q;
        const u32 w0 = v.x, w1 = v.y, w2 = v.z, w3 = v.w;
#else
        const u32 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
#endif
        m[4 * u + 0] = hb_bswap(w3);
        m[4 * u + 1] = hb_bswap(w2);
        m[4 * u + 2] = hb_bswap(w1);
        m[4 * u + 3] = hb_bswap(w0);
    }
}

// A whole ss-byte sector at data + off (ALIGN = 16: full-width, 16-byte aligned).
template <int NL, int ALIGN>
HB_HD void hb_load_full16_or_bytes(const unsigned char *data, u64 off, u32 ss, u32 m[NL]) {
    if (ALIGN == 16) hb_load_full16<NL>(data, off, m);
    else hb_load_be_bytes<NL>(data, off, ss, m);
}

template <int NL>
#ifndef HB_GROUP8
#define HB_GROUP8 2
#endif
struct HbGroup { static constexpr int v = NL <= 8 ? HB_GROUP8 : (NL <= 16 ? 2 : 1); };

// tag = (F + sum_j alpha_j m_j) mod p for block `blk` of the call
// (PySwizzle.py:297-307), with alpha in Montgomery form (alpha_j R mod p):
//   acc = F R + sum_j (alpha_j R) m_j  <  (S+1) p R
//   REDC(acc) = F + sum_j alpha_j m_j (mod p),  < (S+2) p
// then one small quotient-estimate reduction.  Sector j of the block is
// data[blk*C + j*ss : min(.. + ss, len)] as a big-endian integer (0 if empty);
// sectors after a short one are empty by construction, which is the
// reference's break at the first short read (PySwizzle.py:304-306).
template <int NL, int ALIGN>
HB_HD void hb_block_tag(const unsigned char *data, u64 len, u64 blk, u64 C, u32 ss, u32 S,
                        const u32 *alpha_mont, const ModP<NL> &M, const u32 F[NL], u32 tag[NL]) {
    u32 acc[2 * NL + 1];
    HB_UNROLL
    for (int t = 0; t < NL; ++t) { acc[t] = 0; acc[NL + t] = F[t]; }
    acc[2 * NL] = 0;
    const u64 base = blk * C;
    if (base + C <= len) {
        if (ALIGN == 16) {
            constexpr int G = HbGroup<NL>::v;
            u32 j = 0;
            HB_NOUNROLL
            for (; j + G <= S; j += G) {
                u32 m[G][NL];
                HB_UNROLL
                for (int g = 0; g < G; ++g) hb_load_full16<NL>(data, base + (u64)(j + g) * ss, m[g]);
                HB_UNROLL
                for (int g = 0; g < G; ++g) hb_mac<NL>(acc, alpha_mont + (u64)(j + g) * NL, m[g]);
            }
            HB_NOUNROLL
            for (; j < S; ++j) {
                u32 m[NL];
                hb_load_full16<NL>(data, base + (u64)j * ss, m);
                hb_mac<NL>(acc, alpha_mont + (u64)j * NL, m);
            }
        } else {
            HB_NOUNROLL
            for (u32 j = 0; j < S; ++j) {
                u32 m[NL];
                hb_load_be_bytes<NL>(data, base + (u64)j * ss, ss, m);
                hb_mac<NL>(acc, alpha_mont + (u64)j * NL, m);
            }
        }
    } else {
        HB_NOUNROLL
        for (u32 j = 0; j < S; ++j) {
            const u64 off = base + (u64)j * ss;
            if (off >= len) break;
            const u32 r = (u32)(len - off < ss ? len - off : ss);
            u32 m[NL];
            hb_load_be_bytes<NL>(data, off, r, m);
            hb_mac<NL>(acc, alpha_mont + (u64)j * NL, m);
            if (r != ss) break;
        }
    }
    u32 v[NL + 1];
    hb_redc<NL>(acc, M, v);
    hb_reduce_small<NL>(v, M, tag);
}

// x R mod p (x < R): REDC(x * (R^2 mod p)).
template <int NL>
HB_HD void hb_to_mont(const u32 x[NL], const u32 *r2, const ModP<NL> &M, u32 out[NL]) {
    u32 acc[2 * NL + 1];
    HB_UNROLL
    for (int t = 0; t <= 2 * NL; ++t) acc[t] = 0;
    hb_mac<NL>(acc, r2, x);
    u32 v[NL + 1];
    hb_redc<NL>(acc, M, v);
    hb_reduce_small<NL>(v, M, out);
}
