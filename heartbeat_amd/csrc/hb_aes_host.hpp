// hb_aes_host.hpp -- host-side AES tables and key schedule (FIPS-197).
//
// Used by the host runtime to build (a) the 1 KiB T0 table that every encode /
// PRF workgroup expands into its LDS-resident, bank-replicated T0/T1 image and
// (b) the round keys that the kernels read as wave-uniform (scalar) operands.
// Also provides a small host AES-CFB8 for PySwizzle State encryption
// (heartbeat/PySwizzle/PySwizzle.py:162-195), which is 64 bytes per call.
#pragma once
#include <stdint.h>
#include <string.h>

namespace hbhost {

struct AesTables {
    uint8_t sbox[256];
    uint32_t t0[256];   // little-endian column word (2s, s, s, 3s)
};

inline uint8_t gf_xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

inline uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t r = 0;
    while (b) {
        if (b & 1) r ^= a;
        a = gf_xtime(a);
        b >>= 1;
    }
    return r;
}

inline const AesTables &aes_tables() {
    static AesTables T = [] {
        AesTables t;
        for (int x = 0; x < 256; ++x) {
            // multiplicative inverse in GF(2^8) (0 -> 0), then the affine map
            uint8_t inv = 0;
            if (x) {
                for (int y = 1; y < 256; ++y)
                    if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
            }
            uint8_t s = inv;
            uint8_t r = inv;
            for (int i = 0; i < 4; ++i) {
                r = (uint8_t)((r << 1) | (r >> 7));
                s ^= r;
            }
            t.sbox[x] = (uint8_t)(s ^ 0x63);
        }
        for (int x = 0; x < 256; ++x) {
            uint8_t s = t.sbox[x];
            uint8_t s2 = gf_xtime(s), s3 = (uint8_t)(s2 ^ s);
            t.t0[x] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
        }
        return t;
    }();
    return T;
}

// Expanded key: nr+1 round keys, 4 little-endian column words each
// (word c of round r = bytes 4c..4c+3 of round key r, byte 4c in bits 0..7).
struct AesKey {
    int nr = 0;
    uint32_t rk[60];
    uint8_t bytes[240];
};

inline bool aes_expand(const uint8_t *key, size_t key_len, AesKey &k) {
    if (key_len != 16 && key_len != 24 && key_len != 32) return false;
    const AesTables &T = aes_tables();
    int nk = (int)key_len / 4;
    k.nr = nk + 6;
    int total = 4 * (k.nr + 1);
    uint8_t *w = k.bytes;
    memcpy(w, key, key_len);
    uint8_t rcon = 1;
    for (int i = nk; i < total; ++i) {
        uint8_t t[4];
        memcpy(t, w + 4 * (i - 1), 4);
        if (i % nk == 0) {
            uint8_t u = t[0];
            t[0] = (uint8_t)(T.sbox[t[1]] ^ rcon);
            t[1] = T.sbox[t[2]];
            t[2] = T.sbox[t[3]];
            t[3] = T.sbox[u];
            rcon = gf_xtime(rcon);
        } else if (nk > 6 && i % nk == 4) {
            for (int j = 0; j < 4; ++j) t[j] = T.sbox[t[j]];
        }
        for (int j = 0; j < 4; ++j) w[4 * i + j] = (uint8_t)(w[4 * (i - nk) + j] ^ t[j]);
    }
    for (int i = 0; i < total; ++i)
        k.rk[i] = (uint32_t)w[4 * i] | ((uint32_t)w[4 * i + 1] << 8) |
                  ((uint32_t)w[4 * i + 2] << 16) | ((uint32_t)w[4 * i + 3] << 24);
    return true;
}

// Round-1 constants of CFB-8 steps whose register starts with z = 1..3 zero
// words (device: hb_aes_round1_z, PrfParams::r1z): for z and output column c,
// round key 1 word c XOR the T-table lookups of column c that read a word
// w_j = rk[j], j < z (column c reads byte r of word (c + r) mod 4 through
// T_r = rotl(T0, 8 r)).
inline void aes_round1_zero_consts(const AesKey &k, uint32_t out[12]) {
    const AesTables &T = aes_tables();
    for (int z = 1; z <= 3; ++z)
        for (int c = 0; c < 4; ++c) {
            uint32_t v = k.rk[4 + c];
            for (int r = 0; r < 4; ++r) {
                const int j = (c + r) & 3;
                if (j >= z) continue;
                const uint32_t t = T.t0[(k.rk[j] >> (8 * r)) & 0xffu];
                v ^= r ? (t << (8 * r)) | (t >> (32 - 8 * r)) : t;
            }
            out[4 * (z - 1) + c] = v;
        }
}

// Plain byte-oriented AES encryption of one block (host; State encryption only).
inline void aes_encrypt_block(const AesKey &k, const uint8_t in[16], uint8_t out[16]) {
    const AesTables &T = aes_tables();
    uint8_t s[16];
    for (int i = 0; i < 16; ++i) s[i] = (uint8_t)(in[i] ^ k.bytes[i]);
    for (int r = 1; r <= k.nr; ++r) {
        uint8_t t[16];
        for (int i = 0; i < 16; ++i) t[i] = T.sbox[s[i]];
        // ShiftRows: row r of column c comes from column (c + r) mod 4
        for (int c = 0; c < 4; ++c)
            for (int row = 0; row < 4; ++row) s[4 * c + row] = t[4 * ((c + row) & 3) + row];
        if (r != k.nr) {
            for (int c = 0; c < 4; ++c) {
                uint8_t a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
                uint8_t x = (uint8_t)(a0 ^ a1 ^ a2 ^ a3);
                s[4 * c] = (uint8_t)(a0 ^ x ^ gf_xtime((uint8_t)(a0 ^ a1)));
                s[4 * c + 1] = (uint8_t)(a1 ^ x ^ gf_xtime((uint8_t)(a1 ^ a2)));
                s[4 * c + 2] = (uint8_t)(a2 ^ x ^ gf_xtime((uint8_t)(a2 ^ a3)));
                s[4 * c + 3] = (uint8_t)(a3 ^ x ^ gf_xtime((uint8_t)(a3 ^ a0)));
            }
        }
        for (int i = 0; i < 16; ++i) s[i] ^= k.bytes[16 * r + i];
    }
    memcpy(out, s, 16);
}

// AES-CFB with 8-bit segments (PyCrypto MODE_CFB default, util.py:88).
inline void aes_cfb8(const AesKey &k, const uint8_t iv[16], const uint8_t *in, uint8_t *out,
                     size_t n, bool encrypt) {
    uint8_t sr[16], o[16];
    memcpy(sr, iv, 16);
    for (size_t i = 0; i < n; ++i) {
        aes_encrypt_block(k, sr, o);
        uint8_t c = encrypt ? (uint8_t)(in[i] ^ o[0]) : in[i];
        out[i] = (uint8_t)(in[i] ^ o[0]);
        memmove(sr, sr + 1, 15);
        sr[15] = c;
    }
}

// Full-block CFB (CFB-128, Crypto++ CFB_Mode<AES>, a stream mode: no padding,
// a final partial block uses the first bytes of its keystream block).
inline void aes_cfb128(const AesKey &k, const uint8_t iv[16], const uint8_t *in, uint8_t *out,
                       size_t n, bool encrypt) {
    uint8_t reg[16], o[16];
    memcpy(reg, iv, 16);
    for (size_t i = 0; i < n; i += 16) {
        aes_encrypt_block(k, reg, o);
        const size_t m = n - i < 16 ? n - i : 16;
        for (size_t b = 0; b < m; ++b) {
            const uint8_t x = in[i + b];
            out[i + b] = (uint8_t)(x ^ o[b]);
            reg[b] = encrypt ? out[i + b] : x;   // feedback = ciphertext
        }
    }
}

}  // namespace hbhost
