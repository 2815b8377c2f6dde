// hb_cpu_swizzle.cpp -- the "cxx Swizzle" CPU counterpart (BASELINE.md 3,
// SURVEY.md 8d): a competent native host encoder, timed beside the GPU in
// bench.py's cpu_baseline.  MEASUREMENT INFRASTRUCTURE, not the product and
// not the oracle: heartbeat_amd never loads it.
//
// Same function as hb_encode / PySwizzle.encode (heartbeat/PySwizzle/
// PySwizzle.py:279-314): tag_i = (F(i) + sum_j alpha_j m_ij) mod p with
// F = KeyedPRF(f_key, p), alpha_j = KeyedPRF(alpha_key, p)(j)
// (heartbeat/util.py:83-96); the reference's native loop is
// cxx/shacham_waters_private.cxx:672-697 (Crypto++ Integer per sector).
// Built the way a native host implementation would be:
//   * AES with AES-NI (aesenc), the key schedule expanded ONCE per key (the
//     reference re-keys per eval, util.py:88, but the schedule is the same);
//     CFB-8 keeps the 16-byte register in an XMM register, byte 0 of each
//     AES output is the keystream byte;
//   * 8 evaluations interleaved per thread (independent aesenc chains hide
//     the instruction latency); after every try accepted lanes take the next
//     block, rejected ones continue their stream -- the GPU engine's re-deal;
//   * SHA-256 of decimal(i) through OpenSSL (SHA-NI where the CPU has it);
//   * the MAC in 64-bit limbs with unsigned __int128: acc = F R +
//     sum_j (alpha_j R mod p) m_ij, one Montgomery reduction per block;
//   * std::thread over contiguous block ranges.
// Pinned to tests/golden/encode_cases.json by tests/test_cpu_baseline.py and
// cross-checked against the GPU tags in every bench run.
#define OPENSSL_SUPPRESS_DEPRECATED   // SHA256_Transform: the direct compression
#include <immintrin.h>
#include <openssl/sha.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "../heartbeat_amd/csrc/hb_aes_host.hpp"

typedef uint64_t u64;
typedef unsigned __int128 u128;

namespace {

// ------------------------------------------------------------------ AES
struct Aes {
    int nr = 0;
    hbhost::AesKey k;
    __m128i rk[15];
};

bool aes_init(const uint8_t *key, size_t len, Aes &a) {
    if (!hbhost::aes_expand(key, len, a.k)) return false;
    a.nr = a.k.nr;
    for (int r = 0; r <= a.nr; ++r) a.rk[r] = _mm_loadu_si128((const __m128i *)(a.k.bytes + 16 * r));
    return true;
}

// The fast path needs AES-NI + SSE4.1 (the CFB-8 engine) and BMI2 + ADX
// (mulx / adcx in the MAC); without any of them everything runs the portable
// byte AES and the unsigned __int128 MAC.
bool have_aesni() {
    static const bool v = __builtin_cpu_supports("aes") && __builtin_cpu_supports("sse4.1") &&
                          __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx");
    return v;
}

// Byte 0 of AES_k(reg[l]) for W registers (AES-NI, interleaved rounds).
template <int W>
__attribute__((target("aes,sse4.1"))) inline void aes_byte0_ni(const Aes &a, const __m128i *reg, uint8_t *o) {
    __m128i s[W];
    for (int l = 0; l < W; ++l) s[l] = _mm_xor_si128(reg[l], a.rk[0]);
    for (int r = 1; r < a.nr; ++r)
        for (int l = 0; l < W; ++l) s[l] = _mm_aesenc_si128(s[l], a.rk[r]);
    for (int l = 0; l < W; ++l) o[l] = (uint8_t)_mm_cvtsi128_si32(_mm_aesenclast_si128(s[l], a.rk[a.nr]));
}

// CFB-8 register shift: drop byte 0, append c as byte 15.
__attribute__((target("sse4.1"))) inline __m128i cfb_shift(__m128i r, uint8_t c) {
    return _mm_insert_epi8(_mm_srli_si128(r, 1), c, 15);
}

// ------------------------------------------------------------------ KeyedPRF
struct Prf {
    Aes aes;
    uint8_t R[512];   // range, nb big-endian bytes
    u64 nb = 0;       // ceil(bitlen(R) / 8): keystream bytes per try
    uint8_t topmask = 0xff;
};

int bitlen_be(const uint8_t *b, size_t n) {
    for (size_t i = 0; i < n; ++i)
        if (b[i]) return (int)(8 * (n - i) - __builtin_clz((unsigned)b[i]) + 24);
    return 0;
}

bool prf_init(const uint8_t *key, size_t key_len, const uint8_t *r_be, size_t r_len, Prf &P) {
    if (!aes_init(key, key_len, P.aes)) return false;
    const int bits = bitlen_be(r_be, r_len);
    if (bits == 0 || bits > 8 * 512) return false;
    P.nb = (u64)(bits + 7) / 8;
    memset(P.R, 0, sizeof P.R);
    memcpy(P.R + P.nb - std::min<u64>(P.nb, r_len), r_be + (r_len > P.nb ? r_len - P.nb : 0),
           std::min<u64>(P.nb, r_len));
    // mask = 2^bitlen(R) - 1 (util.py:81) on the most significant byte
    P.topmask = (uint8_t)((bits % 8) ? (1u << (bits % 8)) - 1 : 0xffu);
    return true;
}

// SHA-256 of ASCII decimal(x) (str(x).encode(), util.py:91): at most 20
// digits, so ONE compression of a block padded here, through OpenSSL's
// SHA256_Transform (SHA-NI where present).  The one-shot SHA256() of
// OpenSSL 3 fetches the algorithm from its provider on every call (~1 us and
// a lock), which would make this baseline measure OpenSSL, not the encode.
void digest_decimal(u64 x, uint8_t d[32]) {
    uint8_t blk[64];
    memset(blk, 0, sizeof blk);
    char t[24];
    int n = 0;
    do {
        t[n++] = (char)('0' + x % 10);
        x /= 10;
    } while (x);
    for (int i = 0; i < n; ++i) blk[i] = (uint8_t)t[n - 1 - i];
    blk[n] = 0x80;
    blk[63] = (uint8_t)(8 * n);
    SHA256_CTX c;
    SHA256_Init(&c);
    SHA256_Transform(&c, blk);
    for (int i = 0; i < 8; ++i) {
        d[4 * i] = (uint8_t)(c.h[i] >> 24);
        d[4 * i + 1] = (uint8_t)(c.h[i] >> 16);
        d[4 * i + 2] = (uint8_t)(c.h[i] >> 8);
        d[4 * i + 3] = (uint8_t)c.h[i];
    }
}

// Lanes of one thread's engine: W evaluations, each its own job.
template <int W>
struct Lanes {
    __m128i reg[W];
    uint8_t pt[W][512];   // plaintext: digest zero-padded / truncated to nb
    uint8_t out[W][512];
    u64 job[W];
    u64 tries[W];
    bool active[W];
};

// One try (nb CFB-8 steps) for every active lane; returns accepted mask bits.
template <int W>
__attribute__((target("aes,sse4.1"))) unsigned prf_try(const Prf &P, Lanes<W> &L) {
    for (u64 b = 0; b < P.nb; ++b) {
        uint8_t o[W];
        aes_byte0_ni<W>(P.aes, L.reg, o);
        for (int l = 0; l < W; ++l) {
            const uint8_t c = (uint8_t)(L.pt[l][b] ^ o[l]);
            L.out[l][b] = c;
            L.reg[l] = cfb_shift(L.reg[l], c);
        }
    }
    unsigned acc = 0;
    for (int l = 0; l < W; ++l) {
        if (!L.active[l]) continue;
        L.out[l][0] &= P.topmask;
        ++L.tries[l];
        if (memcmp(L.out[l], P.R, P.nb) < 0) acc |= 1u << l;
    }
    return acc;
}

// Portable single-lane path (no AES-NI): byte-oriented AES.
bool prf_eval_portable(const Prf &P, const uint8_t dig[32], uint8_t *out, u64 *tries) {
    uint8_t reg[16] = {0}, o[16], pt[512];
    memset(pt, 0, sizeof pt);
    memcpy(pt, dig, std::min<u64>(32, P.nb));
    for (u64 t = 0; t < 4096; ++t) {
        for (u64 b = 0; b < P.nb; ++b) {
            hbhost::aes_encrypt_block(P.aes.k, reg, o);
            const uint8_t c = (uint8_t)(pt[b] ^ o[0]);
            out[b] = c;
            memmove(reg, reg + 1, 15);
            reg[15] = c;
        }
        out[0] &= P.topmask;
        ++*tries;
        if (memcmp(out, P.R, P.nb) < 0) return true;
    }
    return false;
}

// ------------------------------------------------------------------ mod p
template <int N>
struct Mod {
    u64 p[N];
    u64 pinv;        // -p^-1 mod 2^64
    u64 r2[N];       // R^2 mod p, R = 2^(64 N)
};

template <int N>
bool geq(const u64 *a, const u64 *b) {   // a >= b, N limbs
    for (int i = N - 1; i >= 0; --i)
        if (a[i] != b[i]) return a[i] > b[i];
    return true;
}

template <int N>
void sub_in(u64 *a, const u64 *b) {
    u64 br = 0;
    for (int i = 0; i < N; ++i) {
        const u128 d = (u128)a[i] - b[i] - br;
        a[i] = (u64)d;
        br = (u64)(d >> 64) & 1;
    }
}

// BE bytes -> N little-endian limbs (right-aligned)
template <int N>
void from_be(const uint8_t *b, size_t n, u64 *x) {
    memset(x, 0, 8 * N);
    for (size_t i = 0; i < n; ++i) {
        const size_t pos = n - 1 - i;   // byte weight
        x[pos / 8] |= (u64)b[i] << (8 * (pos % 8));
    }
}

template <int N>
void to_be(const u64 *x, uint8_t *b, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const size_t pos = n - 1 - i;
        b[i] = (uint8_t)(x[pos / 8] >> (8 * (pos % 8)));
    }
}

// acc (2N+1 limbs) += a * b
template <int N>
inline void mac(u64 *acc, const u64 *a, const u64 *b) {
    for (int i = 0; i < N; ++i) {
        u64 carry = 0;
        for (int j = 0; j < N; ++j) {
            const u128 t = (u128)a[i] * b[j] + acc[i + j] + carry;
            acc[i + j] = (u64)t;
            carry = (u64)(t >> 64);
        }
        for (int k = i + N; carry && k <= 2 * N; ++k) {
            const u128 t = (u128)acc[k] + carry;
            acc[k] = (u64)t;
            carry = (u64)(t >> 64);
        }
    }
}

// v = REDC(acc) = acc / R mod-ish (N+1 limbs), then v mod p.
template <int N>
void redc_reduce(const Mod<N> &M, u64 *acc, u64 *out) {
    for (int i = 0; i < N; ++i) {
        const u64 q = acc[i] * M.pinv;
        u64 carry = 0;
        for (int j = 0; j < N; ++j) {
            const u128 t = (u128)q * M.p[j] + acc[i + j] + carry;
            acc[i + j] = (u64)t;
            carry = (u64)(t >> 64);
        }
        for (int k = i + N; carry && k <= 2 * N; ++k) {
            const u128 t = (u128)acc[k] + carry;
            acc[k] = (u64)t;
            carry = (u64)(t >> 64);
        }
    }
    u64 v[N + 1];
    for (int i = 0; i <= N; ++i) v[i] = acc[N + i];
    // v < (S + 2) p: quotient estimate from the top two limbs, then exact steps
    const u128 top = ((u128)v[N] << 64) | v[N - 1];
    const u128 q = top / ((u128)M.p[N - 1] + 1);
    if (q) {
        u64 carry = 0, br = 0;
        for (int i = 0; i <= N; ++i) {
            const u128 pr = (u128)(u64)q * (i < N ? M.p[i] : 0) + carry;
            carry = (u64)(pr >> 64);
            const u128 d = (u128)v[i] - (u64)pr - br;
            v[i] = (u64)d;
            br = (u64)(d >> 64) & 1;
        }
        // q fits 64 bits: v < 2^32 p here (S < 2^32), so top / (p_top + 1) < 2^33
    }
    u64 pp[N + 1];
    for (int i = 0; i < N; ++i) pp[i] = M.p[i];
    pp[N] = 0;
    while (geq<N + 1>(v, pp)) sub_in<N + 1>(v, pp);
    for (int i = 0; i < N; ++i) out[i] = v[i];
}

template <int N>
void mod_init(const uint8_t *p_be, size_t p_len, Mod<N> &M) {
    from_be<N>(p_be, p_len, M.p);
    u64 inv = 1;   // Newton: inv = p^-1 mod 2^64
    for (int i = 0; i < 7; ++i) inv *= 2 - M.p[0] * inv;
    M.pinv = 0 - inv;
    // R^2 mod p by doubling 1 (2 * 64 N) times
    u64 x[N + 1];
    memset(x, 0, sizeof x);
    x[0] = 1;
    u64 pp[N + 1];
    for (int i = 0; i < N; ++i) pp[i] = M.p[i];
    pp[N] = 0;
    for (int k = 0; k < 128 * N; ++k) {
        u64 c = 0;
        for (int i = 0; i <= N; ++i) {
            const u64 nc = x[i] >> 63;
            x[i] = (x[i] << 1) | c;
            c = nc;
        }
        if (geq<N + 1>(x, pp)) sub_in<N + 1>(x, pp);
    }
    for (int i = 0; i < N; ++i) M.r2[i] = x[i];
}

// x R mod p
template <int N>
void to_mont(const Mod<N> &M, const u64 *x, u64 *out) {
    u64 acc[2 * N + 1];
    memset(acc, 0, sizeof acc);
    mac<N>(acc, x, M.r2);
    redc_reduce<N>(M, acc, out);
}

// ------------------------------------------------------------------ encode
struct Job {
    const uint8_t *data;
    u64 len, C, block_base;
    u64 ss, tw;
    uint32_t S;
};

// (hi:mid:lo) += (y:x), 192-bit accumulator
__attribute__((target("bmi2,adx"))) inline void acc3(u64 &lo, u64 &mid, u64 &hi, u64 x, u64 y) {
    unsigned long long l = lo, m = mid;
    unsigned char c = _addcarry_u64(0, l, x, &l);
    c = _addcarry_u64(c, m, y, &m);
    lo = l;
    mid = m;
    hi += c;
}

// (hi:mid:lo) += a * b
__attribute__((target("bmi2,adx"))) inline void mulacc(u64 &lo, u64 &mid, u64 &hi, u64 a, u64 b) {
    unsigned long long ph;
    const u64 pl = _mulx_u64(a, b, &ph);
    acc3(lo, mid, hi, pl, ph);
}

// whole sector of 8N big-endian bytes: N byte-swapped word loads
template <int N>
inline void load_full(const uint8_t *b, u64 *m) {
    for (int i = 0; i < N; ++i) {
        u64 w;
        memcpy(&w, b + 8 * (N - 1 - i), 8);
        m[i] = __builtin_bswap64(w);
    }
}

template <int N>
__attribute__((target("bmi2,adx"))) void tag_block(const Job &J, const Mod<N> &M, const std::vector<u64> &am, u64 blk, const uint8_t *F_be,
               u64 nbF, uint8_t *tag) {
    // the block's sectors as limbs (m[j]), then sum_j a_j m_j by product
    // scanning: column k = sum_j sum_{i + l = k} a_ji m_jl in three registers
    // (lo, mid, hi), carries resolved once per column
    u64 mm[64 * N];
    u64 *m = (J.S <= 64) ? mm : nullptr;
    std::vector<u64> big;
    if (!m) {
        big.resize((size_t)J.S * N);
        m = big.data();
    }
    u64 F[N];
    from_be<N>(F_be, nbF, F);
    const u64 base = blk * J.C;
    const bool full = J.ss == 8 * N;
    uint32_t ns = 0;
    for (uint32_t j = 0; j < J.S; ++j) {
        const u64 off = base + (u64)j * J.ss;
        if (off >= J.len) break;
        const u64 r = std::min<u64>(J.ss, J.len - off);
        if (full && r == J.ss) load_full<N>(J.data + off, m + (size_t)j * N);
        else from_be<N>(J.data + off, r, m + (size_t)j * N);
        ++ns;
        if (r != J.ss) break;   // the reference's stop at the first short read
    }
    const u64 *a = am.data();
    u64 acc[2 * N + 1];
    u64 c0 = 0, c1 = 0;   // carry into the next column (128 bits)
    for (int k = 0; k < 2 * N; ++k) {
        // two independent accumulator chains (even / odd sectors) for ILP
        u64 lo[2] = {c0, 0}, mid[2] = {c1, 0}, hi[2] = {0, 0};
        if (k >= N) acc3(lo[0], mid[0], hi[0], F[k - N], 0);   // + F R
        const int i0 = k < N ? 0 : k - N + 1, i1 = k < N ? k : N - 1;
        uint32_t j = 0;
        for (; j + 1 < ns; j += 2)
            for (int i = i0; i <= i1; ++i) {
                mulacc(lo[0], mid[0], hi[0], a[(size_t)j * N + i], m[(size_t)j * N + k - i]);
                mulacc(lo[1], mid[1], hi[1], a[(size_t)(j + 1) * N + i], m[(size_t)(j + 1) * N + k - i]);
            }
        for (; j < ns; ++j)
            for (int i = i0; i <= i1; ++i) mulacc(lo[0], mid[0], hi[0], a[(size_t)j * N + i], m[(size_t)j * N + k - i]);
        acc3(lo[0], mid[0], hi[0], lo[1], mid[1]);
        hi[0] += hi[1];
        acc[k] = lo[0];
        c0 = mid[0];
        c1 = hi[0];
    }
    acc[2 * N] = c0;   // c1 == 0: the total is < (S + 1) p R < 2^(64 (2N + 1))
    u64 t[N];
    redc_reduce<N>(M, acc, t);
    to_be<N>(t, tag, J.tw);
}

// The same tag without BMI2 / ADX: operand scanning in unsigned __int128.
template <int N>
void tag_block_portable(const Job &J, const Mod<N> &M, const std::vector<u64> &am, u64 blk, const uint8_t *F_be,
                        u64 nbF, uint8_t *tag) {
    u64 acc[2 * N + 1];
    memset(acc, 0, sizeof acc);
    u64 F[N], m[N];
    from_be<N>(F_be, nbF, F);
    for (int i = 0; i < N; ++i) {   // + F R
        u64 c = F[i];
        for (int k = N + i; c && k <= 2 * N; ++k) {
            const u128 t = (u128)acc[k] + c;
            acc[k] = (u64)t;
            c = (u64)(t >> 64);
        }
    }
    const u64 base = blk * J.C;
    for (uint32_t j = 0; j < J.S; ++j) {
        const u64 off = base + (u64)j * J.ss;
        if (off >= J.len) break;
        const u64 r = std::min<u64>(J.ss, J.len - off);
        from_be<N>(J.data + off, r, m);
        mac<N>(acc, am.data() + (size_t)j * N, m);
        if (r != J.ss) break;
    }
    u64 t[N];
    redc_reduce<N>(M, acc, t);
    to_be<N>(t, tag, J.tw);
}

template <int N, int W>
__attribute__((target("aes,sse4.1"))) void encode_range(const Job &J, const Prf &P, const Mod<N> &M,
                                                        const std::vector<u64> &am, u64 b0, u64 b1,
                                                        uint8_t *tags, u64 *tries_out, int *fail) {
    Lanes<W> L;
    u64 next = b0, tries = 0;
    auto load = [&](int l) {
        L.active[l] = next < b1;
        L.reg[l] = _mm_setzero_si128();   // fresh cipher per eval (util.py:88)
        L.tries[l] = 0;
        if (!L.active[l]) return;
        L.job[l] = next++;
        uint8_t d[32];
        digest_decimal(J.block_base + L.job[l], d);
        memset(L.pt[l], 0, P.nb);
        memcpy(L.pt[l], d, std::min<u64>(32, P.nb));
    };
    for (int l = 0; l < W; ++l) load(l);
    for (;;) {
        bool any = false;
        for (int l = 0; l < W; ++l) any |= L.active[l];
        if (!any) break;
        const unsigned acc = prf_try<W>(P, L);
        for (int l = 0; l < W; ++l) {
            if (!L.active[l]) continue;
            if (acc >> l & 1) {
                tries += L.tries[l];
                tag_block<N>(J, M, am, L.job[l], L.out[l], P.nb, tags + L.job[l] * J.tw);
                load(l);
            } else if (L.tries[l] >= 4096) {
                *fail = 1;
                L.active[l] = false;
            }
        }
    }
    *tries_out = tries;
}

template <int N>
int encode_n(const uint8_t *p_be, size_t p_len, uint32_t S, const uint8_t *f_key, const uint8_t *a_key,
             size_t key_len, u64 block_base, const uint8_t *data, u64 len, u64 nblocks, uint8_t *tags,
             int threads, u64 *tries_out) {
    Mod<N> M;
    mod_init<N>(p_be, p_len, M);
    Prf Pf, Pa;
    if (!prf_init(f_key, key_len, p_be, p_len, Pf) || !prf_init(a_key, key_len, p_be, p_len, Pa)) return -1;
    const int bits = bitlen_be(p_be, p_len);
    Job J{data, len, 0, block_base, (u64)bits / 8, (u64)(bits + 7) / 8, S};
    J.C = J.ss * S;
    // alpha_j R mod p (PySwizzle.py:291, 302)
    std::vector<u64> am((size_t)S * N);
    for (uint32_t j = 0; j < S; ++j) {
        uint8_t d[32], out[512];
        digest_decimal(j, d);
        u64 tr = 0;
        if (!prf_eval_portable(Pa, d, out, &tr)) return -2;
        u64 a[N];
        from_be<N>(out, Pa.nb, a);
        to_mont<N>(M, a, am.data() + (size_t)j * N);
    }
    threads = std::max(1, threads);
    const u64 T = std::min<u64>((u64)threads, std::max<u64>(1, nblocks));
    std::vector<std::thread> ts;
    std::vector<u64> tr(T, 0);
    std::vector<int> fl(T, 0);
    for (u64 t = 0; t < T; ++t) {
        const u64 b0 = nblocks * t / T, b1 = nblocks * (t + 1) / T;
        ts.emplace_back([&, t, b0, b1] {
            if (have_aesni()) {
                encode_range<N, 8>(J, Pf, M, am, b0, b1, tags, &tr[t], &fl[t]);
            } else {
                for (u64 b = b0; b < b1; ++b) {
                    uint8_t d[32], out[512];
                    digest_decimal(block_base + b, d);
                    if (!prf_eval_portable(Pf, d, out, &tr[t])) fl[t] = 1;
                    tag_block_portable<N>(J, M, am, b, out, Pf.nb, tags + b * J.tw);
                }
            }
        });
    }
    for (auto &th : ts) th.join();
    u64 sum = 0;
    int f = 0;
    for (u64 t = 0; t < T; ++t) {
        sum += tr[t];
        f |= fl[t];
    }
    if (tries_out) *tries_out = sum;
    return f ? -3 : 0;
}

// ------------------------------------------------------------------ prove
// KeyedPRF(P)(x0 + k) for k < n, nb big-endian bytes each: the encode's
// interleaved AES-NI engine (W evaluations per thread, re-dealt per try).
template <int W>
__attribute__((target("aes,sse4.1"))) void prf_range_ni(const Prf &P, u64 x0, u64 n, uint8_t *out, int *fail) {
    Lanes<W> L;
    u64 next = 0;
    auto load = [&](int l) {
        L.active[l] = next < n;
        L.reg[l] = _mm_setzero_si128();
        L.tries[l] = 0;
        if (!L.active[l]) return;
        L.job[l] = next++;
        uint8_t d[32];
        digest_decimal(x0 + L.job[l], d);
        memset(L.pt[l], 0, P.nb);
        memcpy(L.pt[l], d, std::min<u64>(32, P.nb));
    };
    for (int l = 0; l < W; ++l) load(l);
    for (;;) {
        bool any = false;
        for (int l = 0; l < W; ++l) any |= L.active[l];
        if (!any) break;
        const unsigned acc = prf_try<W>(P, L);
        for (int l = 0; l < W; ++l) {
            if (!L.active[l]) continue;
            if (acc >> l & 1) {
                memcpy(out + L.job[l] * P.nb, L.out[l], P.nb);
                load(l);
            } else if (L.tries[l] >= 4096) {
                *fail = 1;
                L.active[l] = false;
            }
        }
    }
}

void prf_range(const Prf &P, u64 x0, u64 n, uint8_t *out, int *fail) {
    if (have_aesni()) return prf_range_ni<8>(P, x0, n, out, fail);
    u64 tr = 0;
    for (u64 k = 0; k < n; ++k) {
        uint8_t d[32];
        digest_decimal(x0 + k, d);
        if (!prf_eval_portable(P, d, out + k * P.nb, &tr)) *fail = 1;
    }
}

// acc (2N + 1 limbs) -> acc mod p: REDC gives acc R^-1 mod p, one more
// Montgomery multiplication by R^2 gives acc mod p.
template <int N>
void acc_mod(const Mod<N> &M, u64 *acc, u64 *out) {
    u64 t[N];
    redc_reduce<N>(M, acc, t);
    to_mont<N>(M, t, out);
}

// PySwizzle.prove (heartbeat/PySwizzle/PySwizzle.py:333-370): idx_i =
// KeyedPRF(key, ntags)(i), v_i = KeyedPRF(key, v_max)(i); mu_j = sum_i v_i
// m_{idx_i, j} mod p (sector j of block idx_i read at idx_i C + j ss, a short
// read counts as its bytes and ends the block), sigma = sum_i v_i tag[idx_i]
// mod p.  The reference's native loop is cxx/shacham_waters_private.cxx:731-789.
// Threads take contiguous slices of the challenge; every sum stays exact in
// 2N + 1 limbs until the end.
template <int N>
int prove_n(const uint8_t *p_be, size_t p_len, uint32_t S, const uint8_t *key, size_t key_len, u64 chunks,
            const uint8_t *vmax_be, size_t vmax_len, u64 ntags, const uint8_t *tags, const uint8_t *data, u64 len,
            int threads, uint8_t *mu_out, uint8_t *sigma_out) {
    Mod<N> M;
    mod_init<N>(p_be, p_len, M);
    const int bits = bitlen_be(p_be, p_len);
    const u64 ss = (u64)bits / 8, tw = (u64)(bits + 7) / 8, C = ss * S;
    if (bitlen_be(vmax_be, vmax_len) > 64 * N) return -4;
    uint8_t nbe[8];
    for (int k = 0; k < 8; ++k) nbe[k] = (uint8_t)(ntags >> (56 - 8 * k));
    Prf Pi, Pv;
    if (!prf_init(key, key_len, nbe, 8, Pi) || !prf_init(key, key_len, vmax_be, vmax_len, Pv)) return -1;
    threads = std::max(1, threads);
    const u64 T = std::min<u64>((u64)threads, std::max<u64>(1, chunks / 64));
    const size_t W = 2 * N + 1;
    std::vector<u64> accs((size_t)T * (S + 1) * W, 0);
    std::vector<int> fl(T, 0);
    std::vector<std::thread> ts;
    for (u64 t = 0; t < T; ++t) {
        ts.emplace_back([&, t] {
            const u64 i0 = chunks * t / T, i1 = chunks * (t + 1) / T, n = i1 - i0;
            std::vector<uint8_t> ib((size_t)n * Pi.nb), vb((size_t)n * Pv.nb);
            prf_range(Pi, i0, n, ib.data(), &fl[t]);
            prf_range(Pv, i0, n, vb.data(), &fl[t]);
            u64 *acc = &accs[(size_t)t * (S + 1) * W];
            u64 v[N], m[N];
            for (u64 k = 0; k < n; ++k) {
                u64 ix = 0;
                for (u64 b = 0; b < Pi.nb; ++b) ix = (ix << 8) | ib[(size_t)(k * Pi.nb + b)];
                from_be<N>(&vb[(size_t)(k * Pv.nb)], Pv.nb, v);
                const u64 base = ix * C;
                for (uint32_t j = 0; j < S; ++j) {
                    const u64 off = base + (u64)j * ss;
                    if (off >= len) break;
                    const u64 r = std::min<u64>(ss, len - off);
                    from_be<N>(data + off, r, m);
                    mac<N>(acc + (size_t)j * W, v, m);
                    if (r != ss) break;
                }
                from_be<N>(tags + ix * tw, tw, m);
                mac<N>(acc + (size_t)S * W, v, m);
            }
        });
    }
    for (auto &th : ts) th.join();
    for (u64 t = 0; t < T; ++t)
        if (fl[t]) return -3;
    for (uint32_t j = 0; j <= S; ++j) {
        u64 sum[2 * N + 1];
        memset(sum, 0, sizeof sum);
        for (u64 t = 0; t < T; ++t) {
            const u64 *a = &accs[((size_t)t * (S + 1) + j) * W];
            u64 c = 0;
            for (size_t k = 0; k < W; ++k) {
                const u128 x = (u128)sum[k] + a[k] + c;
                sum[k] = (u64)x;
                c = (u64)(x >> 64);
            }
        }
        u64 r[N];
        acc_mod<N>(M, sum, r);
        to_be<N>(r, j < S ? mu_out + (size_t)j * tw : sigma_out, tw);
    }
    return 0;
}

}  // namespace

extern "C" {

// hb_encode's contract on host memory (include/hbswizzle.h): tags of blocks
// block_base .. block_base + nblocks - 1 of `data`, tw big-endian bytes each.
// Returns 0, -1 (bad key / prime), -2 / -3 (PRF did not terminate), -4
// (prime above 2048 bits).
int hbcpu_encode(const uint8_t *p_be, size_t p_len, uint32_t S, const uint8_t *f_key, const uint8_t *a_key,
                 size_t key_len, uint64_t block_base, const uint8_t *data, uint64_t len, uint64_t nblocks,
                 uint8_t *tags, int threads, uint64_t *tries_out) {
    const int bits = bitlen_be(p_be, p_len);
    if (bits < 8 || !(p_be[p_len - 1] & 1)) return -1;
    if (bits <= 64) return encode_n<1>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    if (bits <= 128) return encode_n<2>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    if (bits <= 256) return encode_n<4>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    if (bits <= 512) return encode_n<8>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    if (bits <= 1024) return encode_n<16>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    if (bits <= 2048) return encode_n<32>(p_be, p_len, S, f_key, a_key, key_len, block_base, data, len, nblocks, tags, threads, tries_out);
    return -4;
}

// PySwizzle.prove on host memory (hb_prove's contract, include/hbswizzle.h):
// mu (S x tw bytes) and sigma (tw bytes), big-endian.  Every index must be
// < ntags (KeyedPRF(key, ntags) guarantees it).  Returns 0, -1 (bad key /
// prime), -3 (PRF did not terminate), -4 (prime or v_max too wide).
int hbcpu_prove(const uint8_t *p_be, size_t p_len, uint32_t S, const uint8_t *key, size_t key_len,
                uint64_t chunks, const uint8_t *vmax_be, size_t vmax_len, uint64_t ntags, const uint8_t *tags,
                const uint8_t *data, uint64_t len, int threads, uint8_t *mu_out, uint8_t *sigma_out) {
    const int bits = bitlen_be(p_be, p_len);
    if (bits < 8 || !(p_be[p_len - 1] & 1) || ntags == 0) return -1;
#define HB_PROVE_N(N) prove_n<N>(p_be, p_len, S, key, key_len, chunks, vmax_be, vmax_len, ntags, tags, data, len, \
                                 threads, mu_out, sigma_out)
    if (bits <= 64) return HB_PROVE_N(1);
    if (bits <= 128) return HB_PROVE_N(2);
    if (bits <= 256) return HB_PROVE_N(4);
    if (bits <= 512) return HB_PROVE_N(8);
    if (bits <= 1024) return HB_PROVE_N(16);
    if (bits <= 2048) return HB_PROVE_N(32);
#undef HB_PROVE_N
    return -4;
}

// Whether the AES-NI path runs on this host (else the portable byte AES).
int hbcpu_aesni(void) { return have_aesni() ? 1 : 0; }

// SplitMix64 synthetic bytes of the GPU's hb_fill_random stream (bench.py):
// 16-byte unit k = two u64 words x(seed, 2k), x(seed, 2k + 1), little-endian.
void hbcpu_fill(uint8_t *dst, uint64_t start, uint64_t n, uint64_t seed, int threads) {
    auto word = [seed](u64 i) {
        u64 x = seed ^ (i * 0xD1B54A32D192ED03ull);
        x += 0x9E3779B97F4A7C15ull;
        x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
        x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
        return x ^ (x >> 31);
    };
    threads = std::max(1, threads);
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) {
        const u64 a = n * t / threads, b = n * (t + 1) / threads;
        ts.emplace_back([=] {
            for (u64 i = a; i < b;) {
                const u64 pos = start + i, wi = pos / 8, o = pos % 8;
                const u64 w = word(wi);
                const u64 take = std::min<u64>(8 - o, b - i);
                memcpy(dst + i, (const uint8_t *)&w + o, take);
                i += take;
            }
        });
    }
    for (auto &th : ts) th.join();
}

}  // extern "C"
