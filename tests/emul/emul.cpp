// CPU emulation of ONE GPU lane of the Swizzle kernels (test tool only).
//
// Compiles heartbeat_amd/csrc/hb_lane.hpp as plain C++ and runs the exact lane
// logic of the encode / PRF kernels sequentially -- same LDS table layout
// (built for a chosen lane id), same CFB-8 byte-0 AES, same SHA-256 message
// builder, same Montgomery MAC / reduction -- so it can be compared with the
// CPU oracle without a GPU (tests/test_emul.py).  Not part of the product.
#include "../../heartbeat_amd/csrc/hb_lane.hpp"
#include "../../heartbeat_amd/csrc/hb_aes_host.hpp"
#include "../../heartbeat_amd/csrc/hb_bignum_host.hpp"
#include <stdlib.h>
#include <string.h>
#include <map>
#include <string>
#include <vector>

using namespace hbhost;

static std::vector<char> g_tab(HB_TAB_BYTES);

static LaneTab make_tab(int lane) {
    const AesTables &T = aes_tables();
    for (int e = 0; e < 256; ++e)
        for (int t = 0; t < 4; ++t)
            for (int r = 0; r < 32; ++r) {
                uint32_t v = T.t0[e];
                if (t) v = (v << (8 * t)) | (v >> (32 - 8 * t));
                memcpy(&g_tab[(t >> 1) * 65536 + e * 256 + (t & 1) * 128 + r * 4], &v, 4);
            }
    LaneTab L;
    L.tab = g_tab.data();
    const uint32_t r4 = (uint32_t)(lane & 31) * 4u;
    L.lb[0] = r4;
    L.lb[1] = 128u + r4;
    L.lb[2] = 0x10000u | r4;
    L.lb[3] = 0x10000u | (128u + r4);
    return L;
}

template <int NL>
static bool make_prf(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen,
                     PrfParams<NL> &P, int &nr) {
    AesKey k;
    if (!aes_expand(key, keylen, k)) return false;
    nr = k.nr;
    memset(&P, 0, sizeof P);
    memcpy(P.rk, k.rk, sizeof(uint32_t) * 4 * (k.nr + 1));
    aes_round1_zero_consts(k, P.r1z);
    Limbs R = from_be(range_be, rlen, NL);
    for (int t = 0; t < NL; ++t) P.R[t] = R[t];
    int bits = bitlen_be(range_be, rlen);
    P.nb = (uint32_t)(bits + 7) / 8;
    int top = bits - 8 * ((int)P.nb - 1);
    P.topmask = (1u << top) - 1u;
    return bits > 0 && (int)P.nb <= 4 * NL;
}

// Prefix image of the two-pass encode (hb_lane.hpp, CFB prefix), filled
// independently of the lane code: P1 and P2 completely and P3 on demand, each
// entry from the byte-oriented host AES of the register bytes the entry stands
// for.  Entries of P3 never filled stay 0, so a lane that indexes the image
// wrongly reads a wrong keystream byte and the tags differ.
struct Prefix {
    AesKey k;
    uint8_t o0 = 0;
    std::vector<uint8_t> img;
    std::vector<uint8_t> have3;
    static uint8_t byte0(const AesKey &k, const uint8_t reg[16]) {
        uint8_t o[16];
        aes_encrypt_block(k, reg, o);
        return o[0];
    }
    void init(const uint8_t *key, size_t keylen) {
        aes_expand(key, keylen, k);
        img.assign(HB_PFX_BYTES, 0);
        have3.assign(1u << 24, 0);
        uint8_t reg[16] = {0};
        o0 = byte0(k, reg);
        for (int c0 = 0; c0 < 256; ++c0) {
            memset(reg, 0, 16);
            reg[15] = (uint8_t)c0;
            img[HB_PFX_P1 + c0] = byte0(k, reg);
            for (int c1 = 0; c1 < 256; ++c1) {
                memset(reg, 0, 16);
                reg[14] = (uint8_t)c0;
                reg[15] = (uint8_t)c1;
                img[HB_PFX_P2 + (c0 | c1 << 8)] = byte0(k, reg);
            }
        }
    }
    // make sure the P3 entry the eval of digest word d needs is present
    void need(uint32_t d) {
        uint8_t reg[16] = {0};
        uint8_t c0 = (uint8_t)((d >> 24) ^ o0);
        reg[15] = c0;
        uint8_t c1 = (uint8_t)((d >> 16) ^ byte0(k, reg));
        memset(reg, 0, 16);
        reg[14] = c0;
        reg[15] = c1;
        uint8_t c2 = (uint8_t)((d >> 8) ^ byte0(k, reg));
        uint32_t ix = (uint32_t)c0 | (uint32_t)c1 << 8 | (uint32_t)c2 << 16;
        if (have3[ix]) return;
        memset(reg, 0, 16);
        reg[13] = c0;
        reg[14] = c1;
        reg[15] = c2;
        img[HB_PFX_P3 + ix] = byte0(k, reg);
        have3[ix] = 1;
    }
};

static Prefix *prefix_for(const uint8_t *key, size_t keylen) {
    static std::map<std::string, Prefix> cache;
    std::string kk((const char *)key, keylen);
    auto it = cache.find(kk);
    if (it == cache.end()) {
        it = cache.emplace(kk, Prefix()).first;
        it->second.init(key, keylen);
    }
    return &it->second;
}

// pfx != NULL: the first try goes through the prefix image (two-pass
// encode's first pass), later tries resume the stream (retry pass).
template <int NL>
static int prf_eval(const LaneTab &L, const PrfParams<NL> &P, int nr, uint64_t x, uint32_t out[NL],
                    Prefix *pfx = nullptr) {
    uint32_t dig[8], sr[4] = {0, 0, 0, 0};
    hb_sha256_decimal(x, dig);
    for (int tries = 1; tries < 100000; ++tries) {
        uint32_t ok = 0;
        if (tries == 1 && pfx && P.nb >= 4) {
            pfx->need(dig[0]);
            const unsigned char *img = pfx->img.data();
            // as hb_encode_first_kernel: the prefix steps, the early-listing
            // decision (HB_RETRY_DIGEST), then the rest of the try
            hb_prf_prefix<NL>(img, pfx->o0, P, dig[0], sr, out);
            const bool early_reject = out[0] > hb_range_top<NL>(P);
            if (nr == 10) ok = hb_prf_try_from<NL, 10, 1>(L, P, sr, dig, out);
            else if (nr == 12) ok = hb_prf_try_from<NL, 12, 1>(L, P, sr, dig, out);
            else ok = hb_prf_try_from<NL, 14, 1>(L, P, sr, dig, out);
            if (early_reject && ok) return -2;   // the early listing's premise broken
        } else if (nr == 10) ok = hb_prf_try<NL, 10>(L, P, sr, dig, out);
        else if (nr == 12) ok = hb_prf_try<NL, 12>(L, P, sr, dig, out);
        else ok = hb_prf_try<NL, 14>(L, P, sr, dig, out);
        if (ok) return tries;
    }
    return -1;
}

// The prefix kernel's entries: byte 0 of the lane AES of (0, 0, 0,
// hb_pfx_s3(i)) against the host AES, for every P1 / P2 entry and `n3`
// P3 entries spread over the table.  Returns the number of mismatches.
extern "C" int emul_prefix_check(const uint8_t *key, size_t keylen, uint32_t n3, int lane) {
    Prefix ref;
    ref.init(key, keylen);
    AesKey k;
    aes_expand(key, keylen, k);
    LaneTab L = make_tab(lane);
    int bad = 0;
    auto lane_byte = [&](uint32_t i) -> uint8_t {
        uint32_t s3 = hb_pfx_s3(i);
        if (k.nr == 10) return (uint8_t)hb_aes_byte0<10>(L, k.rk, 0, 0, 0, s3);
        if (k.nr == 12) return (uint8_t)hb_aes_byte0<12>(L, k.rk, 0, 0, 0, s3);
        return (uint8_t)hb_aes_byte0<14>(L, k.rk, 0, 0, 0, s3);
    };
    for (uint32_t i = 0; i < HB_PFX_P3; ++i) bad += lane_byte(i) != ref.img[i];
    for (uint32_t t = 0; t < n3; ++t) {
        uint32_t ix = (uint32_t)(((uint64_t)t * 2654435761u) & 0xffffffu);
        uint8_t reg[16] = {0};
        reg[13] = (uint8_t)ix;
        reg[14] = (uint8_t)(ix >> 8);
        reg[15] = (uint8_t)(ix >> 16);
        bad += lane_byte(HB_PFX_P3 + ix) != Prefix::byte0(k, reg);
    }
    return bad;
}

template <int NL>
static int emul_prf_t(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen,
                      uint64_t x, uint8_t *out_be, int lane, int use_prefix) {
    PrfParams<NL> P;
    int nr;
    if (!make_prf<NL>(key, keylen, range_be, rlen, P, nr)) return -1;
    LaneTab L = make_tab(lane);
    uint32_t out[NL];
    int tries = prf_eval<NL>(L, P, nr, x, out, use_prefix ? prefix_for(key, keylen) : nullptr);
    to_be(out, NL, out_be, P.nb);
    return tries;
}

extern "C" int emul_prf(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen,
                        uint64_t x, uint8_t *out_be, int lane, int use_prefix) {
    int bits = bitlen_be(range_be, rlen);
    if (bits <= 64) return emul_prf_t<2>(key, keylen, range_be, rlen, x, out_be, lane, use_prefix);
    if (bits <= 256) return emul_prf_t<8>(key, keylen, range_be, rlen, x, out_be, lane, use_prefix);
    if (bits <= 512) return emul_prf_t<16>(key, keylen, range_be, rlen, x, out_be, lane, use_prefix);
    if (bits <= 1024) return emul_prf_t<32>(key, keylen, range_be, rlen, x, out_be, lane, use_prefix);
    return -2;
}

// The encode's early retry listing (HB_RETRY_DIGEST) over n evals x0..x0+n-1:
// counts[0] first tries rejected, [1] of them decided by the first output
// word alone (listed early), [2] early decisions that the full try
// contradicted (must be 0).
template <int NL>
static int emul_early_t(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen, uint64_t x0,
                        uint64_t n, uint64_t *counts) {
    PrfParams<NL> P;
    int nr;
    if (!make_prf<NL>(key, keylen, range_be, rlen, P, nr) || P.nb < 4) return -1;
    LaneTab L = make_tab(0);
    Prefix *pfx = prefix_for(key, keylen);
    const u32 top = hb_range_top<NL>(P);
    counts[0] = counts[1] = counts[2] = 0;
    for (uint64_t x = x0; x < x0 + n; ++x) {
        uint32_t dig[8], sr[4], out[NL];
        hb_sha256_decimal(x, dig);
        pfx->need(dig[0]);
        hb_prf_prefix<NL>(pfx->img.data(), pfx->o0, P, dig[0], sr, out);
        const bool early = out[0] > top;
        uint32_t ok;
        if (nr == 10) ok = hb_prf_try_from<NL, 10, 1>(L, P, sr, dig, out);
        else if (nr == 12) ok = hb_prf_try_from<NL, 12, 1>(L, P, sr, dig, out);
        else ok = hb_prf_try_from<NL, 14, 1>(L, P, sr, dig, out);
        counts[0] += ok ? 0 : 1;
        counts[1] += early ? 1 : 0;
        counts[2] += early && ok ? 1 : 0;
    }
    return 0;
}

extern "C" int emul_early(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen, uint64_t x0,
                          uint64_t n, uint64_t *counts) {
    int bits = bitlen_be(range_be, rlen);
    if (bits <= 64) return emul_early_t<2>(key, keylen, range_be, rlen, x0, n, counts);
    if (bits <= 256) return emul_early_t<8>(key, keylen, range_be, rlen, x0, n, counts);
    if (bits <= 512) return emul_early_t<16>(key, keylen, range_be, rlen, x0, n, counts);
    if (bits <= 1024) return emul_early_t<32>(key, keylen, range_be, rlen, x0, n, counts);
    return -2;
}

template <int NL>
static int emul_encode_t(const uint8_t *p_be, size_t plen, uint32_t S, const uint8_t *fkey,
                         const uint8_t *akey, size_t keylen, uint64_t block_base,
                         const uint8_t *data, uint64_t len, uint64_t nblocks, uint8_t *tags, int lane,
                         int align, int use_prefix) {
    PrfParams<NL> F, A;
    int nrf, nra;
    if (!make_prf<NL>(fkey, keylen, p_be, plen, F, nrf)) return -1;
    if (!make_prf<NL>(akey, keylen, p_be, plen, A, nra)) return -1;
    LaneTab L = make_tab(lane);
    Limbs p = from_be(p_be, plen, NL);
    ModP<NL> M;
    memset(&M, 0, sizeof M);
    for (int t = 0; t < NL; ++t) M.p[t] = p[t];
    M.pinv = mont_pinv(p[0]);
    M.inv_scaled = inv_scaled(p);
    Limbs r2 = pow2_mod(64u * NL, p);
    std::vector<uint32_t> alpha_mont((size_t)S * NL);
    for (uint32_t j = 0; j < S; ++j) {
        uint32_t a[NL];
        prf_eval<NL>(L, A, nra, j, a);
        hb_to_mont<NL>(a, r2.data(), M, &alpha_mont[(size_t)j * NL]);
    }
    int bits = bitlen_be(p_be, plen);
    uint32_t ss = (uint32_t)bits / 8, tw = (uint32_t)(bits + 7) / 8;
    uint64_t C = (uint64_t)ss * S;
    for (uint64_t b = 0; b < nblocks; ++b) {
        uint32_t f[NL], tag[NL];
        prf_eval<NL>(L, F, nrf, block_base + b, f, use_prefix ? prefix_for(fkey, keylen) : nullptr);
        if (align == 16)
            hb_block_tag<NL, 16>(data, len, b, C, ss, S, alpha_mont.data(), M, f, tag);
        else
            hb_block_tag<NL, 1>(data, len, b, C, ss, S, alpha_mont.data(), M, f, tag);
        hb_store_be<NL>(tags + b * tw, tw, tag);
    }
    return 0;
}

extern "C" int emul_encode(const uint8_t *p_be, size_t plen, uint32_t S, const uint8_t *fkey,
                           const uint8_t *akey, size_t keylen, uint64_t block_base,
                           const uint8_t *data, uint64_t len, uint64_t nblocks, uint8_t *tags,
                           int lane, int align, int use_prefix) {
    int bits = bitlen_be(p_be, plen);
    if (bits <= 256) return emul_encode_t<8>(p_be, plen, S, fkey, akey, keylen, block_base, data, len, nblocks, tags, lane, align, use_prefix);
    if (bits <= 512) return emul_encode_t<16>(p_be, plen, S, fkey, akey, keylen, block_base, data, len, nblocks, tags, lane, align, use_prefix);
    if (bits <= 1024) return emul_encode_t<32>(p_be, plen, S, fkey, akey, keylen, block_base, data, len, nblocks, tags, lane, align, use_prefix);
    return -2;
}

// ------------------------------------------------------------------ cxx prf
// One lane's cxx prf::evaluate (hb_cxx_try + SHA256(LE32)), as hb_engine<MODE 1>
// runs it -- or hb_cxx_try_bytes (MODE 2) when ByteCount(limit) % 16 != 0:
// tries until accepted or HB_CXX_MAX_TRIES.
template <int NL>
static int cxx_prf_eval(const LaneTab &L, const PrfParams<NL> &P, int nr, uint32_t x, uint32_t out[NL]) {
    uint32_t dig[8], sr[4] = {0, 0, 0, 0};
    hb_sha256_le32(x, dig);
    for (uint32_t k = 1;; ++k) {
        uint32_t ok;
        if (P.nb % 16)
            ok = nr == 14 ? hb_cxx_try_bytes<NL, 14>(L, P, sr, dig, out, k - 1)
               : nr == 12 ? hb_cxx_try_bytes<NL, 12>(L, P, sr, dig, out, k - 1)
                          : hb_cxx_try_bytes<NL, 10>(L, P, sr, dig, out, k - 1);
        else
            ok = nr == 14 ? hb_cxx_try<NL, 14>(L, P, sr, dig, out)
               : nr == 12 ? hb_cxx_try<NL, 12>(L, P, sr, dig, out)
                          : hb_cxx_try<NL, 10>(L, P, sr, dig, out);
        if (ok || k >= HB_CXX_MAX_TRIES) return (int)k;
    }
}

template <int NL>
static int emul_cxx_prf_t(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen,
                          uint32_t x, uint8_t *out_be, int lane) {
    PrfParams<NL> P;
    int nr;
    if (!make_prf<NL>(key, keylen, range_be, rlen, P, nr)) return -1;
    LaneTab L = make_tab(lane);
    uint32_t out[NL];
    int tries = cxx_prf_eval<NL>(L, P, nr, x, out);
    to_be(out, NL, out_be, P.nb);
    return tries;
}

extern "C" int emul_cxx_prf(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen,
                            uint32_t x, uint8_t *out_be, int lane) {
    int bits = bitlen_be(range_be, rlen);
    if (bits <= 256) return emul_cxx_prf_t<8>(key, keylen, range_be, rlen, x, out_be, lane);
    if (bits <= 512) return emul_cxx_prf_t<16>(key, keylen, range_be, rlen, x, out_be, lane);
    if (bits <= 1024) return emul_cxx_prf_t<32>(key, keylen, range_be, rlen, x, out_be, lane);
    return -2;
}

// ------------------------------------------------------------------ Merkle chunks
// One lane of hb_merkle_offsets_kernel + hb_hmac_kernel: the seed's own key
// schedule (hb_aes_expand_lane), KeyedPRF(seed, filesz - chunk + 1).eval(0),
// then HMAC-SHA256(seed, data[off .. off + chunk)).  Returns the PRF tries.
template <int NR>
static int merkle_lane(const uint8_t *seed, size_t seed_len, const uint8_t *data, uint64_t len, uint64_t filesz,
                       uint64_t chunksz, int lane, uint64_t *off_out, uint8_t *digest) {
    LaneTab L = make_tab(lane);
    if (filesz < chunksz) chunksz = filesz;
    const uint64_t range = filesz - chunksz + 1;
    constexpr int NK = NR - 6;
    uint32_t key[NK];
    for (int t = 0; t < NK; ++t)
        key[t] = (uint32_t)seed[4 * t] | ((uint32_t)seed[4 * t + 1] << 8) | ((uint32_t)seed[4 * t + 2] << 16) |
                 ((uint32_t)seed[4 * t + 3] << 24);
    PrfParams<2> P;
    memset(&P, 0, sizeof P);
    hb_aes_expand_lane<NR>(L, key, P.rk);
    P.R[0] = (uint32_t)range;
    P.R[1] = (uint32_t)(range >> 32);
    int bits = 0;
    for (uint64_t r = range; r; r >>= 1) ++bits;
    P.nb = (uint32_t)(bits + 7) / 8;
    P.topmask = (1u << (bits - 8 * ((int)P.nb - 1))) - 1u;
    uint32_t dig[8], sr[4] = {0, 0, 0, 0}, out[2] = {0, 0};
    hb_sha256_decimal(0, dig);
    int tries = 0;
    uint32_t ok = 0;
    while (!ok && tries < 100000) {
        ok = hb_prf_try<2, NR>(L, P, sr, dig, out);
        ++tries;
    }
    const uint64_t off = (uint64_t)out[0] | ((uint64_t)out[1] << 32);
    *off_out = off;
    uint32_t kw[16];
    for (int t = 0; t < 16; ++t) {
        uint32_t w = 0;
        for (int k = 0; k < 4; ++k) w = (w << 8) | ((size_t)(4 * t + k) < seed_len ? seed[4 * t + k] : 0u);
        kw[t] = w;
    }
    uint32_t d[8];
    hb_hmac_sha256(kw, data, len, off, chunksz, d);
    for (int t = 0; t < 8; ++t)
        for (int b = 0; b < 4; ++b) digest[4 * t + b] = (uint8_t)(d[t] >> (24 - 8 * b));
    return tries;
}

extern "C" int emul_merkle(const uint8_t *seed, size_t seed_len, const uint8_t *data, uint64_t len, uint64_t filesz,
                           uint64_t chunksz, int lane, uint64_t *off_out, uint8_t *digest) {
    if (seed_len == 16) return merkle_lane<10>(seed, seed_len, data, len, filesz, chunksz, lane, off_out, digest);
    if (seed_len == 24) return merkle_lane<12>(seed, seed_len, data, len, filesz, chunksz, lane, off_out, digest);
    if (seed_len == 32) return merkle_lane<14>(seed, seed_len, data, len, filesz, chunksz, lane, off_out, digest);
    return -1;
}
