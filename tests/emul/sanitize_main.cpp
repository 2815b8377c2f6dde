// sanitize_main.cpp -- ASan/UBSan run of the CPU builds (sanitizers
// on host code).  Built by tests/test_sanitize.py as ONE executable from
// tests/emul/emul.cpp (the kernels' per-lane code, hb_lane.hpp, as plain C++)
// and oracle/swizzle_oracle.c, both under -fsanitize=address,undefined with
// recovery off: any out-of-bounds access, use-after-free, leak or undefined
// shift/overflow aborts the run.  The two implementations are also compared on
// every input (emul lane == oracle), so a sanitizer-clean run is a parity run.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
int emul_prf(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen, uint64_t x,
             uint8_t *out_be, int lane, int use_prefix);
int emul_encode(const uint8_t *p_be, size_t plen, uint32_t S, const uint8_t *fkey, const uint8_t *akey,
                size_t keylen, uint64_t block_base, const uint8_t *data, uint64_t len, uint64_t nblocks,
                uint8_t *tags, int lane, int align, int use_prefix);
int emul_cxx_prf(const uint8_t *key, size_t keylen, const uint8_t *range_be, size_t rlen, uint32_t x,
                 uint8_t *out_be, int lane);
int hbo_prf_eval(const unsigned char *key, size_t keylen, const unsigned char *range_be, size_t range_len,
                 uint64_t x, unsigned char *out_be, size_t out_len);
int hbo_cxx_prf_eval(const unsigned char *key, size_t keylen, const unsigned char *range_be,
                     size_t range_len, uint32_t x, unsigned char *out_be, size_t out_len);
int hbo_encode(const unsigned char *p_be, size_t p_len, uint32_t sectors, const unsigned char *f_key,
               const unsigned char *a_key, size_t keylen, uint64_t block_base, const unsigned char *data,
               uint64_t len, uint64_t nblocks, unsigned char *tags_out, int nthreads);
}

static uint64_t g_state = 0x243f6a8885a308d3ull;
static uint64_t rnd() {   // SplitMix64
    uint64_t z = (g_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static std::vector<uint8_t> hex(const char *h) {
    std::vector<uint8_t> v;
    for (size_t i = 0; h[i] && h[i + 1]; i += 2) {
        unsigned b;
        sscanf(h + i, "%2x", &b);
        v.push_back((uint8_t)b);
    }
    return v;
}

static int fails = 0;
#define CHECK(c, ...)                         \
    do {                                      \
        if (!(c)) {                           \
            fprintf(stderr, __VA_ARGS__);     \
            fputc('\n', stderr);              \
            ++fails;                          \
        }                                     \
    } while (0)

int main() {
    // moduli: 2^61-1, the bench 256-bit prime, 2^255-19 (unaligned sectors)
    // and a 960-bit odd modulus (NL = 32, unaligned 120-byte sectors)
    const char *primes[] = {
        "1fffffffffffffff",
        "db8709c32591ddc589b5c3c0986f92e0d11205b943c23a7e419e6c35b0256e6b",
        "7fffffffffffffffffffffffffffffffffffffffffffffffffffffffffffffed",
        "c90fdaa22168c234c4c6628b80dc1cd129024e088a67cc74020bbea63b139b22514a08798e3404ddef9519b3cd3a431b"
        "302b0a6df25f14374fe1356d6d51c245e485b576625e7ec6f44c42e9a637ed6b0bff5cb6f406b7edee386bfb5a899fa5"
        "ae9f24117c4b1fe649286651ece65381ffffffffffffffff",
    };
    for (const char *ph : primes) {
        std::vector<uint8_t> p = hex(ph);
        for (int keylen : {16, 24, 32}) {
            uint8_t key[32];
            for (int i = 0; i < keylen; ++i) key[i] = (uint8_t)rnd();
            for (int k = 0; k < 24; ++k) {
                uint64_t x = k < 8 ? (uint64_t)k : k < 16 ? rnd() >> (k * 3) : rnd();
                uint8_t a[128] = {0}, b[128] = {0};
                int ta = emul_prf(key, keylen, p.data(), p.size(), x, a, k % 64, k & 1);
                int tb = hbo_prf_eval(key, keylen, p.data(), p.size(), x, b, p.size());
                CHECK(ta >= 1 && tb >= 1 && memcmp(a, b, p.size()) == 0, "prf mismatch p=%.16s keylen=%d x=%llu",
                      ph, keylen, (unsigned long long)x);
                uint8_t c[128] = {0}, d[128] = {0};
                if (p.size() >= 16) {
                    const uint32_t xi = (uint32_t)x;
                    int tc = emul_cxx_prf(key, keylen, p.data(), p.size(), xi, c, k % 64);
                    int td = hbo_cxx_prf_eval(key, keylen, p.data(), p.size(), xi, d, p.size());
                    CHECK(tc == td && memcmp(c, d, p.size()) == 0, "cxx prf mismatch p=%.16s x=%u", ph, xi);
                }
            }
        }
        // encode: lengths around block boundaries, with a tail sector
        const int bits = (int)(p.size() * 8) - __builtin_clz((unsigned)p[0]) + 24;
        const uint32_t ss = (uint32_t)bits / 8, tw = (uint32_t)(bits + 7) / 8;
        for (uint32_t S : {1u, 3u, 16u}) {
            const uint64_t C = (uint64_t)ss * S;
            for (uint64_t len : {(uint64_t)0, (uint64_t)1, C - 1, C, C + 1, 3 * C + 17}) {
                std::vector<uint8_t> data(len);
                for (auto &x : data) x = (uint8_t)rnd();
                const uint64_t nt = len / C + 1;
                std::vector<uint8_t> ta(nt * tw), tb(nt * tw);
                uint8_t fk[32], ak[32];
                for (int i = 0; i < 32; ++i) { fk[i] = (uint8_t)rnd(); ak[i] = (uint8_t)rnd(); }
                const uint32_t nl = bits <= 256 ? 8u : bits <= 512 ? 16u : 32u;
                const int align = ss == 4 * nl ? 16 : 1;   // full-width sectors (emul_encode's NL)
                int ra = emul_encode(p.data(), p.size(), S, fk, ak, 32, 5, data.data(), len, nt, ta.data(),
                                     (int)(len % 64), align, (int)(len & 1));
                int rb = hbo_encode(p.data(), p.size(), S, fk, ak, 32, 5, data.data(), len, nt, tb.data(), 1);
                CHECK(ra == 0 && rb == 0 && ta == tb, "encode mismatch p=%.16s S=%u len=%llu align=%d", ph, S,
                      (unsigned long long)len, align);
            }
        }
    }
    printf("sanitize: %d failures\n", fails);
    return fails ? 1 : 0;
}
