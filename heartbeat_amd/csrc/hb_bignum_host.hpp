// hb_bignum_host.hpp -- the few host-side multiprecision helpers the runtime
// needs to set up a modulus for the kernels (little-endian u32 limbs).
//   * parse / print big-endian byte strings
//   * 2^k mod p by doubling (R mod p, R^2 mod p for Montgomery conversion)
//   * -p^-1 mod 2^32 (Montgomery constant) and the scaled 1/p estimate
// Nothing here runs per block; all per-block arithmetic is on the GPU.
#pragma once
#include <stdint.h>
#include <stddef.h>
#include <vector>

namespace hbhost {

typedef std::vector<uint32_t> Limbs;

inline Limbs from_be(const uint8_t *be, size_t n, size_t nl) {
    Limbs r(nl, 0);
    for (size_t k = 0; k < n; ++k) {
        size_t pos = n - 1 - k;   // byte index from the least significant end
        if (pos / 4 < nl) r[pos / 4] |= (uint32_t)be[k] << (8 * (pos % 4));
    }
    return r;
}

inline void to_be(const uint32_t *v, size_t nl, uint8_t *be, size_t n) {
    for (size_t k = 0; k < n; ++k) {
        size_t pos = n - 1 - k;
        be[k] = pos / 4 < nl ? (uint8_t)(v[pos / 4] >> (8 * (pos % 4))) : 0;
    }
}

inline int bitlen_be(const uint8_t *be, size_t n) {
    for (size_t k = 0; k < n; ++k)
        if (be[k]) {
            int b = 8;
            while (!(be[k] & (1u << (b - 1)))) --b;
            return (int)(8 * (n - 1 - k)) + b;
        }
    return 0;
}

inline int cmp(const Limbs &a, const Limbs &b) {
    for (size_t t = a.size(); t-- > 0;) {
        if (a[t] != b[t]) return a[t] < b[t] ? -1 : 1;
    }
    return 0;
}

inline void sub_in_place(Limbs &a, const Limbs &b) {
    uint64_t borrow = 0;
    for (size_t t = 0; t < a.size(); ++t) {
        uint64_t d = (uint64_t)a[t] - b[t] - borrow;
        a[t] = (uint32_t)d;
        borrow = (d >> 63) & 1;
    }
}

// 2^k mod p; p (nl limbs) > 1.
inline Limbs pow2_mod(unsigned k, const Limbs &p) {
    size_t nl = p.size();
    Limbs x(nl + 1, 0), pp(p);
    pp.push_back(0);
    x[0] = 1;
    if (cmp(x, pp) >= 0) sub_in_place(x, pp);
    for (unsigned i = 0; i < k; ++i) {
        uint32_t carry = 0;
        for (size_t t = 0; t <= nl; ++t) {
            uint32_t nc = x[t] >> 31;
            x[t] = (x[t] << 1) | carry;
            carry = nc;
        }
        if (cmp(x, pp) >= 0) sub_in_place(x, pp);
    }
    x.resize(nl);
    return x;
}

// (a + b) mod p for a, b < p (p.size() limbs).
inline Limbs add_mod(const Limbs &a, const Limbs &b, const Limbs &p) {
    size_t nl = p.size();
    Limbs x(nl + 1, 0), pp(p);
    pp.push_back(0);
    uint64_t c = 0;
    for (size_t t = 0; t < nl; ++t) {
        c += (uint64_t)a[t] + b[t];
        x[t] = (uint32_t)c;
        c >>= 32;
    }
    x[nl] = (uint32_t)c;
    if (cmp(x, pp) >= 0) sub_in_place(x, pp);
    x.resize(nl);
    return x;
}

// x mod p for any limb vector x (bitwise long division).
inline Limbs mod_any(const Limbs &x, const Limbs &p) {
    size_t nl = p.size();
    Limbs r(nl, 0);
    for (size_t t = x.size(); t-- > 0;)
        for (int b = 31; b >= 0; --b) {
            r = add_mod(r, r, p);                       // r = 2r mod p
            if ((x[t] >> b) & 1u) {
                Limbs one(nl, 0);
                one[0] = 1;
                r = add_mod(r, one, p);
            }
        }
    return r;
}

// a * b mod p (a, b < p), shift-and-add.
inline Limbs mul_mod(const Limbs &a, const Limbs &b, const Limbs &p) {
    size_t nl = p.size();
    Limbs r(nl, 0);
    for (size_t t = nl; t-- > 0;)
        for (int k = 31; k >= 0; --k) {
            r = add_mod(r, r, p);
            if ((b[t] >> k) & 1u) r = add_mod(r, a, p);
        }
    return r;
}

// -p^-1 mod 2^32 (p odd), Newton iteration.
inline uint32_t mont_pinv(uint32_t p0) {
    uint32_t inv = 1;
    for (int i = 0; i < 5; ++i) inv *= 2u - p0 * inv;
    return (uint32_t)(0u - inv);
}

// 2^(32 (nl-2)) / p as a double (matches the device-side scaling).
inline double inv_scaled(const Limbs &p) {
    int nl = (int)p.size();
    double pd = 0.0;
    for (int t = nl - 1; t >= 0; --t) {
        double s = 1.0;
        int e = t - (nl - 2);
        if (e < -31) continue;   // dropped as on the device (HbScale)
        for (int i = 0; i < (e >= 0 ? e : -e); ++i) s *= 4294967296.0;
        pd += (double)p[t] * (e >= 0 ? s : 1.0 / s);
    }
    return 1.0 / pd;
}

}  // namespace hbhost
