"""The arithmetic of the split wide-prime MAC (hb_args.hpp WtabArgs / WmacArgs,
hb_wide.hpp, hb_runtime.cpp wide_plan) restated in Python and checked against
the direct sum_j alpha_j m_j mod p (PySwizzle.py:297-307) on the CPU: the
signed digit table, the int8 column sums the MFMA forms, kz, the shift w and
the final reduction's input range.  The device layout (fragments, lane
transposes) is covered by the GPU parity tests."""
import random

import pytest


def plan(bits, tw, C):
    """wide_plan: w, or None when the split MAC does not apply."""
    if C == 0 or C % 16 or C > 32768:
        return None
    lc = (C - 1).bit_length()
    w = lc + 8 * tw + 7 - bits
    return w if 0 <= w <= 29 else None


def digits(r, D):
    """D balanced base-256 digits of r (two's complement below 0) and the carry out."""
    m = r % (1 << (8 * D + 8))
    out, carry = [], 0
    for i in range(D):
        v = ((m >> (8 * i)) & 0xff) + carry
        carry = 1 if v >= 128 else 0
        out.append(v - 256 * carry)
    return out, carry


def wide_tag(p, S, alphas, block, F):
    bits = p.bit_length()
    ss, tw = bits // 8, (bits + 7) // 8
    C = ss * S
    w = plan(bits, tw, C)
    assert w is not None
    half = int.from_bytes(b"\x7f" * tw, "big")
    cols = [0] * tw
    sum_r = 0
    for x in range(C):
        j, k = divmod(x, ss)
        r = alphas[j] * pow(256, ss - 1 - k, p) % p
        sum_r += r
        rr = r - p if r > half else r
        d, carry = digits(rr, tw)
        assert carry == (1 if rr < 0 else 0)          # hb_wtab_kernel's status check
        assert sum(di * 256 ** i for i, di in enumerate(d)) == rr
        u = block[x]
        for c in range(tw):
            cols[c] += d[c] * (u - 128)
    assert all(abs(c) < 2 ** 31 for c in cols)          # int32 MFMA accumulators
    G = sum(pow(256, e, p) for e in range(ss)) % p
    kz = (sum(alphas) * 128 * G) % p + (p << w)
    assert kz == (128 * sum_r) % p + (p << w)
    T = sum(c * 256 ** i for i, c in enumerate(cols)) + kz
    nl = 16 if bits <= 512 else 32 if bits <= 1024 else 64
    assert 0 < T < 3 * p << w and T < 2 ** (32 * (nl + 1))
    assert T + F < (p << 32)                             # hb_reduce_small's range
    return (T + F) % p


def _prime(bits, seed):
    import importlib
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(seed)
    while True:
        p = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(p):
            return p


@pytest.mark.parametrize("bits,S", [(1024, 10), (512, 16), (1020, 16), (384, 4), (1000, 32)])
def test_wide_mac_equals_direct_sum(bits, S):
    p = _prime(bits, bits * 7 + S)
    ss = bits // 8
    C = ss * S
    if plan(bits, (bits + 7) // 8, C) is None:
        pytest.skip("C % 16 != 0: the split MAC does not apply (in-kernel MAC)")
    rng = random.Random(S)
    alphas = [rng.randrange(p) for _ in range(S)]
    for trial in range(3):
        if trial == 0:
            block = bytes([255] * C)                     # extreme bytes
        elif trial == 1:
            block = bytes(C)
        else:
            block = bytes(rng.randrange(256) for _ in range(C))
        F = rng.randrange(p)
        want = (F + sum(a * int.from_bytes(block[j * ss:(j + 1) * ss], "big") for j, a in enumerate(alphas))) % p
        assert wide_tag(p, S, alphas, block, F) == want


def test_plan_limits():
    assert plan(1024, 128, 1280) == 18
    assert plan(2048, 256, 2560) == 19
    assert plan(1017, 128, 127 * 16) is not None
    assert plan(1024, 128, 32768 + 16) is None           # int32 column sums
    assert plan(1024, 128, 1288) is None                 # C % 16 != 0
