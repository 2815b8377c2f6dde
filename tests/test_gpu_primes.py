"""Every limb-count instantiation against the oracle (round 5): primes of
129 to 2048 bits -- including the 257-512-bit range (NL = 16 kernels), which
no golden vector exercises, and the edges of each limb count (256/257,
512/513, 1024/1025, 2047/2048 bits) -- with 1, 3 and 7 sectors per block on
ragged files (a short last sector), encoded from host memory through the
drop-in API and from device memory through the C ABI, then proved
(10 challenged blocks + a 37-index challenge) and verified.  Primes are
drawn from a seeded generator (Miller-Rabin, heartbeat_amd's getPrime test),
so the cases are reproducible.  The oracle (oracle/swizzle_oracle.c, OpenSSL
BIGNUM, any size) is pinned by the reference's golden vectors for 20- to
2048-bit primes.  Bar: bit-exact.  Reference: PySwizzle.py:279-395,
util.py:44-96."""
import ctypes
import hashlib
import importlib
import io
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BITS = [129, 200, 256, 257, 384, 511, 512, 513, 768, 1000, 1024, 1025, 1536, 2047, 2048]


def seeded_prime(bits, seed):
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    rng = random.Random(seed)
    while True:
        x = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
        if pys._is_probable_prime(x):
            return x


@pytest.mark.parametrize("bits", BITS)
def test_prime_sizes_encode_prove_verify(oracle, bits):
    from heartbeat_amd import _native as nat
    from heartbeat_amd.PySwizzle import Challenge
    pys = importlib.import_module("heartbeat_amd.PySwizzle.PySwizzle")
    ctx = nat.context()
    L = nat.lib()
    p = seeded_prime(bits, 1000 + bits)
    w = nat.width_of(p)
    ss = bits // 8
    pb = nat.be(p)
    rng = np.random.default_rng(bits)
    for S in (1, 3, 7):
        C = ss * S
        n = 40 * C + ss // 2 + 1                    # 40 whole blocks + a short sector
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fk = hashlib.sha256(b"pf%d-%d" % (bits, S)).digest()
        ak = hashlib.sha256(b"pa%d-%d" % (bits, S)).digest()
        want = oracle.encode(p, S, fk, ak, data, nthreads=8)
        nb = len(want)
        # host memory through the drop-in API
        tag, n2 = pys.encode_file(p, S, fk, ak, io.BytesIO(data))
        assert n2 == nb and tag.sigma == want, (bits, S, "host")
        # device memory through the C ABI
        d, t = ctypes.c_void_p(), ctypes.c_void_p()
        ctx.check(L.hb_device_malloc(ctx.h, n, ctypes.byref(d)))
        ctx.check(L.hb_device_malloc(ctx.h, nb * w, ctypes.byref(t)))
        try:
            hd = np.frombuffer(data, dtype=np.uint8)
            ctx.check(L.hb_memcpy(ctx.h, d, hd.ctypes.data, n, 1))
            ctx.check(L.hb_encode(ctx.h, pb, len(pb), S, fk, ak, 32, 0, d, n, nb, t, 3, None))
            got = np.empty(nb * w, dtype=np.uint8)
            ctx.check(L.hb_memcpy(ctx.h, got.ctypes.data, t.value, nb * w, 2))
            assert [int.from_bytes(got[i * w:(i + 1) * w].tobytes(), "big") for i in range(nb)] == want, \
                (bits, S, "device")
            for chunks in (10, 37):
                key = hashlib.sha256(b"pc%d-%d-%d" % (bits, S, chunks)).digest()
                mu = ctypes.create_string_buffer(w * S)
                sg = ctypes.create_string_buffer(w)
                ctx.check(L.hb_prove(ctx.h, pb, len(pb), S, key, 32, chunks, pb, len(pb), t, nb, d, n, 3, mu, sg))
                gmu = [int.from_bytes(mu.raw[j * w:(j + 1) * w], "big") for j in range(S)]
                gsg = int.from_bytes(sg.raw, "big")
                omu, osg = oracle.prove(p, S, key, chunks, p, want, data)
                assert (gmu, gsg) == (omu, osg), (bits, S, chunks)
                # the same challenge through the drop-in API from host memory
                beat = pys.PySwizzle(S, b"k" * 32, p)
                proof = beat.prove(io.BytesIO(data), Challenge(chunks, p, key), tag)
                assert (proof.mu, proof.sigma) == (omu, osg)
                rhs = ctypes.create_string_buffer(w)
                ctx.check(L.hb_verify_rhs(ctx.h, pb, len(pb), S, fk, ak, 32, nb, key, 32, chunks, pb, len(pb),
                                          mu.raw, rhs))
                assert int.from_bytes(rhs.raw, "big") == gsg, (bits, S, chunks, "verify")
                assert oracle.verify(p, S, fk, ak, nb, key, chunks, p, omu, osg)
        finally:
            ctx.check(L.hb_device_free(ctx.h, d))
            ctx.check(L.hb_device_free(ctx.h, t))


@pytest.mark.parametrize("bits", [9, 33, 64, 65, 300, 700, 1500, 2048])
def test_keyedprf_ranges_vs_oracle(oracle, bits):
    """KeyedPRF (util.py:83-96) on the GPU for ranges of 9 to 2048 bits (the
    reference KATs stop at 300 bits): 512 inputs each, == the oracle."""
    from heartbeat_amd.PySwizzle import KeyedPRF
    rng = random.Random(bits)
    R = rng.getrandbits(bits) | (1 << (bits - 1))
    key = hashlib.sha256(b"kr%d" % bits).digest()
    xs = list(range(256)) + [rng.getrandbits(63) for _ in range(256)]
    assert KeyedPRF(key, R).eval_many(xs) == [oracle.prf_eval(key, R, x) for x in xs]
